"""Summarise a rocprofv3 --pmc CSV (tools/gpu_pmc_valu.sh) per kernel: VALU busy fraction
(SQ_ACTIVE_INST_VALU quad-cycles / CUs / GRBM_GUI_ACTIVE per XCD), VALU instructions, effective
clock, LDS instructions and bank-conflict cycles.  Writes valu_<config>.json next to the CSV."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d, config = sys.argv[1], sys.argv[2]
batch = int(sys.argv[3]) if len(sys.argv) > 3 else None
f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
acc = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> [per-dispatch values]
disp = defaultdict(lambda: defaultdict(float))
dur = {}
for row in csv.DictReader(open(f)):
    k = row["Kernel_Name"].split("(")[0]
    key = (k, row["Dispatch_Id"])
    disp[key][row["Counter_Name"]] += float(row["Counter_Value"])
    if "End_Timestamp" in row and row.get("Start_Timestamp"):
        dur[key] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
for (k, _), c in disp.items():
    for n, v in c.items():
        acc[k][n].append(v)
N_CU, N_XCD = 256, 8
out = {}
print(f"# VALU issue per kernel, config {config} (rocprofv3 --pmc, mean over dispatches)\n")
print("| kernel | dispatches | SQ_INSTS_VALU | VALU busy | eff. clock GHz | SQ_INSTS_LDS | LDS bank-conflict cycles | SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES |")
print("|---|---|---|---|---|---|---|---|")
for k, c in sorted(acc.items()):
    m = {n: sum(v) / len(v) for n, v in c.items()}
    gui = m.get("GRBM_GUI_ACTIVE", 0.0) / N_XCD            # per-XCD busy cycles (summed over the 8 XCDs)
    busy = 4.0 * m.get("SQ_ACTIVE_INST_VALU", 0.0) / (4 * N_CU) / gui if gui else 0.0
    ds = [v for (kk, _), v in dur.items() if kk == k]
    clk = gui / (sum(ds) / len(ds)) / 1e9 if ds else 0.0
    wait = m.get("SQ_WAIT_INST_ANY", 0) / m["SQ_WAVE_CYCLES"] if m.get("SQ_WAVE_CYCLES") else 0.0
    out[k] = {"valu_insts": m.get("SQ_INSTS_VALU"), "valu_busy": busy, "eff_clock_ghz": clk,
              "lds_insts": m.get("SQ_INSTS_LDS"), "lds_bank_conflict": m.get("SQ_LDS_BANK_CONFLICT"),
              "wait_inst_frac": wait, "dispatches": len(c["SQ_INSTS_VALU"])}
    print(f"| `{k}` | {len(c['SQ_INSTS_VALU'])} | {m.get('SQ_INSTS_VALU', 0):.4g} | {busy:.3f} | {clk:.2f} | "
          f"{m.get('SQ_INSTS_LDS', 0):.4g} | {m.get('SQ_LDS_BANK_CONFLICT', 0):.4g} | {wait:.3f} |")
out["batch"] = batch
json.dump(out, open(os.path.join(d, f"valu_{config}.json"), "w"), indent=1)
