"""Mean per-dispatch counter values for one kernel from a rocprofv3 --pmc CSV directory."""
import csv, glob, os, sys
from collections import defaultdict
d, kern = sys.argv[1], sys.argv[2]
f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
disp = defaultdict(lambda: defaultdict(float))
for row in csv.DictReader(open(f)):
    if row["Kernel_Name"].split("(")[0] == kern:
        disp[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
n = len(disp)
tot = defaultdict(float)
for c in disp.values():
    for k, v in c.items():
        tot[k] += v / n
print(f"{kern}: {n} dispatches")
for k in sorted(tot):
    print(f"  {k:24s} {tot[k]:.4g}")
if tot.get("SQ_WAVE_CYCLES"):
    w = tot["SQ_WAVE_CYCLES"]
    print("  wait_any/wave %.3f  wait_inst/wave %.3f  valu_active/wave %.3f  icache miss/req %.4f" % (
        tot.get("SQ_WAIT_ANY", 0) / w, tot.get("SQ_WAIT_INST_ANY", 0) / w, 4 * tot.get("SQ_ACTIVE_INST_VALU", 0) / w,
        tot.get("SQC_ICACHE_MISSES", 0) / max(1, tot.get("SQC_ICACHE_REQ", 1))))
