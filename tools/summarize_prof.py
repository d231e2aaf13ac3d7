"""Summarise a rocprofv3 session (kernel stats + FETCH_SIZE / WRITE_SIZE passes) into
profiles/: a markdown summary and traffic_<config>.json consumed by bench.py.

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are KiB of
memory-side requests; the guide calibrates them only for 16 B/lane streams ("other access
widths are uncalibrated: calibrate on a known byte count"), and the pipeline kernels move
data 4 B per lane.  So both counters are scaled by the factors measured on k_diag_stream,
which reads and then writes exactly 1 GiB at 4 B per lane (tools/pmc_calibrate.py).
"""
import collections
import csv
import json
import os
import sys

KMAP = {"k_encode": "encode_rm_scramble", "k_modofdm": "modulate_idft_cp", "k_fep": "k_fep<11>", "k_td16": "k_td16",
        "k_chest": "k_chest", "k_rx_llr": "k_rx_llr", "k_rx_level": "k_rx_level"}


def short(name):
    for k, v in KMAP.items():
        if name.startswith(k) or name.startswith("void " + k):
            return v
    return None


def calibration(prof_dir, tag):
    """bytes per counted KiB for FETCH_SIZE and WRITE_SIZE at 4 B/lane (k_diag_stream)."""
    out = {}
    for sub, ctr, mode in (("calfetch", "FETCH_SIZE", 0), ("calwrite", "WRITE_SIZE", 1)):
        rows = [r for r in csv.DictReader(open(os.path.join(prof_dir, f"{sub}_{tag}", "run_counter_collection.csv")))
                if "k_diag_stream" in r["Kernel_Name"] and r["Counter_Name"] == ctr]
        kib = float(rows[mode]["Counter_Value"])       # dispatch 0 = read pass, 1 = write pass
        out[ctr] = (1 << 30) / (kib * 1024.0)
    return out


def main(prof_dir, tag, config, out_dir):
    stats = list(csv.DictReader(open(os.path.join(prof_dir, f"trace_{tag}", "run_kernel_stats.csv"))))
    cal = calibration(prof_dir, tag)
    pmc = collections.defaultdict(list)
    res = {}
    # only the batch launches count: bench.py also times smaller side runs (C5's 2048-subframe rate, on
    # the k_td16 build the per-size dispatch picks below 98304 blocks), so per key keep the largest grid
    grid = collections.defaultdict(int)
    for sub in ("fetch", "write"):
        for r in csv.DictReader(open(os.path.join(prof_dir, f"{sub}_{tag}", "run_counter_collection.csv"))):
            k = short(r["Kernel_Name"])
            if k:
                grid[k] = max(grid[k], int(r["Grid_Size"]))
    for sub, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        for r in csv.DictReader(open(os.path.join(prof_dir, f"{sub}_{tag}", "run_counter_collection.csv"))):
            k = short(r["Kernel_Name"])
            if k and int(r["Grid_Size"]) == grid[k]:
                res[k] = dict(res.get(k, {}), kernel=r["Kernel_Name"].split("(")[0])
                pmc[(k, ctr)].append(float(r["Counter_Value"]))
                res[k].update({x: r[x] for x in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size",
                                            "VGPR_Count", "SGPR_Count")})
    traffic = {}
    lines = [f"# rocprofv3 summary {tag} — config {config}", "",
             "Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline`"
             f" (+ separate `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes)", "",
             "| kernel | calls | avg µs | min µs | max µs | % |", "|---|---|---|---|---|---|"]
    for s in stats:
        lines.append(f"| `{s['Name'][:70]}` | {s['Calls']} | {float(s['AverageNs'])/1e3:.1f} | "
                     f"{float(s['MinNs'])/1e3:.1f} | {float(s['MaxNs'])/1e3:.1f} | {float(s['Percentage']):.1f} |")
    lines += ["", f"Calibration (k_diag_stream, 1 GiB at 4 B/lane): {cal['FETCH_SIZE']:.3f} B per FETCH_SIZE byte, "
              f"{cal['WRITE_SIZE']:.3f} B per WRITE_SIZE byte.", "",
              "| kernel | FETCH_SIZE KiB/launch | WRITE_SIZE KiB/launch | HBM bytes/launch (calibrated) | resources |",
              "|---|---|---|---|---|"]
    for k in sorted({k for k, _ in pmc}):
        f = sum(pmc[(k, "FETCH_SIZE")]) / max(1, len(pmc[(k, "FETCH_SIZE")]))
        w = sum(pmc[(k, "WRITE_SIZE")]) / max(1, len(pmc[(k, "WRITE_SIZE")]))
        b = (f * cal["FETCH_SIZE"] + w * cal["WRITE_SIZE"]) * 1024
        traffic[k] = b
        lines.append(f"| {k} | {f:.0f} | {w:.0f} | {b/1e6:.1f} MB | {res.get(k)} |")
    # per-dispatch durations from the kernel trace: the median over the launches of each kernel is
    # what bench.py reports beside its HIP-event time (roofline.profiler_ms)
    kt = os.path.join(prof_dir, f"trace_{tag}", "run_kernel_trace.csv")
    prof_ms = {}
    if os.path.exists(kt):
        durs = collections.defaultdict(list)
        for r in csv.DictReader(open(kt)):
            k = short(r["Kernel_Name"])
            if k and (k not in grid or int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) == grid[k]):
                durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        lines += ["", "Per-dispatch durations (kernel trace; batch-size launches only):", "",
                  "| kernel | dispatches | median ms | mean ms | min ms |", "|---|---|---|---|---|"]
        for k, v in sorted(durs.items()):
            v = sorted(v)
            med = v[len(v) // 2] if len(v) % 2 else 0.5 * (v[len(v) // 2 - 1] + v[len(v) // 2])
            prof_ms[k] = med
            lines.append(f"| {k} | {len(v)} | {med:.4f} | {sum(v) / len(v):.4f} | {v[0]:.4f} |")
    os.makedirs(out_dir, exist_ok=True)
    open(os.path.join(out_dir, f"rocprof_{tag}_{config}.md"), "w").write("\n".join(lines) + "\n")
    traffic["batch"] = int(os.environ.get("BATCH", {"C3": 8192, "C2": 2048, "C4": 1024, "C5": 49152, "FEP": 8192, "UE": 4096}.get(config, 0)))
    json.dump(traffic, open(os.path.join(out_dir, f"traffic_{config}.json"), "w"), indent=1)
    if prof_ms:
        prof_ms["batch"] = traffic["batch"]
        json.dump(prof_ms, open(os.path.join(out_dir, f"traffic_{config}_ms.json"), "w"), indent=1)
    for s in ("trace", "fetch", "write", "calfetch", "calwrite"):
        d = os.path.join(prof_dir, f"{s}_{tag}")
        for fn in os.listdir(d):
            if fn.endswith("stats.csv") or fn.endswith("counter_collection.csv") or fn.endswith("kernel_trace.csv"):
                src = os.path.join(d, fn)
                dst = os.path.join(out_dir, f"{tag}_{config}_{s}_{fn}")
                open(dst, "w").write(open(src).read())
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4] if len(sys.argv) > 4 else "profiles")
