"""BLER sweep on the GPU against the reference-held AWGN curves (tests/golden/bler_awgn_tx1_nrx1.json).

  python tools/bler_sweep.py --mcs 0 9 16 27 --trials 20000 [--no-dci] [--out gpurun_out/bler.json]

For every CSV row on the waterfall (0.005 < BLER < 0.995) it runs the GPU dlsim loop
(openair4g_amd/dlsim.py) and prints GPU vs reference BLER with the z score of their difference,
then the SNR shift that best aligns the two curves (log-BLER interpolation)."""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mcs", type=int, nargs="+", default=[0, 9, 16, 27])
    ap.add_argument("--trials", type=int, default=20000)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--no-dci", action="store_true")
    ap.add_argument("--llr8", action="store_true", help="the 8-bit turbo decoder (dlsim -L)")
    ap.add_argument("--lo", type=float, default=0.005)
    ap.add_argument("--hi", type=float, default=0.995)
    ap.add_argument("--out", default=None)
    ap.add_argument("--curves", default="awgn_results", choices=["awgn_results", "perf_curves_abs"],
                    help="which reference-held curve set to compare with")
    a = ap.parse_args()
    import dlsim_oracle as D
    from openair4g_amd.dlsim import DlsimBler
    curves = D.load_curves(a.curves)
    res = {}
    for mcs in a.mcs:
        sim = DlsimBler(mcs, batch=a.batch, with_dci=not a.no_dci, llr8=a.llr8)
        rows = []
        t0 = time.time()
        for snr, e, n in curves[mcs]:
            q = e / n
            if not (a.lo < q < a.hi):
                continue
            k, m = sim.run_point(snr, a.trials, seed=int(round(snr * 1000)) + 7919 * mcs)
            p = k / m
            se = math.sqrt(p * (1 - p) / m + q * (1 - q) / n) + 1e-12
            rows.append([snr, k, m, e, n, (p - q) / se])
            print(f"MCS {mcs:2d} SNR {snr:6.2f}: GPU {k:6d}/{m} = {p:.4f}   ref {e:5d}/{n} = {q:.4f}   z {(p - q) / se:+6.2f}",
                  flush=True)
        # shift: ref(snr) ~ gpu(snr + d); fit d minimising squared log-BLER error by interpolation
        s = np.array([r[0] for r in rows])
        pg = np.clip(np.array([r[1] / r[2] for r in rows]), 1e-4, 1)
        pr = np.clip(np.array([r[3] / r[4] for r in rows]), 1e-4, 1)
        best = None
        for d in np.arange(-0.5, 0.5001, 0.005):
            g = np.interp(s + d, s, np.log(pg), left=np.nan, right=np.nan)
            ok = ~np.isnan(g)
            if ok.sum() < 3:
                continue
            err = float(np.mean((g[ok] - np.log(pr[ok])) ** 2))
            if best is None or err < best[1]:
                best = (round(float(d), 3), err)
        print(f"MCS {mcs}: best shift ref(snr) ~ gpu(snr + d), d = {best}  ({time.time() - t0:.1f}s)", flush=True)
        from openair4g_amd.dlsim import wilson
        inside = sum(1 for r in rows if abs(r[5]) <= 1.96)
        in_ci = sum(1 for r in rows if wilson(r[3], r[4])[0] <= r[1] / r[2] <= wilson(r[3], r[4])[1])
        print(f"MCS {mcs}: {inside} of {len(rows)} rows within |z| <= 1.96; {in_ci} inside the reference row's "
              f"95 % (Wilson) interval", flush=True)
        res[mcs] = {"rows": rows, "shift_db": best[0] if best else None, "dci": not a.no_dci, "llr8": a.llr8,
                    "curves": a.curves, "rows_within_z196": inside, "rows_inside_ci": in_ci}
        sim.close()
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
