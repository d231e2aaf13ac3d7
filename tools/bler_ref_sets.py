"""The reference holds two AWGN BLER curve sets for the same dlsim configuration (TM1, 25 PRB, one RX,
same TBS per MCS): AWGN_results/bler_tx1_chan18_nrx1_mcs*.csv and Perf_Curves_Abs/awgn_bler_tx1_mcs*.csv
(tests/golden/bler_awgn_tx1_nrx1.json holds both).  This prints, per MCS, the SNR shift d that best
aligns them, AWGN_results(snr) ~ Perf_Curves_Abs(snr + d), fitted on log-BLER by interpolation over
their common waterfall rows, and each set's 50 % crossing.  CPU only, data only."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import dlsim_oracle as D  # noqa: E402


def crossing(rows, level=0.5):
    s = np.array([r[0] for r in rows])
    p = np.array([r[1] / r[2] for r in rows])
    for i in range(len(p) - 1):
        if p[i] >= level > p[i + 1]:
            return float(s[i] + (s[i + 1] - s[i]) * (p[i] - level) / (p[i] - p[i + 1]))
    return float("nan")


def shift(a_rows, b_rows):
    """d minimising mean (log b(s + d) - log a(s))^2 over a's waterfall rows inside b's range."""
    sa = np.array([r[0] for r in a_rows]); pa = np.array([r[1] / r[2] for r in a_rows])
    sb = np.array([r[0] for r in b_rows]); pb = np.clip(np.array([r[1] / r[2] for r in b_rows]), 1e-4, 1)
    keep = (pa > 0.005) & (pa < 0.995)
    sa, pa = sa[keep], pa[keep]
    best = None
    for d in np.arange(-0.6, 0.6001, 0.005):
        g = np.interp(sa + d, sb, np.log(pb), left=np.nan, right=np.nan)
        ok = ~np.isnan(g)
        if ok.sum() < 3:
            continue
        e = float(np.mean((g[ok] - np.log(pa[ok])) ** 2))
        if best is None or e < best[1]:
            best = (round(float(d), 3), e)
    return best


def main():
    a, b = D.load_curves("awgn_results"), D.load_curves("perf_curves_abs")
    print("MCS  50%-crossing AWGN_results  Perf_Curves_Abs   shift d (AWGN_results(s) ~ Perf(s + d))")
    for m in sorted(a):
        if m not in b:
            continue
        sh = shift(a[m], b[m])
        print(f"{m:3d}  {crossing(a[m]):8.3f}  {crossing(b[m]):8.3f}   {sh[0] if sh else None}")


if __name__ == "__main__":
    main()
