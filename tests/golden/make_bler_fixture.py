"""Generates tests/golden/bler_awgn_tx1_nrx1.json from the reference-held BLER curves
openair1/SIMULATION/LTE_PHY/BLER_SIMULATIONS/AWGN/AWGN_results/bler_tx1_chan18_nrx1_mcs{0..27}.csv
(dlsim, TM1, AWGN = channel model 18, one RX antenna, 25 PRB; columns SNR; MCS; TBS; rate; err0;
trials0; ...) and from the second set the reference holds for the same configuration,
BLER_SIMULATIONS/AWGN/Perf_Curves_Abs/awgn_bler_tx1_mcs{0..27}.csv (same dlsim CSV layout, same TBS
per MCS, another run).  Data only: (SNR, err0, trials0) per row, plus TBS / rate per MCS.  Run in the
container that holds the reference tree: python tests/golden/make_bler_fixture.py"""
import json
import os

BASE = "/root/reference/openair1/SIMULATION/LTE_PHY/BLER_SIMULATIONS/AWGN"
SRC = BASE + "/AWGN_results"
SRC2 = BASE + "/Perf_Curves_Abs"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bler_awgn_tx1_nrx1.json")


def read(path):
    rows, tbs, rate = [], None, None
    with open(path) as f:
        next(f)
        for line in f:
            v = [x.strip() for x in line.split(";")]
            if len(v) < 6:
                continue
            tbs, rate = int(v[2]), float(v[3])
            rows.append([round(float(v[0]), 3), int(v[4]), int(v[5])])
    return {"TBS": tbs, "rate": rate, "rows": rows}


curves = {str(m): read(os.path.join(SRC, f"bler_tx1_chan18_nrx1_mcs{m}.csv")) for m in range(28)}
curves2 = {str(m): read(os.path.join(SRC2, f"awgn_bler_tx1_mcs{m}.csv")) for m in range(28)
           if os.path.exists(os.path.join(SRC2, f"awgn_bler_tx1_mcs{m}.csv"))}
json.dump({"source": SRC + "/bler_tx1_chan18_nrx1_mcs*.csv", "columns": ["snr_db", "err0", "trials0"],
           "curves": curves, "source_perf_curves_abs": SRC2 + "/awgn_bler_tx1_mcs*.csv",
           "curves_perf_curves_abs": curves2}, open(OUT, "w"), separators=(",", ":"))
print("wrote", OUT)
