"""Cases of the lte_est_freq_offset reference pin (tests/test_ref_pin_fo_cpu.py against the TU compiled
here, tests/test_fo_fixture_cpu.py against tests/golden/fo_ref.json from tests/golden/gen_fo_ref.py):
an estimate plane of splitmix64 int16 (antenna 0, 14 rows of ofdm_symbol_size words) per case and a
sequence of (l, reset) calls; expected: the return value and *freq_offset after each call (the
function's static first_run carries across the calls of a case)."""
import numpy as np

from rm_ref_cases import splitmix64

CALLS = [(0, 1), (None, 0), (0, 0), (None, 0), (0, 1), (None, 0), (2, 0)]   # None: 4 - Ncp; l = 2 is refused


def fo_cases():
    return [dict(N_RB_DL=n_rb, Ncp=ncp, amp=amp, seed=0x70F0000 + 64 * i + 8 * ncp + j)
            for i, n_rb in enumerate((6, 15, 25, 50, 100)) for ncp in (0, 1) for j, amp in enumerate((300, 3000, 32767))]


def fo_plane(c, N):
    """int32 words (re | im << 16) with |component| <= amp"""
    w = splitmix64(c["seed"], 14 * N // 2 + 16).view(np.int16)[:2 * (14 * N + 16)].astype(np.int32)
    v = (w % (2 * c["amp"] + 1)) - c["amp"]
    return ((v[0::2] & 0xFFFF) | (v[1::2] << 16)).astype(np.int32)


def calls(c):
    return [(4 - c["Ncp"] if l is None else l, r) for l, r in CALLS]
