"""Cases of the dlsch_llr_computation.c reference pin (tests/test_ref_pin_llr_cpu.py against the TU
compiled here, tests/test_llr_fixture_cpu.py against the fixtures it produced, tests/golden/llr_ref.json
made by tests/golden/gen_llr_ref.py).  Inputs are splitmix64 words, so only the case list and digests
are stored.

Two reference quirks bound what is compared:
  - dlsch_64qam_llr's remainder test is inverted (dlsch_llr_computation.c:866-867: len2 += (len_mod4 ?
    0 : 1)): with len mod 4 != 0 the last len mod 4 REs of the symbol are never written (their LLRs
    are whatever the buffer held), with len mod 4 == 0 one extra quad is written past len (the next
    symbol overwrites it).  The oracle and the library write all len REs;
  - qpsk_qpsk / qpsk_qam16 / qpsk_qam64 step over (len >> 2) quads two at a time (:1077, :1350,
    :1631): 8 ceil((len >> 2) / 2) REs are computed, so with (len >> 2) even and len mod 4 != 0 the
    last len mod 4 REs are not.
Compared: the REs the reference computes; the test also checks that it leaves the others untouched."""
import numpy as np

from rm_ref_cases import digest, splitmix64


def words16(seed, n):
    """n int16 from splitmix64(seed), full range"""
    return splitmix64(seed, n // 4 + 1).view(np.int16)[:n].copy()


def qam_cases():
    cases = []
    k = 0
    for qm in (2, 4, 6):
        for n_rb, ncp, mode1, sym, nb in ((25, 0, 1, 4, 25), (25, 0, 1, 2, 25), (100, 0, 0, 0, 100), (100, 0, 1, 7, 100),
                                          (50, 1, 1, 3, 17), (50, 1, 0, 6, 50), (15, 0, 1, 11, 15), (6, 0, 1, 7, 5),
                                          (6, 1, 0, 0, 6), (75, 0, 0, 8, 33)):
            k += 1
            cases.append(dict(Qm=qm, N_RB_DL=n_rb, Ncp=ncp, mode1_flag=mode1, symbol=sym, nb_rb=nb, seed=0x11A0000 + k))
    return cases


def ia_cases():
    return [dict(qm1=qm1, n=n, seed=0x11B0000 + 16 * i + qm1)
            for qm1 in (2, 4, 6) for i, n in enumerate((8, 10, 12, 100, 250, 600, 800, 1000, 1200))]


def qam_len(c):
    """REs of the symbol (dlsch_*_llr's len, pbch_pss_sss_adjust 0)"""
    sm = c["symbol"] - (7 - c["Ncp"]) if c["symbol"] >= 7 - c["Ncp"] else c["symbol"]
    if sm == 0 or sm == 4 - c["Ncp"]:
        return c["nb_rb"] * (10 if c["mode1_flag"] else 8)
    return c["nb_rb"] * 12


def qam_written(c):
    """REs the reference writes"""
    n = qam_len(c)
    return n - (n & 3) if c["Qm"] == 6 else n


def ia_written(n):
    return min(n, 8 * (((n >> 2) + 1) // 2))


def qam_inputs(c):
    """symbol-major comp, mag, magb (int32 words; the magnitudes packed (m, m) as the compensation writes
    them) and the per-RE magnitudes"""
    W = 14 * c["N_RB_DL"] * 12 + 64
    comp = words16(c["seed"], 2 * W).view(np.int32)
    m = words16(c["seed"] ^ 0x5A5A, W)
    mb = words16(c["seed"] ^ 0xA5A5, W)
    pack = lambda v: ((v.astype(np.int32) & 0xFFFF) | (v.astype(np.int32) << 16)).astype(np.int32)   # noqa: E731
    return comp, pack(m), pack(mb), m, mb


def ia_inputs(c):
    n = c["n"] + 32
    s0, s1, rho = (words16(c["seed"] ^ x, 2 * n) for x in (0, 0x1111, 0x2222))
    m = np.abs(words16(c["seed"] ^ 0x3333, n).astype(np.int32)).clip(0, 32767).astype(np.int16)
    return s0, s1, rho, m


__all__ = ["digest", "qam_cases", "ia_cases", "qam_len", "qam_written", "ia_written", "qam_inputs", "ia_inputs"]
