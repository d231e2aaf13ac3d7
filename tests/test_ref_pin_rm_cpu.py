"""Oracle pinned to the reference's own rate matcher and Gold generator, compiled unmodified here
(oracle/Makefile: _ref/libref_rm.so = PHY/CODING/lte_rate_matching.c, _ref/libref_gold.so =
PHY/LTE_REFSIG/lte_gold.c).  Runs only in the build container, where /root/reference exists; the
results travel to the GPU box as tests/golden/rm_ref.npz (tests/golden/gen_rm_ref.py), which
tests/test_rm_ref_fixture_cpu.py and tests/test_gpu_rm_ref.py check.

Pinned here, bit-exact, oracle (oracle/oai_oracle.c, oai_oracle_td.c, oai_oracle_ctrl.c) against
the reference function of the same role:
  - sub_block_interleaving_turbo (lte_rate_matching.c:51-130): all 188 K, w and the d[3D+2]
    side effect;
  - lte_rate_matching_turbo (:464-634): all 188 K x rv 0-3 x Kmimo 1/2 over several (G, C, r, Qm,
    Nl) geometries, the C1/C2/C3/C5 geometries, the "Exiting, RM condition" exit (E = 0);
  - generate_dummy_w (:293-382): all 188 K, F = 0 and filler sizes F > 0;
  - lte_rate_matching_turbo_rx (:688-831): clear = 1 then clear = 0 HARQ sequences rv 0, 2, 3, 1,
    int16 wrap-around;
  - sub_block_deinterleaving_turbo (:193-243), including its writes in front of d;
  - sub_block_interleaving_cc / lte_rate_matching_cc (:132-190, :637-680: PDCCH / PBCH);
  - lte_gold_generic (lte_gold.c:151-177) and dlsch_scrambling's use of it
    (dlsch_scrambling.c:51-97, restated below around the reference generator), lte_gold's
    cell-specific table (:52-93) for both prefixes and all 504 cell ids.
"""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
from ref_cases import QPP

pytestmark = pytest.mark.skipif(O.ref_rm() is None or O.ref_gold() is None,
                                reason="oracle/_ref/libref_rm.so / libref_gold.so not built (no reference tree)")

KS = sorted(QPP)


def _d_stream(K, rng):
    """A turbo-encoder output d (3K+12 entries of 0/1), the sub-block interleaver's input."""
    return rng.integers(0, 2, 3 * K + 12, dtype=np.uint8)


@pytest.mark.parametrize("K", KS)
def test_subblock_interleaving_all_K(K):
    rng = np.random.default_rng(K)
    D = K + 4
    d = _d_stream(K, rng)
    rtc_r, w_r, buf_r = O.ref_subblock(d, D)
    rtc_o, w_o, buf_o = O.subblock(d, D)
    assert rtc_r == rtc_o
    assert np.array_equal(w_o[:len(w_r)], w_r), K
    # the d[3D+2] = d[2] side effect on the caller's buffer (lte_rate_matching.c:75)
    assert np.array_equal(buf_o[:96 + 3 * D + 16], buf_r[:96 + 3 * D + 16]), K


def _geometries(K):
    """(G, C, r, Qm, Nl) tuples exercising E = floor / ceil, Nl = 2 and wrap-around."""
    out = []
    for C, Qm, Nl in [(1, 2, 1), (3, 4, 1), (6, 6, 1), (5, 4, 2), (13, 6, 1)]:
        for gmul in (1, 3):
            G = Nl * Qm * (C * (K // 2) * gmul + (C // 2))       # G' mod C != 0 when C > 1
            for r in sorted({0, C - 1, C // 2}):
                out.append((G, C, r, Qm, Nl))
    return out


@pytest.mark.parametrize("K", KS)
def test_rate_matching_all_K(K):
    rng = np.random.default_rng(1000 + K)
    D = K + 4
    rtc, w, _ = O.ref_subblock(_d_stream(K, rng), D)
    for (G, C, r, Qm, Nl) in _geometries(K):
        for Kmimo in (1, 2):
            for rv in range(4):
                e_r = O.ref_rate_match(rtc, G, w, C, r, Qm, rvidx=rv, Nl=Nl, Kmimo=Kmimo)
                e_o = O.rate_match(rtc, G, w, C, r, Qm, rvidx=rv, Nl=Nl, Kmimo=Kmimo)
                assert np.array_equal(e_o, e_r), (K, G, C, r, Qm, Nl, Kmimo, rv)


# bench / parity geometries: (K, G, C, Qm, Kmimo, Nl)
GEOMS = {"C1": (960, 1512, 1, 2, 1, 1), "C2": (6144, 60000, 5, 4, 1, 1), "C3": (6144, 86400, 6, 6, 2, 1),
         "C5": (5504, 57600, 8, 4, 1, 1), "TM2": (6144, 57600, 5, 4, 1, 2)}


@pytest.mark.parametrize("name", sorted(GEOMS))
def test_rate_matching_config_geometries(name):
    K, G, C, Qm, Kmimo, Nl = GEOMS[name]
    rng = np.random.default_rng(7)
    rtc, w, _ = O.ref_subblock(_d_stream(K, rng), K + 4)
    total = 0
    for r in range(C):
        for rv in range(4):
            e_r = O.ref_rate_match(rtc, G, w, C, r, Qm, rvidx=rv, Nl=Nl, Kmimo=Kmimo)
            assert np.array_equal(O.rate_match(rtc, G, w, C, r, Qm, rvidx=rv, Nl=Nl, Kmimo=Kmimo), e_r)
            if rv == 0:
                total += len(e_r)
    assert total == G - G % (Nl * Qm)


def test_rm_condition_exit():
    """Ncb < Kw: the reference prints "Exiting, RM condition" and returns E = 0 (:518-521)."""
    rng = np.random.default_rng(3)
    rtc, w, _ = O.ref_subblock(_d_stream(6144, rng), 6148)
    for C, Kmimo in [(13, 2), (7, 2), (26, 1)]:
        assert len(O.ref_rate_match(rtc, 200000, w, C, 0, 6, Kmimo=Kmimo)) == 0
        assert len(O.rate_match(rtc, 200000, w, C, 0, 6, Kmimo=Kmimo)) == 0


@pytest.mark.parametrize("K", KS)
def test_generate_dummy_w_all_K(K):
    D = K + 4
    rtc_r, w_r = O.ref_dummy_w(D, 0)
    assert np.array_equal(O.dummy_w(D)[:len(w_r)] == 2, w_r == 2), K
    for F in (0, 8, 16, 24, 40, 64):
        if F >= K:
            continue
        _, w_r = O.ref_dummy_w(D, F)
        w_o = O.dummy_w_F(D, F)[:len(w_r)]
        assert np.array_equal(w_o == 2, w_r == 2), (K, F)


@pytest.mark.parametrize("K", [40, 512, 960, 1056, 2112, 4032, 5504, 6144])
def test_rate_matching_rx_harq_sequence(K):
    """clear = 1 on round 0, then clear = 0 for rv 2, 3, 1 (dlsim's round loop, dlsim.c:2141): the
    soft sums wrap in int16 exactly as the reference's `w[ind] += soft` does."""
    rng = np.random.default_rng(K + 5)
    D = K + 4
    R = (D + 31) >> 5
    _, dw = O.ref_dummy_w(D, 0)
    for (G, C, r, Qm, Nl, Kmimo) in [(3 * K + 300, 1, 0, 2, 1, 1), (6 * (3 * K) + 24, 2, 1, 6, 1, 2),
                                      (4 * 2 * K, 2, 0, 4, 2, 1)]:
        w_r = np.zeros(3 * 32 * R, np.int16)
        w_o = np.zeros(3 * 32 * R + 64, np.int16)
        for rnd, rv in enumerate((0, 2, 3, 1)):
            soft = rng.integers(-32768, 32768, G, dtype=np.int16)
            ret, E_r, w_r = O.ref_rate_match_rx(R, G, w_r, dw, soft, C, r, Qm, rvidx=rv, clear=1 if rnd == 0 else 0,
                                                Nl=Nl, Kmimo=Kmimo)
            assert ret == 0
            w_o, E_o = O.rate_match_rx(soft, K, G, C, r, Qm, rvidx=rv, Nl=Nl, Kmimo=Kmimo, w=w_o,
                                       clear=1 if rnd == 0 else 0, dw=np.concatenate([dw, np.zeros(64, np.uint8)]))
            assert E_o == E_r
            assert np.array_equal(w_o[:3 * 32 * R], w_r), (K, G, rnd, rv)


def test_rate_matching_rx_invalid_parameters():
    ret, _, _ = O.ref_rate_match_rx(193, 1000, np.zeros(18528, np.int16), np.zeros(18528, np.uint8),
                                    np.zeros(1000, np.int16), 0, 0, 2)
    assert ret == -1
    E = ctypes.c_uint32()
    z = np.zeros(18528 + 64, np.int16)
    assert O.orc().orc_rate_matching_turbo_rx(193, 1000, O.P(z), O.P(np.zeros(18600, np.uint8)), O.P(z), 0, 1827072,
                                              8, 1, 0, 1, 2, 1, 0, ctypes.byref(E)) == -1


@pytest.mark.parametrize("K", KS[::7] + [6144])
def test_subblock_deinterleaving(K):
    rng = np.random.default_rng(K + 9)
    D = K + 4
    R = (D + 31) >> 5
    w = rng.integers(-32768, 32768, 3 * 32 * R, dtype=np.int16)
    d_r = O.ref_deinterleave(D, w)
    buf = np.zeros(96 + 3 * D + 64, dtype=np.int16)
    O.orc().orc_sub_block_deinterleaving_turbo(D, ctypes.c_void_p(buf.ctypes.data + 2 * 96), O.P(w))
    assert np.array_equal(buf, d_r[:len(buf)]), K


@pytest.mark.parametrize("D", [40, 57, 64, 70, 72, 96, 100])
def test_cc_interleaving_and_rate_matching(D):
    """PDCCH / PBCH tail-biting path: sub_block_interleaving_cc + lte_rate_matching_cc."""
    L = O.orc()
    L.orc_sub_block_interleaving_cc.restype = ctypes.c_uint32
    L.orc_lte_rate_matching_cc.restype = ctypes.c_uint32
    L.orc_lte_rate_matching_cc.argtypes = [ctypes.c_uint32, ctypes.c_uint16, ctypes.c_void_p, ctypes.c_void_p]
    rng = np.random.default_rng(D)
    R = (D + 31) >> 5
    buf = np.full(96 + 3 * D + 64, 2, np.uint8)
    buf[96:96 + 3 * D] = rng.integers(0, 2, 3 * D, dtype=np.uint8)
    w_r = np.zeros(3 * 32 * R + 16, np.uint8)
    w_o = np.zeros_like(w_r)
    rr = O.ref_rm().sub_block_interleaving_cc(D, ctypes.c_void_p(buf.ctypes.data + 96), O.P(w_r))
    ro = L.orc_sub_block_interleaving_cc(D, ctypes.c_void_p(buf.ctypes.data + 96), O.P(w_o))
    assert rr == ro
    assert np.array_equal(w_r, w_o)
    for E in (72, 144, 576, 1920, 1728):
        e_r = np.zeros(E + 16, np.uint8)
        e_o = np.zeros_like(e_r)
        assert O.ref_rm().lte_rate_matching_cc(rr, E, O.P(w_r), O.P(e_r)) == L.orc_lte_rate_matching_cc(
            rr, E, O.P(w_o), O.P(e_o))
        assert np.array_equal(e_r, e_o), (D, E)


def test_gold_generic_words():
    rng = np.random.default_rng(5)
    L = O.orc()
    for c_init in [0, 1, 0x1234 << 14, (0x1234 << 14) + (1 << 13) + (7 << 9) + 503, 0x7FFFFFFF,
                   *rng.integers(0, 1 << 31, 40).tolist()]:
        ref = O.ref_gold_words(c_init, 64)
        x1, x2 = ctypes.c_uint32(0), ctypes.c_uint32(c_init)
        orc = [L.orc_gold_generic(ctypes.byref(x1), ctypes.byref(x2), 1 if i == 0 else 0) for i in range(64)]
        assert np.array_equal(np.array(orc, np.uint32), ref), c_init


def _ref_dlsch_scrambling(e, G, rnti, q, Ns, Nid_cell):
    """dlsch_scrambling.c:51-97 around the reference's own lte_gold_generic: c_init, the
    (1 + G/32) * 32-entry loop (the overrun past G kept)."""
    c_init = (rnti << 14) + (q << 13) + ((Ns >> 1) << 9) + Nid_cell
    words = O.ref_gold_words(c_init, 1 + (G >> 5))
    bits = ((words[:, None] >> np.arange(32, dtype=np.uint32)) & 1).astype(np.uint8).ravel()
    out = e.copy()
    n = len(bits)
    out[:n] = (out[:n] & 1) ^ bits
    return out


@pytest.mark.parametrize("G,rnti,q,Ns,Nid", [(1512, 0x1234, 0, 14, 0), (60000, 0x1234, 0, 14, 0),
                                             (86400, 0x1234, 1, 10, 0), (86400, 0xFFFF, 0, 0, 503),
                                             (57600, 0x3D, 1, 18, 17), (31, 1, 0, 2, 5)])
def test_dlsch_scrambling_vs_reference_gold(G, rnti, q, Ns, Nid):
    rng = np.random.default_rng(G + Ns)
    e = rng.integers(0, 2, (1 + (G >> 5)) * 32 + 32, dtype=np.uint8)
    ref = _ref_dlsch_scrambling(e, G, rnti, q, Ns, Nid)
    c_init = (rnti << 14) + (q << 13) + ((Ns >> 1) << 9) + Nid
    assert np.array_equal(O.scramble(e, G, c_init)[:len(ref)], ref)


@pytest.mark.parametrize("Ncp", [0, 1])
def test_lte_gold_cell_table(Ncp):
    for Nid in list(range(0, 504, 7)) + [503]:
        fp = O.frame(6, Nid_cell=Nid, Ncp=Ncp)
        t = np.zeros((20, 2, 14), np.uint32)
        O.orc().orc_lte_gold_table(ctypes.byref(fp), O.P(t))
        assert np.array_equal(t, O.ref_gold_table(Ncp, Nid)), (Ncp, Nid)
