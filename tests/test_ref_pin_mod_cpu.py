"""The oracle's modulation / RE mapping / precoding, scrambling and PCFICH against the reference's own
PHY/LTE_TRANSPORT/dlsch_modulation.c (:1181-1493, with allocate_REs_in_RB :139-982),
dlsch_scrambling.c (:51-97) and pcfich.c (:48-228), compiled unmodified into oracle/_ref/libref_mod.so
(oracle/Makefile, glue oracle/ref_glue_mod.c).  Frame grids must be identical word for word, and dlsch_modulation's
return value (re_allocated) equal.  Skipped where the reference tree was not built here (the GPU box);
tests/test_mod_fixture_cpu.py covers the committed fixtures there."""
import itertools

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.skipif(O.ref_mod() is None, reason="oracle/_ref/libref_mod.so not built (no reference tree)")

FULL = {6: [0x3F, 0, 0, 0], 15: [0x7FFF, 0, 0, 0], 25: [0x1FFFFFF, 0, 0, 0], 50: [0xFFFFFFFF, 0x3FFFF, 0, 0],
        75: [0xFFFFFFFF, 0xFFFFFFFF, 0x7FF, 0], 100: [0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xF]}
NBITS = 14 * 1200 * 6


def _bits(rng):
    return rng.integers(0, 2, NBITS).astype(np.uint8)


def _alloc(rng, n_rb, kind):
    if kind == "full":
        return list(FULL[n_rb])
    m = 0
    while m == 0:
        m = int(rng.integers(0, 1 << n_rb, dtype=np.uint64)) if n_rb < 64 else \
            int.from_bytes(rng.bytes(16), "little") & ((1 << n_rb) - 1)
        if kind == "odd":          # a few scattered RBs, including the DC-straddling one of odd N_RB
            m = (m & int.from_bytes(rng.bytes(16), "little") & int.from_bytes(rng.bytes(16), "little")) | \
                (1 << (n_rb // 2))
    return [(m >> (32 * i)) & 0xFFFFFFFF for i in range(4)]


def _check(fp, amp, sf, npdcch, cws, rho_a=8192, rho_b=8192):
    r_ref, g_ref = O.ref_modulation(fp, amp, sf, npdcch, cws, rho_a, rho_b)
    r_orc, g_orc = O.orc_modulation_grids(fp, amp, sf, npdcch, cws, rho_a, rho_b)
    assert r_orc == r_ref
    for a, (x, y) in enumerate(zip(g_orc, g_ref)):
        d = np.nonzero(x != y)[0]
        assert d.size == 0, f"antenna {a}: {d.size} words differ, first at {d[:4]} ({x[d[:4]]} vs {y[d[:4]]})"
    return r_ref


def test_qam_tables_equal_reference():
    q16 = np.zeros(4, np.int32)
    q64 = np.zeros(8, np.int32)
    O.ref_mod().ref_glue_qam_tables(q16.ctypes.data, q64.ctypes.data)
    # dlsch_modulation.c:79-103 through impl_defs_top.h's QAM16_n1 / QAM64_n1..n3; the outer 64-QAM
    # level exceeds int16 (the oracle keeps int levels)
    assert list(q16) == [10362, 31086, -10362, -31086]
    assert list(q64) == [15169, 5057, 25281, 35393, -15169, -5057, -25281, -35393]


@pytest.mark.parametrize("n_rb", [6, 15, 25, 50, 100])   # init_frame_parms: lte_parms.c:31-145
@pytest.mark.parametrize("Ncp", [0, 1])
def test_siso_every_bandwidth_and_prefix(n_rb, Ncp):
    """TM1 (SISO, one and two TX antennas), QPSK / 16-QAM / 64-QAM, every subframe index (PBCH,
    PSS / SSS exclusions at 0 and 5), 1-3 PDCCH symbols (4 at 6 PRB), full allocations."""
    rng = np.random.default_rng(1000 + 10 * n_rb + Ncp)
    for n_ant in (1, 2):
        fp = O.frame(n_rb, Nid_cell=int(rng.integers(0, 504)), Ncp=Ncp, nb_antennas_tx=n_ant, mode1_flag=1)
        for sf in range(10):
            mcs = (5, 12, 22)[sf % 3]
            npdcch = (1, 2, 3, 4)[sf % 4] if n_rb <= 10 else (1, 2, 3)[sf % 3]
            n = _check(fp, 512, sf, npdcch, [dict(e=_bits(rng), mcs=mcs, mimo_mode=0, rb_alloc=_alloc(rng, n_rb, "full"))])
            assert n > 0


@pytest.mark.parametrize("n_rb", [6, 15, 25, 50, 100])
def test_siso_partial_allocations(n_rb):
    """Random and sparse RB bitmaps (odd N_RB: the DC-straddling RB's half-RB skip, dlsch_modulation.c:245-249)."""
    rng = np.random.default_rng(2000 + n_rb)
    fp = O.frame(n_rb, Nid_cell=7, nb_antennas_tx=1, mode1_flag=1)
    for i, kind in itertools.product(range(6), ("random", "odd")):
        _check(fp, 512, (i * 3) % 10, 1 + i % 3,
               [dict(e=_bits(rng), mcs=(3, 15, 26)[i % 3], mimo_mode=0, rb_alloc=_alloc(rng, n_rb, kind))])


@pytest.mark.parametrize("n_rb", [6, 15, 25, 50, 100])
def test_alamouti(n_rb):
    """TM2 transmit diversity (dlsch_modulation.c:362-546, 868-876): one codeword on two ports,
    the pair written from the accumulated values, with the power offsets rho_A / rho_B."""
    rng = np.random.default_rng(3000 + n_rb)
    fp = O.frame(n_rb, Nid_cell=int(rng.integers(0, 504)), nb_antennas_tx=2, mode1_flag=0)
    for sf in range(10):
        rho = [(8192, 8192), (5793, 8192), (8192, 11585)][sf % 3]
        kind = "full" if sf % 2 == 0 else "random"
        _check(fp, 512, sf, 1 + sf % 3, [dict(e=_bits(rng), mcs=(6, 13, 24)[sf % 3], mimo_mode=1,
                                              rb_alloc=_alloc(rng, n_rb, kind))], *rho)


@pytest.mark.parametrize("n_rb", [6, 15, 25, 50, 100])
@pytest.mark.parametrize("Ncp", [0, 1])
def test_large_cdd_two_codewords(n_rb, Ncp):
    """TM3 LARGE_CDD with two codewords (dlsch_modulation.c:547-749): the floor-halved sum and the
    per-RB-reset alternating sign of the difference, mixed modulation orders."""
    rng = np.random.default_rng(4000 + 10 * n_rb + Ncp)
    fp = O.frame(n_rb, Nid_cell=int(rng.integers(0, 504)), Ncp=Ncp, nb_antennas_tx=2, mode1_flag=0)
    for sf in range(10):
        m0, m1 = [(19, 19), (4, 16), (12, 27), (28, 2)][sf % 4]
        ra = _alloc(rng, n_rb, "full" if sf % 3 else "random")
        _check(fp, 512, sf, 1 + sf % 3, [dict(e=_bits(rng), mcs=m0, mimo_mode=2, rb_alloc=ra),
                                         dict(e=_bits(rng), mcs=m1, mimo_mode=2, rb_alloc=ra)])


def test_c3_headline_subframe_and_amplitudes():
    """The C3 configuration itself (100 PRB, 2 × 64-QAM MCS 19, subframe 7, one PDCCH
    symbol, AMP 512, rho 0 dB) and a few other amplitudes."""
    rng = np.random.default_rng(5)
    fp = O.frame(100, Nid_cell=0, nb_antennas_tx=2, mode1_flag=0)
    for amp in (512, 1024, 4096):
        n = _check(fp, amp, 7, 1, [dict(e=_bits(rng), mcs=19, mimo_mode=2, rb_alloc=FULL[100]),
                                   dict(e=_bits(rng), mcs=19, mimo_mode=2, rb_alloc=FULL[100])])
        assert n == 14400


@pytest.mark.parametrize("G", [0, 1, 31, 32, 33, 1512, 14400, 60000, 86400])
def test_scrambling_equals_reference(G):
    """dlsch_scrambling's XOR loop (c_init = rnti 2^14 + q 2^13 + floor(Ns / 2) 2^9 + Nid_cell)
    against the oracle's orc_scramble on e[0 .. G); the reference also rewrites the entries up to
    32 (1 + G / 32) - 1, which the oracle's buffer is not asked to reproduce."""
    rng = np.random.default_rng(6000 + G)
    for rnti, Nid, q, Ns in [(0x1234, 0, 0, 14), (0xFFFF, 503, 1, 0), (1, 37, 0, 19), (0x8000, 255, 1, 10)]:
        e = rng.integers(0, 2, 32 * (1 + (G >> 5))).astype(np.uint8)
        ref = O.ref_scrambling(e, G, rnti, Nid, q, Ns)
        orc = O.scramble(e, G, (rnti << 14) + (q << 13) + ((Ns >> 1) << 9) + Nid) if G else e
        assert np.array_equal(ref[:G], orc[:G])


@pytest.mark.parametrize("n_rb", [6, 15, 25, 50, 100])
def test_pcfich_reg_mapping_every_cell(n_rb):
    """generate_pcfich_reg_mapping (pcfich.c:48-84): the four REGs and the first-REG index for all 504
    cell ids."""
    for nid in range(504):
        fp = O.frame(n_rb, Nid_cell=nid)
        _, reg, first = O.ref_pcfich(1, 512, fp, 0)
        assert O.pcfich_reg_mapping(fp) == (reg, first), nid


@pytest.mark.parametrize("n_rb", [6, 15, 25, 50, 100])
@pytest.mark.parametrize("Ncp", [0, 1])
def test_pcfich_equals_reference(n_rb, Ncp):
    """generate_pcfich (pcfich.c:144-228): CFI 1-3 codewords, the c_init of 36.211 6.7.1, QPSK at
    amp / sqrt2 (SISO) or amp / 2 (ALAMOUTI pairs), the nushift holes, 1 or 2 TX antennas; whole
    frame grids word for word."""
    rng = np.random.default_rng(7000 + 10 * n_rb + Ncp)
    for n_ant, mode1 in ((1, 1), (2, 1), (2, 0)):
        for cfi in (1, 2, 3):
            for sf in range(10):
                nid = int(rng.integers(0, 504))
                amp = int(rng.choice([512, 1024, 4096, 32767]))
                fp = O.frame(n_rb, Nid_cell=nid, Ncp=Ncp, nb_antennas_tx=n_ant, mode1_flag=mode1)
                ref, _, _ = O.ref_pcfich(cfi, amp, fp, sf)
                orc = [np.zeros_like(g) for g in ref]
                assert O.generate_pcfich(cfi, amp, fp, orc, sf) == 0
                for a in range(n_ant):
                    assert np.array_equal(orc[a], ref[a]), (n_ant, mode1, cfi, sf, nid, amp, a)
