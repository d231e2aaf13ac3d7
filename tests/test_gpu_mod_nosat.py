"""k_modofdm's fused IDFT levels (ibfly4_shr1_ns, oai4g_dft_prims.h) against the saturating levels and
the reference.

C3's kernel folds x0 2^15 into the 32-bit sums of the 256- and 1024-level butterflies and extracts
bits 16..31, which equals the reference's packs_epi32 + wrapping add + >> 1 whenever no value of those
levels leaves int16; its radix-4 adds (leaf, 64-level) rotate the difference once instead of both
operands, equal when nothing saturates.  The host admits the fused form only when a range bound proves that for every
possible bit pattern (mod_nosat_ok in oai4g_host.cpp: the DIT classes' occupied subcarriers x the
largest QAM modulus x the level's scale, plus a truncation margin); OAI4G_MOD_SAT forces the
saturating levels.  The tests:
  - the range check admits C3 at the reference's amplitude (amp 512) and refuses amplitudes whose
    bound exceeds int16;
  - adversarial e bits (every RE the same 64-QAM corner, codewords in opposition so the CDD
    difference is maximal, period-4 and quarter-turn sequences that put the whole band into a
    single bin of a residue class, random corners, random symbols) drive the fused kernel and the
    saturating kernel to bit-identical IQ;
  - on the same adversarial subframes the fused kernel's IQ equals the reference's own
    dlsch_modulation.c -> normal_prefix_mod (ofdm_mod.c) (oracle/_ref, compiled unmodified)."""
import os

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

N_SF = 8
Q64 = [15169, 5057, 25281, 35393, -15169, -5057, -25281, -35393]   # raw 64-QAM levels by index (sign only matters)


def _level_index(v):
    """qam_map's 64-QAM (I, Q) level indices of symbol value v (bit j = the RE's j-th e bit)."""
    ir = ((v & 1) << 2) | (((v >> 2) & 1) << 1) | ((v >> 4) & 1)
    ii = (((v >> 1) & 1) << 2) | (((v >> 3) & 1) << 1) | ((v >> 5) & 1)
    return ir, ii


def _corner(si, sq):
    """the symbol value whose (I, Q) is the outer corner with signs (si, sq)"""
    for v in range(64):
        ir, ii = _level_index(v)
        if abs(Q64[ir]) == 35393 and abs(Q64[ii]) == 35393 and np.sign(Q64[ir]) == si and np.sign(Q64[ii]) == sq:
            return v
    raise AssertionError


PP, MP, MM, PM = _corner(1, 1), _corner(-1, 1), _corner(-1, -1), _corner(1, -1)


def _patterns(n_re, rng):
    """(cw0 symbols, cw1 symbols) per subframe of the batch"""
    idx = np.arange(n_re)
    rot = np.array([PP, MP, MM, PM])
    out = [
        (np.full(n_re, PP), np.full(n_re, PP)),                         # all REs one corner: class DC bins
        (np.full(n_re, PP), np.full(n_re, MM)),                         # opposed codewords: y0 ~ 0, |d| max
        (np.where((idx >> 1) & 1, MM, PP), np.where((idx >> 1) & 1, MM, PP)),   # period 4: the mod-2 classes' Nyquist
        (rot[idx & 3], rot[idx & 3]),                                   # quarter turn per RE
        (rot[(idx >> 1) & 3], rot[3 - ((idx >> 1) & 3)]),              # both codewords, opposite turns
        (rot[rng.integers(0, 4, n_re)], rot[rng.integers(0, 4, n_re)]),   # random corners
        (rng.integers(0, 64, n_re), rng.integers(0, 64, n_re)),         # random symbols
        (np.full(n_re, MM), np.full(n_re, PM)),
    ]
    assert len(out) == N_SF
    return out


def _words(sym, G, n_words):
    bits = ((np.asarray(sym, dtype=np.uint32)[:, None] >> np.arange(6, dtype=np.uint32)) & 1).astype(np.uint8).ravel()
    assert bits.size == G
    buf = np.zeros(n_words * 4, dtype=np.uint8)
    packed = np.packbits(bits, bitorder="little")
    buf[:packed.size] = packed
    return buf.view(np.uint32), bits


def _run(gpu, p, words, sat):
    if sat:
        os.environ["OAI4G_MOD_SAT"] = "1"
    try:
        pipe = gpu.TxPipeline(p, N_SF)
    finally:
        os.environ.pop("OAI4G_MOD_SAT", None)
    nosat = pipe.mod_nosat
    pipe.upload_ebits(words)
    pipe.modulate_only()
    pipe.sync()
    iq = pipe.iq()
    pipe.close()
    return nosat, iq


def _case(gpu, subframe):
    p = gpu.make_params("C3", subframe=subframe, subframe_step=0)
    probe = gpu.TxPipeline(p, N_SF, alloc=False)
    G = [probe.G(cw, subframe) for cw in range(2)]
    ew = probe.ebits_words
    probe.close()
    rng = np.random.default_rng(0xC3 + subframe)
    words = np.zeros((N_SF, 2, ew), dtype=np.uint32)
    bits = []
    for i, syms in enumerate(_patterns(G[0] // 6, rng)):
        row = []
        for cw in range(2):
            words[i, cw], b = _words(syms[cw], G[cw], ew)
            row.append(b)
        bits.append(row)
    return p, words, bits


def test_range_check_admits_c3_and_refuses_large_amplitudes(gpu):
    p = gpu.make_params("C3")
    pipe = gpu.TxPipeline(p, 1, alloc=False)
    assert pipe.mod_nosat                                  # 39 x 782.1 + 128 = 30629 <= 32767
    pipe.close()
    # amp 530: V = 572, 39 x 808.9 + 128 = 31676; amp 560: V = 604, 39 x 854.2 + 128 = 33442
    for amp, ok in ((530, True), (560, False), (1024, False), (4096, False)):
        p = gpu.make_params("C3")
        p.amp = amp
        pipe = gpu.TxPipeline(p, 1, alloc=False)
        assert pipe.mod_nosat == ok, amp
        pipe.close()
    p = gpu.make_params("C2")                              # TM1: no fused kernel
    pipe = gpu.TxPipeline(p, 1, alloc=False)
    assert not pipe.mod_nosat
    pipe.close()


@pytest.mark.parametrize("subframe", [7, 0, 5])
def test_fused_levels_equal_saturating_levels_on_adversarial_bits(gpu, subframe):
    p, words, _ = _case(gpu, subframe)
    ns, iq_ns = _run(gpu, p, words, sat=False)
    s, iq_sat = _run(gpu, p, words, sat=True)
    assert ns and not s
    assert iq_ns.any()
    for i in range(N_SF):
        assert np.array_equal(iq_ns[i], iq_sat[i]), (subframe, i)
    # the adversarial subframes do reach large sample values (the bound is not vacuous)
    pk = np.abs(iq_ns.view(np.int16).reshape(N_SF, -1).astype(np.int32)).max(axis=1)
    print("peak |sample| per pattern:", pk.tolist())
    assert pk[0] > 8000, pk


@pytest.mark.parametrize("subframe", [7, 0])
def test_fused_levels_equal_reference_chain_on_adversarial_bits(gpu, subframe):
    if O.ref_mod() is None or O.ref_ofdm() is None:
        pytest.skip("oracle/_ref not built")
    p, words, bits = _case(gpu, subframe)
    _, iq = _run(gpu, p, words, sat=False)
    fp = O.frame(100, Nid_cell=0, Ncp=0, nb_antennas_tx=2, mode1_flag=0)
    N, nsymb = fp.ofdm_symbol_size, fp.symbols_per_tti
    ra = [int(p.rb_alloc[i]) for i in range(4)]
    for i in (0, 1, 2, 3, 6):
        cws = []
        for cw in range(2):
            e = np.zeros(14 * 1200 * 6, dtype=np.uint8)
            e[:bits[i][cw].size] = bits[i][cw]
            cws.append(dict(e=e, mcs=19, mimo_mode=gpu.LARGE_CDD, rb_alloc=ra))
        ret, grids = O.ref_modulation(fp, p.amp, subframe, p.num_pdcch_symbols, cws)
        for a in range(2):
            g = np.ascontiguousarray(grids[a][subframe * nsymb * N:(subframe + 1) * nsymb * N])
            out = np.zeros(fp.samples_per_tti + 64, dtype=np.int32)
            O.ref_ofdm().ref_glue_normal_prefix_mod(O.P(g), O.P(out), nsymb, O.P(O.frame_geometry(fp)))
            assert np.array_equal(iq[i, a], out[:fp.samples_per_tti]), (subframe, i, a)


def test_full_grid_fused_levels_equal_saturating_levels(gpu):
    """The CRS kernel (CRS + PCFICH / PDCCH + PSS / SSS / PBCH / PHICH in the grid, bench --full-grid):
    the range check covers the static REs' values too; adversarial e bits over subframe indices 0..9
    give identical IQ on the fused and the saturating kernels."""
    import bench
    p = gpu.make_params("C3", subframe=0, subframe_step=1, with_crs=1)
    probe = gpu.TxPipeline(p, 10, alloc=False)
    G = [[probe.G(cw, sf) for cw in range(2)] for sf in range(10)]
    ew = probe.ebits_words
    probe.close()
    rng = np.random.default_rng(0xF6)
    words = np.zeros((10, 2, ew), dtype=np.uint32)
    for sf in range(10):
        syms = _patterns(G[sf][0] // 6, rng)[sf % N_SF]
        for cw in range(2):
            words[sf, cw], _ = _words(syms[cw], G[sf][cw], ew)
    out = []
    for sat in (False, True):
        if sat:
            os.environ["OAI4G_MOD_SAT"] = "1"
        try:
            pipe = gpu.TxPipeline(p, 10)
            bench.full_grid_setup(pipe, p, "C3")
        finally:
            os.environ.pop("OAI4G_MOD_SAT", None)
        assert pipe.mod_nosat == (not sat)
        pipe.upload_ebits(words)
        pipe.modulate_only()
        pipe.sync()
        out.append(pipe.iq())
        pipe.close()
    for sf in range(10):
        assert np.array_equal(out[0][sf], out[1][sf]), sf
