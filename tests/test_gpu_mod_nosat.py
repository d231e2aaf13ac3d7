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
LEVELS = {2: None, 4: [10362, 31086, -10362, -31086], 6: [15169, 5057, 25281, 35393, -15169, -5057, -25281, -35393]}


def _level(v, Qm):
    """qam_map's (I, Q) levels of symbol value v (bit j = the RE's j-th e bit), raw table values;
    QPSK: bit 0 / 1 set = negative I / Q"""
    if Qm == 2:
        return (-1 if v & 1 else 1), (-1 if v & 2 else 1)
    if Qm == 4:
        ir, ii = ((v & 1) << 1) | ((v >> 2) & 1), (v & 2) | ((v >> 3) & 1)
    else:
        ir = ((v & 1) << 2) | (((v >> 2) & 1) << 1) | ((v >> 4) & 1)
        ii = (((v >> 1) & 1) << 2) | (((v >> 3) & 1) << 1) | ((v >> 5) & 1)
    return LEVELS[Qm][ir], LEVELS[Qm][ii]


def _corners(Qm):
    """symbol values of the outer corners (+,+), (-,+), (-,-), (+,-)"""
    top = 1 if Qm == 2 else max(LEVELS[Qm])
    out = []
    for si, sq in ((1, 1), (-1, 1), (-1, -1), (1, -1)):
        out.append(next(v for v in range(1 << Qm) if _level(v, Qm) == (si * top, sq * top)))
    return np.array(out)


def _patterns(n_re, Qm, rng):
    """(cw0 symbols, cw1 symbols) per subframe of the batch"""
    idx = np.arange(n_re)
    rot = _corners(Qm)
    PP, MM, PM = rot[0], rot[2], rot[3]
    out = [
        (np.full(n_re, PP), np.full(n_re, PP)),                         # all REs one corner: class DC bins
        (np.full(n_re, PP), np.full(n_re, MM)),                         # opposed codewords: y0 ~ 0, |d| max
        (np.where((idx >> 1) & 1, MM, PP), np.where((idx >> 1) & 1, MM, PP)),   # period 4: the mod-2 classes' Nyquist
        (rot[idx & 3], rot[idx & 3]),                                   # quarter turn per RE
        (rot[(idx >> 1) & 3], rot[3 - ((idx >> 1) & 3)]),              # both codewords, opposite turns
        (rot[rng.integers(0, 4, n_re)], rot[rng.integers(0, 4, n_re)]),   # random corners
        (rng.integers(0, 1 << Qm, n_re), rng.integers(0, 1 << Qm, n_re)),   # random symbols
        (np.full(n_re, MM), np.full(n_re, PM)),
    ]
    assert len(out) == N_SF
    return out


def _words(sym, Qm, G, n_words):
    bits = ((np.asarray(sym, dtype=np.uint32)[:, None] >> np.arange(Qm, dtype=np.uint32)) & 1).astype(np.uint8).ravel()
    assert bits.size == G
    buf = np.zeros(n_words * 4, dtype=np.uint8)
    packed = np.packbits(bits, bitorder="little")
    buf[:packed.size] = packed
    return buf.view(np.uint32), bits


def _run(gpu, p, words, sat, n_sf=N_SF, setup=None):
    if sat:
        os.environ["OAI4G_MOD_SAT"] = "1"
    try:
        pipe = gpu.TxPipeline(p, n_sf)
        if setup:
            setup(pipe)
    finally:
        os.environ.pop("OAI4G_MOD_SAT", None)
    nosat = pipe.mod_nosat
    pipe.upload_ebits(words)
    pipe.modulate_only()
    pipe.sync()
    iq = pipe.iq()
    pipe.close()
    return nosat, iq


def _case(gpu, subframe, name="C3", step=0, n_sf=N_SF, **over):
    """adversarial packed e-bit words: batch element i (subframe index subframe + i step) carries
    pattern i mod N_SF on every codeword"""
    p = gpu.make_params(name, subframe=subframe, subframe_step=step, **over)
    probe = gpu.TxPipeline(p, n_sf, alloc=False)
    sfs = [(subframe + i * step) % 10 for i in range(n_sf)]
    G = [[probe.G(cw, sf) for cw in range(p.n_cw)] for sf in sfs]
    ew = probe.ebits_words
    probe.close()
    Qm = [gpu.lib().oai4g_get_Qm(p.mcs[cw]) for cw in range(p.n_cw)]
    rng = np.random.default_rng(0xC3 + subframe + 101 * len(name))
    words = np.zeros((n_sf, p.n_cw, ew), dtype=np.uint32)
    bits = []
    for i in range(n_sf):
        row = []
        for cw in range(p.n_cw):
            syms = _patterns(G[i][cw] // Qm[cw], Qm[cw], rng)[i % N_SF][cw]
            words[i, cw], b = _words(syms, Qm[cw], G[i][cw], ew)
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
    for name in ("C2", "TM2", "C4"):                       # every 2048-point transmit mode
        pipe = gpu.TxPipeline(gpu.make_params(name), 1, alloc=False)
        assert pipe.mod_nosat, name
        pipe.close()
    pipe = gpu.TxPipeline(gpu.make_params("C1"), 1, alloc=False)   # 128 points: no fused kernel
    assert not pipe.mod_nosat
    pipe.close()


@pytest.mark.parametrize("name,subframe", [("C3", 7), ("C3", 0), ("C3", 5), ("C2", 7), ("TM2", 7), ("TM2", 0),
                                            ("C4", 7), ("C4", 5)])
def test_fused_levels_equal_saturating_levels_on_adversarial_bits(gpu, name, subframe):
    p, words, _ = _case(gpu, subframe, name)
    ns, iq_ns = _run(gpu, p, words, sat=False)
    s, iq_sat = _run(gpu, p, words, sat=True)
    assert ns and not s
    assert iq_ns.any()
    for i in range(N_SF):
        assert np.array_equal(iq_ns[i], iq_sat[i]), (subframe, i)
    # the adversarial subframes do reach large sample values (the bound is not vacuous)
    pk = np.abs(iq_ns.view(np.int16).reshape(N_SF, -1).astype(np.int32)).max(axis=1)
    print("peak |sample| per pattern:", pk.tolist())
    if name in ("C3", "C2"):
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


@pytest.mark.parametrize("name", ["C3", "C2", "C4"])
def test_full_grid_fused_levels_equal_saturating_levels(gpu, name):
    """The CRS kernels (CRS + PCFICH / PDCCH + PSS / SSS / PBCH / PHICH in the grid, bench --full-grid):
    the range check covers the static REs' values too; adversarial e bits over subframe indices 0..9
    give identical IQ on the fused and the saturating kernels."""
    import bench
    p, words, _ = _case(gpu, 0, name, step=1, n_sf=10, with_crs=1)
    setup = lambda pipe: bench.full_grid_setup(pipe, p, name)   # noqa: E731
    ns, iq_ns = _run(gpu, p, words, False, n_sf=10, setup=setup)
    s, iq_sat = _run(gpu, p, words, True, n_sf=10, setup=setup)
    assert ns and not s
    for sf in range(10):
        assert np.array_equal(iq_ns[sf], iq_sat[sf]), (name, sf)
