"""GPU parity: every drop-in entry point and the batched pipeline against the CPU oracle.

Bit-exact everywhere (integer, byte and fixed-point IQ work).  Inputs are seeded.
"""
import ctypes

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

RNG = np.random.default_rng(20261015)


def _rand_iq(n, amp, rng):
    x = rng.integers(-amp, amp + 1, size=2 * n).astype(np.int16)
    return x


@pytest.mark.parametrize("log2n", [6, 7, 8, 9, 10, 11])
def test_idft_bit_exact(gpu, log2n):
    n = 1 << log2n
    rng = np.random.default_rng(log2n)
    for trial in range(12):
        amp = [512, 3000, 32767][trial % 3]
        x = _rand_iq(n, amp, rng)
        if trial == 11:
            x[:] = rng.choice([-32768, 32767], size=2 * n).astype(np.int16)
        for scale in (1, 0):
            y = gpu.idft(x, scale)
            assert np.array_equal(y, O.idft(x, scale)), (log2n, trial, scale)


@pytest.mark.parametrize("log2n,cp", [(7, 9), (11, 144), (10, 72), (8, 18), (9, 36)])
def test_phy_ofdm_mod(gpu, log2n, cp):
    n = 1 << log2n
    nsym = 6
    grid = RNG.integers(-2000, 2000, size=2 * n * nsym).astype(np.int16).view(np.int32)
    out = gpu.ofdm_mod(grid, log2n, nsym, cp)
    ref = np.zeros(nsym * (n + cp), dtype=np.int32)
    O.orc().orc_ofdm_mod(O.P(grid), O.P(ref), log2n, nsym, cp)
    assert np.array_equal(out, ref)


def test_normal_prefix_mod(gpu):
    fp = gpu.frame_parms(100)
    ofp = O.frame(100)
    grid = RNG.integers(-3000, 3000, size=2 * 2048 * 7).astype(np.int16).view(np.int32)
    out = gpu.normal_prefix_mod(grid, fp, 7, np.zeros(30720, dtype=np.int32))
    ref = np.zeros(30720, dtype=np.int32)
    O.orc().orc_normal_prefix_mod(O.P(grid), O.P(ref), 7, ctypes.byref(ofp))
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("nbits", [8, 24, 936, 30576, 30576 + 5, 75376, 1])
def test_crc24(gpu, nbits):
    data = RNG.integers(0, 256, size=(nbits + 7) // 8 + 4, dtype=np.uint8)
    assert gpu.crc24a(data, nbits) == O.crc24a(data, nbits)
    assert gpu.crc24b(data, nbits) == O.crc24b(data, nbits)


def _qpp(K):
    import openair4g_amd  # noqa: F401
    idx = _qpp_index(K)
    return _QPP[idx]


_QPP = None


def _load_qpp():
    global _QPP
    rows = []
    import re
    src = open(O.ROOT + "/include/oai4g_qpp.c").read()
    for m in re.finditer(r"\{\s*(\d+),\s*(\d+),\s*(\d+)\}", src):
        rows.append(tuple(int(v) for v in m.groups()))
    _QPP = {k: (f1, f2) for k, f1, f2 in rows}
    return _QPP


@pytest.mark.parametrize("K", [40, 48, 104, 512, 528, 960, 1056, 2112, 5504, 6144])
def test_turbo_encoder(gpu, K):
    qpp = _QPP or _load_qpp()
    f1, f2 = qpp[K]
    c = RNG.integers(0, 256, size=K // 8, dtype=np.uint8)
    assert np.array_equal(gpu.turbo_encode(c, f1, f2), O.turbo_encode(c, f1, f2))


@pytest.mark.parametrize("K", [40, 960, 6144, 5504, 1056])
def test_subblock_and_rate_matching(gpu, K):
    qpp = _QPP or _load_qpp()
    f1, f2 = qpp[K]
    c = RNG.integers(0, 256, size=K // 8, dtype=np.uint8)
    d = O.turbo_encode(c, f1, f2)
    D = K + 4
    rtc_o, w_o, dfull_o = O.subblock(d, D)
    dfull = np.full(96 + 3 * D + 16, 2, dtype=np.uint8)
    dfull[96:96 + len(d)] = d
    rtc_g, w_g = gpu.subblock_interleave(dfull, D)
    assert rtc_g == rtc_o
    assert np.array_equal(w_g, w_o)
    for (G, C, r, Qm, rv) in [(60000, 5, 1, 4, 0), (1512, 1, 0, 2, 0), (86400, 6, 5, 6, 2), (30000, 3, 2, 2, 3)]:
        e_g = gpu.rate_match(rtc_o, G, w_o, C, r, Qm, rvidx=rv)
        e_o = O.rate_match(rtc_o, G, w_o, C, r, Qm, rvidx=rv)
        assert np.array_equal(e_g, e_o), (G, C, r, Qm, rv)


def test_rate_matching_rm_condition(gpu):
    """Kmimo=2 at large C hits the reference's limited-buffer refusal: E = 0."""
    K = 6144
    w = np.zeros(3 * 32 * ((K + 4 + 31) // 32), dtype=np.uint8)
    e = gpu.rate_match((K + 4 + 31) // 32, 200000, w, 13, 0, 6, Kmimo=2)
    assert len(e) == 0


@pytest.mark.parametrize("name,subframe", [("C1", 7), ("C2", 7), ("C3", 7), ("C2", 0), ("C3", 5), ("TM2", 7),
                                          ("TM2", 0), ("TM2S", 5)])
def test_dlsch_encoding_scrambling_modulation(gpu, name, subframe):
    """The drop-in dlsch_encoding -> dlsch_scrambling -> dlsch_modulation chain vs the oracle."""
    p = gpu.make_params(name, subframe=subframe)
    cfg = O.tx_cfg_from_params(p, subframe)
    fp = gpu.frame_parms(p.N_RB_DL, p.Nid_cell, 0, p.nb_antennas_tx, p.mode1_flag, 0)
    payloads = [RNG.integers(0, 256, size=p.TBS[cw] // 8 + 8, dtype=np.uint8) for cw in range(p.n_cw)]
    txd_o, txF_o, e_o = O.tx_subframe(cfg, [pl.copy() for pl in payloads], want_e=True)
    dls = []
    for cw in range(p.n_cw):
        dl = gpu.DlschHandle(Kmimo=p.Kmimo, Mdlharq=8, N_RB_DL=p.N_RB_DL)
        h = dl.h
        h.TBS = p.TBS[cw]
        h.mcs = p.mcs[cw]
        h.rvidx = 0
        h.round = 0
        h.mimo_mode = p.mimo_mode
        for i in range(4):
            h.rb_alloc[i] = p.rb_alloc[i]
        h.nb_rb = p.nb_rb
        h.Nl = 1
        dl.d.rnti = p.rnti
        a = payloads[cw].copy()
        assert gpu.dlsch_encoding(a, fp, p.num_pdcch_symbols, dl, subframe) == 0
        # CRC appended in place into the caller's buffer
        crc = O.crc24a(payloads[cw], p.TBS[cw]) >> 8
        A = p.TBS[cw] // 8
        assert list(a[A:A + 3]) == [(crc >> 16) & 255, (crc >> 8) & 255, crc & 255]
        G = O.get_G(p.N_RB_DL, 0, p.mode1_flag, 0, p.nb_rb, list(p.rb_alloc), gpu.lib().oai4g_get_Qm(p.mcs[cw]), 1,
                    p.num_pdcch_symbols, subframe)
        gpu.dlsch_scrambling(fp, dl, G, 0, 2 * subframe)
        e = dl.view("e", G)
        assert np.array_equal(e, e_o[cw][:G]), (name, cw)
        dls.append(dl)
    N = p.N_RB_DL and fp.ofdm_symbol_size
    txF = [np.zeros(10 * 14 * N, dtype=np.int32) for _ in range(p.nb_antennas_tx)]
    n_re = gpu.dlsch_modulation(txF, 512, subframe, fp, p.num_pdcch_symbols, dls[0], dls[1] if p.n_cw > 1 else None)
    assert n_re == _re_allocated(p, subframe), name
    for aa in range(p.nb_antennas_tx):
        got = txF[aa][subframe * 14 * N:(subframe + 1) * 14 * N]
        assert np.array_equal(got, txF_o[aa]), (name, aa)


def _re_allocated(p, subframe):
    """dlsch_modulation's return value from the oracle (ALAMOUTI also counts the pilot it steps
    over inside a pair, dlsch_modulation.c:868-876)."""
    cfg = O.tx_cfg_from_params(p, subframe)
    return O.modulation_count(cfg)


def _pipeline_check(gpu, name, n_sf, first_sf, step, check_idx=None, seed=7, **over):
    p = gpu.make_params(name, subframe=first_sf, subframe_step=step, **over)
    pipe = gpu.TxPipeline(p, n_sf)
    rng = np.random.default_rng(seed)
    pay = rng.integers(0, 256, size=(n_sf, p.n_cw, p.payload_stride), dtype=np.uint8)
    pipe.upload_payload(pay)
    pipe.run()
    pipe.sync()
    iq = pipe.iq()
    eb = pipe.ebits()
    idxs = range(n_sf) if check_idx is None else check_idx
    for i in idxs:
        sf = (first_sf + i * step) % 10
        cfg = O.tx_cfg_from_params(p, sf)
        txd_o, _, e_o = O.tx_subframe(cfg, [pay[i, cw] for cw in range(p.n_cw)], want_e=True)
        for cw in range(p.n_cw):
            G = pipe.G(cw, sf)
            assert np.array_equal(gpu.unpack_bits(eb[i, cw], G), e_o[cw][:G]), (name, i, cw)
        assert np.array_equal(iq[i], txd_o), (name, i)
    pipe.close()
    return iq


@pytest.mark.parametrize("name,n_sf,first,step", [("C1", 10, 0, 1), ("C2", 3, 7, 0), ("C3", 10, 0, 1),
                                                  ("C2", 10, 3, 1), ("TM2", 10, 0, 1), ("TM2S", 10, 0, 1),
                                                  ("C4", 10, 0, 1)])
def test_pipeline_bit_exact(gpu, name, n_sf, first, step):
    _pipeline_check(gpu, name, n_sf, first, step)


@pytest.mark.parametrize("name", ["C1", "C2", "C3", "TM2"])
def test_pipeline_extended_cp(gpu, name):
    """Extended cyclic prefix (12 symbols, one 512-sample-equivalent prefix): RE map with the
    extended pilot symbols, 6-symbol slots through PHY_ofdm_mod (ofdm_mod.c:252-259)."""
    _pipeline_check(gpu, name, 10, 0, 1, seed=3, Ncp=1)


@pytest.mark.parametrize("name", ["C3", "TM2"])
def test_pipeline_extended_cp_with_crs(gpu, name):
    p = gpu.make_params(name, subframe=0, subframe_step=1, Nid_cell=13, with_crs=1, Ncp=1)
    pipe = gpu.TxPipeline(p, 10)
    pay = np.random.default_rng(5).integers(0, 256, size=(10, p.n_cw, p.payload_stride), dtype=np.uint8)
    pipe.upload_payload(pay)
    pipe.run()
    pipe.sync()
    iq = pipe.iq()
    for i in range(10):
        txd_o, _, _ = O.tx_subframe(O.tx_cfg_from_params(p, i), [pay[i, cw] for cw in range(p.n_cw)])
        assert np.array_equal(iq[i], txd_o), (name, i)
    pipe.close()


@pytest.mark.parametrize("nid", [0, 1, 2, 5])
def test_pipeline_tm2_odd_bandwidth(gpu, nid):
    """ALAMOUTI on 15 PRB (odd N_RB: the middle RB straddles DC; PBCH/sync half-RB exclusions in
    subframes 0 and 5), every CRS shift class."""
    _pipeline_check(gpu, "TM2S", 10, 0, 1, seed=nid, N_RB_DL=15, rb_alloc=gpu.FULL_ALLOC_15, nb_rb=15,
                    num_pdcch_symbols=2, Nid_cell=nid)


@pytest.mark.parametrize("name,N_RB", [("C2", 25), ("C3", 25), ("TM2", 25), ("C2", 50), ("C3", 50), ("TM2", 50),
                                       ("C3", 15), ("C3", 6)])
def test_pipeline_bandwidths(gpu, name, N_RB):
    """5 MHz (25 PRB, idft512, odd N_RB: DC-straddling middle RB), 10 MHz (50 PRB, idft1024) and
    64-QAM TM3 on 3 / 1.4 MHz grids through the batched path, every subframe of a frame
    (PBCH/sync exclusions in 0 and 5)."""
    mcs = gpu.CONFIGS[name]["mcs"]
    alloc = {6: gpu.FULL_ALLOC_6, 15: gpu.FULL_ALLOC_15, 25: gpu.FULL_ALLOC_25, 50: gpu.FULL_ALLOC_50}[N_RB]
    _pipeline_check(gpu, name, 10, 0, 1, seed=N_RB, N_RB_DL=N_RB, rb_alloc=alloc, nb_rb=N_RB, num_pdcch_symbols=2,
                    TBS=tuple(gpu.tbs_bits(m, N_RB) if m else 0 for m in mcs))


@pytest.mark.parametrize("nid,ncp,crs", [(0, 0, 0), (13, 0, 1), (301, 0, 1), (5, 1, 0), (8, 1, 1)])
def test_pipeline_c4(gpu, nid, ncp, crs):
    """C4 (4 TX, 4-port large-delay CDD, build-defined): every subframe of a frame, every CRS
    shift class, normal / extended CP, with and without the 4-port CRS."""
    _pipeline_check(gpu, "C4", 10, 0, 1, seed=nid + 1, Nid_cell=nid, Ncp=ncp, with_crs=crs)


def test_pipeline_full_size_c4(gpu):
    """Bench-size C4 batch (1024 subframes per GPU): sampled bit-exact checks."""
    _pipeline_check(gpu, "C4", 1024, 7, 0, check_idx=[0, 511, 1023], seed=21)


def test_pipeline_full_size_c3(gpu):
    """Bench-size batch (C3, 2048 subframes): sampled bit-exact checks + determinism."""
    n_sf = 2048
    iq1 = _pipeline_check(gpu, "C3", n_sf, 7, 0, check_idx=[0, 1, 777, n_sf - 1], seed=11)
    iq2 = _pipeline_check(gpu, "C3", n_sf, 7, 0, check_idx=[], seed=11)
    assert np.array_equal(iq1, iq2)
    # every subframe carries signal on both antennas
    assert np.all(np.abs(iq1.view(np.int16)).reshape(n_sf, -1).max(axis=1) > 0)


# ---------------------------------------------------------------- CRS (A12)
@pytest.mark.parametrize("name,n_sf,first,step,nid", [("C1", 10, 0, 1, 0), ("C2", 4, 4, 1, 77), ("C3", 10, 0, 1, 301),
                                                      ("TM2", 10, 0, 1, 41)])
def test_pipeline_with_crs_bit_exact(gpu, name, n_sf, first, step, nid):
    p = gpu.make_params(name, subframe=first, subframe_step=step, Nid_cell=nid, with_crs=1)
    pipe = gpu.TxPipeline(p, n_sf)
    rng = np.random.default_rng(nid + n_sf)
    pay = rng.integers(0, 256, size=(n_sf, p.n_cw, p.payload_stride), dtype=np.uint8)
    pipe.upload_payload(pay)
    pipe.run()
    pipe.sync()
    iq = pipe.iq()
    for i in range(n_sf):
        sf = (first + i * step) % 10
        txd_o, _, _ = O.tx_subframe(O.tx_cfg_from_params(p, sf), [pay[i, cw] for cw in range(p.n_cw)])
        assert np.array_equal(iq[i], txd_o), (name, i)
    pipe.close()


@pytest.mark.parametrize("N_RB,nid,n_ant,mode1", [(6, 0, 1, 1), (100, 5, 2, 0), (50, 200, 2, 1), (15, 9, 2, 0)])
def test_generate_pilots_drop_in(gpu, N_RB, nid, n_ant, mode1):
    fp_o = O.frame(N_RB, nid, 0, n_ant, mode1)
    ref = O.generate_pilots(fp_o, 512, ntti=10)
    fp = gpu.FrameParms()
    gpu.lib().oai4g_init_frame_parms(ctypes.byref(fp), N_RB, nid, 0, n_ant, mode1, 0)
    rng = np.random.default_rng(N_RB)
    grids = [rng.integers(-1000, 1000, len(ref[a])).astype(np.int32) for a in range(n_ant)]
    pre = [g.copy() for g in grids]
    gpu.generate_pilots(grids, 512, fp, 10)
    for a in range(n_ant):
        pil = ref[a] != 0
        assert np.array_equal(grids[a][pil], ref[a][pil])          # pilots overwritten (=)
        assert np.array_equal(grids[a][~pil], pre[a][~pil])        # everything else untouched
    sym = np.zeros(fp.ofdm_symbol_size, dtype=np.int32)
    gpu.lte_dl_cell_spec(sym, 512, fp, 3, 1, 0)
    N = fp.ofdm_symbol_size
    assert np.array_equal(sym, ref[0][(1 * 14 + 11) * N:(1 * 14 + 12) * N])   # slot 3 = subframe 1, symbol 11


# k_encode stages the e words per half of the code blocks (blocks [0, ceil(C/2)) then the rest,
# a word shared by the halves carried over): every MCS at 100 PRB TM1 covers C = 1..13, odd and
# even C, half boundaries inside and on word edges, and circular-buffer repetition (E > Nnn at
# low MCS with C > 1); each subframe index varies G and the per-block E split
@pytest.mark.parametrize("mcs", [0, 3, 5, 7, 9, 12, 16, 20, 24, 27])
def test_pipeline_every_block_count(gpu, mcs):
    _pipeline_check(gpu, "C2", 10, 0, 1, mcs=[mcs], TBS=None)


def test_tx_batch_refuses_misaligned_iq(gpu):
    """The 2048-point modulator stores sample pairs as 8-byte words: oai4g_tx_batch refuses an IQ
    buffer that is not 8-byte aligned (returns -1 with a message) instead of faulting."""
    pipe = gpu.TxPipeline(gpu.make_params("C3"), 1)
    L = pipe.L
    assert L.oai4g_tx_batch(pipe.cfg, 1, pipe.d_payload, pipe.d_work, pipe.d_iq + 4, None) == -1
    assert b"8-byte aligned" in L.oai4g_last_error()
    ms = (ctypes.c_float * 2)()
    assert L.oai4g_tx_batch_timed(pipe.cfg, 1, pipe.d_payload, pipe.d_work, pipe.d_iq + 4, None, ms) == -1
    pipe.run()   # the aligned buffer still works
    pipe.sync()
