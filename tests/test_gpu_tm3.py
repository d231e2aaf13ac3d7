"""GPU parity of the TM3 (LARGE_CDD, 2 TX ports) receive chain — dlsch_extract_rbs_dual,
dlsch_channel_level_TM3, prec2A_TM3 + dlsch_channel_compensation_TM3, dlsch_detection_mrc, the
codeword-0 LLRs (k_rx_level_tm3 / k_rx_llr_tm3) — against the oracle restatement
(tests/test_rx_tm3_cpu.py pins it by the decoding loop): the drop-in on full-range random grids and
estimates (saturation / wrap paths, 1 and 2 receive antennas, odd N_RB_DL with the PBCH / sync
subframes), and the headline configuration's receive loop on the GPU: C3 TxPipeline (both ports'
CRS) -> channel H = I -> FepBatch over 2 antennas -> 4 channel-estimation batches -> RxBatchTM3 ->
RM-rx / deinterleaving / turbo decoding: codeword 0 comes back, LLRs bit-exact vs the oracle."""
import numpy as np
import pytest

import oracle_lib as O
from test_rx_cpu import alloc, decode_tb, dual_alloc
from test_rx_tm3_cpu import c3_params

pytestmark = pytest.mark.gpu

RAND = [(100, 6, 6, 19, 1, 7, 2, None), (50, 4, 2, 12, 2, 3, 2, None), (100, 6, 4, 22, 3, 0, 2, None),
        (25, 6, 6, 19, 1, 6, 2, None), (25, 4, 4, 14, 2, 4, 1, None), (15, 6, 6, 20, 1, 3, 2, None),
        (50, 6, 6, 19, 1, 5, 2, None),
        (100, 4, 6, 10, 2, 8, 1, [0xF0F0F0F0, 0x0000FFFF, 0, 0x3])]


@pytest.mark.parametrize("N_RB,Qm0,Qm1,mcs,npd,sf,nb_rx,ra", RAND)
def test_gpu_tm3_random_inputs(gpu, N_RB, Qm0, Qm1, mcs, npd, sf, nb_rx, ra):
    ra = ra or dual_alloc(N_RB)
    fo = O.frame(N_RB, Nid_cell=N_RB + sf, nb_antennas_tx=2, mode1_flag=0)
    fg = gpu.frame_parms(N_RB, Nid_cell=N_RB + sf, nb_antennas_tx=2, mode1_flag=0)
    n = fo.symbols_per_tti * fo.ofdm_symbol_size
    rng = np.random.default_rng(N_RB * 7 + Qm0 + sf)
    for scale in (2 ** 31 - 1, 3000):
        rx = [rng.integers(-scale, scale, n, dtype=np.int64).astype(np.int32) for _ in range(nb_rx)]
        est = {(p, a): rng.integers(-scale, scale, n, dtype=np.int64).astype(np.int32) for p in (0, 1)
               for a in range(nb_rx)}
        lo, so = O.rx_pdsch_tm3(fo, rx, est, ra, Qm0, Qm1, mcs, npd, sf)
        lg, sg = gpu.rx_pdsch_tm3(fg, rx, est, ra, Qm0, Qm1, mcs, npd, sf)
        assert sg == so and np.array_equal(lg, lo), (scale, so, sg)


@pytest.mark.parametrize("N_RB,sf", [(25, 7), (15, 3)])
def test_gpu_dual_extraction_odd_full_allocation_refused(gpu, N_RB, sf):
    """Odd N_RB_DL, every RB allocated: the reference's dl_ch0_ext moves 144 slots per full RB in
    non-pilot symbols (dlsch_demodulation.c:3932-3936), so its port-0 estimates go stale from the
    second full RB on — refused by the TM3 and TM2 drop-ins, as by the oracle."""
    fg = gpu.frame_parms(N_RB, nb_antennas_tx=2, mode1_flag=0)
    fo = O.frame(N_RB, nb_antennas_tx=2, mode1_flag=0)
    n = fg.symbols_per_tti * fg.ofdm_symbol_size
    z = np.ones(n, np.int32)
    est = {(p, a): z for p in (0, 1) for a in (0, 1)}
    with pytest.raises(gpu.OAI4GError):
        gpu.rx_pdsch_tm3(fg, [z, z], est, alloc(N_RB), 6, 6, 19, 1, sf)
    with pytest.raises(gpu.OAI4GError):
        gpu.rx_pdsch_tm2(fg, [z, z], est, alloc(N_RB), 4, 1, sf)
    assert O.rx_pdsch_tm2(fo, [z, z], est, alloc(N_RB), 4, 1, sf, check=False)[0] is None


def test_gpu_tm3_refuses_holes(gpu):
    """Odd N_RB_DL, subframe 0: the dual extraction's skip_half = 2 pilot branch (symbol 7 of the
    PBCH rows) leaves ext slots unwritten that the stream reaches — refused on both sides."""
    fg = gpu.frame_parms(25, nb_antennas_tx=2, mode1_flag=0)
    n = fg.symbols_per_tti * fg.ofdm_symbol_size
    z = np.zeros(n, np.int32)
    with pytest.raises(gpu.OAI4GError):
        gpu.rx_pdsch_tm3(fg, [z, z], {(p, a): z for p in (0, 1) for a in (0, 1)}, alloc(25), 6, 6, 19, 1, 0)


@pytest.mark.parametrize("N_RB,mcs,npd,sf", [(100, 19, 1, 7), (100, 16, 2, 3), (50, 19, 1, 8)])
def test_gpu_tm3_receive_loop(gpu, N_RB, mcs, npd, sf):
    n_tx, n_sf = 3, 2
    p = c3_params(N_RB, mcs, npd, sf)
    p.subframe_step = 1
    pipe = gpu.TxPipeline(p, n_tx)
    rng = np.random.default_rng(mcs + N_RB)
    pay = rng.integers(0, 256, size=(n_tx, 2, p.payload_stride), dtype=np.uint8)
    pipe.upload_payload(pay)
    pipe.run()
    pipe.sync()
    iq = pipe.iq()                                      # [n_tx][2 antennas][spt]: H = I, RX a <- TX a
    fg = gpu.frame_parms(N_RB, nb_antennas_tx=2, mode1_flag=0)
    fep = gpu.FepBatch(fg, n_tx, 2)
    fep.upload(iq)
    fep.run()
    Qm = 4 if mcs < 17 else 6
    rx = gpu.RxBatchTM3(fg, dual_alloc(N_RB), Qm, Qm, mcs, npd, p.rnti, n_sf, nb_rx=2, first_subframe=sf)
    rx.estimate(fep.d_rxF, first_subframe=sf)
    rx.launch(fep.d_rxF, unscramble=1)
    llr = rx.llrs()
    rxF = fep.result()                                   # [n_tx][2][nsymb][N]
    N = fg.ofdm_symbol_size
    fo = O.frame(N_RB, nb_antennas_tx=2, mode1_flag=0)
    for i in range(n_sf):
        s = (sf + i) % 10
        est = {(pp, a): O.chest_subframe(fo, rxF[i, a].ravel(), rxF[i + 1, a, 0], s, p=pp) for pp in (0, 1)
               for a in (0, 1)}
        lo, _ = O.rx_pdsch_tm3(fo, [rxF[i, 0].ravel(), rxF[i, 1].ravel()], est, alloc(N_RB), Qm, Qm, mcs, npd, s)
        G = rx.llr_count(s)
        u = np.zeros(32 * (1 + G // 32), np.int16)
        u[:G] = lo
        O.dlsch_unscrambling(u, G, (p.rnti << 14) + (s << 9) + fo.Nid_cell)
        assert len(lo) == G and np.array_equal(llr[i, :G], u[:G]), s
        res, tb = decode_tb(llr[i, :G], G, p.TBS[0], Qm)
        assert all(it <= 4 for it, _ in res), (s, [it for it, _ in res])
        assert np.array_equal(tb, pay[i, 0, :p.TBS[0] // 8]), s
    rx.close()
    fep.close()
    pipe.close()


QQ_RAND = [(100, 9, 1, 7, 2, None), (50, 5, 2, 3, 1, None), (25, 7, 1, 6, 2, None), (15, 3, 2, 4, 2, None),
           (100, 8, 3, 8, 2, [0xF0F0F0F0, 0x0000FFFF, 0, 0x3])]


@pytest.mark.parametrize("N_RB,mcs,npd,sf,nb_rx,ra", QQ_RAND)
def test_gpu_tm3_qpsk_two_codewords_random_inputs(gpu, N_RB, mcs, npd, sf, nb_rx, ra):
    """Both codewords QPSK: the dual-stream correlation and the interference-aware qpsk_qpsk LLRs of
    both streams, bit-exact against the oracle on full-range random grids and estimates."""
    ra = ra or dual_alloc(N_RB)
    fo = O.frame(N_RB, Nid_cell=N_RB + sf, nb_antennas_tx=2, mode1_flag=0)
    fg = gpu.frame_parms(N_RB, Nid_cell=N_RB + sf, nb_antennas_tx=2, mode1_flag=0)
    n = fo.symbols_per_tti * fo.ofdm_symbol_size
    rng = np.random.default_rng(N_RB * 5 + mcs + sf)
    for scale in (2 ** 31 - 1, 3000):
        rx = [rng.integers(-scale, scale, n, dtype=np.int64).astype(np.int32) for _ in range(nb_rx)]
        est = {(p, a): rng.integers(-scale, scale, n, dtype=np.int64).astype(np.int32) for p in (0, 1)
               for a in range(nb_rx)}
        a0, a1, so = O.rx_pdsch_tm3_qq(fo, rx, est, ra, mcs, npd, sf)
        g0, g1, sg = gpu.rx_pdsch_tm3_2cw(fg, rx, est, ra, mcs, npd, sf)
        assert sg == so and np.array_equal(g0, a0) and np.array_equal(g1, a1), (scale, so, sg)


@pytest.mark.parametrize("N_RB,mcs,npd,sf,nb_rx", [(100, 9, 1, 7, 2), (50, 6, 2, 3, 1)])
def test_gpu_tm3_qpsk_receive_loop_both_codewords(gpu, N_RB, mcs, npd, sf, nb_rx):
    """C3-shaped TM3 with both codewords QPSK through the GPU: TxPipeline -> channel H = [[2, 1],
    [1, 2]] -> FepBatch -> 4 estimations -> RxBatchTM3.launch_2cw -> both transport blocks decode."""
    n_tx, n_sf = 3, 2
    p = c3_params(N_RB, mcs, npd, sf)
    p.subframe_step = 1
    pipe = gpu.TxPipeline(p, n_tx)
    rng = np.random.default_rng(mcs + N_RB + 3)
    pay = rng.integers(0, 256, size=(n_tx, 2, p.payload_stride), dtype=np.uint8)
    pipe.upload_payload(pay)
    pipe.run()
    pipe.sync()
    t16 = pipe.iq().view(np.int16).astype(np.int64)              # [n_tx][2][spt * 2]
    H = [[2, 1], [1, 2]][:nb_rx]
    rxs = [np.clip(H[a][0] * t16[:, 0] + H[a][1] * t16[:, 1], -32768, 32767).astype(np.int16).view(np.int32)
           for a in range(nb_rx)]
    iq = np.ascontiguousarray(np.stack(rxs, axis=1))
    fg = gpu.frame_parms(N_RB, nb_antennas_tx=2, mode1_flag=0)
    fep = gpu.FepBatch(fg, n_tx, nb_rx)
    fep.upload(iq)
    fep.run()
    rx = gpu.RxBatchTM3(fg, dual_alloc(N_RB), 2, 2, mcs, npd, p.rnti, n_sf, nb_rx=nb_rx, first_subframe=sf)
    rx.estimate(fep.d_rxF, first_subframe=sf)
    rx.launch_2cw(fep.d_rxF, unscramble=1)
    l0, l1 = rx.llrs(), rx.llrs1()
    rxF = fep.result()
    fo = O.frame(N_RB, nb_antennas_tx=2, mode1_flag=0)
    for i in range(n_sf):
        s_ = (sf + i) % 10
        est = {(pp, a): O.chest_subframe(fo, rxF[i, a].ravel(), rxF[i + 1, a, 0], s_, p=pp) for pp in (0, 1)
               for a in range(nb_rx)}
        a0, a1, _ = O.rx_pdsch_tm3_qq(fo, [rxF[i, a].ravel() for a in range(nb_rx)], est, alloc(N_RB), mcs, npd, s_)
        G = rx.llr_count(s_)
        for cw, (gl, ol) in enumerate(((l0, a0), (l1, a1))):
            u = np.zeros(32 * (1 + G // 32), np.int16)
            u[:G] = ol
            O.dlsch_unscrambling(u, G, (p.rnti << 14) + (s_ << 9) + fo.Nid_cell)
            assert len(ol) == G and np.array_equal(gl[i, :G], u[:G]), (s_, cw)
            res, tb = decode_tb(gl[i, :G], G, p.TBS[cw], 2)
            assert all(it <= 4 for it, _ in res), (s_, cw, [it for it, _ in res])
            assert np.array_equal(tb, pay[i, cw, :p.TBS[cw] // 8]), (s_, cw)
    rx.close()
    fep.close()
    pipe.close()


QX_RAND = [(100, 4, 9, 1, 7, 2, None), (50, 6, 5, 2, 3, 1, None), (25, 4, 7, 1, 6, 2, None),
           (15, 6, 3, 2, 4, 2, None), (100, 6, 8, 3, 8, 2, [0xF0F0F0F0, 0x0000FFFF, 0, 0x3]),
           (50, 2, 6, 1, 2, 2, None)]


@pytest.mark.parametrize("N_RB,Qm1,mcs,npd,sf,nb_rx,ra", QX_RAND)
def test_gpu_tm3_qpsk_codeword0_random_inputs(gpu, N_RB, Qm1, mcs, npd, sf, nb_rx, ra):
    """Codeword 0 QPSK through the drop-in rx_pdsch_tm3: qpsk_qam16 / qpsk_qam64 against a 16 / 64-QAM
    codeword 1 (interferer magnitude dl_ch_mag1 of antenna 0), qpsk_qpsk's codeword 0 when both are
    QPSK; bit-exact against the oracle on full-range random grids and estimates."""
    ra = ra or dual_alloc(N_RB)
    fo = O.frame(N_RB, Nid_cell=N_RB + sf, nb_antennas_tx=2, mode1_flag=0)
    fg = gpu.frame_parms(N_RB, Nid_cell=N_RB + sf, nb_antennas_tx=2, mode1_flag=0)
    n = fo.symbols_per_tti * fo.ofdm_symbol_size
    rng = np.random.default_rng(N_RB * 3 + Qm1 + mcs + sf)
    for scale in (2 ** 31 - 1, 3000, 300):
        rx = [rng.integers(-scale, scale, n, dtype=np.int64).astype(np.int32) for _ in range(nb_rx)]
        est = {(p, a): rng.integers(-scale, scale, n, dtype=np.int64).astype(np.int32) for p in (0, 1)
               for a in range(nb_rx)}
        lo, so = O.rx_pdsch_tm3(fo, rx, est, ra, 2, Qm1, mcs, npd, sf)
        lg, sg = gpu.rx_pdsch_tm3(fg, rx, est, ra, 2, Qm1, mcs, npd, sf)
        assert sg == so and np.array_equal(lg, lo), (scale, so, sg)


@pytest.mark.parametrize("N_RB,mcs0,mcs1,npd,sf", [(100, 9, 19, 1, 7), (50, 7, 14, 2, 3)])
def test_gpu_tm3_qpsk_with_qam_interferer_receive_loop(gpu, N_RB, mcs0, mcs1, npd, sf):
    """TM3 with codeword 0 QPSK and codeword 1 16 / 64-QAM through the GPU: TxPipeline -> H = [[2, 1],
    [1, 2]] -> FepBatch -> 4 estimations -> RxBatchTM3 (qpsk_qam16 / qpsk_qam64) -> codeword 0 decodes,
    LLRs bit-exact against the oracle's loop."""
    import openair4g_amd as oai
    n_tx, n_sf = 3, 2
    p = oai.make_params("C3", subframe=sf, N_RB_DL=N_RB, nb_rb=N_RB, rb_alloc=alloc(N_RB), mcs=[mcs0, mcs1], TBS=None,
                        num_pdcch_symbols=npd, with_crs=1, Nid_cell=0)
    p.subframe_step = 1
    pipe = gpu.TxPipeline(p, n_tx)
    rng = np.random.default_rng(mcs0 + mcs1 + N_RB)
    pay = rng.integers(0, 256, size=(n_tx, 2, p.payload_stride), dtype=np.uint8)
    pipe.upload_payload(pay)
    pipe.run()
    pipe.sync()
    t16 = pipe.iq().view(np.int16).astype(np.int64)
    H = [[2, 1], [1, 2]]
    rxs = [np.clip(H[a][0] * t16[:, 0] + H[a][1] * t16[:, 1], -32768, 32767).astype(np.int16).view(np.int32)
           for a in range(2)]
    iq = np.ascontiguousarray(np.stack(rxs, axis=1))
    fg = gpu.frame_parms(N_RB, nb_antennas_tx=2, mode1_flag=0)
    fep = gpu.FepBatch(fg, n_tx, 2)
    fep.upload(iq)
    fep.run()
    Qm1 = 4 if mcs1 < 17 else 6
    rx = gpu.RxBatchTM3(fg, dual_alloc(N_RB), 2, Qm1, mcs0, npd, p.rnti, n_sf, nb_rx=2, first_subframe=sf)
    rx.estimate(fep.d_rxF, first_subframe=sf)
    rx.launch(fep.d_rxF, unscramble=1)
    llr = rx.llrs()
    rxF = fep.result()
    fo = O.frame(N_RB, nb_antennas_tx=2, mode1_flag=0)
    for i in range(n_sf):
        s_ = (sf + i) % 10
        est = {(pp, a): O.chest_subframe(fo, rxF[i, a].ravel(), rxF[i + 1, a, 0], s_, p=pp) for pp in (0, 1)
               for a in range(2)}
        lo, _ = O.rx_pdsch_tm3(fo, [rxF[i, 0].ravel(), rxF[i, 1].ravel()], est, alloc(N_RB), 2, Qm1, mcs0, npd, s_)
        G = rx.llr_count(s_)
        u = np.zeros(32 * (1 + G // 32), np.int16)
        u[:G] = lo
        O.dlsch_unscrambling(u, G, (p.rnti << 14) + (s_ << 9) + fo.Nid_cell)
        assert len(lo) == G and np.array_equal(llr[i, :G], u[:G]), s_
        res, tb = decode_tb(llr[i, :G], G, p.TBS[0], 2)
        assert all(it <= 4 for it, _ in res), (s_, [it for it, _ in res])
        assert np.array_equal(tb, pay[i, 0, :p.TBS[0] // 8]), s_
    rx.close()
    fep.close()
    pipe.close()


@pytest.mark.parametrize("N_RB,Qm0,Qm1,mcs,npd,sf,nb_rx,ecp", [(100, 6, 6, 19, 1, 7, 2, 0), (50, 4, 2, 12, 2, 3, 1, 0),
                                                               (25, 2, 6, 7, 1, 6, 2, 0), (100, 2, 2, 9, 3, 8, 2, 0),
                                                               (50, 6, 4, 20, 1, 2, 2, 1), (15, 4, 4, 12, 2, 6, 2, 1)])
def test_gpu_tm3_from_pilot_rows_equals_estimate_planes(gpu, N_RB, Qm0, Qm1, mcs, npd, sf, nb_rx, ecp):
    """oai4g_chest_batch_pilots + oai4g_rx_batch_tm3_pilots (the demodulator forms the estimate rows
    from the 5 pilot rows with the estimator's temporal interpolation) against the four 14-row
    estimate planes + oai4g_rx_batch_tm3: bit-identical LLRs on random FEP outputs, both CP types,
    every codeword-0 LLR family (both codewords too when both are QPSK)."""
    import ctypes
    fg = gpu.frame_parms(N_RB, Nid_cell=N_RB + sf, nb_antennas_tx=2, mode1_flag=0, Ncp=ecp)
    n_sf, N, nsymb = 3, fg.ofdm_symbol_size, fg.symbols_per_tti
    rng = np.random.default_rng(N_RB + mcs + 17 * ecp)
    for scale in (3000, 2 ** 31 - 1):
        rxF = rng.integers(-scale, scale, (n_sf + 1) * nb_rx * nsymb * N, dtype=np.int64).astype(np.int32)
        L = gpu.lib()
        d = L.oai4g_dev_alloc(rxF.nbytes)
        assert d and L.oai4g_memcpy_h2d(d, rxF.ctypes.data, rxF.nbytes) == 0
        rx = gpu.RxBatchTM3(fg, dual_alloc(N_RB), Qm0, Qm1, mcs, npd, 0x1234, n_sf, nb_rx=nb_rx, first_subframe=sf)
        two = Qm0 == 2 and Qm1 == 2
        rx.estimate(d, first_subframe=sf)
        rx.launch_2cw(d) if two else rx.launch(d)
        a0 = rx.llrs()
        a1 = rx.llrs1() if two else None
        rx.estimate_pilots(d, first_subframe=sf)
        rx.launch_2cw_pilots(d) if two else rx.launch_pilots(d)
        b0 = rx.llrs()
        assert np.array_equal(a0, b0), scale
        if two:
            assert np.array_equal(a1, rx.llrs1()), scale
        rx.close()
        L.oai4g_dev_free(ctypes.c_void_p(d))
