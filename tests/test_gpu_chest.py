"""GPU parity of the downlink channel estimation (lte_dl_channel_estimation, high_speed_flag = 1;
SURVEY §8f item 3) against the oracle restatement (tests/test_chest_cpu.py pins it to the
reference's filt96_32.h and to the decoding loop): the drop-in call by call on full-range random
grids (the saturating adds of overlapping filter responses, the mulhi/shift wraps, the temporal
interpolation rows), the batched estimator of consecutive subframes, and the closed loop on the
GPU: TX (with CRS) -> FEP -> estimation -> demodulation -> turbo decoding recovers the payload."""
import numpy as np
import pytest

import oracle_lib as O
from test_rx_cpu import alloc, decode_tb, params

pytestmark = pytest.mark.gpu


def test_gpu_filters_equal_oracle(gpu):
    for k in range(6):
        assert np.array_equal(gpu.chest_filters(k), O.chest_filters(k)), k
        assert np.array_equal(gpu.chest_dc_filters(k), O.chest_dc_filters(k)), k


CASES = [(100, 0, 0, 0), (100, 301, 1, 0), (50, 7, 0, 1), (6, 2, 1, 0), (6, 11, 0, 1), (50, 4, 1, 1), (100, 88, 1, 1),
         # odd N_RB_DL: the 25-PRB DC pair, the 15-PRB second-half start 1 + nushift + 3 p
         (25, 0, 0, 0), (25, 13, 1, 0), (25, 30, 0, 1), (15, 4, 0, 0), (15, 9, 1, 1), (15, 2, 1, 0)]


@pytest.mark.parametrize("N_RB,nid,p,Ncp", CASES)
def test_gpu_drop_in_call_sequence(gpu, N_RB, nid, p, Ncp):
    fo = O.frame(N_RB, Nid_cell=nid, Ncp=Ncp, nb_antennas_tx=2, mode1_flag=0)
    fg = gpu.frame_parms(N_RB, Nid_cell=nid, Ncp=Ncp, nb_antennas_tx=2, mode1_flag=0)
    N, nsymb = fo.ofdm_symbol_size, fo.symbols_per_tti
    lp = 4 if Ncp == 0 else 3
    rng = np.random.default_rng(N_RB + nid)
    g = O.gold_table(fo)
    e0 = rng.integers(-2**31, 2**31 - 1, nsymb * N, dtype=np.int64).astype(np.int32)
    eo, eg = e0.copy(), e0.copy()
    for sf in (0, 4, 9):
        for scale in (2**15, 700):
            y = (rng.integers(-scale, scale, (nsymb * N, 2)).astype(np.int16)).view(np.int32).ravel()
            for Ns, l, sym in ((2 * sf, 0, 0), (2 * sf, lp, lp), (2 * sf + 1, 0, nsymb // 2),
                               (2 * sf + 1, lp, nsymb // 2 + lp)):
                O.dl_channel_estimation(fo, g, y, eo, Ns, p, l, sym)
                gpu.lte_dl_channel_estimation(fg, y, eg, Ns, p, l, sym)
                assert np.array_equal(eg, eo), (sf, scale, sym)


def test_gpu_drop_in_rejects(gpu):
    fg = gpu.frame_parms(50)
    est = np.zeros(14 * fg.ofdm_symbol_size, np.int32)
    y = np.zeros_like(est)
    with pytest.raises(gpu.OAI4GError):
        gpu.lte_dl_channel_estimation(fg, y, est, 0, 2, 0, 0)        # port 2
    with pytest.raises(gpu.OAI4GError):
        gpu.lte_dl_channel_estimation(fg, y, est, 0, 0, 0, 3)        # not a pilot symbol


@pytest.mark.parametrize("N_RB,nid,Ncp,first", [(100, 17, 0, 3), (6, 1, 0, 8), (50, 40, 1, 0), (100, 5, 1, 9),
                                                 (25, 3, 0, 7), (25, 11, 1, 0), (15, 2, 0, 2)])
def test_gpu_batch_matches_oracle(gpu, N_RB, nid, Ncp, first):
    fo = O.frame(N_RB, Nid_cell=nid, Ncp=Ncp)
    fg = gpu.frame_parms(N_RB, Nid_cell=nid, Ncp=Ncp)
    N, nsymb = fo.ofdm_symbol_size, fo.symbols_per_tti
    n_sf = 12
    rng = np.random.default_rng(nid)
    y = (rng.integers(-2**15, 2**15, ((n_sf + 1) * nsymb * N, 2)).astype(np.int16)).view(np.int32).ravel()
    cb = gpu.ChestBatch(fg, n_sf, first_subframe=first)
    got = cb.run(y[:n_sf * nsymb * N].reshape(n_sf, -1), y[n_sf * nsymb * N:][:N])
    cb.close()
    for i in range(n_sf):
        sf = (first + i) % 10
        want = O.chest_subframe(fo, y[i * nsymb * N:(i + 1) * nsymb * N], y[(i + 1) * nsymb * N:][:N], sf)
        assert np.array_equal(got[i], want), i


@pytest.mark.parametrize("N_RB,mcs,npd,sf", [(100, 16, 1, 7), (100, 27, 2, 3), (6, 9, 2, 2), (50, 24, 3, 1),
                                              (25, 16, 1, 7), (25, 27, 2, 3), (25, 0, 1, 7)])
def test_gpu_estimated_channel_loop(gpu, N_RB, mcs, npd, sf):
    """dlsim's receive path with perfect_ce = 0, all on the GPU: TxPipeline (TM1, CRS) over three
    consecutive subframes -> FepBatch -> ChestBatch (the FEP output buffer, its third subframe's
    symbol 0 closing the second's rows 12 / 13) -> RxBatch -> per-block RM-rx / deinterleave /
    turbo_decoder16: the first two subframes' transport blocks come back."""
    n_tx, n_sf = 3, 2
    p = params("C2", N_RB, mcs, npd, sf, subframe_step=1)
    pipe = gpu.TxPipeline(p, n_tx)
    rng = np.random.default_rng(mcs + N_RB)
    pay = rng.integers(0, 256, size=(n_tx, 1, p.payload_stride), dtype=np.uint8)
    pipe.upload_payload(pay)
    pipe.run()
    pipe.sync()
    fg = gpu.frame_parms(N_RB)
    fep = gpu.FepBatch(fg, n_tx, 1)
    fep.upload(pipe.iq())
    fep.run()
    cb = gpu.ChestBatch(fg, n_sf, first_subframe=sf)
    est = cb.run(None, None, d_rxdataF=fep.d_rxF)
    rxF = fep.result()[:, 0].reshape(n_tx, -1)
    # the batch equals the oracle's call sequence on the same FEP output
    fo = O.frame(N_RB)
    for i in range(n_sf):
        assert np.array_equal(est[i], O.chest_subframe(fo, rxF[i], rxF[i + 1][:fo.ofdm_symbol_size], (sf + i) % 10))
    cb.close()
    fep.close()
    pipe.close()
    Qm = 2 if mcs < 10 else 4 if mcs < 17 else 6
    rx = gpu.RxBatch(fg, alloc(N_RB), Qm, npd, p.rnti, n_sf, first_subframe=sf, subframe_step=1)
    llr = rx.run(rxF[:n_sf], est, unscramble=1)
    for i in range(n_sf):
        s = (sf + i) % 10
        G = rx.llr_count(s)
        res, tb = decode_tb(llr[i], G, p.TBS[0], Qm)
        assert all(it <= 4 for it, _ in res), (s, [it for it, _ in res])
        assert np.array_equal(tb, pay[i, 0, :p.TBS[0] // 8]), s
    rx.close()


@pytest.mark.parametrize("N_RB,Qm,npd,first,Ncp", [(100, 4, 1, 3, 0), (50, 6, 2, 8, 0), (6, 2, 3, 0, 0),
                                                    (100, 6, 1, 9, 0), (50, 4, 2, 1, 1),
                                                    (25, 4, 1, 3, 0), (25, 6, 2, 7, 0), (15, 4, 1, 1, 0), (25, 6, 1, 2, 1)])
def test_gpu_fused_estimation_demodulation(gpu, N_RB, Qm, npd, first, Ncp):
    """oai4g_rx_batch_estimated (k_rx_chest) = oai4g_chest_batch then oai4g_rx_batch, and = the
    oracle's chain, on full-range random grids (saturating estimates and LLRs)."""
    fo = O.frame(N_RB, Nid_cell=N_RB + first, Ncp=Ncp)
    fg = gpu.frame_parms(N_RB, Nid_cell=N_RB + first, Ncp=Ncp)
    N, nsymb = fo.ofdm_symbol_size, fo.symbols_per_tti
    n_sf = 10
    rng = np.random.default_rng(N_RB * Qm + first)
    y = (rng.integers(-2**15, 2**15, ((n_sf + 1) * nsymb * N, 2)).astype(np.int16)).view(np.int32).ravel()
    cb = gpu.ChestBatch(fg, n_sf, first_subframe=first)
    rb = gpu.RxBatch(fg, alloc(N_RB), Qm, npd, 0x2345, n_sf, first_subframe=first, subframe_step=1)
    yin = np.ascontiguousarray(y[:n_sf * nsymb * N + N])          # the batch + the next symbol 0
    assert gpu.lib().oai4g_memcpy_h2d(cb.d_rx, gpu._ptr(yin), yin.nbytes) == 0
    cb.launch(cb.d_rx)
    rb.launch(cb.d_rx, cb.d_est, 1)
    two = rb.llrs()
    rb.launch_estimated(cb, cb.d_rx, 1)
    fused = rb.llrs()
    for i in range(n_sf):
        sf = (first + i) % 10
        G = rb.llr_count(sf)
        assert np.array_equal(fused[i, :G], two[i, :G]), i
        if i in (0, n_sf - 1) and Ncp == 0:
            est = O.chest_subframe(fo, y[i * nsymb * N:(i + 1) * nsymb * N], y[(i + 1) * nsymb * N:][:N], sf)
            lo, _ = O.rx_pdsch_siso(fo, y[i * nsymb * N:(i + 1) * nsymb * N], est, alloc(N_RB), Qm, npd, sf)
            u = np.zeros(32 * (1 + len(lo) // 32), np.int16)
            u[:len(lo)] = lo
            O.dlsch_unscrambling(u, len(lo), (0x2345 << 14) + (sf << 9) + fo.Nid_cell)
            assert np.array_equal(fused[i, :G], u[:G]), i
    cb.close()
    rb.close()
