"""GPU parity of the TM2 (ALAMOUTI, 2 TX ports) receive chain — dlsch_extract_rbs_dual,
dlsch_channel_level over both ports, dlsch_channel_compensation per (port, RX antenna),
dlsch_detection_mrc, dlsch_alamouti, the LLRs (k_rx_level_tm2 / k_rx_llr_tm2) — against the oracle
restatement (tests/test_rx_tm2_cpu.py pins it by the decoding loop): the drop-in on full-range random
grids and estimates (saturation / wrap paths, QPSK / 16 / 64-QAM, 1 and 2 receive antennas, odd
N_RB_DL, partial allocations), and a receive loop on the GPU: TM2 TxPipeline (both ports' CRS) ->
channel H -> FepBatch over the receive antennas -> 4 channel-estimation batches -> RxBatchTM2 ->
RM-rx / deinterleaving / turbo decoding: the TB comes back, LLRs bit-exact vs the oracle."""
import numpy as np
import pytest

import oracle_lib as O
from test_rx_cpu import alloc, decode_tb, dual_alloc
from test_rx_tm2_cpu import qm_of, tm2_params

pytestmark = pytest.mark.gpu

RAND = [(100, 2, 1, 7, 2, None), (50, 4, 2, 3, 2, None), (100, 6, 3, 1, 1, None), (25, 6, 1, 6, 2, None),
        (25, 4, 2, 2, 1, None), (15, 2, 1, 4, 2, None), (6, 4, 3, 8, 1, None),
        (100, 6, 2, 8, 2, [0xF0F0F0F0, 0x0000FFFF, 0, 0x3])]


@pytest.mark.parametrize("N_RB,Qm,npd,sf,nb_rx,ra", RAND)
def test_gpu_tm2_random_inputs(gpu, N_RB, Qm, npd, sf, nb_rx, ra):
    ra = ra or dual_alloc(N_RB)
    fo = O.frame(N_RB, Nid_cell=N_RB + sf, nb_antennas_tx=2, mode1_flag=0)
    fg = gpu.frame_parms(N_RB, Nid_cell=N_RB + sf, nb_antennas_tx=2, mode1_flag=0)
    n = fo.symbols_per_tti * fo.ofdm_symbol_size
    rng = np.random.default_rng(N_RB * 7 + Qm + sf)
    for scale in (2 ** 31 - 1, 3000):
        rx = [rng.integers(-scale, scale, n, dtype=np.int64).astype(np.int32) for _ in range(nb_rx)]
        est = {(p, a): rng.integers(-scale, scale, n, dtype=np.int64).astype(np.int32) for p in (0, 1)
               for a in range(nb_rx)}
        lo, so = O.rx_pdsch_tm2(fo, rx, est, ra, Qm, npd, sf)
        lg, sg = gpu.rx_pdsch_tm2(fg, rx, est, ra, Qm, npd, sf)
        assert sg == so and np.array_equal(lg, lo), (scale, so, sg)


@pytest.mark.parametrize("N_RB,mcs,npd,sf,nb_rx", [(100, 16, 1, 7, 2), (50, 9, 2, 3, 1), (100, 24, 1, 8, 2)])
def test_gpu_tm2_receive_loop(gpu, N_RB, mcs, npd, sf, nb_rx):
    n_tx, n_sf = 3, 2
    p = tm2_params(N_RB, mcs, npd, sf)
    p.subframe_step = 1
    pipe = gpu.TxPipeline(p, n_tx)
    rng = np.random.default_rng(mcs + N_RB)
    pay = rng.integers(0, 256, size=(n_tx, 1, p.payload_stride), dtype=np.uint8)
    pipe.upload_payload(pay)
    pipe.run()
    pipe.sync()
    iq = pipe.iq()                                      # [n_tx][2 antennas][spt]
    if nb_rx == 1:                                      # H = [1 1]: the antennas' sum (int16 saturation)
        t16 = iq.view(np.int16).astype(np.int64)
        s = np.clip(t16[:, 0] + t16[:, 1], -32768, 32767).astype(np.int16)
        iq = np.ascontiguousarray(s.view(np.int32)[:, None, :])
    fg = gpu.frame_parms(N_RB, nb_antennas_tx=2, mode1_flag=0)
    fep = gpu.FepBatch(fg, n_tx, nb_rx)
    fep.upload(iq)
    fep.run()
    Qm = qm_of(mcs)
    rx = gpu.RxBatchTM2(fg, dual_alloc(N_RB), Qm, npd, p.rnti, n_sf, nb_rx=nb_rx, first_subframe=sf)
    rx.estimate(fep.d_rxF, first_subframe=sf)
    rx.launch(fep.d_rxF, unscramble=1)
    llr = rx.llrs()
    rxF = fep.result()                                   # [n_tx][nb_rx][nsymb][N]
    fo = O.frame(N_RB, nb_antennas_tx=2, mode1_flag=0)
    for i in range(n_sf):
        s_ = (sf + i) % 10
        est = {(pp, a): O.chest_subframe(fo, rxF[i, a].ravel(), rxF[i + 1, a, 0], s_, p=pp) for pp in (0, 1)
               for a in range(nb_rx)}
        lo, _ = O.rx_pdsch_tm2(fo, [rxF[i, a].ravel() for a in range(nb_rx)], est, alloc(N_RB), Qm, npd, s_)
        G = rx.llr_count(s_)
        u = np.zeros(32 * (1 + G // 32), np.int16)
        u[:G] = lo
        O.dlsch_unscrambling(u, G, (p.rnti << 14) + (s_ << 9) + fo.Nid_cell)
        assert len(lo) == G and np.array_equal(llr[i, :G], u[:G]), s_
        res, tb = decode_tb(llr[i, :G], G, p.TBS[0], Qm)
        assert all(it <= 4 for it, _ in res), (s_, [it for it, _ in res])
        assert np.array_equal(tb, pay[i, 0, :p.TBS[0] // 8]), s_
    rx.close()
    fep.close()
    pipe.close()
