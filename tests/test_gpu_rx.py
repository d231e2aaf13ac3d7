"""GPU parity of the UE PDSCH demodulation (rx_pdsch's extraction, channel level, compensation and
LLRs, dlsch_unscrambling) against the oracle restatement
(tests/test_rx_cpu.py), and the closed loop on the GPU: transmit (k_encode + k_modofdm) -> FEP
(k_fep) -> demodulation (k_rx_*) -> RX rate matching, sub-block deinterleaving and the 16-bit turbo
decoder -> every code block's CRC passes and the transport block comes back."""
import numpy as np
import pytest

import oracle_lib as O
from test_rx_cpu import alloc, decode_tb, loop_llr, params, perfect_ce

pytestmark = pytest.mark.gpu

RAND = [(100, 2, 1, 7, None), (100, 4, 2, 0, None), (100, 6, 3, 5, None), (50, 6, 1, 0, None), (6, 4, 3, 9, None),
        (50, 2, 2, 5, [0x0F0F0F0F, 0x3, 0, 0]), (100, 6, 1, 1, [0xFFFF0000, 0xFFFFFFFF, 0x0000FFFF, 0x3]),
        # odd N_RB_DL: the DC split, PBCH / PSS / SSS RBs dropped and halved in subframes 0 / 5
        (25, 2, 1, 7, None), (25, 4, 2, 0, None), (25, 6, 1, 5, None), (15, 6, 3, 0, None), (25, 2, 2, 3, [0x1F0F0F0, 0, 0, 0]),
        (15, 4, 1, 5, [0x7F80, 0, 0, 0]), (25, 6, 3, 0, [0x00FFF000, 0, 0, 0])]


@pytest.mark.parametrize("N_RB,Qm,npdcch,sf,ra", RAND)
def test_gpu_rx_pdsch_random_inputs(gpu, N_RB, Qm, npdcch, sf, ra):
    """Full-range random grids and estimates (saturating madd / packs / subs paths)."""
    ra = ra or alloc(N_RB)
    fo, fg = O.frame(N_RB), gpu.frame_parms(N_RB)
    n = fo.symbols_per_tti * fo.ofdm_symbol_size
    rng = np.random.default_rng(N_RB * 7 + Qm + sf)
    for scale in (2**31 - 1, 3000):
        y = rng.integers(-scale, scale, n, dtype=np.int64).astype(np.int32)
        h = rng.integers(-scale, scale, n, dtype=np.int64).astype(np.int32)
        lo, so = O.rx_pdsch_siso(fo, y, h, ra, Qm, npdcch, sf)
        lg, sg = gpu.rx_pdsch_siso(fg, y, h, ra, Qm, npdcch, sf)
        assert sg == so and np.array_equal(lg, lo), (scale, so, sg)


def test_gpu_rx_batch_and_unscrambling(gpu):
    N_RB, Qm, npd, rnti = 100, 4, 2, 0x1234
    fo, fg = O.frame(N_RB, Nid_cell=17), gpu.frame_parms(N_RB, Nid_cell=17)
    n = fo.symbols_per_tti * fo.ofdm_symbol_size
    rng = np.random.default_rng(5)
    n_sf = 10
    y = rng.integers(-3000, 3000, (n_sf, n), dtype=np.int64).astype(np.int32)
    h = rng.integers(-1500, 1500, (n_sf, n), dtype=np.int64).astype(np.int32)
    rx = gpu.RxBatch(fg, alloc(N_RB), Qm, npd, rnti, n_sf, first_subframe=3, subframe_step=1)
    out = rx.run(y, h, unscramble=1)
    for i in range(n_sf):
        sf = (3 + i) % 10
        lo, _ = O.rx_pdsch_siso(fo, y[i], h[i], alloc(N_RB), Qm, npd, sf)
        assert rx.llr_count(sf) == len(lo)
        u = np.zeros(32 * (1 + len(lo) // 32) + 32, np.int16)
        u[:len(lo)] = lo
        O.dlsch_unscrambling(u, len(lo), (rnti << 14) + (sf << 9) + 17)
        assert np.array_equal(out[i, :len(lo)], u[:len(lo)]), sf
        v = np.zeros_like(u)
        v[:len(lo)] = lo
        gpu.dlsch_unscrambling(fg, rnti, len(lo), v, 0, 2 * sf)
        assert np.array_equal(v[:len(lo)], u[:len(lo)])
        # PMCH (mbsfn_flag = 1): c_init = (Ns / 2) 2^9 + Nid_cell_mbsfn (dlsch_scrambling.c:115-118)
        fg.Nid_cell_mbsfn = 37 + sf
        m = np.zeros_like(u)
        m[:len(lo)] = lo
        O.dlsch_unscrambling(m, len(lo), (sf << 9) + 37 + sf)
        v[:] = 0
        v[:len(lo)] = lo
        gpu.dlsch_unscrambling(fg, rnti, len(lo), v, 0, 2 * sf, mbsfn_flag=1)
        assert np.array_equal(v[:len(lo)], m[:len(lo)])
        fg.Nid_cell_mbsfn = 0
    rx.close()


@pytest.mark.parametrize("N_RB,mcs,npd,sf", [(100, 16, 1, 7), (100, 27, 2, 3), (50, 9, 3, 8), (100, 22, 1, 1),
                                              (25, 16, 1, 7), (25, 9, 2, 3)])
def test_gpu_tx_fep_rx_decode_loop(gpu, N_RB, mcs, npd, sf):
    """TM1 with CRS, two consecutive subframes: the GPU transmit batch -> IQ -> batched FEP ->
    batched demodulation with dlsim's perfect channel estimate (AMP, 0) and unscrambling, LLRs
    bit-exact against the oracle's loop (test_rx_cpu.loop_llr) -> per code block RX rate matching,
    deinterleaving and the 16-bit turbo decoder on the GPU: every CRC passes, the TB comes back."""
    n_sf = 2
    p = params("C2", N_RB, mcs, npd, sf, subframe_step=1)
    pipe = gpu.TxPipeline(p, n_sf)
    rng = np.random.default_rng(mcs)
    pay = rng.integers(0, 256, size=(n_sf, 1, p.payload_stride), dtype=np.uint8)
    pipe.upload_payload(pay)
    pipe.run()
    pipe.sync()
    fg = gpu.frame_parms(N_RB)
    fep = gpu.FepBatch(fg, n_sf, 1)
    fep.upload(pipe.iq())
    fep.run()
    rxF = fep.result()[:, 0].reshape(n_sf, -1)
    fep.close()
    pipe.close()
    Qm = 2 if mcs < 10 else 4 if mcs < 17 else 6
    rx = gpu.RxBatch(fg, alloc(N_RB), Qm, npd, p.rnti, n_sf, first_subframe=sf, subframe_step=1)
    llr = rx.run(rxF, np.stack([perfect_ce(fg)] * n_sf), unscramble=1)
    ops = (lambda soft, K, G, C, r, Qm_: _gpu_rm(soft, K, G, C, r, Qm_),
           lambda w, K: gpu.sub_block_deinterleaving_turbo(K + 4, w)[96:96 + 3 * K + 12],
           lambda d, K, ct, F: gpu.turbo_decoder16(d, K, max_iterations=4, crc_type=ct, F=F))
    for i in range(n_sf):
        s = (sf + i) % 10
        G = rx.llr_count(s)
        want, G_o, _ = loop_llr(params("C2", N_RB, mcs, npd, s), s, pay[i, 0])
        assert G == G_o and np.array_equal(llr[i, :G], want), s
        res, tb = decode_tb(llr[i], G, p.TBS[0], Qm, C_ops=ops)
        assert all(it <= 4 for it, _ in res), (s, [it for it, _ in res])
        assert np.array_equal(tb, pay[i, 0, :p.TBS[0] // 8]), s
    rx.close()


def _gpu_rm(soft, K, G, C, r, Qm):
    D = K + 4
    R = (D + 31) >> 5
    w = np.zeros(3 * 32 * R + 64, np.int16)
    E = gpu_mod().rate_matching_turbo_rx(R, G, w, O.dummy_w(D), soft, C, r, Qm)
    return w, E


def gpu_mod():
    import openair4g_amd
    return openair4g_amd


def test_gpu_pmch_scrambling(gpu):
    """dlsch_scrambling with mbsfn_flag = 1 (PMCH, dlsch_scrambling.c:70-72): c_init =
    (Ns / 2) 2^9 + Nid_cell_mbsfn, independent of the RNTI and the cell id."""
    fg = gpu.frame_parms(50, Nid_cell=11)
    fg.Nid_cell_mbsfn = 201
    dl = gpu.DlschHandle(Kmimo=1, Mdlharq=8, N_RB_DL=50)
    dl.d.rnti = 0x4321
    G = 5000
    rng = np.random.default_rng(8)
    e0 = rng.integers(0, 2, 32 * (1 + G // 32), dtype=np.uint8)
    e = dl.view("e", len(e0))
    e[:] = e0
    gpu.dlsch_scrambling(fg, dl, G, 0, 14, mbsfn_flag=1)
    want = O.scramble(e0.copy(), G, (7 << 9) + 201)
    assert np.array_equal(dl.view("e", G), np.asarray(want)[:G])
    dl.close()
