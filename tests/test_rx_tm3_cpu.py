"""TM3 (LARGE_CDD, 2 TX ports) receive chain on the oracle (oracle/oai_oracle_rx.c:
orc_rx_pdsch_tm3 — dlsch_extract_rbs_dual, dlsch_channel_level_TM3, prec2A_TM3_128,
dlsch_channel_compensation_TM3, dlsch_detection_mrc, the single-stream LLRs of codeword 0, as
dlsim's TM3 UE runs rx_pdsch with dual_stream_flag = 0).  The reference translation units are
unbuildable here (PHY/defs.h), so the restatement is pinned by the closed loop: the oracle's C3
transmit subframe (2 antennas, both ports' CRS) -> per receive antenna slot_fep -> the estimates of
ports 0 / 1 -> TM3 demodulation -> codeword 0's transport block comes back, over the channel
H = I (each receive antenna sees one transmit antenna: the large-delay CDD precoding and the
receiver's prec2A_TM3 + MRC then separate the two streams exactly), with 2 and with 1 receive
antenna and the two-antenna MRC.  The LLR stream has exactly G entries."""
import numpy as np
import pytest

import oracle_lib as O
from test_rx_cpu import alloc, decode_tb, dual_alloc, n_alloc


def c3_params(N_RB, mcs, npdcch, sf, Nid=0):
    import openair4g_amd as oai
    ra = dual_alloc(N_RB, dc=False)
    return oai.make_params("C3", subframe=sf, N_RB_DL=N_RB, nb_rb=n_alloc(ra), rb_alloc=ra, mcs=[mcs, mcs], TBS=None,
                           num_pdcch_symbols=npdcch, with_crs=1, Nid_cell=Nid)


def tm3_loop(p, sf, pays, H, nb_rx=2):
    """TX of subframes sf, sf + 1 (C3 with CRS) -> flat channel H[rx][tx] (int) -> per RX antenna the
    FEP of subframe sf and symbol 0 of the next -> estimates of ports 0 / 1 -> orc_rx_pdsch_tm3."""
    cfg = O.tx_cfg_from_params(p, sf)
    fp = cfg.fp
    spt, N = fp.samples_per_tti, fp.ofdm_symbol_size
    frames = [np.zeros(10 * spt + N, np.int32) for _ in range(nb_rx)]
    for d, pay in enumerate(pays):
        s = (sf + d) % 10
        txd, _, _ = O.tx_subframe(O.tx_cfg_from_params(p, s), [pay[0], pay[1]])
        t16 = txd.view(np.int16).reshape(2, spt, 2).astype(np.int64)
        for a in range(nb_rx):
            r = H[a][0] * t16[0] + H[a][1] * t16[1]
            frames[a][s * spt:(s + 1) * spt] = np.clip(r, -32768, 32767).astype(np.int16).reshape(-1).view(np.int32)
    rxF, est = [], {}
    for a in range(nb_rx):
        g = np.zeros(15 * N, np.int32)
        for Ns in (2 * sf, 2 * sf + 1):
            for l in range(7):
                assert O.slot_fep([frames[a]], [g], fp, l, Ns) == 0
        nxt = np.zeros(15 * N, np.int32)
        assert O.slot_fep([frames[a]], [nxt], fp, 0, (2 * sf + 2) % 20) == 0
        rxF.append(g[:14 * N].copy())
        for port in (0, 1):
            est[(port, a)] = O.chest_subframe(fp, g[:14 * N].copy(), nxt[:N].copy(), sf, p=port)
    return fp, rxF, est


# (N_RB, mcs, PDCCH symbols, subframe, RX antennas).  One RX antenna: the channel [1, 1] (dlsim's AWGN
# sum of the transmit antennas) carries stream 0 alone on every other RE (s = +1) and erases it on
# the rest (h0' = 0): a low-rate 16-QAM codeword still decodes.
CASES = [(100, 19, 1, 7, 2), (50, 16, 2, 3, 2), (100, 11, 3, 8, 1), (25, 19, 1, 7, 2), (100, 12, 1, 1, 2)]


@pytest.mark.parametrize("N_RB,mcs,npdcch,sf,nb_rx", CASES)
def test_tm3_loop_decodes_codeword0(N_RB, mcs, npdcch, sf, nb_rx):
    p = c3_params(N_RB, mcs, npdcch, sf)
    rng = np.random.default_rng(N_RB * mcs + sf)
    pays = [[rng.integers(0, 256, p.payload_stride, dtype=np.uint8) for _ in range(2)] for _ in range(2)]
    H = [[1, 0], [0, 1]] if nb_rx == 2 else [[1, 1]]
    fp, rxF, est = tm3_loop(p, sf, pays, H, nb_rx)
    Qm = 4 if mcs < 17 else 6
    llr, sh = O.rx_pdsch_tm3(fp, rxF[:nb_rx], est, dual_alloc(N_RB, dc=False), Qm, Qm, mcs, npdcch, sf)
    G = O.get_G(N_RB, 0, 0, 0, n_alloc(dual_alloc(N_RB, dc=False)), dual_alloc(N_RB, dc=False), Qm, 1, npdcch, sf)
    assert len(llr) == G
    u = np.zeros(32 * (1 + G // 32), np.int16)
    u[:G] = llr
    O.dlsch_unscrambling(u, G, (p.rnti << 14) + (sf << 9) + fp.Nid_cell)
    res, tb = decode_tb(u[:G], G, p.TBS[0], Qm)
    assert all(it <= 4 for it, _ in res), [it for it, _ in res]
    assert np.array_equal(tb, pays[0][0][:p.TBS[0] // 8])


def test_tm3_qpsk_codeword0_and_garbage_free_lengths():
    fp = O.frame(50, nb_antennas_tx=2, mode1_flag=0)
    N = fp.ofdm_symbol_size
    rng = np.random.default_rng(1)
    rx = [rng.integers(-3000, 3000, 14 * N).astype(np.int32) for _ in range(2)]
    est = {(pp, a): rng.integers(-3000, 3000, 14 * N).astype(np.int32) for pp in (0, 1) for a in (0, 1)}
    # Qm0 = 2: codeword 0 of the interference-aware path (qpsk_qpsk with Qm1 = 2)
    l0, sh0 = O.rx_pdsch_tm3(fp, rx, est, alloc(50), 2, 2, 5, 1, 7)
    q0, _, shq = O.rx_pdsch_tm3_qq(fp, rx, est, alloc(50), 5, 1, 7)
    assert np.array_equal(l0, q0) and sh0 == shq
    # subframes 0 / 5 drop the PBCH / sync RBs (unlike the single-antenna extraction) and shorten by
    # adjust_G2 (16-QAM: pilot symbols by 2/3 of it)
    for sf in (0, 5, 7):
        llr, _ = O.rx_pdsch_tm3(fp, rx, est, alloc(50), 4, 4, 14, 2, sf)
        assert len(llr) % 4 == 0 and len(llr) > 0


# Both codewords QPSK: rx_pdsch runs the interference-aware dlsch_qpsk_qpsk_llr for each stream
# (dlsch_demodulation.c:643-669), so dlsim decodes codeword 1 too.  Stream 1 is demodulated from
# receive antenna 0 alone (dlsch_detection_mrc leaves it uncombined with dual_stream_flag 0), so the
# channel's first row must keep the precoded streams apart: H = [[2, 1], [1, 2]].
QQ = [(100, 9, 1, 7, 2), (50, 5, 2, 3, 2), (25, 7, 1, 6, 2), (100, 4, 3, 8, 1)]


@pytest.mark.parametrize("N_RB,mcs,npdcch,sf,nb_rx", QQ)
def test_tm3_qpsk_loop_decodes_both_codewords(N_RB, mcs, npdcch, sf, nb_rx):
    p = c3_params(N_RB, mcs, npdcch, sf)
    rng = np.random.default_rng(N_RB * mcs + sf + 1)
    pays = [[rng.integers(0, 256, p.payload_stride, dtype=np.uint8) for _ in range(2)] for _ in range(2)]
    H = [[2, 1], [1, 2]][:nb_rx]
    fp, rxF, est = tm3_loop(p, sf, pays, H, nb_rx)
    l0, l1, sh = O.rx_pdsch_tm3_qq(fp, rxF[:nb_rx], est, dual_alloc(N_RB, dc=False), mcs, npdcch, sf)
    G = O.get_G(N_RB, 0, 0, 0, n_alloc(dual_alloc(N_RB, dc=False)), dual_alloc(N_RB, dc=False), 2, 1, npdcch, sf)
    assert len(l0) == G and len(l1) == G
    for cw, llr in enumerate((l0, l1)):
        u = np.zeros(32 * (1 + G // 32), np.int16)
        u[:G] = llr
        O.dlsch_unscrambling(u, G, (p.rnti << 14) + (sf << 9) + fp.Nid_cell)   # q = 0 for both (dlsim.c:2642-2647)
        res, tb = decode_tb(u[:G], G, p.TBS[cw], 2)
        assert all(it <= 4 for it, _ in res), (cw, [it for it, _ in res])
        assert np.array_equal(tb, pays[0][cw][:p.TBS[cw] // 8]), cw


# Codeword 0 QPSK, codeword 1 16 / 64-QAM: rx_pdsch runs dlsch_qpsk_16qam_llr / dlsch_qpsk_64qam_llr
# for codeword 0 only (dlsch_demodulation.c:670-690), stream 1 and dl_ch_mag1 from receive antenna 0.
QX = [(50, 9, 16, 1, 7), (50, 9, 22, 1, 7), (25, 5, 12, 2, 3), (100, 7, 19, 1, 8)]


@pytest.mark.parametrize("N_RB,mcs0,mcs1,npdcch,sf", QX)
def test_tm3_qpsk_with_qam_interferer_decodes_codeword0(N_RB, mcs0, mcs1, npdcch, sf):
    import openair4g_amd as oai
    ra = dual_alloc(N_RB, dc=False)
    p = oai.make_params("C3", subframe=sf, N_RB_DL=N_RB, nb_rb=n_alloc(ra), rb_alloc=ra, mcs=[mcs0, mcs1], TBS=None,
                        num_pdcch_symbols=npdcch, with_crs=1, Nid_cell=0)
    rng = np.random.default_rng(N_RB + mcs0 + mcs1)
    pays = [[rng.integers(0, 256, p.payload_stride, dtype=np.uint8) for _ in range(2)] for _ in range(2)]
    Qm1 = 4 if mcs1 < 17 else 6
    for H in ([[1, 0], [0, 1]], [[2, 1], [1, 2]]):
        fp, rxF, est = tm3_loop(p, sf, pays, H, 2)
        llr, sh = O.rx_pdsch_tm3(fp, rxF, est, ra, 2, Qm1, mcs0, npdcch, sf)
        G = O.get_G(N_RB, 0, 0, 0, n_alloc(dual_alloc(N_RB, dc=False)), dual_alloc(N_RB, dc=False), 2, 1, npdcch, sf)
        assert len(llr) == G
        u = np.zeros(32 * (1 + G // 32), np.int16)
        u[:G] = llr
        O.dlsch_unscrambling(u, G, (p.rnti << 14) + (sf << 9) + fp.Nid_cell)
        res, tb = decode_tb(u[:G], G, p.TBS[0], 2)
        assert all(it <= 4 for it, _ in res), (H, [it for it, _ in res])
        assert np.array_equal(tb, pays[0][0][:p.TBS[0] // 8]), H


@pytest.mark.parametrize("N_RB", [15, 25])
def test_tm3_odd_nrb_full_allocation_refused(N_RB):
    """Odd N_RB_DL, every RB allocated: from the second full RB of a non-pilot symbol on, the
    reference's dl_ch0_ext has moved 144 slots per RB (dlsch_demodulation.c:3932-3936) and the
    port-0 estimates it reads are stale, so the oracle refuses (as the library does)."""
    fp = O.frame(N_RB, nb_antennas_tx=2, mode1_flag=0)
    N = fp.ofdm_symbol_size
    rng = np.random.default_rng(N_RB)
    rx = [rng.integers(-3000, 3000, 14 * N).astype(np.int32) for _ in range(2)]
    est = {(pp, a): rng.integers(-3000, 3000, 14 * N).astype(np.int32) for pp in (0, 1) for a in (0, 1)}
    import ctypes
    out = np.zeros(14 * 1200 * 6 + 64, dtype=np.int16)
    rp = (ctypes.c_void_p * 2)(*[r.ctypes.data for r in rx])
    ep = (ctypes.c_void_p * 4)(*[est[(p_, a)].ctypes.data for p_ in (0, 1) for a in (0, 1)])
    sh = ctypes.c_uint8()
    ra = (ctypes.c_uint32 * 4)(*alloc(N_RB))
    for sf in (3, 7):
        assert O.orc().orc_rx_pdsch_tm3(ctypes.byref(fp), 2, rp, ep, ra, 6, 6, 19, 1, sf, O.P(out), ctypes.byref(sh)) < 0
    # the DC RB and the next one stay defined
    llr, _ = O.rx_pdsch_tm3(fp, rx, est, dual_alloc(N_RB), 6, 6, 19, 1, 7)
    assert len(llr) > 0
