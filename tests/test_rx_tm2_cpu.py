"""TM2 (ALAMOUTI, 2 TX ports) receive chain on the oracle (oracle/oai_oracle_rx.c: orc_rx_pdsch_tm2 —
dlsch_extract_rbs_dual, dlsch_channel_level, dlsch_channel_compensation per (port, RX antenna),
dlsch_detection_mrc, dlsch_alamouti, the single-stream LLRs, as dlsim's TM2 UE runs rx_pdsch).  The
reference translation units are unbuildable here (PHY/defs.h), so the restatement is pinned by the
closed loop: the oracle's TM2 transmit subframe (space-frequency block code over 2 antennas, both
ports' CRS) -> per receive antenna slot_fep -> the estimates of ports 0 / 1 -> TM2 demodulation ->
the transport block comes back, over H = I with 2 RX antennas and H = [1 1] with one (dlsim's AWGN
sum of the transmit antennas).  The LLR stream has exactly G entries."""
import numpy as np
import pytest

import oracle_lib as O
from test_rx_cpu import alloc, decode_tb, dual_alloc, n_alloc


def tm2_params(N_RB, mcs, npdcch, sf, Nid=0):
    import openair4g_amd as oai
    ra = dual_alloc(N_RB, dc=False)
    return oai.make_params("TM2", subframe=sf, N_RB_DL=N_RB, nb_rb=n_alloc(ra), rb_alloc=ra, mcs=[mcs, 0], TBS=None,
                           num_pdcch_symbols=npdcch, with_crs=1, Nid_cell=Nid)


def tm2_loop(p, sf, pays, H, nb_rx=2):
    """TX of subframes sf, sf + 1 (TM2 with CRS) -> flat channel H[rx][tx] -> per RX antenna the FEP
    of subframe sf and symbol 0 of the next -> estimates of ports 0 / 1."""
    fp = O.tx_cfg_from_params(p, sf).fp
    spt, N = fp.samples_per_tti, fp.ofdm_symbol_size
    frames = [np.zeros(10 * spt + N, np.int32) for _ in range(nb_rx)]
    for d, pay in enumerate(pays):
        s = (sf + d) % 10
        txd, _, _ = O.tx_subframe(O.tx_cfg_from_params(p, s), [pay])
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


def qm_of(mcs):
    return 2 if mcs < 10 else (4 if mcs < 17 else 6)


# (N_RB, mcs, PDCCH symbols, subframe, RX antennas)
CASES = [(100, 16, 1, 7, 2), (50, 9, 2, 3, 2), (100, 22, 1, 8, 1), (25, 12, 1, 7, 2), (6, 9, 3, 2, 1), (100, 5, 3, 1, 1)]


@pytest.mark.parametrize("N_RB,mcs,npdcch,sf,nb_rx", CASES)
def test_tm2_loop_decodes(N_RB, mcs, npdcch, sf, nb_rx):
    p = tm2_params(N_RB, mcs, npdcch, sf)
    rng = np.random.default_rng(N_RB * mcs + sf)
    pays = [rng.integers(0, 256, p.payload_stride, dtype=np.uint8) for _ in range(2)]
    H = [[1, 0], [0, 1]] if nb_rx == 2 else [[1, 1]]
    fp, rxF, est = tm2_loop(p, sf, pays, H, nb_rx)
    Qm = qm_of(mcs)
    llr, sh = O.rx_pdsch_tm2(fp, rxF[:nb_rx], est, dual_alloc(N_RB, dc=False), Qm, npdcch, sf)
    G = O.get_G(N_RB, 0, 0, 0, n_alloc(dual_alloc(N_RB, dc=False)), dual_alloc(N_RB, dc=False), Qm, 1, npdcch, sf)
    assert len(llr) == Qm * (G // Qm) and len(llr) == G
    u = np.zeros(32 * (1 + G // 32), np.int16)
    u[:G] = llr
    O.dlsch_unscrambling(u, G, (p.rnti << 14) + (sf << 9) + fp.Nid_cell)
    res, tb = decode_tb(u[:G], G, p.TBS[0], Qm)
    assert all(it <= 4 for it, _ in res), [it for it, _ in res]
    assert np.array_equal(tb, pays[0][:p.TBS[0] // 8])


def test_tm2_alamouti_combining_is_exact_for_identity_channel():
    """With H = I and both receive antennas, the combined symbol of every pair is the transmitted QAM
    point scaled by a common gain: its sign pattern equals the sent bits (hard decisions of the QPSK
    LLRs equal the scrambled e bits).  Even N_RB_DL: at 15 / 25 PRB the reference's dual extraction
    reads the DC RB's second half from bins 0..5 (extract_dual), which shifts the pairs there."""
    N_RB, mcs, npdcch, sf = 50, 5, 2, 6
    p = tm2_params(N_RB, mcs, npdcch, sf)
    rng = np.random.default_rng(5)
    pays = [rng.integers(0, 256, p.payload_stride, dtype=np.uint8) for _ in range(2)]
    fp, rxF, est = tm2_loop(p, sf, pays, [[1, 0], [0, 1]], 2)
    llr, _ = O.rx_pdsch_tm2(fp, rxF, est, alloc(N_RB), 2, npdcch, sf)
    G = len(llr)
    _, _, e = O.tx_subframe(O.tx_cfg_from_params(p, sf), [pays[0]], want_e=True)
    e0 = np.asarray(e[0], dtype=np.uint8)[:G]                # scrambled e bits (QPSK: bit 1 -> negative)
    assert np.all(llr != 0)
    assert np.array_equal((llr < 0).astype(np.uint8), e0)
