"""The oracle's transmit chain pinned end to end to the independent 36.211/36.212 model
(tests/spec_model.py): payload -> CRC24A -> segmentation -> turbo -> sub-block interleaving ->
rate matching -> scrambling (the e bits) -> QAM -> PDSCH resource mapping -> TM1 single-port or
TM3 two-port large-delay CDD precoding (the frequency grid txdataF), for the configurations the
bench and the GPU parity suite use (C1, C2, C3) and a bandwidth sweep 6 ... 100 PRB, in
subframes 0 (PBCH + sync exclusions), 5 (sync) and 7 (none).

The model shares nothing with the oracle's code; its departures from the spec are the
reference's, written as cited parameters: A6q filler bits encoded as 0, the int Q15 QAM tables
(the 64-QAM outer level 35393 exceeds int16 until the amp scaling; LTE_TRANSPORT/vars.h:72),
floor halving with the sign after the floor in CDD, and
the CDD sign reset per resource block (checked to coincide with the spec's global (-1)^i here:
every RB contributes an even number of REs)."""
import numpy as np
import pytest

import oracle_lib as O
import spec_model as S

FULL = {6: (0x3F, 0, 0, 0), 15: (0x7FFF, 0, 0, 0), 25: (0x1FFFFFF, 0, 0, 0),
        50: (0xFFFFFFFF, 0x3FFFF, 0, 0), 100: (0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xF)}


def run_case(name, N_RB, mcs, sf, nid, npdcch, tbs=None):
    import openair4g_amd as oai
    tbs = tbs or tuple(oai.tbs_bits(m, N_RB) if m else 0 for m in mcs)
    kw = dict(N_RB_DL=N_RB, rb_alloc=FULL[N_RB], nb_rb=N_RB, num_pdcch_symbols=npdcch, mcs=mcs, TBS=tbs)
    p = oai.make_params(name, subframe=sf, Nid_cell=nid, **kw)
    cfg = O.tx_cfg_from_params(p, sf)
    rng = np.random.default_rng(1000 * N_RB + 10 * sf + nid)
    pays = [rng.integers(0, 256, tbs[cw] // 8 + 8, dtype=np.uint8) for cw in range(p.n_cw)]
    _, txF, es = O.tx_subframe(cfg, pays, want_e=True)
    fp = cfg.fp
    N = fp.ofdm_symbol_size
    crs_ports = 1 if p.mode1_flag else 2
    res = S.pdsch_res(N_RB, N, fp.first_carrier_offset, nid % 6, npdcch, sf, crs_ports, rb_alloc=FULL[N_RB])
    e_spec = []
    for cw in range(p.n_cw):
        Qm = 2 if mcs[cw] < 10 else (4 if mcs[cw] < 17 else 6)
        G = O.get_G(N_RB, 0, p.mode1_flag, 0, N_RB, list(FULL[N_RB]), Qm, 1, npdcch, sf)
        assert G == Qm * len(res), (cw, G, len(res))                 # get_G == the model's RE count
        c_init = (p.rnti << 14) + (cw << 13) * 0 + (sf << 9) + nid     # dlsim passes q = 0 for both CWs
        e = S.dlsch_e(pays[cw][:tbs[cw] // 8], tbs[cw], G, Qm, Kmimo=p.Kmimo, c_init=c_init)
        assert np.array_equal(es[cw][:G], np.array(e, dtype=np.uint8)), f"e bits of CW{cw}"
        e_spec.append((e, Qm))
    if p.n_cw == 1:
        ref, used = S.siso_grid(e_spec[0][0], res, e_spec[0][1], p.nb_antennas_tx, N)
    else:
        ref, used = S.cdd2_grid(e_spec[0][0], e_spec[1][0], res, e_spec[0][1], e_spec[1][1], N)
        ref_rb, _ = S.cdd2_grid(e_spec[0][0], e_spec[1][0], res, e_spec[0][1], e_spec[1][1], N, sign_reset_per_rb=True)
        assert np.array_equal(ref, ref_rb)
    assert np.array_equal(txF, ref)
    assert O.modulation_count(cfg) == len(res)


@pytest.mark.parametrize("sf", [0, 5, 7])
@pytest.mark.parametrize("case", [("C1", 6, (9, 0), 0, 3), ("C2", 100, (16, 0), 0, 1),
                                  ("C3", 100, (19, 19), 0, 1)], ids=lambda c: c[0])
def test_config_grid_matches_spec(case, sf):
    name, N_RB, mcs, nid, npdcch = case
    run_case(name, N_RB, mcs, sf, nid, npdcch)


@pytest.mark.parametrize("N_RB,nid,sf", [(15, 1, 0), (25, 2, 5), (50, 4, 7), (15, 5, 5), (25, 3, 0), (50, 0, 0)])
@pytest.mark.parametrize("name,mcs", [("C2", (12, 0)), ("C3", (17, 22))])
def test_bandwidth_sweep_matches_spec(name, mcs, N_RB, nid, sf):
    """odd N_RB (DC-straddling RB, half-RB PBCH/sync edges) and every CRS shift class"""
    run_case(name, N_RB, mcs, sf, nid, 2)


@pytest.mark.parametrize("case", [("C1", 6, (9, 0), (1008, 0)), ("C2", 100, (16, 0), (10008, 0)),
                                  ("C3", 100, (19, 19), (30008, 20000))], ids=lambda c: c[0])
def test_filler_bits_match_spec(case):
    """Non-table TBS whose segmentation leaves F > 0 filler bits (A6q: encoded as 0,
    3gpplte_sse.c:380-476 / lte_segmentation.c:137-139), end to end through the grid."""
    name, N_RB, mcs, tbs = case
    B = tbs[0] + 24
    assert S.segment([0] * B)[1] > 0
    run_case(name, N_RB, mcs, 7, 1, 2, tbs=tbs)
