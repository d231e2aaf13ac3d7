"""The batched transmit path carrying the eNB's whole downlink grid: PDSCH, cell-specific RS, the
control region of oai4g_tx_config_set_control (PCFICH + PDCCH) and the common signals of
oai4g_tx_config_set_common (PSS + SSS in subframes 0 / 5, PBCH in subframe 0, PHICHs) —
phy_procedures_lte_eNb.c's txdataF — through the IDFT + CP.  Bit-exact IQ against the oracle:
orc_tx_subframe_dci's grid with the oracle's generate_pss / _sss / _pbch / _phich applied in a
frame grid, then orc_normal_prefix_mod, for all 10 subframe indices."""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
from test_gpu_control_batch import _items

pytestmark = pytest.mark.gpu


def _oracle_iq(p, sf, pay, items, n_common, pdu, fm4, phich, pbch_state):
    cfg = O.tx_cfg_from_params(p, sf)
    _, txF, _ = O.tx_subframe(cfg, [pay[cw] for cw in range(p.n_cw)], dci=items, n_common=n_common)
    fp = cfg.fp
    N, nsymb, n_ant = fp.ofdm_symbol_size, fp.symbols_per_tti, fp.nb_antennas_tx
    frame = [np.zeros(10 * nsymb * N + N, np.int32) for _ in range(n_ant)]
    for a in range(n_ant):
        frame[a][sf * nsymb * N:(sf + 1) * nsymb * N] = txF[a][:nsymb * N]
    nsl = nsymb // 2
    if sf in (0, 5):                                   # phy_procedures_lte_eNb.c:1547-1556, 1700-1711
        assert O.generate_pss(frame, p.amp, fp, nsl - 1, 2 * sf) == 0
        assert O.generate_sss(frame, p.amp, fp, nsl - 2, 2 * sf) == 0
    if sf == 0 and pdu is not None:                    # :1662 (frame_mod4 0 encodes, the others map)
        scratch = [np.zeros_like(f) for f in frame]
        assert O.generate_pbch(pbch_state, scratch, p.amp, fp, pdu, 0) == 0
        assert O.generate_pbch(pbch_state, frame, p.amp, fp, pdu, fm4) == 0
    for (psf, g, q, h) in phich:
        if psf == sf:
            assert O.generate_phich(fp, p.amp, q, g, h, sf, frame) == 0
    txd = [np.zeros(fp.samples_per_tti, np.int32) for _ in range(n_ant)]
    for a in range(n_ant):
        sub = np.ascontiguousarray(frame[a][sf * nsymb * N:(sf + 1) * nsymb * N])
        O.orc().orc_normal_prefix_mod(O.P(sub), O.P(txd[a]), nsymb, ctypes.byref(fp))
    return np.stack(txd)


@pytest.mark.parametrize("name,nid,fm4,dci", [("C3", 0, 0, True), ("C3", 13, 2, True), ("C2", 7, 1, False),
                                               ("TM2", 41, 3, True), ("C1", 2, 0, True)])
def test_batch_full_grid(gpu, name, nid, fm4, dci):
    p = gpu.make_params(name, subframe=0, subframe_step=1, Nid_cell=nid, with_crs=1)
    n_ant = p.nb_antennas_tx
    items, n_common = _items(gpu, name, p, False) if dci else ([], 0)
    fo = O.frame(p.N_RB_DL, nid, p.Ncp, n_ant, p.mode1_flag)
    ng = len(O.phich_reg_mapping(fo))
    rng = np.random.default_rng(nid + 11)
    phich = [] if (p.mode1_flag == 1 and n_ant > 1) or nid % 6 >= 3 else \
        [(int(sf), int(rng.integers(0, ng)), int(rng.integers(0, 8)), int(rng.integers(0, 2))) for sf in (0, 3, 3, 7, 9)]
    pdu = rng.integers(0, 256, 3, dtype=np.uint8)
    pipe = gpu.TxPipeline(p, 10)
    if items:
        pipe.set_control(items, n_common)
    pipe.set_common(pss_sss=True, pbch_pdu=pdu, frame_mod4=fm4, phich=phich)
    pay = rng.integers(0, 256, size=(10, p.n_cw, p.payload_stride), dtype=np.uint8)
    pipe.upload_payload(pay)
    pipe.run()
    pipe.sync()
    iq = pipe.iq()
    st = O.OrcPbch()
    for sf in range(10):
        want = _oracle_iq(p, sf, pay[sf], items, n_common, pdu, fm4, phich, st)
        assert np.array_equal(iq[sf], want), (name, sf)
    # switching the common signals off restores the PDSCH + CRS (+ control) grid
    pipe.set_common()
    pipe.run()
    pipe.sync()
    txd, _, _ = O.tx_subframe(O.tx_cfg_from_params(p, 0), [pay[0, cw] for cw in range(p.n_cw)],
                              dci=items or None, n_common=n_common)
    assert np.array_equal(pipe.iq()[0], txd)
    pipe.close()
