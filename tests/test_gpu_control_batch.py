"""The batched transmit path with the control region (oai4g_tx_config_set_control): every
subframe of the batch carries generate_dci_top's PCFICH + PDCCH (dlsim.c:2553) beside the PDSCH
and, with with_crs, the cell-specific RS (dlsim.c:2681) — dlsim's complete txdataF — through the
IDFT + CP.  Bit-exact IQ against the oracle (orc_tx_subframe_dci) for all 10 subframe indices."""
import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

# dlsim's DCIs: format 1 (TM1/TM2: 23 bits at 1.4 MHz, 39 at 20 MHz), 2A (TM3, 48 bits), L = 1
DCI_LEN = {"C1": 23, "C2": 39, "C3": 48, "C4": 48, "TM2": 39, "TM2S": 23}


def _items(gpu, name, p, extra_common=False):
    fp = O.frame(p.N_RB_DL, p.Nid_cell, p.Ncp, p.nb_antennas_tx, p.mode1_flag)
    npd = p.num_pdcch_symbols
    nCCE = O.get_nCCE(npd, fp)
    table = np.zeros(800, np.int32)
    rng = np.random.default_rng(len(name) + p.Nid_cell)
    items = []
    if extra_common:                              # an SI-RNTI format 1A DCI (dlsim.c:1292-1297)
        items.append((28, 2, O.get_nCCE_offset(table, 4, nCCE, 1, 0xFFFF, 7), 0xFFFF,
                      rng.integers(0, 256, 8, dtype=np.uint8)))
    items.append((DCI_LEN[name], 1, O.get_nCCE_offset(table, 2, nCCE, 0, p.rnti, 7), p.rnti,
                  rng.integers(0, 256, 8, dtype=np.uint8)))
    return items, (1 if extra_common else 0)


@pytest.mark.parametrize("name,crs,nid,common", [("C1", 1, 0, False), ("C2", 1, 0, False), ("C3", 1, 0, False),
                                                 ("C3", 0, 77, True), ("TM2", 1, 41, True), ("C4", 1, 5, False),
                                                 ("TM2S", 1, 3, False)])
def test_batch_with_control(gpu, name, crs, nid, common):
    p = gpu.make_params(name, subframe=0, subframe_step=1, Nid_cell=nid, with_crs=crs)
    if name in ("C2", "C3", "C4", "TM2"):
        p.num_pdcch_symbols = 2 if common else 1
    items, n_common = _items(gpu, name, p, common)
    pipe = gpu.TxPipeline(p, 10)
    pipe.set_control(items, n_common)
    pay = np.random.default_rng(nid + 5).integers(0, 256, size=(10, p.n_cw, p.payload_stride), dtype=np.uint8)
    pipe.upload_payload(pay)
    pipe.run()
    pipe.sync()
    iq = pipe.iq()
    for sf in range(10):
        txd, _, _ = O.tx_subframe(O.tx_cfg_from_params(p, sf), [pay[sf, cw] for cw in range(p.n_cw)],
                                  dci=items, n_common=n_common)
        assert np.array_equal(iq[sf], txd), (name, sf)
    # switching the control region off restores the plain PDSCH (+ CRS) grid
    pipe.set_control([])
    pipe.run()
    pipe.sync()
    txd, _, _ = O.tx_subframe(O.tx_cfg_from_params(p, 3), [pay[3, cw] for cw in range(p.n_cw)])
    assert np.array_equal(pipe.iq()[3], txd)
    pipe.close()
