"""F > 0 filler bits on the GPU: non-table transport block sizes whose code
block segmentation leaves filler bits (lte_segmentation.c:137-139; the reference encodes them
as 0, 3gpplte_sse.c:380-476).  Batch path and drop-in dlsch_encoding, bit-exact against the
oracle, which tests/test_spec_grid_cpu.py::test_filler_bits_match_spec pins to the spec model."""
import numpy as np
import pytest

import oracle_lib as O
from test_gpu_parity import _pipeline_check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,tbs", [("C1", (1008, 0)), ("C2", (10008, 0)), ("C3", (30008, 20000))])
def test_pipeline_filler(gpu, name, tbs):
    _pipeline_check(gpu, name, 10, 0, 1, seed=11, TBS=tbs)


@pytest.mark.parametrize("tbs", [1008, 10008, 6200])
def test_drop_in_dlsch_encoding_filler(gpu, tbs):
    p = gpu.make_params("C2", subframe=7, TBS=(tbs, 0))
    cfg = O.tx_cfg_from_params(p, 7)
    fp = gpu.frame_parms(p.N_RB_DL, p.Nid_cell, 0, p.nb_antennas_tx, p.mode1_flag, 0)
    pay = np.random.default_rng(tbs).integers(0, 256, size=tbs // 8 + 8, dtype=np.uint8)
    _, _, e_o = O.tx_subframe(cfg, [pay.copy()], want_e=True)
    dl = gpu.DlschHandle(Kmimo=p.Kmimo, Mdlharq=8, N_RB_DL=p.N_RB_DL)
    h = dl.h
    h.TBS, h.mcs, h.rvidx, h.round, h.mimo_mode, h.Nl = tbs, p.mcs[0], 0, 0, p.mimo_mode, 1
    for i in range(4):
        h.rb_alloc[i] = p.rb_alloc[i]
    h.nb_rb = p.nb_rb
    dl.d.rnti = p.rnti
    assert gpu.dlsch_encoding(pay.copy(), fp, p.num_pdcch_symbols, dl, 7) == 0
    G = O.get_G(p.N_RB_DL, 0, p.mode1_flag, 0, p.nb_rb, list(p.rb_alloc), gpu.lib().oai4g_get_Qm(p.mcs[0]), 1,
                p.num_pdcch_symbols, 7)
    gpu.dlsch_scrambling(fp, dl, G, 0, 14)
    assert np.array_equal(dl.view("e", G), e_o[0][:G])
