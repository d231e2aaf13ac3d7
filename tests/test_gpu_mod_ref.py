"""The library's drop-in dlsch_modulation, dlsch_scrambling and generate_pcfich (C ABI
oai4g_dlsch_modulation / oai4g_dlsch_scrambling / oai4g_generate_pcfich, HIP kernels) against the
fixtures the reference's own dlsch_modulation.c, dlsch_scrambling.c and pcfich.c produced here
(tests/golden/mod_ref.json): frame grids digest for digest, the return value (re_allocated) equal,
scrambled e bits equal, the PCFICH REG mapping equal."""
import ctypes
import json
import os

import numpy as np
import pytest

from mod_ref_cases import NBITS, e_bits, grid_digests, symbol0_digests
from rm_ref_cases import digest

pytestmark = pytest.mark.gpu

FIX = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mod_ref.json")))


def _dlsch(gpu, c, cw, rnti=0):
    dl = gpu.DlschHandle(Kmimo=1, Mdlharq=8, N_RB_DL=c["N_RB_DL"])
    h = dl.h
    h.mcs = c["mcs"][cw]
    h.mimo_mode = c["mimo_mode"]
    for i in range(4):
        h.rb_alloc[i] = c["rb_alloc"][i]
    h.nb_rb = sum(bin(int(w)).count("1") for w in c["rb_alloc"])
    h.Nl = 1
    h.Nlayers = 1
    h.TBS = 1024         # the drop-in derives a coding geometry it does not use for the grid
    dl.d.rnti = rnti
    return dl


@pytest.mark.parametrize("i", range(len(FIX["modulation"])))
def test_dlsch_modulation_equals_reference(gpu, i):
    m = FIX["modulation"][i]
    c = m["case"]
    fp = gpu.frame_parms(c["N_RB_DL"], c["Nid_cell"], c["Ncp"], c["n_ant"], c["mode1_flag"], 0)
    dls = []
    for cw in range(c["n_cw"]):
        dl = _dlsch(gpu, c, cw)
        dl.view("e", NBITS)[:] = e_bits(c["seed"][cw])
        dl.d.sqrt_rho_a, dl.d.sqrt_rho_b = c["rho"]
        dls.append(dl)
    nsymb = 12 if c["Ncp"] else 14
    grids = [np.zeros(10 * nsymb * fp.ofdm_symbol_size, dtype=np.int32) for _ in range(c["n_ant"])]
    ret = gpu.dlsch_modulation(grids, c["amp"], c["subframe"], fp, c["num_pdcch"], dls[0],
                               dls[1] if c["n_cw"] > 1 else None)
    assert ret == m["ret"]
    assert grid_digests(grids, c, fp.ofdm_symbol_size) == m["digests"]


@pytest.mark.parametrize("i", range(len(FIX["scrambling"])))
def test_dlsch_scrambling_equals_reference(gpu, i):
    s = FIX["scrambling"][i]
    c = s["case"]
    G = c["G"]
    dl = gpu.DlschHandle(Kmimo=1, Mdlharq=8, N_RB_DL=100)
    dl.d.rnti = c["rnti"]
    fp = gpu.frame_parms(100, c["Nid_cell"], 0, 1, 1, 0)
    e = dl.view("e", NBITS)
    e[:] = e_bits(c["seed"])
    gpu.dlsch_scrambling(fp, dl, G, c["q"], c["Ns"])
    assert digest(dl.view("e", G)) == s["digest"]


@pytest.mark.parametrize("i", range(len(FIX["pcfich"])))
def test_generate_pcfich_equals_reference(gpu, i):
    p = FIX["pcfich"][i]
    c = p["case"]
    fp = gpu.frame_parms(c["N_RB_DL"], c["Nid_cell"], c["Ncp"], c["n_ant"], c["mode1_flag"], 0)
    reg = (ctypes.c_uint16 * 4)()
    first = ctypes.c_uint8()
    gpu.lib().oai4g_generate_pcfich_reg_mapping(fp, reg, ctypes.byref(first))
    assert (list(reg), first.value) == (p["reg"], p["first"])
    nsymb = 12 if c["Ncp"] else 14
    grids = [np.zeros(10 * nsymb * fp.ofdm_symbol_size, dtype=np.int32) for _ in range(c["n_ant"])]
    assert gpu.generate_pcfich(c["cfi"], c["amp"], fp, grids, c["subframe"]) == 0
    assert symbol0_digests(grids, c, fp.ofdm_symbol_size) == p["digests"]
