"""GPU parity of the PCFICH drop-in (oai4g_generate_pcfich, pcfich.c:144-228; SURVEY.md 8f item
2) against the oracle restatement, which tests/test_pcfich_cpu.py pins to the 36.211 model.
Bit-exact on the whole frame grid (only the 16 PCFICH REs per antenna may change)."""
import numpy as np
import pytest

import oracle_lib as O
from test_pcfich_cpu import CASES

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N_RB,Nid,cfi,mode1,subframe", CASES)
def test_gpu_pcfich_drop_in(gpu, N_RB, Nid, cfi, mode1, subframe):
    n_ant = 1 if mode1 else 2
    fp_o = O.frame(N_RB, Nid_cell=Nid, nb_antennas_tx=n_ant, mode1_flag=mode1)
    fp_g = gpu.frame_parms(N_RB, Nid_cell=Nid, nb_antennas_tx=n_ant, mode1_flag=mode1)
    N, nsymb = fp_o.ofdm_symbol_size, fp_o.symbols_per_tti
    rng = np.random.default_rng(N_RB + Nid)
    base = [rng.integers(-2**31, 2**31 - 1, 10 * nsymb * N, dtype=np.int64).astype(np.int32) for _ in range(n_ant)]
    g_o = [b.copy() for b in base]
    g_g = [b.copy() for b in base]
    assert O.generate_pcfich(cfi, 1024, fp_o, g_o, subframe) == 0
    assert gpu.generate_pcfich(cfi, 1024, fp_g, g_g, subframe) == 0
    for a in range(n_ant):
        assert np.array_equal(g_g[a], g_o[a]), a


def test_gpu_pcfich_reg_mapping_and_errors(gpu):
    import ctypes
    for N_RB, Nid in ((6, 0), (25, 13), (100, 377), (50, 99)):
        fp = gpu.frame_parms(N_RB, Nid_cell=Nid)
        reg = (ctypes.c_uint16 * 4)()
        first = ctypes.c_uint8()
        gpu.lib().oai4g_generate_pcfich_reg_mapping(fp, reg, ctypes.byref(first))
        assert (list(reg), first.value) == O.pcfich_reg_mapping(O.frame(N_RB, Nid_cell=Nid))
    fp = gpu.frame_parms(25)
    g = [np.zeros(10 * 14 * fp.ofdm_symbol_size, np.int32)]
    assert gpu.generate_pcfich(0, 512, fp, g, 0) == -1
    assert gpu.generate_pcfich(4, 512, fp, g, 0) == -1
