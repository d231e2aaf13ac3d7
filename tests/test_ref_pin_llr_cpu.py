"""The oracle's LLR stages against the reference's own PHY/LTE_TRANSPORT/dlsch_llr_computation.c
(dlsch_qpsk_llr :636, dlsch_16qam_llr :688, dlsch_64qam_llr :810, qpsk_qpsk :1041, qpsk_qam16 :1300,
qpsk_qam64 :1584), compiled unmodified into oracle/_ref/libref_llr.so (oracle/Makefile, glue
oracle/ref_glue_llr.c).  Full-range int16 inputs (saturation, abs(-32768) included).  The oracle's
receivers (orc_rx_pdsch_siso / _tm2 / _tm3 / _tm3_q2) run these per-RE stages.  Skipped where the
reference tree was not built (the GPU box); tests/test_llr_fixture_cpu.py covers the committed fixtures."""
import numpy as np
import pytest

import oracle_lib as O
from llr_ref_cases import ia_cases, ia_inputs, ia_written, qam_cases, qam_inputs, qam_len, qam_written

pytestmark = pytest.mark.skipif(O.ref_llr() is None, reason="oracle/_ref/libref_llr.so not built (no reference tree)")
SENT = 12345


def ref_qam(c):
    comp, mag, magb, _, _ = qam_inputs(c)
    comp, mag, magb = O.aligned(comp), O.aligned(mag), O.aligned(magb)
    llr = O.aligned(np.full(6 * (c["N_RB_DL"] * 12 + 16), SENT, np.int16))
    n = O.ref_llr().ref_glue_qam_llr(c["Qm"], c["N_RB_DL"], c["Ncp"], c["mode1_flag"], comp.ctypes.data, mag.ctypes.data,
                                     magb.ctypes.data, llr.ctypes.data, c["symbol"], c["nb_rb"], 0)
    return n, llr


def ref_ia(c):
    s0, s1, rho, m = (O.aligned(x) for x in ia_inputs(c))
    mag = O.aligned(np.repeat(m, 2))
    out = O.aligned(np.full(2 * c["n"] + 64, SENT, np.int16))
    R = O.ref_llr()
    if c["qm1"] == 2:
        R.qpsk_qpsk(s0.ctypes.data, s1.ctypes.data, out.ctypes.data, rho.ctypes.data, c["n"])
    elif c["qm1"] == 4:
        R.qpsk_qam16(s0.ctypes.data, s1.ctypes.data, mag.ctypes.data, out.ctypes.data, rho.ctypes.data, c["n"])
    else:
        R.qpsk_qam64(s0.ctypes.data, s1.ctypes.data, mag.ctypes.data, out.ctypes.data, rho.ctypes.data, c["n"])
    return out


@pytest.mark.parametrize("c", qam_cases(), ids=lambda c: f"Qm{c['Qm']}-{c['N_RB_DL']}prb-cp{c['Ncp']}-m{c['mode1_flag']}-l{c['symbol']}-nb{c['nb_rb']}")
def test_qam_llr_equals_reference(c):
    n, llr = ref_qam(c)
    L = qam_len(c)
    assert n == c["Qm"] * L                         # the output pointer advance: len REs
    w = qam_written(c)
    _, _, _, m, mb = qam_inputs(c)
    comp, _, _, _, _ = qam_inputs(c)
    o = c["symbol"] * c["N_RB_DL"] * 12
    orc = O.orc_llr_qam(c["Qm"], comp[o:o + L].view(np.int16), m[o:o + L], mb[o:o + L], L)
    assert np.array_equal(orc[:c["Qm"] * w], llr[:c["Qm"] * w])
    assert np.all(llr[c["Qm"] * w:c["Qm"] * L] == SENT)    # the 64-QAM remainder the reference skips


@pytest.mark.parametrize("c", ia_cases(), ids=lambda c: f"qm1{c['qm1']}-n{c['n']}")
def test_interference_aware_llr_equals_reference(c):
    out = ref_ia(c)
    s0, s1, rho, m = ia_inputs(c)
    orc = O.orc_llr_ia(c["qm1"], s0, s1, m, rho, c["n"])
    w = ia_written(c["n"])
    assert np.array_equal(orc[:2 * w], out[:2 * w])
    assert np.all(out[2 * w:2 * c["n"]] == SENT)
