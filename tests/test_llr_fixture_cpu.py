"""The oracle's LLR stages against the fixtures the reference's own dlsch_llr_computation.c produced
here (tests/golden/llr_ref.json, tests/golden/gen_llr_ref.py; cases and quirks in
tests/llr_ref_cases.py).  Runs everywhere, the reference tree not needed."""
import json
import os

import numpy as np
import pytest

import oracle_lib as O
from llr_ref_cases import digest, ia_inputs, ia_written, qam_inputs, qam_len, qam_written

FIX = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "llr_ref.json")))


@pytest.mark.parametrize("i", range(len(FIX["qam"])))
def test_oracle_qam_llr_equals_reference_fixture(i):
    f = FIX["qam"][i]
    c = f["case"]
    L = qam_len(c)
    assert f["advance"] == c["Qm"] * L
    comp, _, _, m, mb = qam_inputs(c)
    o = c["symbol"] * c["N_RB_DL"] * 12
    orc = O.orc_llr_qam(c["Qm"], comp[o:o + L].view(np.int16), m[o:o + L], mb[o:o + L], L)
    assert digest(orc[:c["Qm"] * qam_written(c)]) == f["digest"]


@pytest.mark.parametrize("i", range(len(FIX["ia"])))
def test_oracle_interference_aware_llr_equals_reference_fixture(i):
    f = FIX["ia"][i]
    c = f["case"]
    s0, s1, rho, m = ia_inputs(c)
    orc = O.orc_llr_ia(c["qm1"], s0, s1, m, rho, c["n"])
    assert digest(orc[:2 * ia_written(c["n"])]) == f["digest"]
