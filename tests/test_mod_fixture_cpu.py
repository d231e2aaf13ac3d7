"""The oracle's modulation / RE mapping / precoding, scrambling and PCFICH against the fixtures the
reference's own dlsch_modulation.c / dlsch_scrambling.c / pcfich.c produced here (tests/golden/mod_ref.json,
tests/golden/gen_mod_ref.py).  Runs everywhere, the reference tree not needed."""
import json
import os

import numpy as np
import pytest

import oracle_lib as O
from mod_ref_cases import cws_of, e_bits, frame_of, grid_digests, symbol0_digests
from rm_ref_cases import digest

FIX = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mod_ref.json")))


@pytest.mark.parametrize("i", range(len(FIX["modulation"])))
def test_oracle_modulation_equals_reference_fixture(i):
    m = FIX["modulation"][i]
    c = m["case"]
    fp = frame_of(O, c)
    ret, grids = O.orc_modulation_grids(fp, c["amp"], c["subframe"], c["num_pdcch"], cws_of(c), *c["rho"])
    assert ret == m["ret"]
    assert grid_digests(grids, c, fp.ofdm_symbol_size) == m["digests"]


@pytest.mark.parametrize("i", range(len(FIX["scrambling"])))
def test_oracle_scrambling_equals_reference_fixture(i):
    s = FIX["scrambling"][i]
    c = s["case"]
    G = c["G"]
    e = e_bits(c["seed"])[:32 * (1 + (G >> 5))]
    got = O.scramble(e, G, (c["rnti"] << 14) + (c["q"] << 13) + ((c["Ns"] >> 1) << 9) + c["Nid_cell"])
    assert digest(got[:G]) == s["digest"]


@pytest.mark.parametrize("i", range(len(FIX["pcfich"])))
def test_oracle_pcfich_equals_reference_fixture(i):
    p = FIX["pcfich"][i]
    c = p["case"]
    fp = frame_of(O, c)
    assert O.pcfich_reg_mapping(fp) == (p["reg"], p["first"])
    n = 10 * (12 if c["Ncp"] else 14) * fp.ofdm_symbol_size
    grids = [np.zeros(n, np.int32) for _ in range(c["n_ant"])]
    assert O.generate_pcfich(c["cfi"], c["amp"], fp, grids, c["subframe"]) == 0
    assert symbol0_digests(grids, c, fp.ofdm_symbol_size) == p["digests"]
