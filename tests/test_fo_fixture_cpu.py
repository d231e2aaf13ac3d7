"""The oracle's lte_est_freq_offset against the fixtures the reference's own lte_est_freq_offset.c
produced here (tests/golden/fo_ref.json, tests/golden/gen_fo_ref.py; cases in tests/fo_ref_cases.py).
Runs everywhere, the reference tree not needed."""
import json
import os

import pytest

from test_ref_pin_fo_cpu import orc_sequence

FIX = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fo_ref.json")))


@pytest.mark.parametrize("i", range(len(FIX["cases"])))
def test_oracle_freq_offset_equals_reference_fixture(i):
    f = FIX["cases"][i]
    assert orc_sequence(f["case"]) == [tuple(x) for x in f["calls"]]
