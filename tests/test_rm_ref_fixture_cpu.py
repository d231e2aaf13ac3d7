"""The oracle's rate matcher and Gold generator reproduce the reference-generated fixtures
(tests/golden/rm_ref.{json,npz}, made by tests/golden/gen_rm_ref.py from the reference's
lte_rate_matching.c / lte_gold.c compiled unmodified).  Runs everywhere (the fixtures travel;
the reference does not): the pin of tests/test_ref_pin_rm_cpu.py, carried to the GPU box."""
import json
import os

import numpy as np
import pytest

import oracle_lib as O
import rm_ref_cases as RC

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "rm_ref.json")))
ARR = np.load(os.path.join(HERE, "golden", "rm_ref.npz"))
IMPL = RC.oracle_impl(O)


def check_sweeps(impl, ks=None):
    """Every digest of rm_ref.json against `impl` (shared with tests/test_gpu_rm_ref.py)."""
    for K in (ks or RC.KS):
        R, w = RC.run_sbi(impl, K)
        assert [int(R), RC.digest(w)] == FIX["sbi"][str(K)], ("sbi", K)
        Es, e = RC.run_rm_sweep(impl, K)
        assert [Es, RC.digest(e)] == FIX["rm"][str(K)], ("rm", K)
        assert RC.digest(RC.run_dummy_w(impl, K)) == FIX["dummy_w"][str(K)], ("dummy_w", K)
    for K in RC.RX_KS:
        Es, w = RC.run_rm_rx(impl, K)
        assert [Es, RC.digest(w)] == FIX["rm_rx"][str(K)], ("rm_rx", K)
    for K in RC.DEINT_KS:
        assert RC.digest(RC.run_deint(impl, K)) == FIX["deint"][str(K)], ("deint", K)
    assert RC.digest(RC.run_gold(impl)) == FIX["gold"]


def test_oracle_reproduces_reference_digests():
    check_sweeps(IMPL)


@pytest.mark.parametrize("name", sorted(RC.MAP_GEOMS))
def test_oracle_rm_map_equals_reference(name):
    K, G, C, Qm, Kmimo, Nl = RC.MAP_GEOMS[name]
    for r in sorted({0, C - 1}):
        assert np.array_equal(RC.rm_map(IMPL, K, G, C, r, Qm, Kmimo, Nl), ARR["map_" + name].astype(np.int32))


def test_oracle_gold_words_equal_reference():
    for sf in range(10):
        assert np.array_equal(IMPL["gold"](RC.c_init(0x1234, 0, sf, 0), 2701), ARR["gold_sf"][sf])


def test_fixture_shapes():
    assert len(FIX["sbi"]) == 188 and len(FIX["rm"]) == 188 and len(FIX["dummy_w"]) == 188
    assert ARR["map_C3"].shape == (14400,) and ARR["map_C2"].shape == (12000,) and ARR["map_C1"].shape == (1512,)
    # the composed map is a selection without repeats at these geometries (E < Kw - NULLs)
    for n in ("map_C1", "map_C2", "map_C3"):
        assert len(np.unique(ARR[n])) == len(ARR[n])
