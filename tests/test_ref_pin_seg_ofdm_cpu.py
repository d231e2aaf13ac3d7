"""Oracle pinned to the reference's own code-block segmentation and OFDM modulator, compiled
unmodified here (oracle/Makefile: _ref/libref_seg.so = PHY/CODING/lte_segmentation.c,
_ref/libref_ofdm.so = PHY/MODULATION/ofdm_mod.c).  Runs only in the build container, where
/root/reference exists; the results travel as tests/golden/seg_ofdm_ref.{json,npz}
(tests/golden/gen_seg_ofdm_ref.py), which tests/test_seg_ofdm_fixture_cpu.py and
tests/test_gpu_seg_ofdm_ref.py check.

Pinned here, bit-exact, oracle against reference, array by array:
  - lte_segmentation (:39-176): C, C+/C-, K+/K-, F for every B < 20000, every TBS + 24 of the TBS
    table and the C > 16 refusal; the code-block buffers (filler bytes :141-143, payload :154-159,
    CRC-24B :161-169) for every 17th byte-aligned B and the multi-block edges;
  - PHY_ofdm_mod (:85-230), CYCLIC_PREFIX: N = 128 (static temp) .. 2048, 1..14 symbols;
  - normal_prefix_mod (:47-83): 6/15/25/50/100 PRB, normal and extended prefix, nsymb 1..14;
  - do_OFDM_mod (:233-284): slot offsets of whole-frame buffers, 1/2/4 antennas, both prefixes.
"""
import numpy as np
import pytest

import oracle_lib as O
import seg_ofdm_ref_cases as SC
from test_seg_ofdm_fixture_cpu import oracle_frame

pytestmark = pytest.mark.skipif(O.ref_seg() is None or O.ref_ofdm() is None,
                                reason="oracle/_ref/libref_seg.so / libref_ofdm.so not built (no reference tree)")
REF = SC.ref_impl(O) if O.ref_seg() is not None and O.ref_ofdm() is not None else None
ORC = SC.oracle_impl(O)


def test_segmentation_parameters_all_B():
    Bs = np.arange(0, 20000)
    assert np.array_equal(SC.run_seg_params(ORC, Bs), SC.run_seg_params(REF, Bs))
    big = np.array(SC.SEG_EXTRA_B + tuple(range(20000, 97921, 97)) + (97928, 98304, 120000), np.int64)
    assert np.array_equal(SC.run_seg_params(ORC, big), SC.run_seg_params(REF, big))


@pytest.mark.parametrize("B", [8, 40, 48, 512, 520, 1024, 1032, 2048, 2056, 6144, 6152, 6168, 12240, 12288, 18360,
                               30576 + 24, 36720, 61200, 75376 + 24, 97920])
def test_segmentation_buffers(B):
    data = SC.seg_payload(B)
    r_ret, r_vals, r_bufs = O.ref_segmentation(B, data)
    o_ret, o_vals, o_bufs = ORC["seg"](B, data)
    assert r_ret == o_ret == 0 and r_vals == o_vals
    for r in range(r_vals[0]):
        assert np.array_equal(o_bufs[r], r_bufs[r]), (B, r)


@pytest.mark.parametrize("case", SC.OFDM_CASES)
def test_phy_ofdm_mod(case):
    assert np.array_equal(SC.run_ofdm_mod(ORC, case), SC.run_ofdm_mod(REF, case))


@pytest.mark.parametrize("n_rb,ncp", SC.NPM_FRAMES)
def test_normal_prefix_mod(n_rb, ncp):
    fp = oracle_frame(n_rb, ncp, 1)
    for nsymb in SC.NPM_NSYMB:
        assert np.array_equal(SC.run_npm(ORC, fp, nsymb), SC.run_npm(REF, fp, nsymb)), nsymb


@pytest.mark.parametrize("n_rb,ncp,na", SC.DO_OFDM_FRAMES)
def test_do_ofdm_mod(n_rb, ncp, na):
    fp = oracle_frame(n_rb, ncp, na)
    for slot in SC.DO_OFDM_SLOTS:
        assert np.array_equal(SC.run_do_ofdm(ORC, fp, 3, slot), SC.run_do_ofdm(REF, fp, 3, slot)), slot


def test_normal_prefix_mod_full_grid_subframe():
    """A C3-shaped subframe (100 PRB, both slots) through do_OFDM_mod twice, as dlsim's
    do_OFDM_mod_l loop does, equals the oracle."""
    fp = oracle_frame(100, 0, 2)
    for slot in (14, 15):
        assert np.array_equal(SC.run_do_ofdm(ORC, fp, 0, slot), SC.run_do_ofdm(REF, fp, 0, slot))
