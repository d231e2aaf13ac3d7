"""GPU parity against the reference's own segmentation and OFDM modulator (lte_segmentation.c,
ofdm_mod.c compiled unmodified in the build container; their outputs travel as
tests/golden/seg_ofdm_ref.{json,npz}, made by tests/golden/gen_seg_ofdm_ref.py).

  - the drop-ins oai4g_lte_segmentation, oai4g_PHY_ofdm_mod, oai4g_normal_prefix_mod and
    oai4g_do_OFDM_mod reproduce every parameter row and digest of the fixture
    (tests/seg_ofdm_ref_cases.py defines the cases);
  - the C3 bench batch (8192 subframes, bench.py's seed, the fused k_modofdm path): the payloads the
    device generated equal the restated generator, and the sampled subframes' IQ equals the
    reference's do_OFDM_mod (IDFT, CP, slot layout) applied to the oracle's grid of that subframe;
  - every CP region of all 8192 x 2 antennas x 14 symbols equals the tail of its symbol
    (ofdm_mod.c:167-171) at the reference's slot layout (:57-79)."""
import numpy as np
import pytest

import seg_ofdm_ref_cases as SC
from test_seg_ofdm_fixture_cpu import FIX, check_ofdm, check_seg, oracle_frame

pytestmark = pytest.mark.gpu


def test_dropin_segmentation_reproduces_reference(gpu):
    check_seg(SC.gpu_impl(gpu))


def test_dropin_ofdm_reproduces_reference(gpu):
    check_ofdm(SC.gpu_impl(gpu), oracle_frame)


def _cp_layout(fp):
    """(start of the symbol body, prefix length) of the 14 symbols of a subframe, as
    normal_prefix_mod lays them out (ofdm_mod.c:57-79): per slot, symbol 0 with nb_prefix_samples0,
    then 6 with nb_prefix_samples."""
    N, half = fp.ofdm_symbol_size, fp.samples_per_tti // 2
    cp0, cp = fp.nb_prefix_samples0, fp.nb_prefix_samples
    out = []
    for slot in range(2):
        out.append((slot * half + cp0, cp0))
        for j in range(6):
            out.append((slot * half + N + cp0 + j * N + (1 + j) * cp, cp))
    return out


def test_c3_bench_batch_against_reference_ofdm(gpu):
    p = gpu.make_params("C3", subframe=7)
    pipe = gpu.TxPipeline(p, SC.BENCH_N_SF)
    pipe.fill_payload(seed=SC.BENCH_SEED)
    pipe.run()
    pipe.sync()
    pay = pipe.download_payload()
    assert np.array_equal(pay, SC.bench_payload(SC.BENCH_SEED, SC.BENCH_N_SF, p.n_cw, p.payload_stride))
    del pay
    iq = pipe.iq()
    pipe.close()
    for i in SC.BENCH_C3_SAMPLES:
        assert [SC.digest(iq[i, a]) for a in range(iq.shape[1])] == FIX["bench_C3"][str(i)], i
    fp = oracle_frame(100, 0, 2)
    N = fp.ofdm_symbol_size
    assert _cp_layout(fp)[-1][0] + N == fp.samples_per_tti
    for start, cp in _cp_layout(fp):
        assert np.array_equal(iq[:, :, start - cp:start], iq[:, :, start + N - cp:start + N]), start
