"""GPU parity of the opt-in limited-buffer rate matching (the build's
extension, not the reference): TM3 MCS >= 20 transport blocks whose code blocks do not fit the
soft buffer (Ncb < Kw), which the reference refuses (lte_rate_matching.c:518-521).  The batch
path with oai4g_tx_params_t.rm_limited_buffer = 1 is compared bit-exactly with the oracle whose
rate matcher is pinned to 36.212 5.1.4.1.2 by test_oracle_cpu.py."""
import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mcs,tbs,rv,sf", [(28, 75376, 0, 7), (22, 43816, 2, 7), (28, 75376, 3, 5)])
def test_gpu_limited_buffer_rm_batch(gpu, mcs, tbs, rv, sf):
    p = gpu.make_params("C3", subframe=sf, mcs=[mcs, mcs], TBS=[tbs, tbs])
    p.rm_limited_buffer = 1
    for cw in range(p.n_cw):
        p.rvidx[cw] = rv
    n_sf = 2
    pipe = gpu.TxPipeline(p, n_sf)
    rng = np.random.default_rng(mcs + rv)
    pay = rng.integers(0, 256, size=(n_sf, p.n_cw, p.payload_stride), dtype=np.uint8)
    pipe.upload_payload(pay)
    pipe.run()
    pipe.sync()
    iq = pipe.iq().copy()
    pipe.close()
    O.set_rm_limited(True)
    try:
        for i in range(n_sf):
            ref, _, _ = O.tx_subframe(O.tx_cfg_from_params(p, sf), [pay[i, cw] for cw in range(p.n_cw)])
            assert np.array_equal(iq[i], np.asarray(ref)), i
    finally:
        O.set_rm_limited(False)


def test_gpu_limited_buffer_off_keeps_reference_exit(gpu):
    p = gpu.make_params("C3", subframe=7, mcs=[28, 28], TBS=[75376, 75376])
    with pytest.raises(Exception):
        gpu.TxPipeline(p, 1)
