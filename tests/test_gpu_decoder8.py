"""GPU parity of the 8-bit turbo decoder (k_td8, oai4g_decode8.hip) against the oracle restatement
(oracle/oai_oracle_td8.c, pinned by tests/test_td8_cpu.py): iteration counts and decoded bytes
bit-exact for the drop-in and the batch (blocks stopping at different iterations in one wave),
over block sizes of both hard-decision branches (K mod 128 = 0 or not), every input-scaling
shift, CRC24A / CRC24B, filler F > 0 and saturating inputs."""
import numpy as np
import pytest

import oracle_lib as O
from ref_cases import QPP, crc_block, llrs

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("K", [512, 528, 1024, 1056, 4160, 5504, 6144])
def test_gpu_decoder8_drop_in(gpu, K):
    rng = np.random.default_rng(K)
    for amp, sigma, crc, max_it in ((32, 24, 0, 8), (8, 6, 1, 6), (100, 90, 0, 8), (300, 220, 1, 4), (64, 0, 0, 2),
                                    (40, 45, 1, 3)):
        c = crc_block(rng, K, crc)
        y = llrs(O.turbo_encode(c, *QPP[K]), amp, sigma, rng)
        it_o, d_o = O.turbo_decode8(y, K, max_it=max_it, crc_type=crc)
        it_g, d_g = gpu.turbo_decoder8(y, K, max_iterations=max_it, crc_type=crc)
        assert it_g == it_o, (K, amp, sigma)
        if max_it > 1:
            assert np.array_equal(d_g, d_o), (K, amp, sigma)


def test_gpu_decoder8_saturating_inputs(gpu):
    rng = np.random.default_rng(3)
    for K in (1024, 2112):
        y = rng.choice([-32768, 32767, -32767, 0, 1, -1, 200, -200], size=3 * K + 12).astype(np.int16)
        it_o, d_o = O.turbo_decode8(y, K, max_it=4)
        it_g, d_g = gpu.turbo_decoder8(y, K, max_iterations=4)
        assert it_g == it_o and np.array_equal(d_g, d_o), K


def test_gpu_decoder8_filler(gpu):
    rng = np.random.default_rng(9)
    for K, F in ((1056, 24), (2048, 64)):
        for sigma in (0, 20):
            c = crc_block(rng, K, 0, F)
            y = llrs(O.turbo_encode(c, *QPP[K]), 32, sigma, rng)
            it_o, d_o = O.turbo_decode8(y, K, crc_type=0, F=F)
            it_g, d_g = gpu.turbo_decoder8(y, K, crc_type=0, F=F)
            assert it_g == it_o and np.array_equal(d_g, d_o), (K, F, sigma)


@pytest.mark.parametrize("K,n_cb", [(5504, 61), (1056, 40)])
def test_gpu_decoder8_batch(gpu, K, n_cb):
    rng = np.random.default_rng(K + n_cb)
    ys = []
    for i in range(n_cb):
        c = crc_block(rng, K, 1)
        sigma = (0, 20, 28, 34, 40)[i % 5]
        ys.append(llrs(O.turbo_encode(c, *QPP[K]), 32, sigma, rng))
    ys = np.stack(ys)
    dec = gpu.TurboDecoder8Batch(K, n_cb)
    dec.upload(ys)
    dec.run(max_iterations=8, crc_type=1)
    its, outs = dec.results()
    dec.close()
    assert len(set(its.tolist())) > 1                  # blocks stop at different iterations
    for i in range(n_cb):
        it, d = O.turbo_decode8(ys[i], K, max_it=8, crc_type=1)
        assert its[i] == it and np.array_equal(outs[i], d), i
