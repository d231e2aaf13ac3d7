"""GPU decoder parity on the shared decoder cases of tests/ref_cases.py (noisy codewords at
several SNRs, CRC24_A / CRC24_B, filler F > 0, unstructured and saturating LLRs,
max_iterations 1..8) and the turbo encoder on every table K class: bit-exact against the oracle
(decoded bytes AND the returned iteration count), through the drop-in and the batched API.
The oracle is pinned to the textbook models (tests/test_td_spec_cpu.py, tests/test_oracle_cpu.py)."""
from collections import defaultdict

import numpy as np
import pytest

import oracle_lib as O
from ref_cases import QPP, decoder_cases, encoder_cases

pytestmark = pytest.mark.gpu
CASES = decoder_cases()


def test_gpu_turbo_encoder_matches_oracle(gpu):
    for K, c in encoder_cases():
        assert np.array_equal(gpu.turbo_encode(c, *QPP[K])[:3 * K + 12], O.turbo_encode(c, *QPP[K])), K


def test_gpu_drop_in_decoder16_matches_oracle(gpu):
    for name, K, y, max_it, crc_type, F in CASES:
        it_o, dec_o = O.turbo_decode(y, K, max_it, crc_type, F)
        it, dec = gpu.turbo_decoder16(y, K, max_iterations=max_it, crc_type=crc_type, F=F)
        assert it == it_o, name
        assert np.array_equal(dec[:K // 8], dec_o), name


def test_gpu_batch_decoder_matches_oracle(gpu):
    """Every case of one (K, max_it, crc_type, F) class in one batched launch."""
    groups = defaultdict(list)
    for name, K, y, max_it, crc_type, F in CASES:
        groups[(K, max_it, crc_type, F)].append(y)
    for (K, max_it, crc_type, F), ys in groups.items():
        b = gpu.TurboDecoderBatch(K, len(ys))
        b.upload(np.stack(ys))
        b.run(max_iterations=max_it, crc_type=crc_type, F=F)
        its, outs = b.results()
        b.close()
        for j, y in enumerate(ys):
            it_o, dec_o = O.turbo_decode(y, K, max_it, crc_type, F)
            assert its[j] == it_o, (K, j)
            assert np.array_equal(outs[j][:K // 8], dec_o), (K, j)
