"""GPU parity against the REFERENCE's own coding outputs (tests/golden/ref_coding.npz, made by
tests/golden/gen_ref_coding.py from oracle/_ref/libref_coding.so = the reference's 3gpplte_sse.c
and 3gpplte_turbo_decoder_sse_16bit.c compiled unmodified).  Bit-exact: decoded bytes and the
returned iteration count; encoder output except the 14 positions the reference leaves undefined
for K/8 odd (A6u, see tests/test_ref_pin_cpu.py)."""
import json
import os
from collections import defaultdict

import numpy as np
import pytest

from ref_cases import QPP, decoder_cases, digest, encoder_cases, undefined_positions

pytestmark = pytest.mark.gpu
FIX = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_coding.npz"))
META = json.loads(FIX["meta"].tobytes().decode())


def test_gpu_turbo_encoder_matches_reference(gpu):
    for i, (K, c) in enumerate(encoder_cases()):
        assert META["enc"][i]["in"] == digest(c), "case inputs drifted from the fixture"
        ref = np.unpackbits(FIX[f"enc_{i}"])[:3 * K + 12]
        got = gpu.turbo_encode(c, *QPP[K])[:3 * K + 12]
        mask = np.ones(3 * K + 12, bool)
        mask[undefined_positions(K)] = False
        assert np.array_equal(got[mask], ref[mask]), K


def test_gpu_drop_in_decoder16_matches_reference(gpu):
    for i, (name, K, y, max_it, crc_type, F) in enumerate(decoder_cases()):
        assert META["dec"][i]["in"] == digest(y), name
        ref = FIX[f"dec_{i}"]
        it, dec = gpu.turbo_decoder16(y, K, max_iterations=max_it, crc_type=crc_type, F=F)
        assert it == ref[0], name
        assert np.array_equal(dec[:K // 8], ref[1:]), name


def test_gpu_batch_decoder_matches_reference(gpu):
    """Every case of one (K, max_it, crc_type, F) class in one batched launch."""
    groups = defaultdict(list)
    for i, (name, K, y, max_it, crc_type, F) in enumerate(decoder_cases()):
        groups[(K, max_it, crc_type, F)].append((i, y))
    for (K, max_it, crc_type, F), items in groups.items():
        b = gpu.TurboDecoderBatch(K, len(items))
        b.upload(np.stack([y for _, y in items]))
        b.run(max_iterations=max_it, crc_type=crc_type, F=F)
        its, outs = b.results()
        b.close()
        for j, (i, _) in enumerate(items):
            ref = FIX[f"dec_{i}"]
            assert its[j] == ref[0], (K, i)
            assert np.array_equal(outs[j][:K // 8], ref[1:]), (K, i)
