"""Seeded decoder / encoder input cases shared by the CPU pins (tests/test_td_spec_cpu.py) and the
GPU parity tests (tests/test_gpu_decoder_cases.py).  TEST INFRASTRUCTURE: the inputs are built
with the oracle's encoder / CRC, which are pinned to tests/spec_model.py and to the reference's
own crc_byte.c (tests/test_ref_pin_cpu.py)."""
import hashlib
import os
import re

import numpy as np

import oracle_lib as O

QPP = {int(a): (int(b), int(c)) for a, b, c in re.findall(
    r"\{\s*(\d+)\s*,\s*(\d+)\s*,\s*(\d+)\s*\}",
    open(os.path.join(os.path.dirname(O.ORACLE_DIR), "include", "oai4g_qpp.c")).read())}


def undefined_positions(K):
    """Output positions of threegpplte_turbo_encoder that read the never-written last byte of
    systematic2 when K/8 is odd (3gpplte_sse.c:321-367, :408): z'_k for k >= K-8 and the second
    encoder's tail (x', z') x 3."""
    if (K // 8) % 2 == 0:
        return np.zeros(0, dtype=np.int64)
    return np.concatenate([3 * np.arange(K - 8, K) + 2, 3 * K + 6 + np.arange(6)])


def crc_block(rng, K, crc_type, F=0):
    """A code block as lte_segmentation leaves it: F/8 zero filler bytes, payload, CRC (type 0 =
    CRC24_A over the K-24-F payload bits, as the single-block TB; 1 = CRC24_B over K-24)."""
    c = np.zeros(K // 8 + 4, dtype=np.uint8)
    n = (K - 24 - F) // 8
    c[F // 8:F // 8 + n] = rng.integers(0, 256, n, dtype=np.uint8)
    if crc_type == 0:
        v = O.crc24a(c[F // 8:], K - 24 - F) >> 8
    else:
        v = O.crc24b(c, K - 24) >> 8
    c[(K - 24) // 8:(K - 24) // 8 + 3] = [v >> 16, (v >> 8) & 255, v & 255]
    return c[:K // 8]


def llrs(d, amp, sigma, rng):
    y = (d.astype(np.float64) * 2 - 1) * amp
    if sigma:
        y = y + rng.normal(0, sigma, len(d))
    return np.clip(np.round(y), -32768, 32767).astype(np.int16)


def decoder_cases():
    """(name, K, y, max_it, crc_type, F): the cases pinned here and in the golden fixture."""
    rng = np.random.default_rng(14)
    cases = []
    for K in (40, 104, 512, 1024, 2048, 5504, 6144):
        for crc_type in (0, 1):
            for amp, sigma in ((32, 0), (32, 20), (32, 28), (32, 36), (100, 150)):
                c = crc_block(rng, K, crc_type)
                d = O.turbo_encode(c, *QPP[K])
                cases.append((f"K{K}_crc{crc_type}_a{amp}_s{sigma}", K, llrs(d, amp, sigma, rng), 8, crc_type, 0))
        cases.append((f"K{K}_unstructured", K, rng.integers(-40, 41, 3 * K + 12).astype(np.int16), 8, 0, 0))
        cases.append((f"K{K}_saturating", K, rng.integers(-32768, 32768, 3 * K + 12).astype(np.int16), 6, 1, 0))
    for K, F in ((1056, 24), (6144, 64), (512, 8)):     # filler: CRC24_A starts at byte F/8 (:1314-1321)
        for sigma in (0, 30):
            c = crc_block(rng, K, 0, F)
            cases.append((f"K{K}_F{F}_s{sigma}", K, llrs(O.turbo_encode(c, *QPP[K]), 32, sigma, rng), 8, 0, F))
    for max_it in (1, 2, 3, 5):
        c = crc_block(rng, 1024, 0)
        cases.append((f"K1024_maxit{max_it}", 1024, llrs(O.turbo_encode(c, *QPP[1024]), 32, 32, rng), max_it, 0, 0))
    return cases




ENC_K = (40, 48, 56, 104, 512, 528, 1008, 1024, 1056, 2048, 3072, 4096, 5504, 6144)


def encoder_cases():
    """(K, c) turbo-encoder inputs pinned in the fixture."""
    rng = np.random.default_rng(15)
    return [(K, rng.integers(0, 256, K // 8, dtype=np.uint8)) for K in ENC_K for _ in range(2)]


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]
