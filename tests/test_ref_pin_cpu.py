"""Oracle pinned to the reference's own compiled coding translation units (oracle/_ref/libref_coding.so:
PHY/CODING/crc_byte.c, 3gpplte_sse.c, 3gpplte_turbo_decoder_sse_16bit.c, built unmodified by
oracle/Makefile).  Runs only in the build container, where /root/reference exists; the GPU box
gets the same pin through tests/golden/ref_coding.npz (tests/golden/gen_ref_coding.py).

Pinned here:
  - CRC-24A / CRC-24B (crc_byte.c:117-153) on every byte length 1..768 and ragged bit lengths;
  - the SSE turbo encoder (3gpplte_sse.c:380-476) for all 188 QPP sizes, including the A6q
    filler quirk (the encoder ignores F: filler bits are encoded as 0);
  - the 16-bit max-log-MAP decoder (3gpplte_turbo_decoder_sse_16bit.c:945-1385): decoded bytes
    AND the returned iteration count, over unstructured / saturating LLRs, noisy codewords at
    several SNRs, CRC24_A / CRC24_B, filler F > 0 and max_iterations 1..8.

Reference defect found by this pin (A6u): for K/8 odd (K = 40 ... 504 in steps of 16), the SSE
encoder's interleave_compact_byte packs the QPP-permuted stream 16 bits at a time for n >> 1
words (3gpplte_sse.c:321-367), so the last byte of `systematic2` (a stack array, :408) is never
written: the last 8 z' bits and the second encoder's tail are computed from uninitialised stack
memory.  Those 14 output positions are undefined in the reference; the oracle (and the GPU path)
use the spec's interleaved bits there.  The test checks every other position bit for bit, and that
the undefined positions are exactly the ones that depend on that byte.
"""
import re

import numpy as np
import pytest

import oracle_lib as O
from ref_cases import QPP, decoder_cases, encoder_cases, undefined_positions  # noqa: F401

REF = O.ref_coding()
pytestmark = pytest.mark.skipif(REF is None, reason="oracle/_ref/libref_coding.so not built (no reference tree)")


def test_qpp_table_equals_reference_f1f2mat_old():
    """include/oai4g_qpp.c (36.212 Table 5.1.3-3) equals the reference's lte_interleaver2.h:29."""
    src = open("/root/reference/openair1/PHY/CODING/lte_interleaver2.h").read()
    body = src[src.index("f1f2mat_old"):]
    nums = [int(x) for x in re.findall(r"\d+", body[body.index("{"):body.index("}")])]
    pairs = list(zip(nums[0::2], nums[1::2]))
    assert len(pairs) == 188
    assert pairs == [QPP[K] for K in sorted(QPP)]


@pytest.mark.parametrize("kind", ["24a", "24b"])
def test_crc_vs_reference(kind):
    rng = np.random.default_rng(11)
    fn = O.crc24a if kind == "24a" else O.crc24b
    for nbytes in list(range(1, 130)) + [767, 768, 4587, 5466]:
        a = rng.integers(0, 256, nbytes + 4, dtype=np.uint8)
        for bitlen in {8 * nbytes, max(1, 8 * nbytes - 3)}:
            assert fn(a, bitlen) == O.ref_crc(a, bitlen, kind), (nbytes, bitlen)


def test_turbo_encoder_all_sizes_vs_reference():
    rng = np.random.default_rng(12)
    for K in sorted(QPP):
        und = undefined_positions(K)
        mask = np.ones(3 * K + 12, bool)
        mask[und] = False
        for t in range(3):
            c = rng.integers(0, 256, K // 8, dtype=np.uint8)
            ref = O.ref_turbo_encode(c)
            orc = O.turbo_encode(c, *QPP[K])
            assert np.array_equal(ref[mask], orc[mask]), K
            assert set(np.flatnonzero(ref != orc)) <= set(und.tolist()), K


def test_turbo_encoder_filler_quirk_vs_reference():
    """A6q: with F > 0 the SSE encoder still encodes the F leading (zeroed) filler bits as 0 —
    the reference ignores its F argument (3gpplte_sse.c:380-476); the oracle ignores it too."""
    rng = np.random.default_rng(13)
    for K, F in ((1056, 24), (6144, 64), (512, 8), (5504, 40)):
        c = rng.integers(0, 256, K // 8, dtype=np.uint8)
        c[:F // 8] = 0                       # lte_segmentation zeroes the filler bytes (:137-139)
        assert np.array_equal(O.ref_turbo_encode(c, F=F), O.turbo_encode(c, *QPP[K]))


@pytest.mark.parametrize("case", decoder_cases(), ids=lambda c: c[0])
def test_turbo_decoder16_vs_reference(case):
    name, K, y, max_it, crc_type, F = case
    it_r, dec_r = O.ref_turbo_decode(y, K, max_it, crc_type, F)
    it_o, dec_o = O.turbo_decode(y, K, max_it, crc_type, F)
    assert it_o == it_r, name
    assert np.array_equal(dec_o, dec_r), name
