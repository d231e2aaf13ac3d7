"""Oracle pinned to the reference's own compiled coding translation units (oracle/_ref/libref_coding.so:
PHY/CODING/crc_byte.c and ccoding_byte_lte.c, built unmodified by oracle/Makefile).  Runs only in
the build container, where /root/reference exists.

Pinned here:
  - CRC-24A / CRC-24B (crc_byte.c:117-153) on every byte length 1..129, long blocks and ragged
    bit lengths;
  - the QPP table (include/oai4g_qpp.c) against the reference's lte_interleaver2.h:29 text.

The turbo encoder and decoder TUs link against the QPP tables of PHY/CODING/lte_interleaver.h,
which the reference lists in .MISSING_LARGE_BLOBS, so they are not built (no stand-ins); those
stages are pinned to the textbook models tests/spec_model.py and tests/td_spec.py instead
(tests/test_oracle_cpu.py, tests/test_td_spec_cpu.py).

Source-reading note (A6u, 3gpplte_sse.c:321-367, :408): for K/8 odd the SSE encoder's
interleave_compact_byte packs the permuted stream 16 bits at a time for n >> 1 words, so the last
byte of the stack array `systematic2` is never written and the last 8 z' bits plus the second
encoder's tail are computed from uninitialised memory.  The oracle and the GPU path use the spec's
interleaved bits there (tests/ref_cases.undefined_positions lists the 14 positions).
"""
import re

import numpy as np
import pytest

import oracle_lib as O
from ref_cases import QPP

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
