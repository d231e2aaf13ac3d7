"""Control-region oracle (oracle/oai_oracle_ctrl.c) pinned to the reference's own compiled
crc_byte.c / ccoding_byte_lte.c (oracle/_ref/libref_coding.so): crc16 on every bit length
(including the reference's partial-byte step) and the tail-biting convolutional encoder with the
RNTI-masked CRC16 of DCIs and PBCH (add_crc = 2) and without CRC (add_crc = 0)."""
import numpy as np
import pytest

import oracle_lib as O

REF = O.ref_coding()
needs_ref = pytest.mark.skipif(REF is None, reason="oracle/_ref/libref_coding.so not built (no reference tree)")


@needs_ref
def test_crc16_vs_reference():
    rng = np.random.default_rng(21)
    for bitlen in list(range(1, 130)) + [255, 256, 1000]:
        a = rng.integers(0, 256, bitlen // 8 + 2, dtype=np.uint8)
        assert O.crc16(a, bitlen) == O.ref_crc(a, bitlen, "16"), bitlen


@needs_ref
@pytest.mark.parametrize("add_crc", [2, 0])
def test_ccodelte_encode_vs_reference(add_crc):
    rng = np.random.default_rng(22 + add_crc)
    for n in range(8, 72):
        for rnti in (0, 0x1234, 0xFFFF, 0x5555, 0xFFFE):
            a = rng.integers(0, 256, n // 8 + 1, dtype=np.uint8)
            assert np.array_equal(O.ccode_encode(a, n, add_crc, rnti), O.ref_ccode_encode(a, n, add_crc, rnti)), (n, rnti)
