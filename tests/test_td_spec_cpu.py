"""The oracle turbo decoder (oracle/oai_oracle_td.c) pinned to the textbook max-log-MAP model
(tests/td_spec.py), SURVEY §8c's fallback criterion for the decoder: at several SNR points, for
CRC24_A and CRC24_B blocks and filler F > 0, every block the oracle reports as CRC-passing
(return value <= max_iterations, 3gpplte_turbo_decoder_sse_16bit.c:1304-1351) carries the same
hard decisions as the textbook decoder, and both equal the transmitted block."""
import numpy as np
import pytest

import oracle_lib as O
import td_spec as T
from ref_cases import QPP, crc_block, llrs

# (K, sigma on +-32 BPSK) -- noiseless, moderate, near the 16-bit decoder's threshold
POINTS = [(40, 0), (40, 24), (40, 32), (512, 0), (512, 28), (512, 34), (1024, 30), (1024, 36),
          (6144, 0), (6144, 32), (6144, 38)]


@pytest.mark.parametrize("K,sigma", POINTS)
@pytest.mark.parametrize("crc_type", [0, 1])
def test_oracle_decoder_agrees_with_textbook(K, sigma, crc_type):
    rng = np.random.default_rng(1000 * K + 10 * sigma + crc_type)
    B = 6 if K < 6144 else 3
    cs = [crc_block(rng, K, crc_type) for _ in range(B)]
    ys = np.stack([llrs(O.turbo_encode(c, *QPP[K]), 32, sigma, rng) for c in cs])
    tb = T.bits_to_bytes(T.decode(ys, K, *QPP[K]))
    n_pass = 0
    for i in range(B):
        it, dec = O.turbo_decode(ys[i], K, crc_type=crc_type)
        if it <= 8:
            n_pass += 1
            assert np.array_equal(dec, cs[i]), (K, sigma, i)
            assert np.array_equal(tb[i], dec), (K, sigma, i)
    if sigma == 0:
        assert n_pass == B


@pytest.mark.parametrize("K,F", [(1056, 24), (512, 8), (2048, 64)])
def test_oracle_decoder_filler_agrees_with_textbook(K, F):
    rng = np.random.default_rng(K + F)
    cs = [crc_block(rng, K, 0, F) for _ in range(4)]
    ys = np.stack([llrs(O.turbo_encode(c, *QPP[K]), 32, 26, rng) for c in cs])
    tb = T.bits_to_bytes(T.decode(ys, K, *QPP[K]))
    for i in range(len(cs)):
        it, dec = O.turbo_decode(ys[i], K, crc_type=0, F=F)
        assert it <= 8
        assert np.array_equal(dec, cs[i]) and np.array_equal(tb[i], dec)


def test_textbook_model_matches_spec_encoder_noiseless():
    """The model itself inverts tests/spec_model.turbo_encode (independent of the oracle)."""
    import spec_model as S
    rng = np.random.default_rng(5)
    for K in (40, 48, 208, 1008):
        c = rng.integers(0, 256, K // 8, dtype=np.uint8)
        d = np.array(S.turbo_encode(S.bytes_to_bits(c, K), *QPP[K]), dtype=np.float64)
        assert np.array_equal(T.bits_to_bytes(T.decode(64 * (2 * d - 1), K, *QPP[K], iterations=1))[0], c)
