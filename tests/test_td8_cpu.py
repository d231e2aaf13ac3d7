"""The 8-bit turbo decoder oracle (oracle/oai_oracle_td8.c, a restatement of
3gpplte_turbo_decoder_sse_8bit.c for n % 16 == 0, n >= 512; the reference TU includes PHY/defs.h
and its interleaver blob is missing, so it cannot be built here) pinned like the 16-bit one
(SURVEY §8c's fallback): every block it reports as CRC-passing carries the transmitted bits and
the textbook max-log-MAP model's hard decisions, at several SNR points and input scales (the
decoder's own |LLR|-mean scaling to int8), for CRC24A / CRC24B and both hard-decision branches
(n mod 128 = 0: extrinsic only; otherwise extrinsic + systematic through pi6)."""
import numpy as np
import pytest

import oracle_lib as O
import td_spec as T
from ref_cases import QPP, crc_block, llrs

# (K, amplitude, sigma): K = 1024 / 6144 / 5504 take the n mod 128 = 0 branch, 1056 / 528 / 4160 not;
# amplitudes 8 / 32 / 100 / 300 cover the 0 / 2 / 3 / (3, 4) input shifts
POINTS = [(1024, 32, 0), (1024, 32, 26), (6144, 100, 80), (5504, 8, 6), (1056, 300, 200), (528, 32, 20),
          (4160, 64, 48), (6144, 32, 30)]


@pytest.mark.parametrize("K,amp,sigma", POINTS)
@pytest.mark.parametrize("crc_type", [0, 1])
def test_decoder8_agrees_with_textbook(K, amp, sigma, crc_type):
    rng = np.random.default_rng(K + amp + sigma + crc_type)
    B = 4
    cs = [crc_block(rng, K, crc_type) for _ in range(B)]
    ys = np.stack([llrs(O.turbo_encode(c, *QPP[K]), amp, sigma, rng) for c in cs])
    tb = T.bits_to_bytes(T.decode(ys, K, *QPP[K]))
    n_pass = 0
    for i in range(B):
        it, dec = O.turbo_decode8(ys[i], K, crc_type=crc_type)
        assert 2 <= it <= 9
        if it <= 8:
            n_pass += 1
            assert np.array_equal(dec, cs[i]), (K, sigma, i)
            assert np.array_equal(tb[i], dec), (K, sigma, i)
    if sigma == 0:
        assert n_pass == B


def test_decoder8_scope():
    assert O.turbo_decode8(np.zeros(3 * 40 + 12, np.int16), 40)[0] == 255     # n < 512
    assert O.turbo_decode8(np.zeros(3 * 520 + 12, np.int16), 520)[0] == 255   # n mod 16 = 8 (reads past its tables)


def test_td8_tables_are_permutations():
    import ctypes
    for K in (512, 1024, 5504, 6144):
        t = [np.zeros(K, np.int32) for _ in range(4)]
        O.orc().orc_td8_tables(K, *[O.P(a) for a in t])
        pi2, pi4, pi5, pi6 = t
        for a in t:
            assert sorted(a.tolist()) == list(range(K))
        assert np.array_equal(pi5[pi4], np.arange(K))   # pi5 inverts pi4 on the window layout
