"""GPU parity of the uplink turbo-decoding chain (A16) against the oracle: decoded bytes and
iteration counts bit-exact, for the drop-ins and the batched decoder (blocks that stop at
different iterations inside one wave)."""
import os
import re

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

QPP = {int(a): (int(b), int(c)) for a, b, c in re.findall(
    r"\{\s*(\d+)\s*,\s*(\d+)\s*,\s*(\d+)\s*\}",
    open(os.path.join(os.path.dirname(O.ORACLE_DIR), "include", "oai4g_qpp.c")).read())}


def crc_block(rng, K, crc="a"):
    msg = rng.integers(0, 256, (K - 24) // 8, dtype=np.uint8)
    c = np.zeros(K // 8 + 4, dtype=np.uint8)
    c[:len(msg)] = msg
    v = (O.crc24a if crc == "a" else O.crc24b)(c, K - 24) >> 8
    c[len(msg):len(msg) + 3] = [v >> 16, (v >> 8) & 255, v & 255]
    return c[:K // 8]


def noisy_llr(rng, K, amp, sigma, crc="a"):
    d = O.turbo_encode(crc_block(rng, K, crc), *QPP[K])
    y = (d.astype(np.float64) * 2 - 1) * amp + rng.normal(0, sigma, len(d))
    return np.clip(np.round(y), -32768, 32767).astype(np.int16)


@pytest.mark.parametrize("K", [40, 48, 512, 1024, 2048, 5504, 6144])
def test_drop_in_decoder_bit_exact(gpu, K):
    rng = np.random.default_rng(K)
    for amp, sigma, crc, max_it in ((32, 20, "a", 8), (100, 110, "a", 8), (8, 10, "b", 6), (32, 0, "b", 2),
                                    (40, 45, "a", 1), (1000, 900, "a", 4)):
        y = noisy_llr(rng, K, amp, sigma, crc)
        ct = 0 if crc == "a" else 1
        it_o, dec_o = O.turbo_decode(y, K, max_it=max_it, crc_type=ct)
        it_g, dec_g = gpu.turbo_decoder16(y, K, max_iterations=max_it, crc_type=ct)
        assert it_g == it_o, (K, amp, sigma, max_it)
        if max_it > 1:
            assert np.array_equal(dec_g, dec_o), (K, amp, sigma)


def test_decoder_saturating_inputs(gpu):
    rng = np.random.default_rng(3)
    K = 1024
    y = rng.choice([-32768, 32767, -32767, 0, 1, -1], size=3 * K + 12).astype(np.int16)
    it_o, dec_o = O.turbo_decode(y, K, max_it=5)
    it_g, dec_g = gpu.turbo_decoder16(y, K, max_iterations=5)
    assert it_g == it_o and np.array_equal(dec_g, dec_o)


@pytest.mark.parametrize("K,n_cb", [(5504, 40), (1024, 19)])
def test_batch_decoder_bit_exact(gpu, K, n_cb):
    """Blocks of one wave stop at different iterations (mixed SNR) and the tail wave is partial."""
    rng = np.random.default_rng(n_cb)
    sig = [(32, 20), (100, 112), (8, 9), (100, 135)]
    llr = np.stack([noisy_llr(rng, K, *sig[i % 4]) for i in range(n_cb)])
    b = gpu.TurboDecoderBatch(K, n_cb)
    b.upload(llr)
    b.run(max_iterations=8)
    it_g, out_g = b.results()
    b.close()
    for i in range(n_cb):
        it_o, dec_o = O.turbo_decode(llr[i], K, max_it=8)
        assert it_g[i] == it_o, i
        assert np.array_equal(out_g[i], dec_o), i
    assert len(set(it_g.tolist())) > 1


@pytest.mark.parametrize("K,C,r,G,Qm,rv,clear", [(1024, 1, 0, 4000, 4, 0, 1), (6144, 2, 1, 30000, 6, 0, 1),
                                                 (5504, 8, 3, 100000, 4, 2, 0), (40, 1, 0, 600, 2, 1, 1)])
def test_rate_matching_rx_and_deinterleave(gpu, K, C, r, G, Qm, rv, clear):
    rng = np.random.default_rng(G + r)
    D = K + 4
    R = (D + 31) >> 5
    E = O.rate_match(R, G, np.zeros(3 * 32 * R, dtype=np.uint8), C, r, Qm, rvidx=rv).size
    soft = rng.integers(-3000, 3000, E).astype(np.int16)
    w0 = rng.integers(-30000, 30000, 3 * 32 * R + 64).astype(np.int16)
    w_o, E_o = O.rate_match_rx(soft, K, G, C, r, Qm, rvidx=rv, w=w0.copy(), clear=clear)
    w_g = w0.copy()
    E_g = gpu.rate_matching_turbo_rx(R, G, w_g, O.dummy_w(D), soft, C, r, Qm, rvidx=rv, clear=clear)
    assert E_g == E_o
    assert np.array_equal(w_g[:3 * 32 * R], w_o[:3 * 32 * R])
    d_o = O.subblock_deinterleave(w_o, K)
    d_g = gpu.sub_block_deinterleaving_turbo(D, w_o)
    assert np.array_equal(d_g[96:96 + 3 * K + 12], d_o)


# every K up to 320 (K1 = K / 8 steps per window): the backward pass's segment schedule changes
# with K1 -- no full segment below the re-run (K1 <= 11), one to six of them with the two-bundle
# operand prefetch taking both its odd and even branches, a partial top segment or none
SMALL_K = [K for K in sorted(QPP) if K <= 320]


def test_drop_in_decoder_every_small_K(gpu):
    rng = np.random.default_rng(320)
    for K in SMALL_K:
        for amp, sigma, crc, max_it in ((32, 24, "a", 8), (32, 40, "b", 5)):
            y = noisy_llr(rng, K, amp, sigma, crc)
            ct = 0 if crc == "a" else 1
            it_o, dec_o = O.turbo_decode(y, K, max_it=max_it, crc_type=ct)
            it_g, dec_g = gpu.turbo_decoder16(y, K, max_iterations=max_it, crc_type=ct)
            assert it_g == it_o, (K, sigma)
            assert np.array_equal(dec_g[:K // 8], dec_o), (K, sigma)
