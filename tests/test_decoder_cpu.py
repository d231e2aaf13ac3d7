"""CPU suite for the uplink turbo-decoding oracle.

The reference decoder's translation unit is not buildable here, so the restatement
(oracle/oai_oracle_td.c) is pinned by properties the reference's own contract implies:
  - the decoder inverts the (spec-pinned) turbo encoder: CRC-terminated blocks come back
    bit-exact, with the first CRC check at iteration 2 succeeding when noiseless;
  - early stop: the returned count is the first iteration >= 2 whose CRC matches, max + 1 when
    none does (3gpplte_turbo_decoder_sse_16bit.c:1304-1351), CRC24_A and CRC24_B, filler F;
  - the receive rate matcher / sub-block deinterleaver invert the transmit ones (36.212
    5.1.4.1), including repetition (E > Ncb), every rv, NULL skipping and C > 1;
  - the decoder is deterministic and iterates below threshold (counts above 2 appear).
"""
import re
import os

import numpy as np
import pytest

import oracle_lib as O

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


def llr(d, amp, sigma, rng):
    y = (d.astype(np.float64) * 2 - 1) * amp
    if sigma:
        y = y + rng.normal(0, sigma, len(d))
    return np.clip(np.round(y), -32768, 32767).astype(np.int16)


@pytest.mark.parametrize("K", [40, 512, 1024, 5504, 6144])
@pytest.mark.parametrize("crc", ["a", "b"])
def test_noiseless_round_trip(K, crc):
    rng = np.random.default_rng(K)
    c = crc_block(rng, K, crc)
    d = O.turbo_encode(c, *QPP[K])
    it, dec = O.turbo_decode(llr(d, 32, 0, rng), K, crc_type=0 if crc == "a" else 1)
    assert it == 2
    assert np.array_equal(dec, c)


def test_noisy_iterations_and_failure():
    rng = np.random.default_rng(7)
    K = 1024
    its = []
    for _ in range(6):
        c = crc_block(rng, K)
        it, dec = O.turbo_decode(llr(O.turbo_encode(c, *QPP[K]), 100, 110, rng), K)
        its.append(it)
        if it <= 8:
            assert np.array_equal(dec, c)
    assert max(its) > 2                                   # iterative gain is exercised
    # no codeword: every CRC check fails -> max_iterations + 1
    it, _ = O.turbo_decode(rng.integers(-50, 50, 3 * K + 12).astype(np.int16), K, max_it=4)
    assert it == 5


def test_decoder_deterministic():
    rng = np.random.default_rng(9)
    K = 5504
    y = llr(O.turbo_encode(crc_block(rng, K), *QPP[K]), 32, 30, rng)
    a, b = O.turbo_decode(y, K), O.turbo_decode(y, K)
    assert a[0] == b[0] and np.array_equal(a[1], b[1])


@pytest.mark.parametrize("K,C,r,G,Qm,rv", [(1024, 1, 0, 4000, 4, 0), (6144, 2, 1, 30000, 6, 0),
                                           (5504, 8, 3, 100000, 4, 0), (512, 1, 0, 3000, 2, 2),
                                           (40, 1, 0, 600, 2, 1), (2048, 3, 2, 14400, 4, 3)])
def test_rx_rate_matching_inverts_tx(K, C, r, G, Qm, rv):
    """TX: turbo -> sub-block interleave -> rate match; RX: +-A soft bits -> rate_matching_rx ->
    deinterleave -> decode recovers the block (E > Ncb exercises repetition)."""
    rng = np.random.default_rng(K + G)
    c = crc_block(rng, K)
    d = O.turbo_encode(c, *QPP[K])
    R, w, _ = O.subblock(d, K + 4)
    e = O.rate_match(R, G, w, C, r, Qm, rvidx=rv)
    soft = ((e.astype(np.int16) * 2 - 1) * 20).astype(np.int16)
    wr, E = O.rate_match_rx(soft, K, G, C, r, Qm, rvidx=rv)
    assert E == len(e)
    y = O.subblock_deinterleave(wr, K)
    # every systematic / parity position that was transmitted carries its bit's sign
    sent = y != 0
    assert np.array_equal((y[sent] > 0).astype(np.uint8), d[sent])
    it, dec = O.turbo_decode(y, K)
    assert it == 2 and np.array_equal(dec, c)
