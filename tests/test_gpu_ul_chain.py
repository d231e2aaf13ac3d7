"""GPU parity of the batched UL receive chain (oai4g_ul_decode_batch: ulsch_decoding.c:1208-1350 --
RM-rx + sub-block deinterleaving fused in k_ul_rm_deint, then k_td16 per block size) against the
oracle's per-block chain (tests/test_ul_chain_cpu.py): iteration counts and decoded code blocks
bit-exact per TB, for C5's 8 x 5504 blocks, a single block with filler bits (F = 24, CRC24A over
the non-filler bits) and K- / K+ blocks (C = 2, F = 32), at SNRs where blocks stop at different
iterations or fail."""
import numpy as np
import pytest

import oracle_lib as O
from test_ul_chain_cpu import UL, ul_e

pytestmark = pytest.mark.gpu


def _batch(tbs, G, Qm, n_tb, seed, amp, sigma, n_unique=None):
    """n_tb noisy TBs; the coded bits of n_unique payloads are reused with fresh noise per TB."""
    rng = np.random.default_rng(seed)
    n_unique = n_unique or n_tb
    codes = []
    for _ in range(n_unique):
        pay = rng.integers(0, 256, tbs // 8 + 8, dtype=np.uint8)
        codes.append(np.array(ul_e(pay, tbs, G, Qm), dtype=np.float64))
    es = [np.clip(np.round((2 * codes[t % n_unique] - 1) * amp + rng.normal(0, sigma, G)), -32768, 32767)
          .astype(np.int16) for t in range(n_tb)]
    return np.stack(es)


@pytest.mark.parametrize("tbs,G,Qm", UL)
@pytest.mark.parametrize("amp,sigma,max_it", [(40, 45, 6), (30, 60, 8), (60, 0, 3)])
def test_gpu_ul_chain_matches_oracle(gpu, tbs, G, Qm, amp, sigma, max_it):
    n_tb = 6
    e = _batch(tbs, G, Qm, n_tb, tbs + amp, amp, sigma)
    ub = gpu.UlDecodeBatch(tbs + 24, G, Qm, n_tb, max_iterations=max_it)
    ub.upload(e)
    ub.launch()
    its, c = ub.results()
    for t in range(n_tb):
        ref = O.ulsch_decode(e[t], tbs + 24, G, Qm, max_it=max_it)
        assert len(ref) == ub.C
        for r, (it, d) in enumerate(ref):
            assert its[t, r] == it, (t, r, its[t, r], it)
            assert np.array_equal(c[t, r, :len(d)], d), (t, r)
    ub.close()


def test_gpu_ul_chain_c5_batch(gpu):
    """C5's configuration at a few hundred TBs (8 blocks each), sampled against the oracle."""
    tbs, G, Qm, n_tb = 43816, 57600, 4, 256
    e = _batch(tbs, G, Qm, n_tb, 5, 60, 25, n_unique=8)
    ub = gpu.UlDecodeBatch(tbs + 24, G, Qm, n_tb, max_iterations=8)
    ub.upload(e)
    ub.launch()
    its, c = ub.results()
    for t in (0, 17, 128, n_tb - 1):
        ref = O.ulsch_decode(e[t], tbs + 24, G, Qm, max_it=8)
        for r, (it, d) in enumerate(ref):
            assert its[t, r] == it and np.array_equal(c[t, r, :len(d)], d), (t, r)
    assert np.all(its <= 8)                     # this SNR decodes every block
    ub.close()


def test_gpu_ul_chain_rows_beyond_grid_y_limit(gpu):
    """n_tb x C above gridDim.y's 65 535: k_ul_rm_deint runs in row chunks; the TBs on both sides
    of every chunk boundary decode as the oracle does."""
    tbs, G, Qm, n_tb = 16, 288, 2, 70000
    e = _batch(tbs, G, Qm, n_tb, 9, 50, 20, n_unique=4)
    ub = gpu.UlDecodeBatch(tbs + 24, G, Qm, n_tb, max_iterations=4)
    assert ub.C == 1
    ub.upload(e)
    ub.launch()
    its, c = ub.results()
    for t in (0, 1, 65534, 65535, 65536, n_tb - 1):
        ref = O.ulsch_decode(e[t], tbs + 24, G, Qm, max_it=4)
        for r, (it, d) in enumerate(ref):
            assert its[t, r] == it and np.array_equal(c[t, r, :len(d)], d), (t, r)
    ub.close()


@pytest.mark.parametrize("tbs,G,Qm", UL)
def test_gpu_ul_chain_harq_rounds_match_oracle(gpu, tbs, G, Qm):
    """oai4g_ul_decode_batch_harq over dlsim's four-round sequence rv 0, 2, 3, 1 (clear = 1 on round
    0, then soft combining in the kept buffers; dlsch_decoding.c:348-383, dlsim.c:2141): iteration
    counts, decoded blocks and the soft buffers bit-exact per round against the oracle chain,
    whose lte_rate_matching_turbo_rx is pinned to the reference's own (tests/test_ref_pin_rm_cpu.py).
    Large soft values make the int16 sums wrap."""
    import spec_model as S
    from test_ul_chain_cpu import ul_e
    n_tb, rng = 4, np.random.default_rng(tbs)
    pays = [rng.integers(0, 256, tbs // 8 + 8, dtype=np.uint8) for _ in range(n_tb)]
    blocks, _ = S.segment([0] * (tbs + 24))
    w_o = [[np.zeros(3 * 32 * ((len(b) + 4 + 31) // 32) + 64, np.int16) for b in blocks] for _ in range(n_tb)]
    ub = gpu.UlDecodeBatch(tbs + 24, G, Qm, n_tb, max_iterations=4)
    for rnd, rv in enumerate((0, 2, 3, 1)):
        amp = 12000 if rnd == 3 else 20
        e = np.stack([np.clip(np.round((2 * np.array(ul_e(pays[t], tbs, G, Qm, rv=rv), np.float64) - 1) * amp
                                       + rng.normal(0, 30, G)), -32768, 32767).astype(np.int16) for t in range(n_tb)])
        ub.upload(e)
        ub.launch_harq(rv, 1 if rnd == 0 else 0)
        its, c = ub.results()
        wg = ub.soft_buffers()
        for t in range(n_tb):
            ref = O.ulsch_decode_harq(e[t], tbs + 24, G, Qm, rv, 1 if rnd == 0 else 0, w_o[t], max_it=4)
            for r, (it, d) in enumerate(ref):
                Ncb = 3 * 32 * ((len(blocks[r]) + 4 + 31) // 32)
                assert np.array_equal(wg[t, r, :Ncb], w_o[t][r][:Ncb]), (rnd, t, r)
                assert its[t, r] == it, (rnd, t, r, its[t, r], it)
                assert np.array_equal(c[t, r, :len(d)], d), (rnd, t, r)
    ub.close()
