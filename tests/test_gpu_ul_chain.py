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
