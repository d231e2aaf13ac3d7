"""GPU parity of lte_est_freq_offset (lte_est_freq_offset.c:104-193) and of the time-domain
channel estimate dl_ch_estimates_time (lte_dl_channel_estimation.c:704-738) against the oracle
(tests/test_freq_offset_cpu.py pins it: dot_product / log2_approx to the reference TU, the rest
to the rotation-recovery model, the idft to lte_dfts.c).  Bit-exact: omega and the filtered
estimate over call sequences (resets, l = 0 and 4 - Ncp, full-range and wrapping inputs), the
batched omegas and time estimates of ChestBatch's planes."""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
from test_freq_offset_cpu import _rotated_planes

pytestmark = pytest.mark.gpu

SIZES = [(6, 0), (15, 0), (25, 0), (25, 1), (50, 0), (50, 1), (100, 0), (100, 1)]


@pytest.mark.parametrize("N_RB,Ncp", SIZES)
def test_gpu_freq_offset_drop_in_sequence(gpu, N_RB, Ncp):
    fo = O.frame(N_RB, Ncp=Ncp)
    fg = gpu.frame_parms(N_RB, Ncp=Ncp)
    lp = 4 - Ncp
    rng = np.random.default_rng(N_RB * 3 + Ncp)
    st = O.FreqOffsetState()
    f = ctypes.c_int(12345)
    seq = []
    for k in range(12):
        kind = k % 4
        l = lp if k % 3 else 0
        if kind == 0:
            plane = _rotated_planes(fo, rng.uniform(-1700, 1700), rng.uniform(50, 1200), rng, l)
        elif kind == 1:          # full range: wrapping level sums, saturating packs
            plane = rng.integers(-2**31, 2**31 - 1, fo.symbols_per_tti * fo.ofdm_symbol_size + 8,
                                 dtype=np.int64).astype(np.int32)
        elif kind == 2:          # extremes (-32768 products, sign_epi16 of -32768)
            v = rng.choice(np.array([-32768, 32767, -1, 0, 1], np.int16), (fo.symbols_per_tti * fo.ofdm_symbol_size + 8) * 2)
            plane = v.view(np.int32)
        else:
            plane = _rotated_planes(fo, rng.uniform(-300, 300), 300.0, rng, l)
        reset = 1 if k in (0, 7) else 0
        want = st.call(fo, plane, l, reset=reset)
        got = gpu.lte_est_freq_offset([plane], fg, l, f, reset=reset)
        seq.append((want, got))
        assert got == want, (k, seq)


def test_gpu_freq_offset_rejects_bad_symbol(gpu):
    fg = gpu.frame_parms(50)
    plane = np.zeros(14 * fg.ofdm_symbol_size + 8, np.int32)
    f = ctypes.c_int(77)
    with pytest.raises(gpu.OAI4GError):
        gpu.lte_est_freq_offset([plane], fg, 2, f)
    assert f.value == 77


@pytest.mark.parametrize("N_RB,Ncp", SIZES)
def test_gpu_estimates_time_drop_in(gpu, N_RB, Ncp):
    fo = O.frame(N_RB, Ncp=Ncp, nb_antennas_tx=2, mode1_flag=0)
    fg = gpu.frame_parms(N_RB, Ncp=Ncp, nb_antennas_tx=2, mode1_flag=0)
    N = fo.ofdm_symbol_size
    rng = np.random.default_rng(N_RB)
    planes = [None] * 8
    for i in (0, 1, 2):            # (p, aarx) = (0, 0), (0, 1), (1, 0); plane 3 NULL
        planes[i] = (rng.integers(-2**15, 2**15, (fo.symbols_per_tti * N, 2)).astype(np.int16)).view(np.int32).ravel()
    outs = [np.full(N, 0x5A5A5A5A, np.int32) for _ in range(8)]
    gpu.dl_ch_estimates_time(fg, 2, planes, outs)
    for i in range(8):
        if planes[i] is not None:
            assert np.array_equal(outs[i], O.chest_time(fo, planes[i])), i
        else:
            assert np.all(outs[i] == 0x5A5A5A5A), i       # NULL planes and planes past (p, aarx) untouched


@pytest.mark.parametrize("N_RB,Ncp,first", [(100, 0, 3), (25, 0, 0), (50, 1, 7), (6, 0, 9), (15, 0, 2)])
def test_gpu_batch_omegas_and_time_estimates(gpu, N_RB, Ncp, first):
    """ChestBatch planes (estimates of random grids) -> the batched omegas and time estimates equal the
    oracle applied to each subframe's plane; the drop-in sequence over the same planes equals
    the update chain of the batched omegas."""
    fo = O.frame(N_RB, Ncp=Ncp)
    fg = gpu.frame_parms(N_RB, Ncp=Ncp)
    N, nsymb = fo.ofdm_symbol_size, fo.symbols_per_tti
    lp = 4 - Ncp
    n_sf = 6
    rng = np.random.default_rng(N_RB + first)
    y = (rng.integers(-2**12, 2**12, ((n_sf + 1) * nsymb * N, 2)).astype(np.int16)).view(np.int32).ravel()
    cb = gpu.ChestBatch(fg, n_sf, first_subframe=first)
    est = cb.run(y[:n_sf * nsymb * N].reshape(n_sf, -1), y[n_sf * nsymb * N:][:N])
    om = cb.freq_offset_omegas(lp)
    om0 = cb.freq_offset_omegas(0)
    tt = cb.time_estimates()
    cb.close()
    st = O.FreqOffsetState()
    f, first_run = ctypes.c_int(0), ctypes.c_int(1)
    for i in range(n_sf):
        plane = np.concatenate([est[i], np.zeros(8, np.int32)])
        assert om[i] == O.fo_omega(fo, plane, lp), i
        assert om0[i] == O.fo_omega(fo, plane, 0), i
        assert np.array_equal(tt[i], O.chest_time(fo, plane)), i
        for _ in range(2):       # slot_fep calls it in both slots of the subframe (l = 4 - Ncp)
            assert gpu.freq_offset_update(fg, om[i], f, first_run) == st.call(fo, plane, lp)
