"""CPU checks of the frequency-offset estimator and the time-domain channel estimate (SURVEY §8f
item 3, the UE front end's remaining pieces):
  - orc_dot_product equals the reference's own dot_product (PHY/TOOLS/cdot_prod.c:40-118 compiled
    unmodified into oracle/_ref/libref_tools.so, when the reference tree is present), extreme
    inputs included (-32768 products, the sign_epi16 of -32768, wrapping sums, packs saturation);
  - orc_log2_approx equals the reference's log2_approx (PHY/TOOLS/log2_approx.c:29-45);
  - lte_est_freq_offset's restatement recovers a frequency offset applied as a phase rotation
    between the pilot rows: estimate = -f within the int16 rounding (the reference's own sign:
    omega = conj(row l) . row 0, lte_est_freq_offset.c:148-168), and its filter follows
    (est 2^10 + f (32767 - 2^10)) >> 15 after the first call;
  - dl_ch_estimates_time of the restatement is the reference idft (oracle pinned to lte_dfts.c)
    of the plane from word 8.
The whole of lte_est_freq_offset is also pinned to the TU itself, which builds unmodified here once
PHY/defs.h is skipped by its guard (tests/test_ref_pin_fo_cpu.py, tests/test_fo_fixture_cpu.py).  That
pin showed the reference's omega alias: omega = twice the upper-half dot product, not the sum of the
two halves; the rotation test below holds either way (both halves carry the same rotation)."""
import ctypes
import math

import numpy as np
import pytest

import oracle_lib as O


def _aligned_i16(a):
    b = O._aligned(a.size, np.int16)
    b[:] = a
    return b


@pytest.mark.parametrize("N,shift,kind", [(8, 15, "small"), (132, 6, "full"), (588, 13, "full"), (24, 0, "full"),
                                          (1200, 9, "extreme"), (64, 3, "extreme"), (12, 15, "full")])
def test_dot_product_equals_reference(N, shift, kind):
    R = O.ref_tools()
    if R is None or not hasattr(R, "dot_product"):
        pytest.skip("reference tree absent (oracle/_ref/libref_tools.so not built)")
    rng = np.random.default_rng(N * 31 + shift)
    for trial in range(20):
        if kind == "small":
            x = rng.integers(-300, 300, 2 * N).astype(np.int16)
            y = rng.integers(-300, 300, 2 * N).astype(np.int16)
        elif kind == "full":
            x = rng.integers(-2**15, 2**15, 2 * N).astype(np.int16)
            y = rng.integers(-2**15, 2**15, 2 * N).astype(np.int16)
        else:
            x = rng.choice(np.array([-32768, 32767, -32767, 0, 1, -1], np.int16), 2 * N)
            y = rng.choice(np.array([-32768, 32767, -32767, 0, 1, -1], np.int16), 2 * N)
        xa, ya = _aligned_i16(x), _aligned_i16(y)
        want = R.dot_product(O.P(xa), O.P(ya), N, shift)
        assert O.dot_product(x, y, N, shift) == want, (trial, N, shift)


def test_log2_approx_equals_reference():
    R = O.ref_tools()
    if R is None or not hasattr(R, "log2_approx"):
        pytest.skip("reference tree absent")
    rng = np.random.default_rng(5)
    vals = list(rng.integers(0, 2**32, 2000, dtype=np.uint64)) + [0, 1, 2, 3, 2**30, 2**31 - 1, 2**31, 2**32 - 1]
    for v in vals:
        assert O.orc().orc_log2_approx(ctypes.c_uint32(int(v))) == R.log2_approx(int(v)), v


def _rotated_planes(fp, f_hz, amp, rng, l):
    """An estimate plane whose row l is row prev rotated by 2 pi f dt (dt = 285.8 us / 250 us)."""
    N, nsymb = fp.ofdm_symbol_size, fp.symbols_per_tti
    lp = 4 - fp.Ncp
    dt = 285.8e-6 if fp.Ncp == 0 else 2.5e-4
    phi = 2 * math.pi * f_hz * dt
    h = amp * np.exp(1j * rng.uniform(0, 2 * np.pi, N))
    plane = np.zeros((nsymb * N + 8, 2), np.int16)
    rows = (0, lp) if l == lp else (lp, 0)          # (prev, current)
    for r, ph in ((rows[0], 0.0), (rows[1], phi)):
        z = h * np.exp(1j * ph)
        plane[r * N:(r + 1) * N, 0] = np.round(z.real).astype(np.int16)
        plane[r * N:(r + 1) * N, 1] = np.round(z.imag).astype(np.int16)
    return plane.view(np.int32).ravel()


@pytest.mark.parametrize("N_RB,Ncp", [(25, 0), (50, 0), (100, 0), (6, 0), (50, 1), (15, 0)])
@pytest.mark.parametrize("l_kind", ["pilot", "zero"])
def test_freq_offset_recovers_rotation(N_RB, Ncp, l_kind):
    fp = O.frame(N_RB, Ncp=Ncp)
    lp = 4 - Ncp
    l = lp if l_kind == "pilot" else 0
    rng = np.random.default_rng(N_RB + Ncp)
    for f in (-1500.0, -300.0, 0.0, 120.0, 700.0, 1700.0):
        plane = _rotated_planes(fp, f, 1000.0, rng, l)   # level below the int32 wrap at 100 PRB
        st = O.FreqOffsetState()
        est = st.call(fp, plane, l)
        # the per-RE floor of ">> dl_ch_shift" biases both components by -1/2 (a few % of |f|)
        assert abs(est + f) <= 0.03 * abs(f) + 60, (f, est)


def test_channel_level_wraps_as_the_reference():
    """dl_channel_level sums re^2 + im^2 in 4 int32 lanes and adds the lanes as int: above
    ~2^32 / (N_RB 12) per RE the sum wraps (the reference's arithmetic, kept): at 100 PRB and
    amplitude 4000 the level, and so dl_ch_shift, come from the wrapped sum."""
    L = O.orc()
    L.orc_fo_channel_level.restype = ctypes.c_int32
    rng = np.random.default_rng(3)
    for amp in (100, 1500, 4000, 20000):
        x = np.round(amp * np.exp(1j * rng.uniform(0, 2 * np.pi, 1200)))
        v = np.stack([x.real, x.imag], 1).astype(np.int16)
        s = int((v.astype(np.int64) ** 2).sum()) & 0xFFFFFFFF
        s = s - (1 << 32) if s >= 1 << 31 else s
        want = int(np.trunc(s / 1200))
        assert L.orc_fo_channel_level(O.P(np.ascontiguousarray(v)), 100) == want, amp


def test_freq_offset_filter_and_reset():
    fp = O.frame(50)
    rng = np.random.default_rng(1)
    st = O.FreqOffsetState()
    p1 = _rotated_planes(fp, 1000.0, 1500.0, rng, 4)
    p2 = _rotated_planes(fp, -500.0, 1500.0, rng, 4)
    e1 = st.call(fp, p1, 4)
    e2_raw = O.FreqOffsetState().call(fp, p2, 4)
    assert st.call(fp, p2, 4) == (e2_raw * 1024 + e1 * (32767 - 1024)) >> 15
    assert st.call(fp, p2, 4, reset=1) == e2_raw
    assert O.fo_omega(fp, p1, 2) == -2**31        # l must be 0 or 4 - Ncp


@pytest.mark.parametrize("N_RB,Ncp", [(6, 0), (25, 0), (50, 1), (100, 0)])
def test_chest_time_is_idft_from_word8(N_RB, Ncp):
    fp = O.frame(N_RB, Ncp=Ncp)
    N = fp.ofdm_symbol_size
    rng = np.random.default_rng(N_RB)
    plane = (rng.integers(-2**15, 2**15, (fp.symbols_per_tti * N, 2)).astype(np.int16)).view(np.int32).ravel()
    want = O.idft(plane[8:8 + N].view(np.int16).copy(), scale=1).view(np.int32)
    assert np.array_equal(O.chest_time(fp, plane), want)
