"""UE receive front end, CPU side: the oracle's forward DFT
(oracle/oai_oracle.c orc_dft, restating lte_dfts.c dft64..dft2048) and slot_fep restatement
(orc_slot_fep, slot_fep.c:40-177).

Pinning: the oracle's DFT is checked bit for bit against the reference's own outputs
(tests/golden/dft_ref.npz, made by gen_golden.py from the unmodified lte_dfts.c) and, where
oracle/_ref is built (this container), against the reference library itself on fresh random and
saturating inputs; the oracle's twiddle rule against the reference's tables.  slot_fep's window
arithmetic is checked against an independent numpy restatement, including the frame wrap.
"""
import os

import numpy as np
import pytest

import oracle_lib as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _aligned_i16(n):
    buf = np.zeros(n + 32, np.int16)
    off = (-buf.ctypes.data % 64) // 2
    return buf[off:off + n]


def test_oracle_dft_matches_reference_outputs():
    z = np.load(os.path.join(GOLDEN, "dft_ref.npz"))
    n = 0
    for key in z.files:
        if key.startswith("x_"):
            _, size, vi, scale = key.split("_")
            assert np.array_equal(O.dft(z[key], int(scale)), z[f"y_{size}_{vi}_{scale}"]), key
            n += 1
    assert n == 30


def _ms(radix3, M):
    return [j * k for j in (1, 2, 3) for k in range(M)] if radix3 else list(range(M))


@pytest.mark.parametrize("name,N,radix3,M", [("tw16", 16, 1, 4), ("tw64", 64, 1, 16), ("tw128", 128, 0, 64),
                                             ("tw256", 256, 1, 64), ("tw512", 512, 0, 256)])
def test_oracle_forward_twiddles_match_reference_tables(name, N, radix3, M):
    """packed_cmult2 operand tables twNa / twNb (lte_dfts.c:1412-1422, 1734-1744, 1951-1953,
    2162-2167, 2344-2350), including tw256a's different rounding"""
    z = np.load(os.path.join(GOLDEN, "dft_ref.npz"))
    ta, tb = z["table_" + name + "a"].reshape(-1, 2), z["table_" + name + "b"].reshape(-1, 2)
    for i, m in enumerate(_ms(radix3, M)):
        a, b = O.dft_twiddle_ab(N, m)
        assert list(a) == list(ta[i]) and list(b) == list(tb[i]), (name, m)


@pytest.mark.parametrize("name,N,radix3,M", [("tw1024", 1024, 1, 256), ("tw2048", 2048, 0, 1024)])
def test_oracle_cmult_twiddles_match_reference_tables(name, N, radix3, M):
    z = np.load(os.path.join(GOLDEN, "dft_ref.npz"))
    t = z["table_" + name].reshape(-1, 2)
    for i, m in enumerate(_ms(radix3, M)):
        a, b = O.dft_twiddle_ab(N, m)      # a = (Wr, -Wi), b = (Wi, Wr)
        assert (int(a[0]), int(b[0])) == (int(t[i][0]), int(t[i][1])) and int(a[1]) == -int(t[i][1]), (name, m)


@pytest.mark.skipif(O.ref_dfts() is None, reason="oracle/_ref (the reference's lte_dfts.c) not built here")
@pytest.mark.parametrize("log2n", [6, 7, 8, 9, 10, 11])
def test_oracle_dft_matches_reference_library(log2n):
    ref = O.ref_dfts()
    n = 1 << log2n
    fn = getattr(ref, f"dft{n}")
    rng = np.random.default_rng(log2n)
    for t in range(12):
        amp = (64, 1000, 12000, 32767)[t % 4]
        x = _aligned_i16(2 * n)
        x[:] = rng.integers(-amp, amp + 1, 2 * n) if t < 8 else rng.choice([-32768, 32767, -amp, amp], 2 * n)
        y = _aligned_i16(2 * n)
        fn(O.P(x), O.P(y), 1)
        assert np.array_equal(O.dft(x, 1), y), (n, t)


def test_oracle_dft_is_a_dft():
    """size-independent property: the fixed-point DFT tracks numpy's FFT (scaled 1/sqrt(N)) at
    amplitudes where the unscaled dft16 leaves do not saturate"""
    rng = np.random.default_rng(5)
    for log2n in range(6, 12):
        n = 1 << log2n
        x = rng.integers(-1000, 1000, 2 * n).astype(np.int16)
        y = O.dft(x, 1)
        X = np.fft.fft(x[0::2] + 1j * x[1::2]) / np.sqrt(n)
        Y = y[0::2] + 1j * y[1::2]
        err = np.sqrt(np.mean(np.abs(Y - X) ** 2))
        assert err < 4.0, (n, err)


def window_start(fp, l, Ns, sample_offset, no_prefix):
    """independent restatement of slot_fep.c:87-150 in unsigned 32-bit arithmetic"""
    N = fp.ofdm_symbol_size
    cp = 0 if no_prefix else fp.nb_prefix_samples
    cp0 = 0 if no_prefix else fp.nb_prefix_samples0
    if no_prefix:
        sfo, slo = N * fp.symbols_per_tti * (Ns >> 1), N * (fp.symbols_per_tti >> 1) * (Ns % 2)
    else:
        sfo, slo = fp.samples_per_tti * (Ns >> 1), (fp.samples_per_tti >> 1) * (Ns % 2)
    r = (sample_offset + slo + cp0 + sfo) & 0xFFFFFFFF
    r -= r % 4
    if l > 0:
        r = (r + (N + cp) * l) & 0xFFFFFFFF
    return r


def fep_cases(fp):
    nsl = 7 - fp.Ncp
    return [(0, 0, 0, 0), (nsl - 1, 1, 0, 0), (3, 7, 5, 0), (0, 19, 0, 0), (nsl - 1, 19, 0, 0),
            (2, 19, fp.samples_per_tti // 2, 0), (1, 5, 3, 1), (nsl - 1, 18, 17, 1)]


@pytest.mark.parametrize("N_RB,Ncp", [(6, 0), (25, 0), (100, 0), (15, 1), (50, 1)])
def test_oracle_slot_fep_windows(N_RB, Ncp):
    fp = O.frame(N_RB, Ncp=Ncp)
    N, fl = fp.ofdm_symbol_size, fp.samples_per_tti * 10
    rng = np.random.default_rng(N_RB)
    frame = rng.integers(-2000, 2000, 2 * fl).astype(np.int16).view(np.int32)
    nsl = 7 - Ncp
    for (l, Ns, so, nop) in fep_cases(fp):
        rx = np.zeros(fl + N, np.int32)
        rx[:fl] = frame
        rxF = np.zeros(fp.symbols_per_tti * N, np.int32)
        assert O.slot_fep([rx], [rxF], fp, l, Ns, so, nop) == 0
        st = window_start(fp, l, Ns, so, nop)
        win = np.concatenate([frame, frame])[st % fl: st % fl + N]
        sym = l + nsl * (Ns & 1)
        assert np.array_equal(rxF[sym * N:(sym + 1) * N], O.dft(win.view(np.int16), 1).view(np.int32)), (l, Ns, so)
        if st > fl - N:                                          # the reference's wrap copy (:123, :153)
            assert np.array_equal(rx[fl:], frame[:N])


def test_oracle_slot_fep_rejects_bad_symbol():
    fp = O.frame(25)
    rx = np.zeros(fp.samples_per_tti * 10 + fp.ofdm_symbol_size, np.int32)
    rxF = np.zeros(14 * fp.ofdm_symbol_size, np.int32)
    assert O.slot_fep([rx], [rxF], fp, 7, 0) == -1
    assert O.slot_fep([rx], [rxF], fp, 0, 20) == -1
    fpe = O.frame(25, Ncp=1)
    assert O.slot_fep([rx], [rxF], fpe, 6, 0) == -1
