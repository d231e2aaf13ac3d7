"""Downlink channel estimation oracle (oracle/oai_oracle_chest.c: lte_dl_channel_estimation with
high_speed_flag = 1, the 6 / 50 / 100, 25 and 15 PRB branches).  Pinned
  - to the reference's own interpolation filters entry by entry (PHY/LTE_ESTIMATION/filt96_32.h,
    read as data when the reference tree is present): the oracle (and the library, test_gpu_chest)
    derive them from one formula with three cited exceptions, and
  - by dlsim's closed loop with perfect_ce = 0: the oracle's transmit subframe with CRS -> IQ ->
    slot_fep -> this estimator -> rx_pdsch -> unscrambling -> RX rate matching -> the 16-bit
    turbo decoder recovers the transport block, also at 6 PRB where slot_fep's 4-sample alignment
    shifts the window (the estimate absorbs the phase ramp that a constant estimate cannot).
No GPU needed."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle_lib as O
from test_rx_cpu import decode_tb, params

REF = "/root/reference/openair1/PHY/LTE_ESTIMATION/filt96_32.h"


def _ref_filters():
    src = re.sub(r"/\*.*?\*/", "", re.sub(r"//[^\n]*", "", open(REF).read()), flags=re.S)
    return {m.group(1): [int(v) for v in re.findall(r"-?\d+", m.group(2))]
            for m in re.finditer(r"short\s+(filt24_\w+)\[24\][^=]*=\s*\{([^}]*)\}", src)}


@pytest.mark.skipif(not os.path.exists(REF), reason="reference tree absent")
def test_filters_equal_reference_header():
    ref = _ref_filters()
    for k in range(6):
        # lte_dl_channel_estimation.c:105-180
        names = (["filt24_0", "filt24_2", "filt24_0", "filt24_2", "filt24_0r2", "filt24_2r"] if k == 0 else
                 [f"filt24_{k}l", f"filt24_{k + 2}l2", f"filt24_{k}", f"filt24_{k + 2}", f"filt24_{k}r2",
                  f"filt24_{k + 2}r"])
        got = O.chest_filters(k)
        for i, nm in enumerate(names):
            want = (ref[nm] + [0] * 24)[:24]          # filt24_0_dcr has 23 initialisers (the 24th is 0)
            assert got[i].tolist() == want, (k, nm)
        # the DC pair of the 25-PRB branch (:116-173): filt24_k_dcr, filt24_(k+2)_dcl
        got = O.chest_dc_filters(k)
        for i, nm in enumerate((f"filt24_{k}_dcr", f"filt24_{k + 2}_dcl")):
            assert got[i].tolist() == (ref[nm] + [0] * 24)[:24], (k, nm)


def _frame_loop(p, sf, pays, fp):
    """Two consecutive subframes sf, sf + 1 through the oracle's TX (CRS on) into one frame, then
    slot_fep of slots 2 sf, 2 sf + 1 and symbol 0 of slot 2 sf + 2."""
    spt, N = fp.samples_per_tti, fp.ofdm_symbol_size
    frame = np.zeros(10 * spt + N, np.int32)
    for d, pay in enumerate(pays):
        s = (sf + d) % 10
        txd, _, _ = O.tx_subframe(O.tx_cfg_from_params(params("C2", fp.N_RB_DL, p.mcs[0], p.num_pdcch_symbols, s,
                                                             Nid_cell=fp.Nid_cell), s),
                                  [pay])
        frame[s * spt:(s + 1) * spt] = txd[0]
    rxF = np.zeros(15 * N, np.int32)                      # slot_fep writes row l + 7 (Ns & 1)
    for Ns in (2 * sf, 2 * sf + 1):
        for l in range(7):
            assert O.slot_fep([frame], [rxF], fp, l, Ns) == 0
    nxt = np.zeros(15 * N, np.int32)
    assert O.slot_fep([frame], [nxt], fp, 0, (2 * sf + 2) % 20) == 0
    return rxF[:14 * N].copy(), nxt[:N].copy()


LOOP = [(6, 9, 2, 2), (6, 16, 3, 7), (50, 16, 1, 3), (100, 27, 2, 7), (100, 4, 1, 8), (50, 24, 3, 1),
        # odd N_RB_DL: the 25-PRB branch with its DC-pair filters (15 PRB: below)
        (25, 16, 1, 7), (25, 0, 1, 7), (25, 27, 2, 3), (25, 9, 3, 8)]


@pytest.mark.parametrize("N_RB,mcs,npdcch,sf", LOOP)
def test_estimated_channel_loop_decodes(N_RB, mcs, npdcch, sf):
    p = params("C2", N_RB, mcs, npdcch, sf)
    fp = O.tx_cfg_from_params(p, sf).fp
    rng = np.random.default_rng(N_RB + mcs)
    pays = [rng.integers(0, 256, p.payload_stride, dtype=np.uint8) for _ in range(2)]
    # the frame grid is indexed by subframe inside the frame: rxF rows start at slot 2 sf
    rxF_sf, next0 = _frame_loop(p, sf, pays, fp)
    est = O.chest_subframe(fp, rxF_sf, next0, sf)
    N = fp.ofdm_symbol_size
    # every row carries an estimate over the allocated band
    band = np.r_[5:5 + 12 * N_RB]
    assert all(np.count_nonzero(est[r * N:(r + 1) * N][band]) > 0.9 * len(band) for r in range(14))
    Qm = 2 if mcs < 10 else 4 if mcs < 17 else 6
    llr, _ = O.rx_pdsch_siso(fp, rxF_sf, est, list(p.rb_alloc), Qm, npdcch, sf)
    G = len(llr)
    u = np.zeros(32 * (1 + G // 32), np.int16)
    u[:G] = llr
    O.dlsch_unscrambling(u, G, (p.rnti << 14) + (sf << 9) + fp.Nid_cell)
    res, tb = decode_tb(u[:G], G, p.TBS[0], Qm)
    assert all(it <= 4 for it, _ in res), [it for it, _ in res]
    assert np.array_equal(tb, pays[0][:p.TBS[0] // 8])


@pytest.mark.parametrize("Nid_cell", [0, 4])
def test_15prb_second_half_quirk(Nid_cell):
    """The 15-PRB branch (:535-623) starts the second half of every pilot symbol at 1 + nushift + 3 p
    (:582) instead of 1 + k, k = (nu + nushift) mod 6.  For port 0 that is right at l = 0 (nu = 0)
    and 3 bins off at l > 0 (nu = 3): the upper half of the estimate rows 4 / 11 is built from data
    REs.  Reproduced as written, so on a flat noiseless channel row 0 is flat across the band while
    row 4 is flat only below DC (the reference's 15-PRB receiver cannot close dlsim's loop)."""
    p = params("C2", 15, 9, 2, 3, Nid_cell=Nid_cell)
    fp = O.tx_cfg_from_params(p, 3).fp
    rng = np.random.default_rng(Nid_cell)
    pays = [rng.integers(0, 256, p.payload_stride, dtype=np.uint8) for _ in range(2)]
    rxF_sf, next0 = _frame_loop(p, 3, pays, fp)
    est = O.chest_subframe(fp, rxF_sf, next0, 3)
    N = fp.ofdm_symbol_size
    iq = est.view(np.int16).reshape(14, N, 2).astype(float)
    lo, hi = slice(5 + 12, 5 + 84), slice(5 + 96, 5 + 168)    # away from the band edges and from DC
    spread = lambda r, sl: np.ptp(iq[r, sl, 0]) + np.ptp(iq[r, sl, 1])
    assert spread(0, lo) < 40 and spread(0, hi) < 40 and spread(4, lo) < 40
    assert spread(4, hi) > 200


def test_constant_channel_interior_is_flat():
    """A flat channel (received grid = the CRS of amplitude AMP = 1024 themselves) gives an interior
    estimate of (AMP, 0) within the filters' floor rounding: conj(pilot) * rx sums two products of
    ONE_OVER_SQRT2 amplitudes (>> 15), and neighbouring triangle taps sum to 16383 / 16384."""
    fp = O.frame(50, Nid_cell=5)
    N = fp.ofdm_symbol_size
    g = O.gold_table(fp)
    grid = np.zeros(14 * N, np.int32)
    O.orc().orc_generate_pilots_subframe((O.ctypes.c_void_p * 1)(grid.ctypes.data), 1024, O.ctypes.byref(fp), 3)
    est = np.zeros(14 * N, np.int32)
    O.dl_channel_estimation(fp, g, grid, est, 6, 0, 0, 0)
    row = est[:N].view(np.int16).reshape(-1, 2)[5 + 24:5 + 12 * 50 - 24]
    assert np.all(np.abs(row[:, 0].astype(int) - 1024) <= 8) and np.all(np.abs(row[:, 1]) <= 8), row[:4]


# ---- the estimator's vector primitives pinned to the reference's own PHY/TOOLS/cmult_sv.c ----
@pytest.mark.parametrize("zero_flag", [0, 1])
@pytest.mark.parametrize("N", [4, 128, 2048])
def test_multadd_complex_vector_real_scalar_equals_reference(zero_flag, N):
    R = O.ref_tools()
    if R is None or not hasattr(R, "multadd_complex_vector_real_scalar"):
        pytest.skip("reference tree absent (oracle/_ref/libref_tools.so not built)")
    R.multadd_complex_vector_real_scalar.argtypes = [ctypes.c_void_p, ctypes.c_int16, ctypes.c_void_p, ctypes.c_uint8,
                                                     ctypes.c_uint32]
    L = O.orc()
    L.orc_multadd_complex_vector_real_scalar.argtypes = [ctypes.c_void_p, ctypes.c_int16, ctypes.c_void_p,
                                                         ctypes.c_uint8, ctypes.c_uint32]
    rng = np.random.default_rng(N + zero_flag)
    for alpha in (21845, 10923, 24576, 8192, 16384, 32767, -32768, 1):
        x = O._aligned(2 * N, np.int16)
        x[:] = rng.integers(-2**15, 2**15, 2 * N)
        x[:8] = [-32768, 32767, -32768, -1, 0, 1, 32767, -32767][:min(8, 2 * N)]
        y0 = rng.integers(-2**15, 2**15, 2 * N).astype(np.int16)
        yr, yo = O._aligned(2 * N, np.int16), O._aligned(2 * N, np.int16)
        yr[:] = y0
        yo[:] = y0
        R.multadd_complex_vector_real_scalar(O.P(x), alpha, O.P(yr), zero_flag, N)
        L.orc_multadd_complex_vector_real_scalar(O.P(x), alpha, O.P(yo), zero_flag, N)
        assert np.array_equal(yr, yo), alpha


def test_multadd_real_vector_complex_scalar_equals_reference():
    R = O.ref_tools()
    if R is None or not hasattr(R, "multadd_real_vector_complex_scalar"):
        pytest.skip("reference tree absent")
    R.multadd_real_vector_complex_scalar.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
    L = O.orc()
    L.orc_multadd_real_vector_complex_scalar.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                         ctypes.c_uint32]
    rng = np.random.default_rng(9)
    for trial in range(200):
        N = 24 if trial % 2 else 8 * int(rng.integers(1, 40))
        x = O._aligned(N, np.int16)
        x[:] = rng.integers(-2**15, 2**15, N) if trial % 3 else rng.choice([-32768, 32767, 0, 16384, -16384], N)
        a = O._aligned(2, np.int16)
        a[:] = rng.integers(-2**15, 2**15, 2)
        y0 = rng.integers(-2**15, 2**15, 2 * N).astype(np.int16)
        yr, yo = O._aligned(2 * N, np.int16), O._aligned(2 * N, np.int16)
        yr[:] = y0
        yo[:] = y0
        R.multadd_real_vector_complex_scalar(O.P(x), O.P(a), O.P(yr), N)
        L.orc_multadd_real_vector_complex_scalar(O.P(x), O.P(a), O.P(yo), N)
        assert np.array_equal(yr, yo), trial
