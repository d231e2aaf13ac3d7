"""GPU parity of the UE receive front end through the C ABI:
oai4g_dft* (lte_dfts.c dft64..dft2048), oai4g_slot_fep (slot_fep.c:40-177) and the batched
oai4g_fep_batch, bit-exact against the reference's own DFT outputs (tests/golden/dft_ref.npz)
and the oracle restatement (orc_dft / orc_slot_fep), which test_fep_cpu.py pins to the
reference library."""
import os

import numpy as np
import pytest

import oracle_lib as O
from test_fep_cpu import fep_cases, window_start

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_gpu_dft_matches_reference_outputs(gpu):
    z = np.load(os.path.join(GOLDEN, "dft_ref.npz"))
    n = 0
    for key in z.files:
        if key.startswith("x_"):
            _, size, vi, scale = key.split("_")
            assert np.array_equal(gpu.dft(z[key], int(scale)), z[f"y_{size}_{vi}_{scale}"]), key
            n += 1
    assert n == 30


@pytest.mark.parametrize("log2n", [6, 7, 8, 9, 10, 11])
def test_gpu_dft_matches_oracle(gpu, log2n):
    n = 1 << log2n
    rng = np.random.default_rng(100 + log2n)
    for t in range(8):
        amp = (50, 2000, 16000, 32767)[t % 4]
        x = (rng.integers(-amp, amp + 1, 2 * n) if t < 4 else
             rng.choice(np.array([-32768, 32767, -amp, amp]), 2 * n)).astype(np.int16)
        for scale in (0, 1):
            assert np.array_equal(gpu.dft(x, scale), O.dft(x, scale)), (n, t, scale)


@pytest.mark.parametrize("N_RB,Ncp", [(6, 0), (15, 0), (25, 0), (50, 0), (100, 0), (25, 1), (100, 1)])
def test_gpu_slot_fep_drop_in(gpu, N_RB, Ncp):
    fp_o = O.frame(N_RB, Ncp=Ncp)
    fp_g = gpu.frame_parms(N_RB, Ncp=Ncp)
    N, fl = fp_o.ofdm_symbol_size, fp_o.samples_per_tti * 10
    rng = np.random.default_rng(7 * N_RB + Ncp)
    frames = [rng.integers(-4000, 4000, 2 * fl).astype(np.int16).view(np.int32) for _ in range(2)]
    for (l, Ns, so, nop) in fep_cases(fp_o):
        rx_g = [np.r_[f, np.zeros(N, np.int32)] for f in frames]
        rx_o = [a.copy() for a in rx_g]
        rxF_g = [np.full(fp_o.symbols_per_tti * N, 7, np.int32) for _ in range(2)]
        rxF_o = [a.copy() for a in rxF_g]
        assert O.slot_fep(rx_o, rxF_o, fp_o, l, Ns, so, nop) == 0
        assert gpu.slot_fep(rx_g, rxF_g, fp_g, l, Ns, so, nop) == 0
        for aa in range(2):
            assert np.array_equal(rxF_g[aa], rxF_o[aa]), (l, Ns, so, nop, aa)
            assert np.array_equal(rx_g[aa], rx_o[aa]), "wrap-extension side effect differs"
        assert window_start(fp_o, l, Ns, so, nop) == gpu.lib().oai4g_slot_fep_offset(fp_g, l, Ns, so, nop)


def test_gpu_slot_fep_errors(gpu):
    fp = gpu.frame_parms(25)
    rx = [np.zeros(fp.samples_per_tti * 10 + fp.ofdm_symbol_size, np.int32)]
    rxF = [np.zeros(14 * fp.ofdm_symbol_size, np.int32)]
    assert gpu.slot_fep(rx, rxF, fp, 7, 0) == -1
    assert gpu.slot_fep(rx, rxF, fp, 0, 20) == -1


def _oracle_fep_subframe(fp_o, rx_sf):
    """every symbol of one subframe (slots 0 and 1, sample_offset 0) by the oracle's slot_fep"""
    N, spt = fp_o.ofdm_symbol_size, fp_o.samples_per_tti
    fl = spt * 10
    nsl = fp_o.symbols_per_tti // 2
    rx = np.zeros(fl + N, np.int32)
    rx[:spt] = rx_sf
    rxF = np.zeros(fp_o.symbols_per_tti * N, np.int32)
    for Ns in (0, 1):
        for l in range(nsl):
            assert O.slot_fep([rx], [rxF], fp_o, l, Ns, 0, 0) == 0
    return rxF.reshape(fp_o.symbols_per_tti, N)


@pytest.mark.parametrize("N_RB,Ncp", [(6, 0), (15, 0), (25, 0), (50, 0), (100, 0), (25, 1), (100, 1)])
def test_gpu_fep_batch(gpu, N_RB, Ncp):
    fp_o = O.frame(N_RB, Ncp=Ncp)
    fp_g = gpu.frame_parms(N_RB, Ncp=Ncp)
    n_sf, n_ant = 3, 2
    rng = np.random.default_rng(N_RB)
    rx = rng.integers(-6000, 6000, (n_sf, n_ant, 2 * fp_o.samples_per_tti)).astype(np.int16).view(np.int32)
    fb = gpu.FepBatch(fp_g, n_sf, n_ant)
    fb.upload(rx)
    fb.run()
    out = fb.result()
    fb.close()
    for s in range(n_sf):
        for a in range(n_ant):
            assert np.array_equal(out[s, a], _oracle_fep_subframe(fp_o, rx[s, a])), (s, a)


def test_gpu_tx_to_fep_loop(gpu):
    """the transmit path's IQ through the receive front end: bit-exact to the oracle's FEP of the
    same IQ, and the PDSCH grid comes back (DFT(IDFT(grid)) = grid up to fixed-point rounding)"""
    p = gpu.make_params("C3", subframe=7)
    n_sf = 4
    pipe = gpu.TxPipeline(p, n_sf)
    rng = np.random.default_rng(11)
    pay = rng.integers(0, 256, size=(n_sf, p.n_cw, p.payload_stride), dtype=np.uint8)
    pipe.upload_payload(pay)
    pipe.run()
    pipe.sync()
    iq = np.ascontiguousarray(pipe.iq()).reshape(n_sf, 2, -1).copy()
    pipe.close()
    fp_o = O.frame(100, nb_antennas_tx=2, mode1_flag=0)
    fp_g = gpu.frame_parms(100, nb_antennas_tx=2, mode1_flag=0)
    fb = gpu.FepBatch(fp_g, n_sf, 2)
    fb.upload(iq)
    fb.run()
    out = fb.result()
    fb.close()
    for s in range(n_sf):
        for a in range(2):
            assert np.array_equal(out[s, a], _oracle_fep_subframe(fp_o, iq[s, a])), (s, a)
    # the transmit grid of subframe 0 (oracle) against the received grid: small residual only
    _, txF, _ = O.tx_subframe(O.tx_cfg_from_params(p, 7), [pay[0, cw] for cw in range(p.n_cw)])
    tx = np.asarray(txF[0]).view(np.int16).reshape(14, -1).astype(np.float64)
    rxg = out[0, 0].view(np.int16).reshape(14, -1).astype(np.float64)
    used = np.abs(tx).sum(axis=1) > 0
    gain = np.sum(rxg[used] * tx[used]) / np.sum(tx[used] ** 2)
    resid = rxg[used] - gain * tx[used]
    assert gain > 0 and np.sqrt(np.mean(resid ** 2)) < 0.05 * np.sqrt(np.mean(tx[used] ** 2))


def test_gpu_fep_batch_full_size(gpu):
    """2048 subframes x 2 antennas at 20 MHz (the bench size): sampled bit-exact checks"""
    fp_o = O.frame(100, nb_antennas_tx=2, mode1_flag=0)
    fp_g = gpu.frame_parms(100, nb_antennas_tx=2, mode1_flag=0)
    n_sf, n_ant = 2048, 2
    rng = np.random.default_rng(3)
    rx = rng.integers(-3000, 3000, (n_sf, n_ant, 2 * fp_o.samples_per_tti), dtype=np.int16).view(np.int32)
    fb = gpu.FepBatch(fp_g, n_sf, n_ant)
    fb.upload(rx)
    fb.run()
    out = fb.result()
    fb.close()
    for s in (0, 1, 777, 2047):
        for a in range(n_ant):
            assert np.array_equal(out[s, a], _oracle_fep_subframe(fp_o, rx[s, a])), (s, a)
