"""Parity at the bench's own batch sizes (bench.py defaults): the exact device-resident inputs
the bench times — transport blocks generated on the device by oai4g_fill_payload with the bench's
seed, the bench's C5 LLRs, FEP IQ of the bench's shape — checked bit-exactly against the oracle
on sampled batch elements (first, last, and seeded random ones), plus determinism."""
import os
import sys

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SEED = 0x5EED0000                           # bench.py: payload_seed(0x5EED0000, rank 0)


def _check_tx(gpu, name, n_sf, samples):
    p = gpu.make_params(name, subframe=7)
    pipe = gpu.TxPipeline(p, n_sf)
    pipe.fill_payload(seed=SEED)
    pipe.run()
    pipe.sync()
    pay = pipe.download_payload()
    iq = pipe.iq()
    eb = pipe.ebits()
    cfg = O.tx_cfg_from_params(p, 7)
    for i in samples:
        txd, _, e_o = O.tx_subframe(cfg, [pay[i, cw] for cw in range(p.n_cw)], want_e=True)
        for cw in range(p.n_cw):
            G = pipe.G(cw, 7)
            assert np.array_equal(gpu.unpack_bits(eb[i, cw], G), e_o[cw][:G]), (name, i, cw)
        assert np.array_equal(iq[i], txd), (name, i)
    # distinct payloads per subframe (the generator really fills the whole batch)
    assert not np.array_equal(pay[0], pay[n_sf - 1])
    pipe.run()
    pipe.sync()
    assert np.array_equal(pipe.iq()[samples], iq[samples])
    pipe.close()


def _samples(n, k=4, seed=1):
    rng = np.random.default_rng(seed)
    return sorted({0, n - 1, n // 2, *rng.integers(0, n, k).tolist()})


def test_c3_bench_batch_8192(gpu):
    _check_tx(gpu, "C3", 8192, _samples(8192))


@pytest.mark.parametrize("n_sf", [1024, 4096])
def test_c4_bench_batches(gpu, n_sf):
    _check_tx(gpu, "C4", n_sf, _samples(n_sf, 3, n_sf))


def test_fep_bench_batch_8192(gpu):
    from test_gpu_fep import _oracle_fep_subframe
    fp_o = O.frame(100, nb_antennas_tx=2, mode1_flag=0)
    fp_g = gpu.frame_parms(100, nb_antennas_tx=2, mode1_flag=0)
    n_sf, n_ant = 8192, 2
    rng = np.random.default_rng(0xFE9)       # bench.py bench_fep, rank 0
    rx = rng.integers(-3000, 3000, (n_sf, n_ant, 2 * fp_o.samples_per_tti), dtype=np.int16).view(np.int32)
    fb = gpu.FepBatch(fp_g, n_sf, n_ant)
    fb.upload(rx)
    fb.run()
    out = fb.result()
    fb.close()
    for s in _samples(n_sf, 3, 5):
        for a in range(n_ant):
            assert np.array_equal(out[s, a], _oracle_fep_subframe(fp_o, rx[s, a])), (s, a)


@pytest.mark.parametrize("mode,n_sf", [("8it", 2048), ("snr", 2048), ("8it", None)])
def test_c5_bench_batch(gpu, mode, n_sf):
    """2048 subframes (16 384 code blocks, 2 waves per SIMD) and the bench's default batch
    (bench.C5_BATCH subframes: 393 216 blocks, many rounds of 3-wave residency)."""
    import bench
    n_cb = (n_sf or bench.C5_BATCH) * bench.C5_CB
    llr = bench.c5_llrs(mode, 0xC5)           # block i = llr[i % 64], as the bench tiles them
    dec = gpu.TurboDecoderBatch(bench.C5_K, n_cb)
    dec.upload_tiled(llr)
    dec.run(max_iterations=8, crc_type=1)
    its, outs = dec.results()
    dec.close()
    for i in _samples(n_cb, 4, 7):
        it, d = O.turbo_decode(llr[i % len(llr)], bench.C5_K, max_it=8, crc_type=1)
        assert its[i] == it and np.array_equal(outs[i], d), i
    if mode == "8it":
        assert np.all(its == 9)                 # unstructured LLRs: every CRC check fails
    else:
        assert np.all(its <= 8)


def test_ue_bench_batch_4096(gpu):
    """bench.py --config UE at its default 4096 subframes: the GPU-transmitted C2 batch through
    FEP -> channel estimation -> demodulation -> unscrambling, sampled subframes checked against the
    oracle's chain on the same IQ (slot_fep, lte_dl_channel_estimation x 5, rx_pdsch,
    dlsch_unscrambling), and their transport blocks decoded back to the device payload."""
    from test_rx_cpu import decode_tb
    n_sf = 4096
    p = gpu.make_params("C2", subframe=0, subframe_step=1, with_crs=1, rnti=0x1234)
    fg, fo = gpu.frame_parms(100), O.frame(100)
    N, spt = fo.ofdm_symbol_size, fo.samples_per_tti
    Qm = gpu.lib().oai4g_get_Qm(p.mcs[0])
    tx = gpu.TxPipeline(p, n_sf + 1)
    tx.fill_payload(0x5EED)                      # bench_ue, rank 0
    tx.run()
    tx.sync()
    iq = tx.iq()
    pay = tx.download_payload()
    tx.close()
    fb = gpu.FepBatch(fg, n_sf + 1, 1)
    fb.upload(iq)
    fb.run()
    cb = gpu.ChestBatch(fg, n_sf, first_subframe=0)
    rb = gpu.RxBatch(fg, list(p.rb_alloc), Qm, p.num_pdcch_symbols, p.rnti, n_sf, first_subframe=0, subframe_step=1)
    cb.launch(fb.d_rxF)
    rb.launch(fb.d_rxF, cb.d_est, 1)
    gpu.lib().oai4g_sync()
    out = np.empty((n_sf, rb.stride), dtype=np.int16)
    gpu.lib().oai4g_memcpy_d2h(gpu._ptr(out), rb.d_llr, out.nbytes)
    for i in _samples(n_sf, 3, 11):
        sf = i % 10
        frame = np.zeros(10 * spt + N, np.int32)
        frame[sf * spt:(sf + 1) * spt] = iq[i, 0]
        nsf = (sf + 1) % 10
        frame[nsf * spt:(nsf + 1) * spt] = iq[i + 1, 0]
        rxF, nxt = np.zeros(15 * N, np.int32), np.zeros(15 * N, np.int32)
        for Ns in (2 * sf, 2 * sf + 1):
            for l in range(7):
                assert O.slot_fep([frame], [rxF], fo, l, Ns) == 0
        assert O.slot_fep([frame], [nxt], fo, 0, (2 * sf + 2) % 20) == 0
        est = O.chest_subframe(fo, rxF[:14 * N], nxt[:N], sf)
        lo, _ = O.rx_pdsch_siso(fo, rxF[:14 * N], est, list(p.rb_alloc), Qm, p.num_pdcch_symbols, sf)
        G = len(lo)
        u = np.zeros(32 * (1 + G // 32), np.int16)
        u[:G] = lo
        O.dlsch_unscrambling(u, G, (p.rnti << 14) + (sf << 9) + fo.Nid_cell)
        assert rb.llr_count(sf) == G and np.array_equal(out[i, :G], u[:G]), i
        if sf not in (0, 5):                    # the reference's even-N_RB extraction of PBCH / sync REs
            res, tb = decode_tb(out[i], G, p.TBS[0], Qm)
            assert np.array_equal(tb, pay[i, 0, :p.TBS[0] // 8]), i
    fb.close()
    cb.close()
    rb.close()
