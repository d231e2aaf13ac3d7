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


@pytest.mark.parametrize("mode", ["8it", "snr"])
def test_c5_bench_batch_16384_blocks(gpu, mode):
    import bench
    n_cb = 2048 * bench.C5_CB
    llr = bench.c5_llrs(n_cb, mode, 0xC5)
    dec = gpu.TurboDecoderBatch(bench.C5_K, n_cb)
    dec.upload(llr)
    dec.run(max_iterations=8, crc_type=1)
    its, outs = dec.results()
    dec.close()
    for i in _samples(n_cb, 4, 7):
        it, d = O.turbo_decode(llr[i], bench.C5_K, max_it=8, crc_type=1)
        assert its[i] == it and np.array_equal(outs[i], d), i
    if mode == "8it":
        assert np.all(its == 9)                 # unstructured LLRs: every CRC check fails
    else:
        assert np.all(its <= 8)
