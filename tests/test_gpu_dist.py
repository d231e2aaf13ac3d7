"""The C ABI's multi-GPU entry points on the GPU box (one GPU: world 1; the N > 1 logic of the
harness is covered by the gloo tests in test_distributed_cpu.py / test_bench_cpu.py):
  - tools/bin/dlsim_tx -g 1 forks its rank, joins an RCCL communicator through
    oai4g_dist_init, broadcasts the parameter block with oai4g_dist_broadcast_params, runs its
    shard and reduces the IQ checksum with oai4g_dist_allreduce_sum_u64: the checksum equals the
    one computed here from TxPipeline over the same global payload stream;
  - shards filled with oai4g_payload_seed concatenate to the global payload stream (payloads
    depend on (seed, global subframe index), not on the world size);
  - the Python path (bench.py's) through the same C calls at world 1."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _checksum(iq_u32, first, per_sf):
    g = (np.uint64(first) * np.uint64(per_sf) + np.arange(iq_u32.size, dtype=np.uint64))
    w = g * np.uint64(0x9E3779B97F4A7C15) + np.uint64(1)
    return int(np.sum(iq_u32.astype(np.uint64) * w, dtype=np.uint64))


def test_c_driver_world1_checksum(gpu):
    B = 16
    exe = os.path.join(ROOT, "tools", "bin", "dlsim_tx")
    out = subprocess.run([exe, "-c", "C3", "-g", "1", "-B", str(B), "-P"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    line = [l for l in out.stdout.splitlines() if "checksum" in l][0]
    got = int(line.split("checksum")[1].split()[0], 16)
    p = gpu.make_params("C3", subframe=7)
    pipe = gpu.TxPipeline(p, B)
    pipe.fill_payload(gpu.lib().oai4g_payload_seed(0x5EED, 0, p.n_cw, p.payload_stride))
    pipe.run()
    pipe.sync()
    iq = pipe.iq().view(np.uint32).ravel()
    pipe.close()
    assert got == _checksum(iq, 0, p.nb_antennas_tx * 30720)


def test_shard_payloads_concatenate(gpu):
    from openair4g_amd import dist as odist
    p = gpu.make_params("C3", subframe=7)
    full = gpu.TxPipeline(p, 24)
    full.fill_payload(odist.global_payload_seed(0x5EED0000, 0, p))
    want = full.download_payload()
    full.close()
    for world in (2, 3):
        parts = []
        for r in range(world):
            lo, hi = odist.shard_range(24, r, world)
            t = gpu.TxPipeline(p, hi - lo)
            t.fill_payload(odist.global_payload_seed(0x5EED0000, lo, p))
            parts.append(t.download_payload())
            t.close()
        assert np.array_equal(np.concatenate(parts), want), world


def test_python_c_dist_world1(gpu):
    """bench.py's N > 1 calls at world 1: unique id, oai4g_dist_init, broadcast of the parameter
    block (a non-root rank would receive these bytes), sum / max reductions, finalize."""
    from openair4g_amd import dist as odist
    L = gpu.lib()
    buf = (ctypes.c_uint8 * 128)()
    assert L.oai4g_dist_unique_id(buf) == 0
    assert L.oai4g_dist_init(0, 1, buf) == 0
    assert L.oai4g_dist_rank() == 0 and L.oai4g_dist_world() == 1
    p = gpu.make_params("C3", subframe=7)
    q = odist.c_broadcast_params(p)
    assert q.to_bytes() == p.to_bytes()
    v = (ctypes.c_uint64 * 3)(1, 2, 3)
    assert L.oai4g_dist_allreduce_sum_u64(v, 3) == 0 and list(v) == [1, 2, 3]
    d = (ctypes.c_double * 1)(2.5)
    assert L.oai4g_dist_allreduce_max_f64(d, 1) == 0 and d[0] == 2.5
    assert L.oai4g_dist_barrier() == 0
    assert L.oai4g_dist_finalize() == 0 and L.oai4g_dist_world() == 0
