"""CPU suite: the N>1 path with world_size 2 over gloo on 127.0.0.1.

Each rank receives the parameter block from rank 0 (the only collective bench.py uses on the
data path's configuration), takes its contiguous shard of global subframes, transmits them
(oracle on CPU here; the HIP pipeline on a GPU box) and the per-rank checksums are reduced.
The reduced checksum must equal a single-process run over all subframes: sharding loses or
duplicates nothing and every rank derived the same configuration.
"""
import hashlib
import os
import socket

import numpy as np
import pytest

N_SUBFRAMES = 5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _subframe_digest(params, g):
    """IQ digest of global subframe g (payload from a per-subframe seed)."""
    import oracle_lib as O
    sf = (params.first_subframe + g * params.subframe_step) % 10
    rng = np.random.default_rng(1000 + g)
    pays = [rng.integers(0, 256, params.TBS[cw] // 8, dtype=np.uint8) for cw in range(params.n_cw)]
    txd, _, _ = O.tx_subframe(O.tx_cfg_from_params(params, sf), pays)
    return int.from_bytes(hashlib.sha256(txd.tobytes()).digest()[:7], "little")


def _worker(rank, world, port, out_path):
    import sys
    tests = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, tests)
    sys.path.insert(0, os.path.dirname(tests))
    import torch
    import torch.distributed as dist
    import openair4g_amd as oai
    from openair4g_amd import dist as odist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    p0 = oai.make_params("C1", subframe=3, subframe_step=1) if rank == 0 else None
    params = odist.broadcast_params(p0, dist)
    # every rank holds the same bytes
    h = torch.tensor([int.from_bytes(hashlib.sha256(params.to_bytes()).digest()[:7], "little")], dtype=torch.int64)
    hs = [torch.zeros_like(h) for _ in range(world)]
    dist.all_gather(hs, h)
    assert len({int(x) for x in hs}) == 1
    lo, hi = odist.shard_range(N_SUBFRAMES, rank, world)
    acc = torch.tensor([sum(_subframe_digest(params, g) for g in range(lo, hi)) % (1 << 62), hi - lo],
                       dtype=torch.int64)
    dist.all_reduce(acc)
    if rank == 0:
        with open(out_path, "w") as f:
            f.write(f"{int(acc[0])} {int(acc[1])}\n")
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_partitions():
    from openair4g_amd.dist import shard_range
    for n in (0, 1, 5, 2048, 8191):
        for world in (1, 2, 3, 8):
            ranges = [shard_range(n, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            assert all(ranges[i][1] == ranges[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1


def test_two_rank_gloo_matches_single_process(tmp_path):
    import torch.multiprocessing as mp
    import openair4g_amd as oai
    out = tmp_path / "sum.txt"
    mp.spawn(_worker, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    total, count = map(int, out.read_text().split())
    params = oai.make_params("C1", subframe=3, subframe_step=1)
    assert count == N_SUBFRAMES
    assert total == sum(_subframe_digest(params, g) for g in range(N_SUBFRAMES)) % (1 << 62)


if __name__ == "__main__":
    pytest.main([__file__, "-q"])


def test_c_shard_range_and_payload_seed():
    """The C ABI's oai4g_shard_range (the one bench.py and tools/dlsim_tx.c -g use) covers
    [0, n) in rank order with sizes differing by at most one; oai4g_payload_seed advances the
    splitmix64 counter (seed + gamma (w + 1) per 8-byte word) by whole subframes (n_cw
    payload_stride / 8 words each)."""
    import ctypes
    import openair4g_amd as oai
    L = oai.load_library()
    for n in (0, 1, 7, 8192, 8193, 65535):
        for world in (1, 2, 3, 8):
            nxt = 0
            sizes = []
            for r in range(world):
                f, c = ctypes.c_int(), ctypes.c_int()
                L.oai4g_shard_range(n, r, world, ctypes.byref(f), ctypes.byref(c))
                assert f.value == nxt
                nxt += c.value
                sizes.append(c.value)
            assert nxt == n and max(sizes) - min(sizes) <= 1
    assert L.oai4g_payload_seed(100, 0, 2, 4608) == 100
    assert L.oai4g_payload_seed(100, 3, 2, 4608) == (100 + 0x9E3779B97F4A7C15 * 3 * 2 * 576) % 2 ** 64
