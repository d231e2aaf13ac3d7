"""Multi-GPU plumbing for the transmit path: one process per GPU, subframes sharded across
ranks (weak scaling), no data-path collective.

The only collective is the broadcast of the POD parameter block (oai4g_tx_params_t, a few
hundred bytes) from rank 0, so every rank derives its configuration from identical bytes;
the RCCL backend ("nccl") carries it over xGMI on MI355X, gloo on CPU-only test hosts.
Each rank then encodes its own contiguous range of global subframe indices, with payloads
generated on-device from (seed, rank).  SURVEY.md section 8(e).
"""
import ctypes


def shard_range(n_total, rank, world):
    """Contiguous [start, stop) of global subframe indices owned by `rank` (sizes differ by <= 1)."""
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def broadcast_params(params, dist, device="cpu", src=0):
    """Broadcast a TxParams block from `src`; returns the TxParams every rank now holds.

    `params` is only read on `src` (pass None elsewhere).  `dist` is torch.distributed with an
    initialised process group; `device` is where the byte tensor lives ("cuda" for RCCL)."""
    import torch
    from . import TxParams
    nbytes = ctypes.sizeof(TxParams)
    if dist.get_rank() == src:
        blob = torch.tensor(list(params.to_bytes()), dtype=torch.uint8, device=device)
    else:
        blob = torch.zeros(nbytes, dtype=torch.uint8, device=device)
    dist.broadcast(blob, src=src)
    return TxParams.from_bytes(bytes(blob.cpu().numpy().tobytes()))


def payload_seed(base_seed, rank):
    """Per-rank seed of the device payload generator (distinct shards, reproducible)."""
    return (base_seed + rank) & 0xFFFFFFFFFFFFFFFF
