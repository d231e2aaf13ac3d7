"""Multi-GPU plumbing for the transmit path: one process per GPU, subframes sharded across
ranks (weak scaling), no data-path collective.

The only collective is the broadcast of the POD parameter block (oai4g_tx_params_t, a few
hundred bytes) from rank 0, so every rank derives its configuration from identical bytes.  On the
GPU it is the C ABI's own RCCL call (oai4g_dist_broadcast_params over xGMI, the same entry the C
host driver tools/dlsim_tx.c -g uses); the torch.distributed group of the timing harness only
carries rank 0's RCCL unique id.  On CPU-only test hosts (gloo) the same block goes through
torch.distributed.  Each rank encodes its own contiguous range of global subframe indices
(oai4g_shard_range), payloads generated on-device from (seed, global subframe index)
(oai4g_payload_seed).  SURVEY.md section 8(e).
"""
import ctypes

from . import OAI4GError, TxParams, lib


def shard_range(n_total, rank, world):
    """Contiguous [start, stop) of global subframe indices owned by `rank` (sizes differ by <= 1):
    the C ABI's oai4g_shard_range."""
    first, count = ctypes.c_int(), ctypes.c_int()
    lib().oai4g_shard_range(n_total, rank, world, ctypes.byref(first), ctypes.byref(count))
    return first.value, first.value + count.value


def global_payload_seed(base_seed, first_subframe, params):
    """oai4g_fill_payload seed of a buffer holding global subframes [first_subframe, ...): the
    payloads depend on (base_seed, global subframe index) only, not on the world size."""
    return lib().oai4g_payload_seed(base_seed, first_subframe, params.n_cw, params.payload_stride)


def c_dist_init(rank, world, dist):
    """Join the C ABI's RCCL communicator: rank 0's unique id through the harness's
    torch.distributed group, then oai4g_dist_init on the device set with oai4g_set_device."""
    L = lib()
    buf = (ctypes.c_uint8 * 128)()
    if rank == 0 and L.oai4g_dist_unique_id(buf) != 0:
        raise OAI4GError(L.oai4g_last_error().decode())
    obj = [bytes(buf) if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    uid = (ctypes.c_uint8 * 128).from_buffer_copy(obj[0])
    if L.oai4g_dist_init(rank, world, uid) != 0:
        raise OAI4GError(L.oai4g_last_error().decode())


def c_broadcast_params(params, root=0):
    """oai4g_dist_broadcast_params: rank root's TxParams to every rank (RCCL)."""
    p = params if params is not None else TxParams()
    if lib().oai4g_dist_broadcast_params(ctypes.byref(p), root) != 0:
        raise OAI4GError(lib().oai4g_last_error().decode())
    return p


def broadcast_params(params, dist, device="cpu", src=0):
    """Broadcast a TxParams block from `src`; returns the TxParams every rank now holds.

    `params` is only read on `src` (pass None elsewhere).  `dist` is torch.distributed with an
    initialised process group; `device` is where the byte tensor lives ("cuda" for RCCL)."""
    import torch
    nbytes = ctypes.sizeof(TxParams)
    if dist.get_rank() == src:
        blob = torch.tensor(list(params.to_bytes()), dtype=torch.uint8, device=device)
    else:
        blob = torch.zeros(nbytes, dtype=torch.uint8, device=device)
    dist.broadcast(blob, src=src)
    return TxParams.from_bytes(bytes(blob.cpu().numpy().tobytes()))
