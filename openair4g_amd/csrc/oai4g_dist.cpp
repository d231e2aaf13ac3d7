/*
 * Multi-GPU plumbing of the C ABI (north_star: "subframes / codewords shard naturally
 * across the 8 GPUs of one node with RCCL broadcast of frame parameters over xGMI only").
 *
 * One process per GPU.  The path has no data-path exchange: every rank encodes its own contiguous
 * range of global subframe indices, payloads generated on its device from (seed, global subframe
 * index).  The collectives are RCCL's (librccl, NCCL API) over xGMI:
 *   - ncclBroadcast of the POD parameter block oai4g_tx_params_t from the root, so every rank
 *     derives its configuration from identical bytes;
 *   - ncclAllReduce of per-rank counters / checksums (sum) and of timings (max) at the end.
 * The unique id travels out of band (a pipe in tools/dlsim_tx.c -g, the torch.distributed store
 * in bench.py).  A communicator per process; the calls are not thread-safe (one host thread drives
 * the rank, as dlsim does).
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <string.h>

#include "oai4g_internal.h"

namespace {
struct dist_t {
  ncclComm_t comm = nullptr;
  hipStream_t s = nullptr;
  void *buf = nullptr;              /* device staging for host-side operands */
  size_t cap = 0;
  int rank = 0, world = 1;
};
dist_t g_dist;

int stage(size_t bytes)
{
  if (bytes <= g_dist.cap) return 0;
  if (g_dist.buf) hipFree(g_dist.buf);
  g_dist.buf = nullptr;
  g_dist.cap = 0;
  if (hipMalloc(&g_dist.buf, bytes) != hipSuccess) return -1;
  g_dist.cap = bytes;
  return 0;
}

#define NCK(x, what)                                                                          \
  do {                                                                                        \
    ncclResult_t r_ = (x);                                                                    \
    if (r_ != ncclSuccess) {                                                                  \
      oai4g_set_error("%s: %s", what, ncclGetErrorString(r_));                               \
      return -1;                                                                              \
    }                                                                                         \
  } while (0)

/* a host array through a device buffer: copy in, collective, copy out, synchronize */
int host_collective(void *v, size_t bytes, int (*op)(void *dbuf))
{
  if (!g_dist.comm) { oai4g_set_error("dist: oai4g_dist_init has not run"); return -1; }
  if (stage(bytes) != 0) { oai4g_set_error("dist: device staging allocation failed"); return -1; }
  if (hipMemcpyAsync(g_dist.buf, v, bytes, hipMemcpyHostToDevice, g_dist.s) != hipSuccess) {
    oai4g_set_error("dist: staging upload failed");
    return -1;
  }
  if (op(g_dist.buf) != 0) return -1;
  if (hipMemcpyAsync(v, g_dist.buf, bytes, hipMemcpyDeviceToHost, g_dist.s) != hipSuccess ||
      hipStreamSynchronize(g_dist.s) != hipSuccess) {
    oai4g_set_error("dist: staging download failed");
    return -1;
  }
  return 0;
}
}  // namespace

extern "C" int oai4g_dist_unique_id(uint8_t id[OAI4G_DIST_ID_BYTES])
{
  ncclUniqueId u;
  static_assert(sizeof(u) == OAI4G_DIST_ID_BYTES, "ncclUniqueId size");
  NCK(ncclGetUniqueId(&u), "dist_unique_id");
  memcpy(id, &u, sizeof(u));
  return 0;
}

extern "C" int oai4g_dist_init(int rank, int world, const uint8_t id[OAI4G_DIST_ID_BYTES])
{
  if (world < 1 || rank < 0 || rank >= world) { oai4g_set_error("dist_init: rank %d of world %d", rank, world); return -1; }
  if (g_dist.comm) { oai4g_set_error("dist_init: already initialised"); return -1; }
  if (oai4g_init() != 0 || oai4g_bind_thread() != 0) return -1;   /* the rank's device: oai4g_set_device before */
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  if (hipStreamCreateWithFlags(&g_dist.s, hipStreamNonBlocking) != hipSuccess) {
    oai4g_set_error("dist_init: stream creation failed");
    return -1;
  }
  ncclResult_t r = ncclCommInitRank(&g_dist.comm, world, u, rank);
  if (r != ncclSuccess) {                              /* leave g_dist as before: a retry starts clean */
    oai4g_set_error("dist_init (ncclCommInitRank): %s", ncclGetErrorString(r));
    hipStreamDestroy(g_dist.s);
    g_dist.s = nullptr;
    g_dist.comm = nullptr;
    return -1;
  }
  g_dist.rank = rank;
  g_dist.world = world;
  return 0;
}

extern "C" int oai4g_dist_broadcast_params(oai4g_tx_params_t *p, int root)
{
  if (!p || root < 0 || root >= g_dist.world) { oai4g_set_error("dist_broadcast_params: bad arguments"); return -1; }
  static int s_root;
  s_root = root;
  return host_collective(p, sizeof(*p), [](void *d) -> int {
    NCK(ncclBroadcast(d, d, sizeof(oai4g_tx_params_t), ncclUint8, s_root, g_dist.comm, g_dist.s),
        "dist_broadcast_params");
    return 0;
  });
}

extern "C" int oai4g_dist_allreduce_sum_u64(uint64_t *v, int n)
{
  if (!v || n < 0) { oai4g_set_error("dist_allreduce_sum_u64: bad arguments"); return -1; }
  if (n == 0) return 0;
  static size_t s_n;
  s_n = (size_t)n;
  return host_collective(v, (size_t)n * 8, [](void *d) -> int {
    NCK(ncclAllReduce(d, d, s_n, ncclUint64, ncclSum, g_dist.comm, g_dist.s), "dist_allreduce_sum_u64");
    return 0;
  });
}

extern "C" int oai4g_dist_allreduce_max_f64(double *v, int n)
{
  if (!v || n < 0) { oai4g_set_error("dist_allreduce_max_f64: bad arguments"); return -1; }
  if (n == 0) return 0;
  static size_t s_n;
  s_n = (size_t)n;
  return host_collective(v, (size_t)n * 8, [](void *d) -> int {
    NCK(ncclAllReduce(d, d, s_n, ncclFloat64, ncclMax, g_dist.comm, g_dist.s), "dist_allreduce_max_f64");
    return 0;
  });
}

extern "C" int oai4g_dist_barrier(void)
{
  uint64_t z = 0;
  return oai4g_dist_allreduce_sum_u64(&z, 1);
}

extern "C" int oai4g_dist_rank(void) { return g_dist.comm ? g_dist.rank : -1; }
extern "C" int oai4g_dist_world(void) { return g_dist.comm ? g_dist.world : 0; }

extern "C" int oai4g_dist_finalize(void)
{
  if (!g_dist.comm) return 0;
  ncclResult_t r = ncclCommDestroy(g_dist.comm);
  g_dist.comm = nullptr;
  if (g_dist.s) hipStreamDestroy(g_dist.s);
  if (g_dist.buf) hipFree(g_dist.buf);
  g_dist = dist_t();
  if (r != ncclSuccess) { oai4g_set_error("dist_finalize: %s", ncclGetErrorString(r)); return -1; }
  return 0;
}

extern "C" void oai4g_shard_range(int n_total, int rank, int world, int *first, int *count)
{
  if (world < 1 || rank < 0 || rank >= world || n_total < 0) {
    *first = 0;
    *count = 0;
    return;
  }
  const int base = n_total / world, extra = n_total % world;
  *first = rank * base + (rank < extra ? rank : extra);
  *count = base + (rank < extra ? 1 : 0);
}

extern "C" uint64_t oai4g_payload_seed(uint64_t seed, uint64_t first_subframe, uint32_t n_cw, uint32_t payload_stride)
{
  /* k_fill: word w of a buffer = splitmix64 output of seed + gamma (w + 1), gamma = 0x9e37...7c15,
   * so the buffer of global subframes [first, ...) equals the global payload when seeded
   * seed + gamma first n_cw stride / 8 (payload_stride is a multiple of 16) */
  return seed + 0x9e3779b97f4a7c15ull * (first_subframe * n_cw * (payload_stride / 8));
}
