/*
 * gfx950 kernels of dlsim's AWGN channel stage (openair1/SIMULATION/LTE_PHY/dlsim.c:2714-2866), the
 * link between the transmit batch and the UE receive batch in a BLER run:
 *   signal_energy   PHY/TOOLS/signal_energy.c:66-110: mean of (re^2 + im^2) >> 4 over the vector,
 *                   minus the squared DC (16-bit lane sums), with the SSE code's wraps and its
 *                   int / uint32_t divisions — dlsim's tx_lev per transmit antenna (:2714-2719)
 *   AWGN            dlsim.c:2852-2866: sigma2_dB = 10 log10(tx_lev) + 10 log10(N / (12 NB_RB)) - SNR
 *                   - pa_dB; r = (short)(s + sqrt(sigma2 / 2) g) per I / Q component, g ~ N(0, 1)
 *                   (the reference draws g from gaussdouble, SIMULATION/TOOLS/rangen_double.c:97, a
 *                   polar Box-Muller over a shuffled 32-bit LCG; here a counter-based Philox-4x32
 *                   stream with the Box-Muller transform in double precision, so a run is
 *                   reproducible from (seed, vector, sample) whatever the launch shape)
 * Both are HBM-streaming (one read + one write of the int16 IQ per sample), one workgroup per
 * vector chunk, coalesced 4-byte lanes.
 */
#include "oai4g_internal.h"

namespace {

constexpr uint32_t SE_WG = 256;
constexpr uint32_t AW_WG = 256;
constexpr uint32_t AW_PER = 4;          /* samples per thread: 1024 per workgroup */

/* Philox-4x32-10 (Salmon et al., "Parallel random numbers: as easy as 1, 2, 3", SC'11) */
__device__ __forceinline__ uint4 philox(uint4 c, uint2 k)
{
  for (int r = 0; r < 10; r++) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    c = make_uint4((uint32_t)(p1 >> 32) ^ c.y ^ k.x, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k.y, (uint32_t)p0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

/* (0, 1] with 53 bits */
__device__ __forceinline__ double u53(uint32_t hi, uint32_t lo)
{
  return ((double)((((uint64_t)hi << 32) | lo) >> 11) + 1.0) * (1.0 / 9007199254740992.0);
}

/* C's (short) of a double: truncation toward zero through int, 16-bit wrap as on x86 */
__device__ __forceinline__ uint32_t to_short(double v) { return (uint32_t)(uint16_t)(int16_t)(int32_t)v; }

}  // namespace

/* energy of vector blockIdx.x: length complex samples at x + blockIdx.x * stride */
__global__ void __launch_bounds__(SE_WG) k_signal_energy(const int32_t *__restrict__ x, size_t stride, uint32_t length,
                                                         int32_t *__restrict__ out)
{
  __shared__ uint32_t s_pw[SE_WG / 64], s_dc[SE_WG / 64];
  const int32_t *v = x + (size_t)blockIdx.x * stride;
  const uint32_t n = length & ~1u;                  /* the SSE loop runs length >> 1 sample pairs */
  uint32_t pw = 0, dre = 0, dim = 0;
  for (uint32_t i = threadIdx.x; i < n; i += SE_WG) {
    const uint32_t w = (uint32_t)v[i];
    const int32_t re = (int16_t)w, im = (int16_t)(w >> 16);
    /* pmaddwd (int32 wrap), psrad 4, paddd (wrap) */
    const int32_t p = (int32_t)((uint32_t)(re * re) + (uint32_t)(im * im));
    pw += (uint32_t)(p >> 4);
    dre += (uint32_t)re;                            /* paddw: only the low 16 bits matter */
    dim += (uint32_t)im;
  }
  const uint32_t dc = (dre & 0xFFFFu) | (dim << 16);
  uint32_t a = pw, lo = dc & 0xFFFFu, hi = dc >> 16;
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o);
    lo += __shfl_xor(lo, o);
    hi += __shfl_xor(hi, o);
  }
  if ((threadIdx.x & 63) == 0) {
    s_pw[threadIdx.x >> 6] = a;
    s_dc[threadIdx.x >> 6] = (lo & 0xFFFFu) | (hi << 16);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t sp = 0, sr = 0, si = 0;
    for (uint32_t w = 0; w < SE_WG / 64; w++) {
      sp += s_pw[w];
      sr += s_dc[w] & 0xFFFFu;
      si += s_dc[w] >> 16;
    }
    /* temp /= length with length unsigned (the int32 sum is converted), then <<= 4 */
    int32_t temp = (int32_t)(sp / length);
    temp = (int32_t)((uint32_t)temp << 4);
    /* the DC term: pmaddwd of the two 16-bit lane sums, / (length * length) as unsigned */
    const int32_t r16 = (int16_t)sr, i16 = (int16_t)si;
    const int32_t t2 = (int32_t)((uint32_t)(r16 * r16) + (uint32_t)(i16 * i16));
    const int32_t temp2 = (int32_t)((uint32_t)t2 / (length * length));
    temp -= temp2;
    out[blockIdx.x] = temp > 0 ? temp : 1;
  }
}

/* vector blockIdx.y, samples [blockIdx.x * 1024, +1024): the transmit samples (tx_len from tx, then
 * tail_len from the common tail) plus noise of standard deviation sqrt(sigma2 / 2) per component */
__global__ void __launch_bounds__(AW_WG) k_awgn(const int32_t *__restrict__ tx, size_t tx_stride, uint32_t tx_len,
                                                const int32_t *__restrict__ tail, uint32_t tail_len,
                                                int32_t *__restrict__ rx, size_t rx_stride,
                                                const int32_t *__restrict__ tx_lev, double offset_db, uint32_t seed_lo,
                                                uint32_t seed_hi, uint32_t vec0)
{
  __shared__ double s_sigma;
  const uint32_t vec = blockIdx.y;
  if (threadIdx.x == 0) {
    /* dlsim.c:2852-2853 */
    const double sigma2_dB = 10.0 * log10((double)tx_lev[vec]) + offset_db;
    s_sigma = sqrt(pow(10.0, sigma2_dB / 10.0) / 2.0);
  }
  __syncthreads();
  const double sigma = s_sigma;
  const uint32_t len = tx_len + tail_len;
  const int32_t *t = tx + (size_t)vec * tx_stride;
  int32_t *r = rx + (size_t)vec * rx_stride;
#pragma unroll
  for (uint32_t u = 0; u < AW_PER; u++) {
    const uint32_t i = blockIdx.x * (AW_WG * AW_PER) + u * AW_WG + threadIdx.x;
    if (i >= len) break;
    const uint32_t w = (uint32_t)(i < tx_len ? t[i] : tail[i - tx_len]);
    const uint4 q = philox(make_uint4(i, vec0 + vec, 0x5EEDu, 0xA3C5u), make_uint2(seed_lo, seed_hi));
    const double u1 = u53(q.x, q.y), u2 = u53(q.z, q.w);
    const double rad = sqrt(-2.0 * log(u1));
    double sn, cs;
    sincospi(2.0 * u2, &sn, &cs);
    const double re = (double)(int16_t)w + sigma * rad * cs, im = (double)(int16_t)(w >> 16) + sigma * rad * sn;
    r[i] = (int32_t)(to_short(re) | (to_short(im) << 16));
  }
}

hipError_t oai4g_launch_signal_energy(const int32_t *d_x, int n, size_t stride, uint32_t length, int32_t *d_out,
                                      hipStream_t s)
{
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_signal_energy, dim3(n), dim3(SE_WG), 0, s, d_x, stride, length, d_out);
  return hipGetLastError();
}

hipError_t oai4g_launch_awgn(const int32_t *d_tx, size_t tx_stride, uint32_t tx_len, const int32_t *d_tail,
                             uint32_t tail_len, int32_t *d_rx, size_t rx_stride, int n, const int32_t *d_tx_lev,
                             double offset_db, uint64_t seed, uint32_t vec0, hipStream_t s)
{
  if (n <= 0) return hipSuccess;
  const uint32_t len = tx_len + tail_len, per = AW_WG * AW_PER;
  hipLaunchKernelGGL(k_awgn, dim3((len + per - 1) / per, n), dim3(AW_WG), 0, s, d_tx, tx_stride, tx_len, d_tail,
                     tail_len, d_rx, rx_stride, d_tx_lev, offset_db, (uint32_t)seed, (uint32_t)(seed >> 32), vec0);
  return hipGetLastError();
}
