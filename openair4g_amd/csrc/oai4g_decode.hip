/*
 * gfx950 uplink turbo decoding:
 *   phy_threegpplte_turbo_decoder16   PHY/CODING/3gpplte_turbo_decoder_sse_16bit.c:945-1385
 *   lte_rate_matching_turbo_rx        PHY/CODING/lte_rate_matching.c:688-831
 *   sub_block_deinterleaving_turbo    PHY/CODING/lte_rate_matching.c:193-243
 *
 * The reference decoder keeps 8 int16 SSE lanes = 8 windows of K/8 trellis steps.  Here one
 * 64-lane wave decodes 8 code blocks at once: lane (g, q) owns window q of block g, i.e. one
 * column of the reference's registers, so every saturating add/sub/max is the reference's own
 * per-lane operation and the results are bit-identical.  Per lane and half-iteration:
 *   - gamma is formed on the fly from the systematic / parity LLRs (compute_gamma16);
 *   - the forward recursion stores alpha for every step (16 B per step and lane);
 *   - the alpha re-run over the first L/8 = 5 steps starts from the previous window's final
 *     alpha (a width-8 shuffle) as in compute_alpha16;
 *   - the backward recursion starts from the lane's own final alpha (the last window from the
 *     termination betas), produces the extrinsic of each step on the way (compute_ext16), and
 *     its re-run over the last 5 steps starts from the next window's beta[0]; the 6 extrinsic
 *     values that depend on re-run betas are produced by the re-run.
 * Between half-iterations the permuted exchanges (pi4 / pi5 / pi6 of init_td16) go through the
 * block's scratch in global memory; the CRC early stop runs per block.
 */
#include "oai4g_internal.h"

typedef const __attribute__((address_space(1))) int16_t gs16_t;

static __device__ __forceinline__ short sadd(short a, short b) { return __builtin_elementwise_add_sat(a, b); }
static __device__ __forceinline__ short ssub(short a, short b) { return __builtin_elementwise_sub_sat(a, b); }
static __device__ __forceinline__ short smax(short a, short b) { return a > b ? a : b; }

#define TD_MAXH 128    /* MAX / 2 */

struct td_blk_t {      /* one block's scratch (int16 element offsets, see td_layout) */
  short *s0, *s1, *s2, *yp1, *yp2, *ext, *ext2;
  uint4 *A;            /* alpha: [(K1 + 1)][8 lanes] x 8 states (16 B) */
};

static __device__ __forceinline__ td_blk_t td_layout(uint8_t *base, uint32_t K)
{
  td_blk_t b;
  short *p = (short *)base;
  const uint32_t n16 = (K + 16 + 7) & ~7u, n128 = K + 128;
  b.s0 = p; p += n16;
  b.s1 = p; p += n16;
  b.s2 = p; p += n16;
  b.yp1 = p; p += n16;
  b.yp2 = p; p += n16;
  b.ext = p; p += n128;
  b.ext2 = p; p += n128;
  b.A = (uint4 *)(((uintptr_t)p + 15) & ~(uintptr_t)15);
  return b;
}

size_t oai4g_td_block_bytes(uint32_t K)
{
  const size_t n16 = (K + 16 + 7) & ~7u, n128 = K + 128;
  return (((5 * n16 + 2 * n128) * 2 + 15) & ~(size_t)15) + (size_t)(K / 8 + 1) * 8 * 16 + 256;
}

static __device__ __forceinline__ uint4 pack8(const short *v)
{
  return make_uint4((uint16_t)v[0] | ((uint32_t)(uint16_t)v[1] << 16), (uint16_t)v[2] | ((uint32_t)(uint16_t)v[3] << 16),
                    (uint16_t)v[4] | ((uint32_t)(uint16_t)v[5] << 16), (uint16_t)v[6] | ((uint32_t)(uint16_t)v[7] << 16));
}
static __device__ __forceinline__ void unpack8(uint4 u, short *v)
{
  v[0] = (short)u.x; v[1] = (short)(u.x >> 16); v[2] = (short)u.y; v[3] = (short)(u.y >> 16);
  v[4] = (short)u.z; v[5] = (short)(u.z >> 16); v[6] = (short)u.w; v[7] = (short)(u.w >> 16);
}

/* forward step (compute_alpha16 :286-367) */
static __device__ __forceinline__ void alpha_step(short *a, short g11, short g10)
{
  short r0 = smax(sadd(a[1], g11), ssub(a[0], g11)), r4 = smax(ssub(a[1], g11), sadd(a[0], g11));
  short r1 = smax(ssub(a[3], g10), sadd(a[2], g10)), r5 = smax(sadd(a[3], g10), ssub(a[2], g10));
  short r2 = smax(sadd(a[5], g10), ssub(a[4], g10)), r6 = smax(ssub(a[5], g10), sadd(a[4], g10));
  short r3 = smax(ssub(a[7], g11), sadd(a[6], g11)), r7 = smax(sadd(a[7], g11), ssub(a[6], g11));
  short mx = smax(smax(smax(r0, r1), smax(r2, r3)), smax(smax(r4, r5), smax(r6, r7)));
  a[0] = ssub(r0, mx); a[1] = ssub(r1, mx); a[2] = ssub(r2, mx); a[3] = ssub(r3, mx);
  a[4] = ssub(r4, mx); a[5] = ssub(r5, mx); a[6] = ssub(r6, mx); a[7] = ssub(r7, mx);
}

/* backward step (compute_beta16 :588-685) */
static __device__ __forceinline__ void beta_step(short *b, short g11, short g10)
{
  short r0 = smax(sadd(b[4], g11), ssub(b[0], g11)), r1 = smax(ssub(b[4], g11), sadd(b[0], g11));
  short r2 = smax(ssub(b[5], g10), sadd(b[1], g10)), r3 = smax(sadd(b[5], g10), ssub(b[1], g10));
  short r4 = smax(sadd(b[6], g10), ssub(b[2], g10)), r5 = smax(ssub(b[6], g10), sadd(b[2], g10));
  short r6 = smax(ssub(b[7], g11), sadd(b[3], g11)), r7 = smax(sadd(b[7], g11), ssub(b[3], g11));
  short mx = smax(smax(smax(r0, r1), smax(r2, r3)), smax(smax(r4, r5), smax(r6, r7)));
  b[0] = ssub(r0, mx); b[1] = ssub(r1, mx); b[2] = ssub(r2, mx); b[3] = ssub(r3, mx);
  b[4] = ssub(r4, mx); b[5] = ssub(r5, mx); b[6] = ssub(r6, mx); b[7] = ssub(r7, mx);
}

/* extrinsic of one step from alpha(k), beta(k+1), gamma(k) (compute_ext16 :733-875) */
static __device__ __forceinline__ short ext_of(const short *a, const short *b, short g11, short g10)
{
  short m00 = smax(smax(sadd(a[0], b[0]), sadd(a[1], b[4])), smax(sadd(a[6], b[7]), sadd(a[7], b[3])));
  short m11 = smax(smax(sadd(a[0], b[4]), sadd(a[1], b[0])), smax(sadd(a[6], b[3]), sadd(a[7], b[7])));
  short m01 = smax(smax(sadd(a[2], b[5]), sadd(a[3], b[1])), smax(sadd(a[4], b[2]), sadd(a[5], b[6])));
  short m10 = smax(smax(sadd(a[2], b[1]), sadd(a[3], b[5])), smax(sadd(a[4], b[6]), sadd(a[5], b[2])));
  m01 = ssub(m01, g10);
  m00 = ssub(m00, g11);
  m10 = sadd(m10, g10);
  m11 = sadd(m11, g11);
  return ssub(smax(m10, m11), smax(m01, m00));
}

static __device__ __forceinline__ void gamma_of(const short *sys, const short *par, uint32_t e, short &g11, short &g10)
{
  const short s = sys[e], p = par[e];
  g11 = (short)(sadd(s, p) >> 1);
  g10 = (short)(ssub(s, p) >> 1);
}

/*
 * log_map16 for the calling lane (window q of its block): sys / par in the reference's vector
 * layout (element 8k + q), extrinsic out likewise.  Lanes of a block exchange re-run seeds with
 * width-8 shuffles; the 8 lanes of a block are always active together.
 */
static __device__ __forceinline__ void log_map(const short *sys, const short *par, short *ext, uint4 *A, uint32_t K,
                                               uint32_t q, int tf)
{
  const uint32_t K1 = K >> 3;
  short a[8], g11, g10;
  /* forward, first run */
#pragma unroll
  for (int s = 0; s < 8; s++) a[s] = (s == 0 && q == 0) ? 0 : -TD_MAXH;
  A[q] = pack8(a);
  for (uint32_t k = 0; k < K1; k++) {
    gamma_of(sys, par, 8 * k + q, g11, g10);
    alpha_step(a, g11, g10);
    A[8 * (k + 1) + q] = pack8(a);
  }
  /* forward re-run over L/8 steps from the previous window's final alpha */
  short fin[8];
#pragma unroll
  for (int s = 0; s < 8; s++) {
    fin[s] = a[s];
    short up = (short)__shfl_up((int)a[s], 1, 8);
    a[s] = q == 0 ? (s == 0 ? 0 : -TD_MAXH) : up;
  }
  A[q] = pack8(a);
  for (uint32_t k = 0; k < 5; k++) {
    gamma_of(sys, par, 8 * k + q, g11, g10);
    alpha_step(a, g11, g10);
    A[8 * (k + 1) + q] = pack8(a);
  }
  /* termination betas of the last window (compute_beta16 :467-521, int16 wrap arithmetic) */
  short t[8];
  {
    short m[3], mm[3];
#pragma unroll
    for (int j = 0; j < 3; j++) gamma_of(sys + 8 * tf, par, K + j, m[j], mm[j]);   /* m_11/m_10[n + j] */
    short beta0 = (short)-m[2], beta1 = m[2];
    short b0_2 = (short)(beta0 - m[1]), b1_2 = (short)(beta0 + m[1]), b2_2 = (short)(beta1 + mm[1]),
          b3_2 = (short)(beta1 - mm[1]);
    t[0] = (short)(b0_2 - m[0]); t[1] = (short)(b0_2 + m[0]); t[2] = (short)(b1_2 + mm[0]); t[3] = (short)(b1_2 - mm[0]);
    t[4] = (short)(b2_2 - mm[0]); t[5] = (short)(b2_2 + mm[0]); t[6] = (short)(b3_2 + m[0]); t[7] = (short)(b3_2 - m[0]);
    short bm = t[0];
#pragma unroll
    for (int s = 1; s < 8; s++) bm = bm > t[s] ? bm : t[s];
#pragma unroll
    for (int s = 0; s < 8; s++) t[s] = (short)(t[s] - bm);
  }
  /* backward, first run: seeded with the lane's own final alpha as stored after the re-run
   * (the re-run reaches step K1 when K1 == 5); extrinsic of steps whose beta the re-run does
   * not touch */
  unpack8(A[8 * K1 + q], fin);
  short b[8], al[8];
#pragma unroll
  for (int s = 0; s < 8; s++) b[s] = q == 7 ? t[s] : fin[s];
  for (int k = (int)K1 - 1; k >= 0; k--) {
    gamma_of(sys, par, 8 * k + q, g11, g10);
    if (k < (int)K1 - 6) {
      unpack8(A[8 * k + q], al);
      ext[8 * k + q] = ext_of(al, b, g11, g10);
    }
    beta_step(b, g11, g10);
  }
  /* backward re-run over the last L/8 steps from the next window's beta[0] */
#pragma unroll
  for (int s = 0; s < 8; s++) {
    short dn = (short)__shfl_down((int)b[s], 1, 8);
    b[s] = q == 7 ? t[s] : dn;
  }
  for (int k = (int)K1 - 1; k >= (int)K1 - 6 && k >= 0; k--) {
    gamma_of(sys, par, 8 * k + q, g11, g10);
    unpack8(A[8 * k + q], al);
    ext[8 * k + q] = ext_of(al, b, g11, g10);
    if (k >= (int)K1 - 5) beta_step(b, g11, g10);
  }
}

__device__ static const uint32_t *td_crc_tab(uint32_t *lds, uint32_t poly)
{
  for (uint32_t v = threadIdx.x; v < 256; v += blockDim.x) {
    uint32_t r = v << 16;
    for (int i = 0; i < 8; i++) r = (r & 0x800000u) ? ((r << 1) ^ poly) & 0xffffffu : (r << 1) & 0xffffffu;
    lds[v] = r;
  }
  return lds;
}

/*
 * Batch decoder: blockIdx.x decodes blocks 8 blockIdx.x .. +7 (one 64-lane wave).
 * llr: [n_cb][llr_stride] int16 (3K + 12 each), out: [n_cb][out_stride] bytes, iters: [n_cb].
 */
__global__ void __launch_bounds__(64) k_td16(int n_cb, uint32_t K, const int16_t *__restrict__ llr, size_t llr_stride,
                                             uint8_t *__restrict__ out, size_t out_stride, uint8_t *__restrict__ iters,
                                             uint32_t max_it, uint32_t crc_type, uint32_t F,
                                             const uint16_t *__restrict__ pi4, const uint16_t *__restrict__ pi5,
                                             const uint16_t *__restrict__ pi6, uint8_t *__restrict__ scratch,
                                             size_t blk_bytes)
{
  __shared__ uint32_t crctab[256];
  __shared__ uint8_t dec[8][6144 / 8 + 8];
  __shared__ uint32_t done_it[8];
  const uint32_t lane = threadIdx.x, g = lane >> 3, q = lane & 7;
  const int cb = (int)(blockIdx.x * 8 + g);
  const bool valid = cb < n_cb;
  const uint32_t K1 = K >> 3, Kb = K >> 3;
  td_crc_tab(crctab, crc_type == 0 ? 0x864cfbu : 0x800063u);
  if (lane < 8) done_it[lane] = 0;
  td_blk_t B = td_layout(scratch + (size_t)(valid ? cb : 0) * blk_bytes, K);
  if (valid) {
    /* demux (:1038-1158): bit i = window q, step v -> element 8v + q */
    gs16_t *y = (gs16_t *)(llr + (size_t)cb * llr_stride);
    for (uint32_t v = 0; v < K1; v++) {
      const uint32_t i = q * K1 + v, j = 8 * v + q;
      B.s0[j] = y[3 * i];
      B.yp1[j] = y[3 * i + 1];
      B.yp2[j] = y[3 * i + 2];
    }
    if (q == 0) {
      for (uint32_t i = 0; i < 3; i++) {   /* tails (:1164-1186) */
        const short s_a = y[3 * K + 2 * i], p_a = y[3 * K + 2 * i + 1];
        const short s_b = y[3 * K + 6 + 2 * i], p_b = y[3 * K + 6 + 2 * i + 1];
        B.s0[K + i] = B.s1[K + i] = B.s2[K + i] = s_a;
        B.yp1[K + i] = p_a;
        B.s0[K + 8 + i] = B.s1[K + 8 + i] = B.s2[K + 8 + i] = s_b;
        B.yp2[K + i] = p_b;
      }
    }
  }
  __syncthreads();
  bool active = valid && max_it > 0;
  if (valid) log_map(B.s0, B.yp1, B.ext, B.A, K, q, 0);
  __syncthreads();
  uint32_t it = 0;
  for (it = 1; it <= max_it; it++) {
    if (active)
      for (uint32_t v = 0; v < K1; v++) B.s2[8 * v + q] = B.ext[pi4[8 * v + q]];
    __syncthreads();
    if (active) log_map(B.s2, B.yp2, B.ext2, B.A, K, q, 1);
    __syncthreads();
    if (active) {
      for (uint32_t v = 0; v < K1; v++) {
        const uint32_t i = 8 * v + q;
        B.s1[i] = sadd(ssub(B.ext2[pi5[i]], B.ext[i]), B.s0[i]);
      }
      if (it > 1)
        for (uint32_t i = q; i < Kb; i += 8) {   /* hard decisions (:1267-1283), MSB first */
          uint32_t byte = 0;
#pragma unroll
          for (int bb = 0; bb < 8; bb++) byte |= (uint32_t)(B.ext2[pi6[8 * i + bb]] > 0) << (7 - bb);
          dec[g][i] = (uint8_t)byte;
          out[(size_t)cb * out_stride + i] = (uint8_t)byte;
        }
    }
    __syncthreads();
    if (active && it > 1 && q == 0) {            /* CRC early stop (:1304-1351) */
      const uint32_t clen = 3, s0b = crc_type == 0 ? (F >> 3) : 0;
      const uint32_t nbytes = crc_type == 0 ? (K - 24 - F) >> 3 : (K - 24) >> 3;
      uint32_t reg = 0;
      for (uint32_t i = 0; i < nbytes; i++) reg = ((reg << 8) & 0xffffffu) ^ crctab[((reg >> 16) ^ dec[g][s0b + i]) & 0xffu];
      const uint32_t oldcrc = (uint32_t)dec[g][Kb - clen] | ((uint32_t)dec[g][Kb - clen + 1] << 8) |
                              ((uint32_t)dec[g][Kb - clen + 2] << 16);
      const uint32_t crc = ((reg & 0xffu) << 16) | (reg & 0xff00u) | ((reg >> 16) & 0xffu);
      if (crc == oldcrc && crc != 0) done_it[g] = it;
    }
    __syncthreads();
    if (active && done_it[g]) active = false;
    if (active && it < max_it) log_map(B.s1, B.yp1, B.ext, B.A, K, q, 0);
    __syncthreads();
    if (active && it < max_it)
      for (uint32_t v = 0; v < K1; v++) {
        const uint32_t i = 8 * v + q;
        B.ext[i] = sadd(ssub(B.ext[i], B.s1[i]), B.s0[i]);
      }
    __syncthreads();
    if (!__any(active)) break;
  }
  if (valid && q == 0) iters[cb] = (uint8_t)(done_it[g] ? done_it[g] : max_it + 1);
}

hipError_t oai4g_launch_td16(int n_cb, uint32_t K, const int16_t *d_llr, size_t llr_stride, uint8_t *d_out,
                             size_t out_stride, uint8_t *d_iters, uint32_t max_it, uint32_t crc_type, uint32_t F,
                             const uint16_t *d_pi, uint8_t *d_scratch, hipStream_t s)
{
  if (n_cb <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_td16, dim3((n_cb + 7) / 8), dim3(64), 0, s, n_cb, K, d_llr, llr_stride, d_out, out_stride,
                     d_iters, max_it, crc_type, F, d_pi, d_pi + K, d_pi + 2 * K, d_scratch, oai4g_td_block_bytes(K));
  return hipGetLastError();
}

/* ======================================================================================
 * RX rate matching + sub-block deinterleaving for one block, thread per w entry:
 * w[p] = sum of the soft inputs that the circular selection maps to p (int16 wrap, the
 * reference's `w[ind] += soft` in any order), then d = deinterleave(w).
 * ==================================================================================== */
__global__ void __launch_bounds__(256) k_rm_rx(const int16_t *__restrict__ soft, uint32_t E, int16_t *__restrict__ w,
                                               const uint8_t *__restrict__ dummy_w, const uint32_t *__restrict__ cidx,
                                               uint32_t Ncb, uint32_t Nnn, uint32_t k0c, int clear)
{
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= Ncb) return;
  int16_t acc = clear ? (int16_t)0 : w[p];
  if (dummy_w[p] != OAI4G_LTE_NULL) {
    /* compact index of p, then every selection round that lands on it */
    const uint32_t c = cidx[p];
    uint32_t k = c >= k0c ? c - k0c : c + Nnn - k0c;
    for (; k < E; k += Nnn) acc = (int16_t)(acc + soft[k]);
  }
  w[p] = acc;
}

__global__ void __launch_bounds__(256) k_subblock_deint(uint32_t D, int16_t *__restrict__ dfull,
                                                        const int16_t *__restrict__ w)
{
  /* dfull = the reference's d buffer from index 0 (the 96-entry prefix included) */
  const uint32_t R = (D + 31) >> 5, Kpi = R << 5, ND = Kpi - D;
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= Kpi) return;
  const uint32_t col = k / R, row = k - col * R;
  const uint32_t index3 = 3 * (__builtin_bitreverse32(col) >> 27) + 96 * row;
  int16_t *d1 = dfull + 96 - 3 * ND;
  d1[index3] = w[k];
  d1[index3 + 1] = w[Kpi + 2 * k];
  d1[index3 + 5] = w[Kpi + 2 * k + 1];
}

hipError_t oai4g_launch_rm_rx(const int16_t *d_soft, uint32_t E, int16_t *d_w, const uint8_t *d_dummy,
                              const uint32_t *d_cidx, uint32_t Ncb, uint32_t Nnn, uint32_t k0c, int clear, hipStream_t s)
{
  hipLaunchKernelGGL(k_rm_rx, dim3((Ncb + 255) / 256), dim3(256), 0, s, d_soft, E, d_w, d_dummy, d_cidx, Ncb, Nnn,
                     k0c, clear);
  return hipGetLastError();
}

hipError_t oai4g_launch_subblock_deint(uint32_t D, int16_t *d_dfull, const int16_t *d_w, hipStream_t s)
{
  const uint32_t Kpi = ((D + 31) >> 5) << 5;
  hipLaunchKernelGGL(k_subblock_deint, dim3((Kpi + 255) / 256), dim3(256), 0, s, D, d_dfull, d_w);
  return hipGetLastError();
}
