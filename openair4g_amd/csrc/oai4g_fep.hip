/*
 * gfx950 kernels for the UE receive front end:
 *   - the reference's fixed-point forward DFT (PHY/TOOLS/lte_dfts.c dft64 :1766, dft128 :1957,
 *     dft256 :2172, dft512 :2359, dft1024 :2574, dft2048 :2689), reproduced operation for
 *     operation — same DIT decomposition, same packed_cmult2 / cmult twiddle products, same
 *     saturating (bfly4_16, bfly2_16, dft16) and wrapping (bfly4) adds, same shifts — so the
 *     output is bit-identical;
 *   - slot_fep's cyclic-prefix removal (PHY/MODULATION/slot_fep.c:40-177): each OFDM symbol's
 *     DFT window is read straight from the time-domain buffer (circularly, as the reference's
 *     wrap copy makes it) and the frequency-domain symbol is written to rxdataF.
 *
 * Organisation mirrors the inverse transform of oai4g_ofdm.hip: an N-point DFT is owned by a
 * unit of T = N/16 threads; thread t runs the radix-16 leaf over inputs x[t + T n] (the
 * digit-reversed leaves of the reference's even/odd and mod-4 splits) in registers, every
 * higher level exchanges operands through LDS (group-major, one pad word per 32), and the last
 * level stores to global memory.  Forward twiddles live in a table of (a, b) operand pairs:
 * x * W = (dot2(x, a), dot2(x, b)) — a = (Wr, -Wi), b = (Wi, Wr) for cmult and for every
 * packed_cmult2 table except tw256a, whose rounding differs (lte_dfts.c:2162), which is why both
 * halves are stored rather than derived.
 */
#include "oai4g_dft_prims.h"

/* forward radix-4 on saturating int16 (bfly4_tw1 lte_dfts.c:860-889, the dft16 stages
 * :1453-1500, bfly4_16 :965-1006): flip = -j x; y1 = (x0 - x2) + (f1 - f3), y3 = (x0 - x2) - (f1 - f3) */
static __device__ __forceinline__ void r4fwd(s16x2 p0, s16x2 p1, s16x2 p2, s16x2 p3, s16x2 &o0, s16x2 &o1,
                                             s16x2 &o2, s16x2 &o3)
{
  s16x2 s02 = cadds(p0, p2), s13 = cadds(p1, p3);
  o0 = cadds(s02, s13);
  o2 = csubs(s02, s13);
  s16x2 d02 = csubs(p0, p2), d13 = csubs(cflip(p1), cflip(p3));
  o1 = cadds(d02, d13);
  o3 = csubs(d02, d13);
}

/* bfly4 (lte_dfts.c:709-745): cmult products kept in 32 bits, one cpack per output, wrapping
 * add of x0 (the forward twin of ibfly4 with y1 / y3 exchanged) */
static __device__ __forceinline__ void bfly4(s16x2 x0, s16x2 x1, s16x2 x2, s16x2 x3, const twp_t &t1,
                                             const twp_t &t2, const twp_t &t3, s16x2 &y0, s16x2 &y1, s16x2 &y2,
                                             s16x2 &y3)
{
  int a1r, a1i, a2r, a2i, a3r, a3i;
  cmulc32(x1, t1, a1r, a1i);   /* with (a, b) operands cmulc32 is cmult */
  cmulc32(x2, t2, a2r, a2i);
  cmulc32(x3, t3, a3r, a3i);
  y0 = caddw(x0, cpack32(wadd(a1r, wadd(a2r, a3r)), wadd(a1i, wadd(a2i, a3i))));
  y1 = caddw(x0, cpack32(wsub(a1i, wadd(a2r, a3i)), wsub(wsub(a3r, a2i), a1r)));
  y2 = caddw(x0, cpack32(wsub(wsub(a2r, a3r), a1r), wsub(wsub(a2i, a3i), a1i)));
  y3 = caddw(x0, cpack32(wsub(wsub(a3i, a2r), a1i), wsub(a1r, wadd(a2i, a3r))));
}

/* bfly2 (lte_dfts.c:396-419, dft2048): cmult(x0, W0 = 32767) and cmult(x1, tw), >>15, packs */
static __device__ __forceinline__ void bfly2(s16x2 x0, s16x2 x1, const twp_t &t, s16x2 &y0, s16x2 &y1)
{
  int a0r = dot2(x0, (s16x2){32767, 0}), a0i = dot2(x0, (s16x2){0, 32767}), a1r, a1i;
  cmulc32(x1, t, a1r, a1i);
  y0 = cpack32(wadd(a0r, a1r), wadd(a0i, a1i));
  y1 = cpack32(wsub(a0r, a1r), wsub(a0i, a1i));
}

/* bfly2_16 (lte_dfts.c:471-483, dft128 / dft512): packed_cmult2 then saturating add / sub */
static __device__ __forceinline__ void bfly2_16(s16x2 x0, s16x2 x1, const twp_t &t, s16x2 &y0, s16x2 &y1)
{
  const s16x2 p = cmulc16(x1, t);
  y0 = cadds(x0, p);
  y1 = csubs(x0, p);
}

__host__ __device__ constexpr int fwd_distinct(int T, int SC, int J) { return T >= SC ? 1 : (SC / T < J ? SC / T : J); }

/* Per-thread twiddle registers: at a level with quarter size SC a thread's butterfly j (operand
 * b = t + T j) uses index q = b mod SC, of which D = min(J, SC/T) are distinct. */
template <int LOG2N>
struct dft_tw_t {
  static constexpr int N = 1 << LOG2N, T = N >> 4;
  static constexpr bool HAS256 = LOG2N >= 8, HAS1024 = LOG2N >= 10, HASR2 = (LOG2N & 1) != 0;
  static constexpr int D64 = fwd_distinct(T, 16, 4), D256 = fwd_distinct(T, 64, 4),
                       D1024 = fwd_distinct(T, 256, 4), DR2 = fwd_distinct(T, N / 2, 8);
  twp_t l16[7];                         /* W16^{0,1,2,3,4,6,9} (tw16a / tw16b) */
  twp_t l64[D64][3];
  twp_t l256[HAS256 ? D256 : 1][3];
  twp_t l1024[HAS1024 ? D1024 : 1][3];
  twp_t r2[HASR2 ? DR2 : 1];

  static __device__ __forceinline__ twp_t ab(const uint32_t *twf, uint32_t i)
  {
    gu32_t *g = (gu32_t *)twf;
    return {u2c(g[i]), u2c(g[OAI4G_TW_TOTAL + i])};
  }
  __device__ __forceinline__ void load(const uint32_t *twf, int t)
  {
    constexpr int i16[7] = {0, 1, 2, 3, 4, 6, 9};
#pragma unroll
    for (int i = 0; i < 7; i++) l16[i] = ab(twf, oai4g_tw_offset(4) + i16[i]);
#pragma unroll
    for (int j = 0; j < D64; j++)
#pragma unroll
      for (int r = 0; r < 3; r++) l64[j][r] = ab(twf, oai4g_tw_offset(6) + (r + 1) * ((t + T * j) & 15));
    if constexpr (HAS256) {
#pragma unroll
      for (int j = 0; j < D256; j++)
#pragma unroll
        for (int r = 0; r < 3; r++) l256[j][r] = ab(twf, oai4g_tw_offset(8) + (r + 1) * ((t + T * j) & 63));
    }
    if constexpr (HAS1024) {
#pragma unroll
      for (int j = 0; j < D1024; j++)
#pragma unroll
        for (int r = 0; r < 3; r++) l1024[j][r] = ab(twf, oai4g_tw_offset(10) + (r + 1) * ((t + T * j) & 255));
    }
    if constexpr (HASR2) {
#pragma unroll
      for (int j = 0; j < DR2; j++) r2[j] = ab(twf, oai4g_tw_offset(LOG2N) + ((t + T * j) & (N / 2 - 1)));
    }
  }
};

/* leaf dft16 in registers (lte_dfts.c:1431-1500): radix-4 without twiddles, transpose, twiddled
 * radix-4 (packed_cmult2 with tw16a / tw16b, including the lossy W^0 = 32767 products) */
static __device__ __forceinline__ void dft16_reg(s16x2 *x, const twp_t *w16)
{
  constexpr int k1[4] = {0, 1, 2, 3}, k2[4] = {0, 2, 4, 5}, k3[4] = {0, 3, 5, 6}; /* slots of k, 2k, 3k */
  s16x2 S[4][4];
#pragma unroll
  for (int j = 0; j < 4; j++) r4fwd(x[j], x[4 + j], x[8 + j], x[12 + j], S[0][j], S[1][j], S[2][j], S[3][j]);
#pragma unroll
  for (int k = 0; k < 4; k++) {
    s16x2 b1 = cmulc16(S[k][1], w16[k1[k]]);
    s16x2 b2 = cmulc16(S[k][2], w16[k2[k]]);
    s16x2 b3 = cmulc16(S[k][3], w16[k3[k]]);
    r4fwd(S[k][0], b1, b2, b3, x[k], x[4 + k], x[8 + k], x[12 + k]);
  }
}

/* radix-4 butterfly of one level: KIND 0 = bfly4_16 (dft64 / dft256 levels) then >> SH,
 * KIND 1 = bfly4 (dft1024 level) then >> 1 */
template <int KIND, int SH>
static __device__ __forceinline__ void fwd_r4(const s16x2 *v, const twp_t *w, s16x2 *y, bool shift)
{
  if constexpr (KIND == 0) {
    r4fwd(v[0], cmulc16(v[1], w[0]), cmulc16(v[2], w[1]), cmulc16(v[3], w[2]), y[0], y[1], y[2], y[3]);
  } else {
    bfly4(v[0], v[1], v[2], v[3], w[0], w[1], w[2], y[0], y[1], y[2], y[3]);
  }
  if (shift) {
#pragma unroll
    for (int m = 0; m < 4; m++) y[m] = (SH == 3) ? shr3(y[m]) : shr1(y[m]);
  }
}

/* intermediate level of size S = 2^LOG2S held in LDS: read all operands, barrier, write all
 * results, barrier.  Sub-transform r of output group g sits at group g + (N/S) r. */
template <int LOG2N, int LOG2S, int KIND, int D>
static __device__ __forceinline__ void dft_level(uint32_t *la, int t, bool active, const twp_t (&tw)[D][3])
{
  constexpr int N = 1 << LOG2N, T = N >> 4, S = 1 << LOG2S, SC = S >> 2, GOUT = N / S;
  s16x2 v[4][4];
  if (active) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int b = t + T * j, q = b & (SC - 1), g = b >> (LOG2S - 2);
#pragma unroll
      for (int r = 0; r < 4; r++) v[j][r] = u2c(la[lphys((uint32_t)((g + GOUT * r) * SC + q))]);
    }
  }
  __syncthreads();
  if (active) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int b = t + T * j, q = b & (SC - 1), g = b >> (LOG2S - 2);
      s16x2 y[4];
      fwd_r4<KIND, (LOG2S == 6) ? 3 : 1>(v[j], tw[j % D], y, true);
      const uint32_t base = (uint32_t)(g * S + q);
#pragma unroll
      for (int m = 0; m < 4; m++) la[lphys(base + m * SC)] = c2u(y[m]);
    }
  }
  __syncthreads();
}

/* One forward N-point DFT by a unit.  prod(x) fills x[n] = input t + T n; cons(f, y) stores
 * output f.  Every thread of the workgroup must call this (barriers), active or not. */
template <int LOG2N, class Prod, class Cons>
static __device__ __forceinline__ void dft_unit(uint32_t *la, int t, bool active, const dft_tw_t<LOG2N> &tw,
                                                Prod prod, Cons cons, int scale)
{
  constexpr int N = 1 << LOG2N, T = N >> 4;
  using TW = dft_tw_t<LOG2N>;
  if (active) {
    s16x2 x[16];
    prod(x);
    dft16_reg(x, tw.l16);
#pragma unroll
    for (int k = 0; k < 16; k++) la[lphys((uint32_t)(t * 16 + k))] = c2u(x[k]);
  }
  __syncthreads();
  if constexpr (LOG2N > 6) dft_level<LOG2N, 6, 0>(la, t, active, tw.l64);
  if constexpr (LOG2N >= 9) dft_level<LOG2N, 8, 0>(la, t, active, tw.l256);
  if constexpr (LOG2N == 11) dft_level<LOG2N, 10, 1>(la, t, active, tw.l1024);
  if (!active) return;
  if constexpr ((LOG2N & 1) != 0) {
    /* final radix-2 level: bfly2_16 (dft128, dft512) or bfly2 (dft2048), then mulhi(23170) << 1 */
    constexpr int SC = N >> 1;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const int q = t + T * j;
      s16x2 y0, y1;
      const s16x2 x0 = u2c(la[lphys((uint32_t)q)]), x1 = u2c(la[lphys((uint32_t)(SC + q))]);
      if constexpr (LOG2N == 11) bfly2(x0, x1, tw.r2[j % TW::DR2], y0, y1);
      else bfly2_16(x0, x1, tw.r2[j % TW::DR2], y0, y1);
      if (scale) { y0 = mulhi2(y0); y1 = mulhi2(y1); }
      cons(q, y0);
      cons(q + SC, y1);
    }
  } else {
    /* final radix-4 level: dft64 (bfly4_16, >>3), dft256 (bfly4_16, >>1), dft1024 (bfly4, >>1) */
    constexpr int SC = N >> 2;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int q = t + T * j;
      s16x2 v[4], y[4];
#pragma unroll
      for (int r = 0; r < 4; r++) v[r] = u2c(la[lphys((uint32_t)(r * SC + q))]);
      if constexpr (LOG2N == 6) fwd_r4<0, 3>(v, tw.l64[j % TW::D64], y, scale != 0);
      else if constexpr (LOG2N == 8) fwd_r4<0, 1>(v, tw.l256[j % TW::D256], y, scale != 0);
      else fwd_r4<1, 1>(v, tw.l1024[j % TW::D1024], y, scale != 0);
#pragma unroll
      for (int m = 0; m < 4; m++) cons(q + m * SC, y[m]);
    }
  }
}

/* ======================================================================================
 * k_fep: per-symbol CP removal + forward DFT.  Unit s = item * nsym + sym; item = (subframe,
 * antenna) with input base item * in_stride and output base item * out_stride; the DFT window of
 * symbol sym starts at in_off[sym] and wraps at in_len (the reference's circular frame buffer).
 * Persistent 128-thread workgroups (twiddle registers loaded once).
 * ==================================================================================== */
template <int LOG2N>
__global__ void __launch_bounds__(128) k_fep(const int32_t *__restrict__ in, int32_t *__restrict__ out,
                                             fep_args_t a, const uint32_t *__restrict__ twf)
{
  constexpr int N = 1 << LOG2N, T = N >> 4, UNITS = 128 / T, LDSW = N + (N >> 5);
  __shared__ uint32_t lds_all[UNITS * LDSW];
  const int unit = threadIdx.x / T, t = threadIdx.x % T;
  dft_tw_t<LOG2N> twr;
  twr.load(twf, t);
  uint32_t *la = lds_all + unit * LDSW;
  for (int s0 = blockIdx.x * UNITS; s0 < a.n_units; s0 += gridDim.x * UNITS) {
    const int s = s0 + unit;
    const bool active = s < a.n_units;
    const int item = active ? s / a.nsym : 0, sym = active ? s - item * a.nsym : 0;
    gu32_t *src = (gu32_t *)in + (size_t)item * a.in_stride;
    uint32_t *dst = (uint32_t *)out + (size_t)item * a.out_stride + a.out_off[sym];
    const uint32_t off = a.in_off[sym], len = a.in_len;
    dft_unit<LOG2N>(
        la, t, active, twr,
        [&](s16x2 *x) {
#pragma unroll
          for (int n = 0; n < 16; n++) {
            uint32_t i = off + (uint32_t)(t + T * n);
            i = (i >= len) ? i - len : i;
            x[n] = u2c(src[i]);
          }
        },
        [&](int f, s16x2 y) { dst[f] = c2u(y); }, a.scale);
    __syncthreads();   /* the next round's leaf stores reuse la */
  }
}

hipError_t oai4g_launch_fep(const int32_t *d_in, int32_t *d_out, int log2n, const fep_args_t &a,
                            const uint32_t *d_twf, int n_cu, hipStream_t s)
{
  if (a.n_units <= 0) return hipSuccess;
  if (a.nsym <= 0 || a.nsym > OAI4G_FEP_MAX_SYM) return hipErrorInvalidValue;
  const int units = 128 / ((1 << log2n) >> 4);
  const int need = (a.n_units + units - 1) / units, cap = n_cu * 8;
  const dim3 grid(need < cap ? need : cap), blk(128);
  switch (log2n) {
  case 6: hipLaunchKernelGGL(k_fep<6>, grid, blk, 0, s, d_in, d_out, a, d_twf); break;
  case 7: hipLaunchKernelGGL(k_fep<7>, grid, blk, 0, s, d_in, d_out, a, d_twf); break;
  case 8: hipLaunchKernelGGL(k_fep<8>, grid, blk, 0, s, d_in, d_out, a, d_twf); break;
  case 9: hipLaunchKernelGGL(k_fep<9>, grid, blk, 0, s, d_in, d_out, a, d_twf); break;
  case 10: hipLaunchKernelGGL(k_fep<10>, grid, blk, 0, s, d_in, d_out, a, d_twf); break;
  case 11: hipLaunchKernelGGL(k_fep<11>, grid, blk, 0, s, d_in, d_out, a, d_twf); break;
  default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
