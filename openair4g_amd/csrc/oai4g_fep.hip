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

#ifndef OAI4G_FEP_WG_PER_CU
#define OAI4G_FEP_WG_PER_CU 16   /* persistent workgroups per CU (64 VGPRs, 9 KB LDS: 8 waves per SIMD) */
#endif

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
 * dft2048 in three register passes and two LDS exchanges (T = 128): the data movement of
 * idft2048_unit (oai4g_ofdm.hip) with the forward butterflies of lte_dfts.c:2689-2777.
 * Input index n = e + 2 r1 + 8 r2 + 32 r3 + 128 n4, output k = k4 + 16 m3 + 64 m2 + 256 m1 + 1024 m0.
 *   pass A: thread t = (e, r1, r2, r3) runs leaf t (dft16 over n4) -> L_t[k4];
 *   pass B: thread u = j + 8 k4 (j = e + 2 r1) runs the 64-level (bfly4_16 over r3, >>3) and the
 *           256-level (bfly4_16 over r2, >>1) in registers -> out256_j[k2], k2 = k4 + 16 m3 + 64 m2;
 *   pass C: thread v, k2 in {v, v + 128}: the 1024-level (bfly4 over r1, >>1) and the 2048-level
 *           (bfly2 over e, mulhi) and the stores.
 * LDS images as in idft2048_unit (E1: L_t[k4] at k4*144 + 2 (t & 31) + ((t >> 5) & 1) + 64 (t >> 6);
 * E2: out256_j[k2] at 8 k2 + j + 2 (k2 >> 3), aliasing E1).
 * ==================================================================================== */
/* (a, b) from a for every table but tw256a/b: b = (Wi, Wr) = (-a.y, a.x) */
static __device__ __forceinline__ twp_t fwd_ab(s16x2 a) { return {a, (s16x2){(short)(-(int)a.y), a.x}}; }

struct dft2048_tw_t {
  static constexpr int X1W = 16 * 144;
  twp_t l16[7];        /* W16^{0,1,2,3,4,6,9} */
  s16x2 b64[3];        /* a of W64^{r k4}, k4 = t >> 3 */
  twp_t b256[4][3];    /* (a, b) of W256^{r (k4 + 16 m3)}: tw256a rounds on its own */
  s16x2 c1024[2][3];   /* a of W1024^{r k2}, k2 = t + 128 h */
  s16x2 c2048[8];      /* a of W2048^{k1}, k1 = t + 128 (h + 2 m1) */

  __device__ __forceinline__ void load(const uint32_t *twf, int t)
  {
    gu32_t *g = (gu32_t *)twf;
    constexpr int i16[7] = {0, 1, 2, 3, 4, 6, 9};
#pragma unroll
    for (int i = 0; i < 7; i++) l16[i] = dft_tw_t<11>::ab(twf, oai4g_tw_offset(4) + i16[i]);
    const int k4 = t >> 3;
#pragma unroll
    for (int r = 0; r < 3; r++) b64[r] = u2c(g[oai4g_tw_offset(6) + (r + 1) * k4]);
#pragma unroll
    for (int m3 = 0; m3 < 4; m3++)
#pragma unroll
      for (int r = 0; r < 3; r++) b256[m3][r] = dft_tw_t<11>::ab(twf, oai4g_tw_offset(8) + (r + 1) * (k4 + 16 * m3));
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
      for (int r = 0; r < 3; r++) c1024[h][r] = u2c(g[oai4g_tw_offset(10) + (r + 1) * (t + 128 * h)]);
#pragma unroll
    for (int i = 0; i < 8; i++) c2048[i] = u2c(g[oai4g_tw_offset(11) + t + 128 * i]);
  }
};

typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));

template <class Prod, class Cons>
static __device__ __forceinline__ void dft2048_unit(uint32_t *lds, int t, bool active, const dft2048_tw_t &tw,
                                                    Prod prod, Cons cons, int scale)
{
  s16x2 x[16];
  /* pass A: leaves */
  if (active) {
    prod(x);
    dft16_reg(x, tw.l16);
    const uint32_t wo = 2u * (t & 31) + ((t >> 5) & 1) + 64u * (t >> 6);
#pragma unroll
    for (int k = 0; k < 16; k++) lds[k * 144 + wo] = c2u(x[k]);
  }
  __syncthreads();
  /* pass B: 64- and 256-levels of the 256-point transform j = t & 7 at k4 = t >> 3 */
  const int j = t & 7, k4 = t >> 3;
  if (active) {
    const uint32_t ro = (uint32_t)k4 * 144u + 2u * j;
#pragma unroll
    for (int r2 = 0; r2 < 4; r2++)
#pragma unroll
      for (int p = 0; p < 2; p++) {
        const u32x2_t v = *(const u32x2_t *)&lds[ro + 16 * r2 + 64 * p];
        x[4 * r2 + 2 * p] = u2c(v.x);
        x[4 * r2 + 2 * p + 1] = u2c(v.y);
      }
  }
  __syncthreads();   /* E2 aliases E1 */
  if (active) {
    const twp_t w64[3] = {fwd_ab(tw.b64[0]), fwd_ab(tw.b64[1]), fwd_ab(tw.b64[2])};
    s16x2 o[4][4];   /* [r2][m3] */
#pragma unroll
    for (int r2 = 0; r2 < 4; r2++) fwd_r4<0, 3>(&x[4 * r2], w64, o[r2], true);
#pragma unroll
    for (int m3 = 0; m3 < 4; m3++) {
      const s16x2 v[4] = {o[0][m3], o[1][m3], o[2][m3], o[3][m3]};
      s16x2 y[4];
      fwd_r4<0, 1>(v, tw.b256[m3], y, true);
#pragma unroll
      for (int m2 = 0; m2 < 4; m2++) {
        const uint32_t k2 = (uint32_t)k4 + 16u * m3 + 64u * m2;
        lds[8u * k2 + j + 2u * (k2 >> 3)] = c2u(y[m2]);
      }
    }
  }
  __syncthreads();
  /* pass C: 1024- and 2048-levels for k2 = t + 128 h */
  if (active) {
    s16x2 v[2][8];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t k2 = (uint32_t)t + 128u * h;
      const uint32_t ro = 8u * k2 + 2u * (k2 >> 3);
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const u32x2_t q = *(const u32x2_t *)&lds[ro + 2 * i];
        v[h][2 * i] = u2c(q.x);
        v[h][2 * i + 1] = u2c(q.y);
      }
    }
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const twp_t w[3] = {fwd_ab(tw.c1024[h][0]), fwd_ab(tw.c1024[h][1]), fwd_ab(tw.c1024[h][2])};
      s16x2 o[2][4];   /* [e][m1] */
#pragma unroll
      for (int e = 0; e < 2; e++) {
        const s16x2 in[4] = {v[h][e], v[h][e + 2], v[h][e + 4], v[h][e + 6]};
        fwd_r4<1, 1>(in, w, o[e], true);
      }
#pragma unroll
      for (int m1 = 0; m1 < 4; m1++) {
        s16x2 y0, y1;
        bfly2(o[0][m1], o[1][m1], fwd_ab(tw.c2048[h + 2 * m1]), y0, y1);
        if (scale) { y0 = mulhi2(y0); y1 = mulhi2(y1); }
        cons(t + 128 * h + 256 * m1, y0);
        cons(t + 128 * h + 256 * m1 + 1024, y1);
      }
    }
  }
}

template <int LOG2N>
struct dft_sel {
  using tw_t = dft_tw_t<LOG2N>;
  static constexpr int XW = (1 << LOG2N) + ((1 << LOG2N) >> 5);
};
template <>
struct dft_sel<11> {
  using tw_t = dft2048_tw_t;
  static constexpr int XW = dft2048_tw_t::X1W;
};

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
  constexpr int N = 1 << LOG2N, T = N >> 4, UNITS = 128 / T, LDSW = dft_sel<LOG2N>::XW;
  __shared__ uint32_t lds_all[UNITS * LDSW];
  const int unit = threadIdx.x / T, t = threadIdx.x % T;
  typename dft_sel<LOG2N>::tw_t twr;
  twr.load(twf, t);
  uint32_t *la = lds_all + unit * LDSW;
  for (int s0 = blockIdx.x * UNITS; s0 < a.n_units; s0 += gridDim.x * UNITS) {
    const int s = s0 + unit;
    const bool active = s < a.n_units;
    const int item = active ? s / a.nsym : 0, sym = active ? s - item * a.nsym : 0;
    gu32_t *src = (gu32_t *)in + (size_t)item * a.in_stride;
    uint32_t *dst = (uint32_t *)out + (size_t)item * a.out_stride + a.out_off[sym];
    const uint32_t off = a.in_off[sym], len = a.in_len;
    auto prod = [&](s16x2 *x) {
#pragma unroll
      for (int n = 0; n < 16; n++) {
        uint32_t i = off + (uint32_t)(t + T * n);
        i = (i >= len) ? i - len : i;
        x[n] = u2c(src[i]);
      }
    };
    auto cons = [&](int f, s16x2 y) { dst[f] = c2u(y); };
    if constexpr (LOG2N == 11) dft2048_unit(la, t, active, twr, prod, cons, a.scale);
    else dft_unit<LOG2N>(la, t, active, twr, prod, cons, a.scale);
    __syncthreads();   /* the next round's leaf stores reuse la */
  }
}

hipError_t oai4g_launch_fep(const int32_t *d_in, int32_t *d_out, int log2n, const fep_args_t &a,
                            const uint32_t *d_twf, int n_cu, hipStream_t s)
{
  if (a.n_units <= 0) return hipSuccess;
  if (a.nsym <= 0 || a.nsym > OAI4G_FEP_MAX_SYM) return hipErrorInvalidValue;
  const int units = 128 / ((1 << log2n) >> 4);
  const int need = (a.n_units + units - 1) / units, cap = n_cu * OAI4G_FEP_WG_PER_CU;
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
