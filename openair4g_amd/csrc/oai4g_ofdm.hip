/*
 * gfx950 kernels for the frequency-domain half of the PDSCH transmit path:
 *   - the reference's fixed-point inverse DFT (PHY/TOOLS/lte_dfts.c idft64..idft2048),
 *     reproduced operation-for-operation (same decomposition, same Q15 twiddles, same
 *     saturating / wrapping adds, same shifts) so the output is bit-identical;
 *   - cyclic-prefix insertion (PHY/MODULATION/ofdm_mod.c:85-171);
 *   - QAM mapping + RE mapping + TM1/TM3 precoding (dlsch_modulation.c:139-1493) fused in
 *     front of the IDFT so the frequency grid never round-trips through HBM.
 *
 * IDFT organisation.  An N-point transform is owned by a "unit" of T = N/16 threads.  Thread t
 * owns the radix-16 leaf that consumes inputs x[t + T n], n = 0..15 (the digit-reversed DIT
 * leaves of the reference's recursive even/odd and mod-4 splits).  The leaf IDFT16 runs in
 * registers; each higher level (64: radix-4 with saturating Q15 products; 256/1024: radix-4
 * with 32-bit accumulation; 128/2048: radix-2) exchanges operands through LDS, stored
 * group-major (pos = group*S + q) with one pad word per 32 to spread LDS banks.  The last level
 * writes straight to global memory, producing the CP in the same pass.
 *
 * The arithmetic is VALU-issue bound, so every step is shaped for instruction count:
 * complex products are two v_dot2_i32_i16 (the reference's madd_epi16), the >>15 + packs_epi32
 * pair is two shifts + one saturating v_cvt_pk_i16_i32, radix adds are packed saturating
 * v_pk_add/sub_i16, and the twiddles a thread needs (a thread's twiddle indices are fixed per
 * level) live in registers for the lifetime of a persistent workgroup.  In the fused kernel a
 * unit transforms every antenna of one (subframe, symbol), so QAM mapping and the e-bit reads
 * are shared between antennas.
 */
#include "oai4g_internal.h"

#include "oai4g_dft_prims.h"

/* ---------------------------------------------------------------------------------------
 * Per-thread twiddle registers.  At a level with quarter size SC a thread's butterfly j
 * (operand b = t + T j) uses index q = b mod SC; only D = min(J, SC/T) of them are distinct.
 * ------------------------------------------------------------------------------------- */
__host__ __device__ constexpr int tw_distinct(int T, int SC, int J) { return T >= SC ? 1 : (SC / T < J ? SC / T : J); }

template <int LOG2N>
struct idft_tw_t {
  static constexpr int N = 1 << LOG2N, T = N >> 4;
  /* final level: radix-2 for odd sizes (idft128/512/2048), radix-4 for idft256/1024 */
  static constexpr bool HAS256 = LOG2N >= 8, HAS1024 = LOG2N >= 10, HASR2 = (LOG2N & 1) != 0;
  static constexpr int D64 = tw_distinct(T, 16, 4), D256 = tw_distinct(T, 64, 4), D1024 = tw_distinct(T, 256, 4),
                       DR2 = tw_distinct(T, N / 2, 8);
  twp_t l16[7];                         /* W16^{0,1,2,3,4,6,9}: wave-uniform (scalar loads) */
  s16x2 l64[D64][3];                    /* per-thread twiddles; companions rebuilt at use */
  s16x2 l256[HAS256 ? D256 : 1][3];
  s16x2 l1024[HAS1024 ? D1024 : 1][3];
  s16x2 r2[HASR2 ? DR2 : 1];

  __device__ __forceinline__ void load(const uint32_t *tw, int t)
  {
    gu32_t *g = (gu32_t *)tw;
    constexpr int i16[7] = {0, 1, 2, 3, 4, 6, 9};
#pragma unroll
    for (int i = 0; i < 7; i++)
      l16[i] = {u2c(g[oai4g_tw_offset(4) + i16[i]]), u2c(g[OAI4G_TW_TOTAL + oai4g_tw_offset(4) + i16[i]])};
#pragma unroll
    for (int j = 0; j < D64; j++) {
      int q = (t + T * j) & 15;
#pragma unroll
      for (int r = 0; r < 3; r++) l64[j][r] = u2c(g[oai4g_tw_offset(6) + (r + 1) * q]);
    }
    if constexpr (HAS256) {
#pragma unroll
      for (int j = 0; j < D256; j++) {
        int q = (t + T * j) & 63;
#pragma unroll
        for (int r = 0; r < 3; r++) l256[j][r] = u2c(g[oai4g_tw_offset(8) + (r + 1) * q]);
      }
    }
    if constexpr (HAS1024) {
#pragma unroll
      for (int j = 0; j < D1024; j++) {
        int q = (t + T * j) & 255;
#pragma unroll
        for (int r = 0; r < 3; r++) l1024[j][r] = u2c(g[oai4g_tw_offset(10) + (r + 1) * q]);
      }
    }
    if constexpr (HASR2) {
#pragma unroll
      for (int j = 0; j < DR2; j++) r2[j] = u2c(g[oai4g_tw_offset(LOG2N) + ((t + T * j) & (N / 2 - 1))]);
    }
  }
};

static __device__ __forceinline__ twp_t tw_of(s16x2 t) { return {t, (s16x2){(short)(-(int)t.y), t.x}}; }
/* The same pair with the companion rebuilt by one v_pk_mul_lo_u16 (lo = t.hi * -1, hi = t.lo * 1,
 * wrapping like (short)-t.y).  `dep` is any per-item value: it is an operand of the asm, so the
 * companion cannot be hoisted out of a persistent item loop, where the compiler would otherwise
 * keep a second register per twiddle for the whole kernel (29 VGPRs at 2048 points). */
static __device__ __forceinline__ twp_t tw_use(s16x2 t, uint32_t dep)
{
  uint32_t tn;
  asm("v_pk_mul_lo_u16 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1] ; %3" : "=v"(tn) : "v"(t), "s"(0x0001FFFFu), "s"(dep));
  return {t, u2c(tn)};
}

#ifndef OAI4G_MOD_W0
#define OAI4G_MOD_W0 1   /* NS leaf: the W^0 products as x - (x > 0) (0: the dot2 form) */
#endif
/* x * conj(W^0) with W^0 = (32767, 0), packed like cmulc16: each lane floor(32767 x / 2^15), which is
 * x - 1 for x > 0 and x for x <= 0 when |x| < 2^15 (NS: no leaf value is -32768).  The lane's x > 0 is
 * the sign bit of -x; the 32-bit subtraction of the two 0/1 flags cannot borrow across lanes (the low
 * flag is 1 only where the low lane is >= 1).  One packed op and three fast ones instead of two dot2,
 * two shifts and a cvt_pk. */
static __device__ __forceinline__ s16x2 w0mul_ns(s16x2 x)
{
  uint32_t n;
  asm("v_pk_sub_u16 %0, 0, %1" : "=v"(n) : "v"(x));
  return u2c(c2u(x) - ((n >> 15) & 0x00010001u));
}

/* leaf IDFT16 in registers (lte_dfts.c:1597-1724); w16 is wave-uniform (scalar loads) */
template <bool FF = false, bool NS = false>
static __device__ __forceinline__ void idft16_reg(s16x2 *x, const twp_t *w16 /* W^{0,1,2,3,4,6,9} */)
{
  constexpr int k1[4] = {0, 1, 2, 3}, k2[4] = {0, 2, 4, 5}, k3[4] = {0, 3, 5, 6}; /* slots of k, 2k, 3k */
  s16x2 S[4][4];
#pragma unroll
  for (int j = 0; j < 4; j++) r4inv<FF, NS>(x[j], x[4 + j], x[8 + j], x[12 + j], S[0][j], S[1][j], S[2][j], S[3][j]);
#pragma unroll
  for (int k = 0; k < 4; k++) {
    /* NS: row 0 multiplies by W^0 = (32767, 0) (companion (0, 32767)), lane by lane floor(32767 x / 2^15)
     * = x - (x > 0) for |x| < 2^15 (w0mul_ns) */
    const bool w0 = NS && OAI4G_MOD_W0 && k == 0;
    s16x2 b1 = w0 ? w0mul_ns(S[k][1]) : cmulc16u(S[k][1], w16[k1[k]]);
    s16x2 b2 = w0 ? w0mul_ns(S[k][2]) : cmulc16u(S[k][2], w16[k2[k]]);
    s16x2 b3 = w0 ? w0mul_ns(S[k][3]) : cmulc16u(S[k][3], w16[k3[k]]);
    r4inv<FF, NS>(S[k][0], b1, b2, b3, x[k], x[4 + k], x[8 + k], x[12 + k]);
  }
}

/*
 * One intermediate combining level of size S = 2^LOG2S over NA transforms of N = 2^LOG2N held
 * in LDS (group-major, NA buffers of LDSW words).  KIND: 0 = ibfly4_16 (64-level) then >>3,
 * 1 = ibfly4 then >>1.  Reads all operands, barrier, writes all results, barrier.
 */
template <int LOG2N, int LOG2S, int KIND, int D>
static __device__ __forceinline__ void idft_level_one(uint32_t *la, int t, const s16x2 (&tw)[D][3])
{
  constexpr int N = 1 << LOG2N, T = N >> 4, S = 1 << LOG2S, SC = S >> 2, GOUT = N / S;
  s16x2 v[4][4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int b = t + T * j, q = b & (SC - 1), g = b >> (LOG2S - 2);
#pragma unroll
    for (int r = 0; r < 4; r++) v[j][r] = u2c(la[lphys((uint32_t)((g + GOUT * r) * SC + q))]);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int b = t + T * j, q = b & (SC - 1), g = b >> (LOG2S - 2);
    const twp_t w[3] = {tw_of(tw[j % D][0]), tw_of(tw[j % D][1]), tw_of(tw[j % D][2])};
    const uint32_t base = (uint32_t)(g * S + q);
    s16x2 y0, y1, y2, y3;
    if (KIND == 0) {
      r4inv(v[j][0], cmulc16(v[j][1], w[0]), cmulc16(v[j][2], w[1]), cmulc16(v[j][3], w[2]), y0, y1, y2, y3);
      y0 = shr3(y0); y1 = shr3(y1); y2 = shr3(y2); y3 = shr3(y3);
    } else {
      ibfly4(v[j][0], v[j][1], v[j][2], v[j][3], w[0], w[1], w[2], y0, y1, y2, y3);
      y0 = shr1(y0); y1 = shr1(y1); y2 = shr1(y2); y3 = shr1(y3);
    }
    la[lphys(base)] = c2u(y0);
    la[lphys(base + SC)] = c2u(y1);
    la[lphys(base + 2 * SC)] = c2u(y2);
    la[lphys(base + 3 * SC)] = c2u(y3);
  }
  __syncthreads();
}

/*
 * One intermediate combining level of size S = 2^LOG2S over NA transforms of N = 2^LOG2N held
 * in LDS (group-major, NA buffers of LDSW words).  KIND: 0 = ibfly4_16 (64-level) then >>3,
 * 1 = ibfly4 then >>1.  Per transform: read all operands, barrier, write all results, barrier
 * (transforms in turn: 16 staged operands per thread instead of 16 NA).
 */
template <int LOG2N, int LOG2S, int KIND, int NA, int D>
static __device__ __forceinline__ void idft_level_lds(uint32_t *lds, int t, const s16x2 (&tw)[D][3])
{
  constexpr int N = 1 << LOG2N, LDSW = N + (N >> 5);
#pragma unroll
  for (int a = 0; a < NA; a++) idft_level_one<LOG2N, LOG2S, KIND, D>(lds + a * LDSW, t, tw);
}

/*
 * NA transforms by one unit.  `prod(n, x)` fills x[a] = input a at t + T n; `cons(a, t, off, y)`
 * stores output sample f = t + off of transform a (off is a compile-time constant after
 * unrolling, so stores can use immediate offsets from a per-thread base).  Every thread of the workgroup must call this (it
 * contains barriers), active or not.
 */
template <int LOG2N, int NA, class Prod, class Cons>
static __device__ __forceinline__ void idft_unit(uint32_t *lds, int t, bool active, const idft_tw_t<LOG2N> &tw,
                                                 Prod prod, Cons cons, int scale)
{
  constexpr int N = 1 << LOG2N, T = N >> 4, LDSW = N + (N >> 5);
  if (active) {
    s16x2 x[NA][16];
    prod(x);   /* fills x[a][n] = input point t + T n of antenna a: one call, so loads batch */
#pragma unroll
    for (int a = 0; a < NA; a++) {
      idft16_reg(x[a], tw.l16);
#pragma unroll
      for (int k = 0; k < 16; k++) lds[a * LDSW + lphys((uint32_t)(t * 16 + k))] = c2u(x[a][k]);
    }
  }
  __syncthreads();
  if constexpr (LOG2N == 6) {
    /* top-level idft64: ibfly4_16 straight to output, >>3 if scale */
    s16x2 v[NA][4][4];
    if (active) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        int q = t + T * j;
#pragma unroll
        for (int a = 0; a < NA; a++)
#pragma unroll
          for (int r = 0; r < 4; r++) v[a][j][r] = u2c(lds[a * LDSW + lphys((uint32_t)(r * 16 + q))]);
      }
    }
    __syncthreads();
    if (active) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const s16x2 *wt = tw.l64[j % idft_tw_t<6>::D64];
        const twp_t w[3] = {tw_of(wt[0]), tw_of(wt[1]), tw_of(wt[2])};
#pragma unroll
        for (int a = 0; a < NA; a++) {
          s16x2 y[4];
          r4inv(v[a][j][0], cmulc16(v[a][j][1], w[0]), cmulc16(v[a][j][2], w[1]), cmulc16(v[a][j][3], w[2]), y[0],
                y[1], y[2], y[3]);
#pragma unroll
          for (int m = 0; m < 4; m++) cons(a, t, T * j + 16 * m, scale ? shr3(y[m]) : y[m]);
        }
      }
    }
  } else {
    idft_level_lds<LOG2N, 6, 0, NA>(lds, t, tw.l64);
    if constexpr (LOG2N >= 9) idft_level_lds<LOG2N, 8, 1, NA>(lds, t, tw.l256);
    if constexpr (LOG2N == 11) idft_level_lds<LOG2N, 10, 1, NA>(lds, t, tw.l1024);
    if constexpr ((LOG2N & 1) != 0) {
      /* final radix-2 level (idft128 / idft512 / idft2048, lte_dfts.c:2058, 2479, 2779): ibfly2 then
       * mulhi scaling */
      constexpr int SC = N >> 1, DR2 = idft_tw_t<LOG2N>::DR2;
      if (active) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
          int q = t + T * j;
#pragma unroll
          for (int a = 0; a < NA; a++) {
            s16x2 y0, y1;
            ibfly2(u2c(lds[a * LDSW + lphys((uint32_t)q)]), u2c(lds[a * LDSW + lphys((uint32_t)(SC + q))]),
                   tw_of(tw.r2[j % DR2]), y0, y1);
            if (scale) { y0 = mulhi2(y0); y1 = mulhi2(y1); }
            cons(a, t, T * j, y0);
            cons(a, t, T * j + SC, y1);
          }
        }
      }
    } else {
      /* final radix-4 level (idft256 / idft1024): ibfly4 then >>1 */
      constexpr int SC = N >> 2;
      if (active) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
          int q = t + T * j;
          const s16x2 *wt = (LOG2N == 8) ? tw.l256[j % idft_tw_t<LOG2N>::D256] : tw.l1024[j % idft_tw_t<LOG2N>::D1024];
          const twp_t w[3] = {tw_of(wt[0]), tw_of(wt[1]), tw_of(wt[2])};
#pragma unroll
          for (int a = 0; a < NA; a++) {
            s16x2 y[4];
            ibfly4(u2c(lds[a * LDSW + lphys((uint32_t)q)]), u2c(lds[a * LDSW + lphys((uint32_t)(SC + q))]),
                   u2c(lds[a * LDSW + lphys((uint32_t)(2 * SC + q))]),
                   u2c(lds[a * LDSW + lphys((uint32_t)(3 * SC + q))]), w[0], w[1], w[2], y[0], y[1], y[2], y[3]);
#pragma unroll
            for (int m = 0; m < 4; m++) cons(a, t, T * j + SC * m, scale ? shr1(y[m]) : y[m]);
          }
        }
      }
    }
  }
}

/* ======================================================================================
 * idft2048 in three register passes and two LDS exchanges (T = 128 threads, NA transforms).
 *
 * Input index n = e + 2 r1 + 8 r2 + 32 r3 + 128 n4 (the reference's even/odd split, then three
 * mod-4 splits, then the idft16 leaf), output index k = k4 + 16 m3 + 64 m2 + 256 m1 + 1024 m0.
 *   pass A: thread t = (e, r1, r2, r3) runs leaf t (idft16 over n4) -> L_t[k4];
 *   pass B: thread u = j + 8 k4 (j = e + 2 r1) holds L_(j, r2, r3)[k4] for all 16 (r2, r3) and
 *           runs both the 64-level (ibfly4_16 over r3, >>3) and the 256-level (ibfly4 over r2,
 *           >>1) in registers -> out256_j[k2], k2 = k4 + 16 m3 + 64 m2;
 *   pass C: thread v holds out256_j[k2] for all 8 j and k2 in {v, v + 128}, runs the 1024-level
 *           (ibfly4 over r1, >>1) and the 2048-level (ibfly2 over e, mulhi) and stores.
 * Every butterfly, twiddle, shift and saturation is the reference's (lte_dfts.c:2779-2866 ->
 * :2630-2687 -> :2284-2357 -> :1856-1946 -> :1597-1724); only the data movement differs from
 * the level-by-level schedule of idft_unit (4 exchanges, 9 barriers per symbol there; 2
 * exchanges, 3 barriers here).
 * LDS images (one region of X1W words per transform, the second aliasing the first):
 *   E1: L_t[k4] at k4*144 + 2 (t & 31) + ((t >> 5) & 1) + 64 (t >> 6)  — pass-A b32 stores 2-way
 *       (free), pass-B ds_read_b64 of the (r3, r3 + 1) pair conflict-free;
 *   E2: out256_j[k2] at 264 j + k2 — pass-B b32 stores conflict-free (264 = 8 mod 64), pass-C
 *       ds_read_b64 of the (k2, k2 + 1) pair conflict-free; pass C takes k2 = 2 t + h, so each
 *       output pair (2 t, 2 t + 1) leaves as one 8-byte store.
 * ==================================================================================== */
struct idft2048_tw_t {
  static constexpr int X1W = 16 * 144;
  twp_t l16[7];        /* W16^{0,1,2,3,4,6,9} (wave-uniform) */
  s16x2 b64[3];        /* W64^{r k4}, r = 1..3, k4 = t >> 3 */
  s16x2 b256[4][3];    /* W256^{r (k4 + 16 m3)} */
  s16x2 c1024[2][3];   /* W1024^{r k2}, k2 = 2 t + h */
  s16x2 c2048[8];      /* W2048^{k1}, k1 = 2 t + h + 256 m1 at [h + 2 m1] */
  static constexpr int E2S = 264;   /* E2 words per 256-point transform j */

  __device__ __forceinline__ void load(const uint32_t *tw, int t)
  {
    gu32_t *g = (gu32_t *)tw;
    constexpr int i16[7] = {0, 1, 2, 3, 4, 6, 9};
#pragma unroll
    for (int i = 0; i < 7; i++)
      l16[i] = {u2c(g[oai4g_tw_offset(4) + i16[i]]), u2c(g[OAI4G_TW_TOTAL + oai4g_tw_offset(4) + i16[i]])};
    const int k4 = t >> 3;
#pragma unroll
    for (int r = 0; r < 3; r++) b64[r] = u2c(g[oai4g_tw_offset(6) + (r + 1) * k4]);
#pragma unroll
    for (int m3 = 0; m3 < 4; m3++)
#pragma unroll
      for (int r = 0; r < 3; r++) b256[m3][r] = u2c(g[oai4g_tw_offset(8) + (r + 1) * (k4 + 16 * m3)]);
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
      for (int r = 0; r < 3; r++) c1024[h][r] = u2c(g[oai4g_tw_offset(10) + (r + 1) * (2 * t + h)]);
#pragma unroll
    for (int i = 0; i < 8; i++) c2048[i] = u2c(g[oai4g_tw_offset(11) + 2 * t + (i & 1) + 256 * (i >> 1)]);
  }
};

typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));

#ifndef OAI4G_DIAG_NOSYNC
#define OAI4G_DIAG_NOSYNC 0   /* timing diagnostic only: 1 = the idft2048 exchanges skip their barriers (wrong output) */
#endif
#if OAI4G_DIAG_NOSYNC
#define IDFT_SYNC() do { } while (0)
#else
#define IDFT_SYNC() __syncthreads()
#endif

/* PSYNC: the producer reads LDS that the exchange aliases (k_modofdm's staged QAM addresses), so
 * the leaf stores wait for every thread's producer */
/* NS: the caller's configuration passed the range check (oai4g_host.cpp mod_nosat_ok: no value of the
 * leaf, 64-, 256-, 1024- or 2048-level leaves int16), so the 256- and 1024-levels take the fused form
 * (ibfly4_shr1_ns), the radix-4 adds rotate once (r4inv NS) and the 2048-level's scale multiplies
 * the unpacked sums (ibfly2_mulhi_ns) */
template <int NA, bool PSYNC, bool NS, class Prod, class Cons2>
static __device__ __forceinline__ void idft2048_unit(uint32_t *lds, int t, bool active, const idft2048_tw_t &tw,
                                                     Prod prod, Cons2 cons2, int scale, uint32_t dep)
{
  constexpr int X1W = idft2048_tw_t::X1W, E2S = idft2048_tw_t::E2S;
  static_assert(7 * E2S + 256 <= X1W, "E2 must fit the exchange");
#ifndef OAI4G_DIAG_MODCUT
#define OAI4G_DIAG_MODCUT 0   /* timing diagnostic only (wrong output): the unit stops after phase 1 = prologue
                                 (QAM / RE map / precoding), 2 = leaf IDFT16, 3 = pass A + B (the 64- and 256-levels
                                 and the E2 stores), 4 = pass C without its IQ stores; the cut values are kept
                                 alive by empty asm operands (no instruction), so the earlier phases still run */
#endif
  auto sink = [&](const s16x2 (&v)[16]) {
#pragma unroll
    for (int k = 0; k < 16; k++) asm volatile("" ::"v"(c2u(v[k])));
  };
  s16x2 x[NA][16];
  /* pass A: leaves */
  if (active) {
    prod(x);
#ifndef OAI4G_MOD_PRIO
/* wave priority 2 from the item's start to a point of the transform, 0 after it: the arbiter issues
 * the latency-bound staging / RE lookups (LDS round trips, little VALU) and the passes that follow
 * ahead of the other waves' pass-C VALU streams (profiles/mod_prio_r06.txt).  Lowered: 1 after the RE
 * lookups (-1.2 %), 5 after the radix-16 leaf (-2.5 %), 6 after the pass-B loads, 7 at pass C, 9 after
 * the first pass-C loads (kept: -4 %), 4 after the staging barrier (slower); 8 = 7 with the leaf and
 * pass B at 1; 2: 1 + the pass-B / pass-C loads at 1; 3: 1 at priority 3 */
#define OAI4G_MOD_PRIO 9
#endif
    if constexpr (OAI4G_MOD_PRIO >= 1 && OAI4G_MOD_PRIO <= 3) __builtin_amdgcn_s_setprio(0);
    if constexpr (OAI4G_MOD_PRIO == 8) __builtin_amdgcn_s_setprio(1);
    if constexpr (OAI4G_DIAG_MODCUT == 1) {
#pragma unroll
      for (int a = 0; a < NA; a++) sink(x[a]);
      return;
    }
    if constexpr (PSYNC)
#pragma unroll
      for (int a = 0; a < NA; a++) idft16_reg<NA == 2, NS>(x[a], tw.l16);
    if constexpr (OAI4G_MOD_PRIO == 5) __builtin_amdgcn_s_setprio(0);
    if constexpr (OAI4G_DIAG_MODCUT == 2) {
#pragma unroll
      for (int a = 0; a < NA; a++) sink(x[a]);
      return;
    }
  }
  if constexpr (OAI4G_DIAG_MODCUT == 1 || OAI4G_DIAG_MODCUT == 2) return;
  if constexpr (PSYNC) IDFT_SYNC();
  if (active) {
#ifndef OAI4G_DIAG_PASSA
#define OAI4G_DIAG_PASSA 0   /* timing diagnostic only: 1 = pass-A stores at bank-distinct (wrong) words */
#endif
    const uint32_t wo = OAI4G_DIAG_PASSA ? (uint32_t)t : 2u * (t & 31) + ((t >> 5) & 1) + 64u * (t >> 6);
#pragma unroll
    for (int a = 0; a < NA; a++) {
      if constexpr (!PSYNC) idft16_reg<NA == 2, NS>(x[a], tw.l16);
#pragma unroll
      for (int k = 0; k < 16; k++) lds[a * X1W + k * 144 + wo] = c2u(x[a][k]);
    }
  }
  IDFT_SYNC();
  /* pass B: 64- and 256-levels of the 256-point transform j = t & 7 at k4 = t >> 3 */
  const int j = t & 7, k4 = t >> 3;
  if constexpr (OAI4G_MOD_PRIO == 2) __builtin_amdgcn_s_setprio(1);
  if (active) {
    const uint32_t ro = (uint32_t)k4 * 144u + 2u * j;
#pragma unroll
    for (int a = 0; a < NA; a++)
#pragma unroll
      for (int r2 = 0; r2 < 4; r2++)
#pragma unroll
        for (int p = 0; p < 2; p++) {
          const u32x2_t v = *(const u32x2_t *)&lds[a * X1W + ro + 16 * r2 + 64 * p];
          x[a][4 * r2 + 2 * p] = u2c(v.x);
          x[a][4 * r2 + 2 * p + 1] = u2c(v.y);
        }
  }
  IDFT_SYNC();   /* E2 aliases E1 */
  if constexpr (OAI4G_MOD_PRIO == 2 || OAI4G_MOD_PRIO == 6) __builtin_amdgcn_s_setprio(0);
  if (active) {
    /* E2 word of out256_j[k2] = E2S j + k2, k2 = k4 + 16 m3 + 64 m2: an affine base plus immediates */
    const uint32_t wb = (uint32_t)E2S * j + k4;
    const twp_t w64[3] = {tw_use(tw.b64[0], dep), tw_use(tw.b64[1], dep), tw_use(tw.b64[2], dep)};
#pragma unroll
    for (int a = 0; a < NA; a++) {
      s16x2 o[4][4];   /* [r2][m3] */
#pragma unroll
      for (int r2 = 0; r2 < 4; r2++) {
        const s16x2 *v = &x[a][4 * r2];
        r4inv<NA == 2, NS>(v[0], cmulc16(v[1], w64[0]), cmulc16(v[2], w64[1]), cmulc16(v[3], w64[2]), o[r2][0], o[r2][1],
              o[r2][2], o[r2][3]);
#pragma unroll
        for (int m = 0; m < 4; m++) o[r2][m] = shr3(o[r2][m]);
      }
#pragma unroll
      for (int m3 = 0; m3 < 4; m3++) {
        /* the 12 companions of this level stay in registers (used once per antenna): 124 VGPRs at
         * 4 waves/SIMD; the other levels' are rebuilt at use */
        const twp_t w[3] = {tw_of(tw.b256[m3][0]), tw_of(tw.b256[m3][1]), tw_of(tw.b256[m3][2])};
        s16x2 y[4];
        if constexpr (NS) {
          ibfly4_shr1_ns(o[0][m3], o[1][m3], o[2][m3], o[3][m3], w[0], w[1], w[2], y[0], y[1], y[2], y[3]);
        } else {
          ibfly4(o[0][m3], o[1][m3], o[2][m3], o[3][m3], w[0], w[1], w[2], y[0], y[1], y[2], y[3]);
#pragma unroll
          for (int m2 = 0; m2 < 4; m2++) y[m2] = shr1(y[m2]);
        }
#pragma unroll
        for (int m2 = 0; m2 < 4; m2++) lds[a * X1W + wb + 16u * m3 + 64u * m2] = c2u(y[m2]);
      }
    }
  }
  IDFT_SYNC();
  if constexpr (OAI4G_DIAG_MODCUT == 3) return;   /* the E2 stores are the cut point's live values */
  /* pass C: 1024- and 2048-levels for k2 = 2 t + h; outputs k2 + 256 m1 (+ 1024) of h = 0, 1 are
   * adjacent and leave through cons2 as one pair.
   * The vector loads still in flight here (a persistent caller's prefetch of its next item, issued
   * before pass A) are waited for now, before this unit's stores: loads and stores share vmcnt, and a
   * later wait for the prefetch would otherwise be a vmcnt(0) that also drains the stores. */
  __builtin_amdgcn_s_waitcnt(0x0F70);   /* vmcnt(0), expcnt / lgkmcnt unconstrained */
  if constexpr (OAI4G_MOD_PRIO == 2) __builtin_amdgcn_s_setprio(1);
  if constexpr (OAI4G_MOD_PRIO == 7 || OAI4G_MOD_PRIO == 8) __builtin_amdgcn_s_setprio(0);
  if (active) {
#ifndef OAI4G_PASSC_TWONCE
#define OAI4G_PASSC_TWONCE 1   /* 1: the pass-C companions are built once for both antennas (0: per antenna) */
#endif
    twp_t wc[2][3], wc2[2][4];
    auto build_wc = [&]() {
#pragma unroll
      for (int h = 0; h < 2; h++) {
#pragma unroll
        for (int r = 0; r < 3; r++) wc[h][r] = tw_use(tw.c1024[h][r], dep);
#pragma unroll
        for (int m1 = 0; m1 < 4; m1++) wc2[h][m1] = tw_use(tw.c2048[h + 2 * m1], dep);
      }
    };
    if (OAI4G_PASSC_TWONCE) build_wc();
#pragma unroll
    for (int a = 0; a < NA; a++) {
      if (!OAI4G_PASSC_TWONCE) build_wc();
      s16x2 v[2][8];   /* [h][j] */
#pragma unroll
      for (int jj = 0; jj < 8; jj++) {
        const u32x2_t q = *(const u32x2_t *)&lds[a * X1W + E2S * jj + 2 * t];
        v[0][jj] = u2c(q.x);
        v[1][jj] = u2c(q.y);
      }
      if constexpr (OAI4G_MOD_PRIO == 2 || OAI4G_MOD_PRIO == 9) __builtin_amdgcn_s_setprio(0);
      s16x2 y[2][2][4];   /* [h][e][m1] */
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const twp_t *w = wc[h];
        s16x2 o[2][4];   /* [e][m1] */
#pragma unroll
        for (int e = 0; e < 2; e++) {
          if constexpr (NS) {
            ibfly4_shr1_ns(v[h][e], v[h][e + 2], v[h][e + 4], v[h][e + 6], w[0], w[1], w[2], o[e][0], o[e][1], o[e][2],
                           o[e][3]);
          } else {
            ibfly4(v[h][e], v[h][e + 2], v[h][e + 4], v[h][e + 6], w[0], w[1], w[2], o[e][0], o[e][1], o[e][2], o[e][3]);
#pragma unroll
            for (int m = 0; m < 4; m++) o[e][m] = shr1(o[e][m]);
          }
        }
#pragma unroll
        for (int m1 = 0; m1 < 4; m1++) {
          if (NS && scale) {
            ibfly2_mulhi_ns(o[0][m1], o[1][m1], wc2[h][m1], y[h][0][m1], y[h][1][m1]);
            continue;
          }
          ibfly2(o[0][m1], o[1][m1], wc2[h][m1], y[h][0][m1], y[h][1][m1]);
          if (scale) {
#pragma unroll
            for (int e = 0; e < 2; e++) y[h][e][m1] = NA == 2 ? mulhi2_f(y[h][e][m1]) : mulhi2(y[h][e][m1]);
          }
        }
      }
#pragma unroll
      for (int m1 = 0; m1 < 4; m1++) {
        if constexpr (OAI4G_DIAG_MODCUT == 4) {
          asm volatile("" ::"v"(c2u(y[0][0][m1])), "v"(c2u(y[1][0][m1])), "v"(c2u(y[0][1][m1])), "v"(c2u(y[1][1][m1])));
          continue;
        }
        cons2(a, 2 * t, 256 * m1, y[0][0][m1], y[1][0][m1]);
        cons2(a, 2 * t, 256 * m1 + 1024, y[0][1][m1], y[1][1][m1]);
      }
    }
  }
}

/* twiddle registers and LDS words per transform of the schedule used for each size */
template <int LOG2N>
struct idft_sel {
  using tw_t = idft_tw_t<LOG2N>;
  static constexpr int XW = (1 << LOG2N) + ((1 << LOG2N) >> 5);
};
template <>
struct idft_sel<11> {
  using tw_t = idft2048_tw_t;
  static constexpr int XW = idft2048_tw_t::X1W;
};
/* dep: a per-item value in persistent loops (see tw_use), 0 elsewhere.  cons(a, t, off, y) takes
 * output t + off of antenna a; cons2(a, tt, off, y0, y1) the adjacent outputs tt + off, tt + off + 1
 * (tt + off even) — the 2048-point schedule produces pairs */
template <int LOG2N, int NA, bool PSYNC = false, bool NS = false, class Prod, class Cons, class Cons2>
static __device__ __forceinline__ void idft_any2(uint32_t *lds, int t, bool active,
                                                 const typename idft_sel<LOG2N>::tw_t &tw, Prod prod, Cons cons,
                                                 Cons2 cons2, int scale, uint32_t dep = 0)
{
  if constexpr (LOG2N == 11) idft2048_unit<NA, PSYNC, NS>(lds, t, active, tw, prod, cons2, scale, dep);
  else idft_unit<LOG2N, NA>(lds, t, active, tw, prod, cons, scale);
}
template <int LOG2N, int NA, bool PSYNC = false, class Prod, class Cons>
static __device__ __forceinline__ void idft_any(uint32_t *lds, int t, bool active,
                                                const typename idft_sel<LOG2N>::tw_t &tw, Prod prod, Cons cons,
                                                int scale, uint32_t dep = 0)
{
  idft_any2<LOG2N, NA, PSYNC>(
      lds, t, active, tw, prod, cons,
      [&](int a, int tt, int off, s16x2 y0, s16x2 y1) {
        cons(a, tt, off, y0);
        cons(a, tt, off + 1, y1);
      },
      scale, dep);
}

/* ======================================================================================
 * Drop-in OFDM modulation: per-symbol IDFT + CP from a frequency grid in global memory.
 * 128-thread workgroups, 128/T units each.
 * ==================================================================================== */
struct ofdm_args_t {
  int nsym;
  int scale;
  ofdm_sym_t sym[28];
};

template <int LOG2N>
__global__ void __launch_bounds__(128) k_ofdm(const int32_t *__restrict__ in, int32_t *__restrict__ out,
                                              ofdm_args_t a, const uint32_t *__restrict__ tw)
{
  constexpr int N = 1 << LOG2N, T = N >> 4, UNITS = 128 / T, LDSW = idft_sel<LOG2N>::XW;
  __shared__ uint32_t lds_all[UNITS * LDSW];
  const int unit = threadIdx.x / T, t = threadIdx.x % T;
  const int s = blockIdx.x * UNITS + unit;
  const bool active = s < a.nsym;
  typename idft_sel<LOG2N>::tw_t twr;
  twr.load(tw, t);
  ofdm_sym_t d = active ? a.sym[s] : a.sym[0];
  const uint32_t *src = (const uint32_t *)in + d.in_off;
  uint32_t *dst = (uint32_t *)out + d.out_off;
  const int cp = (int)d.cp;
  idft_any<LOG2N, 1>(
      lds_all + unit * LDSW, t, active, twr, [&](s16x2 (*x)[16]) {
#pragma unroll
        for (int n = 0; n < 16; n++) x[0][n] = u2c(src[t + T * n]);
      },
      [&](int, int tt, int off, s16x2 y) {
        const int f = tt + off;
        dst[f] = c2u(y);
        if (f >= N - cp) dst[f - N] = c2u(y);
      },
      a.scale);
}

hipError_t oai4g_launch_ofdm(const int32_t *d_in, int32_t *d_out, int log2n, int nsym, const ofdm_sym_t *syms,
                             int scale, const uint32_t *d_tw, hipStream_t s)
{
  if (nsym <= 0) return hipSuccess;
  if (nsym > 28) return hipErrorInvalidValue;
  ofdm_args_t a;
  a.nsym = nsym;
  a.scale = scale;
  for (int i = 0; i < nsym; i++) a.sym[i] = syms[i];
  const int units = 128 / ((1 << log2n) >> 4);
  const dim3 grid((nsym + units - 1) / units), blk(128);
  switch (log2n) {
  case 6: hipLaunchKernelGGL(k_ofdm<6>, grid, blk, 0, s, d_in, d_out, a, d_tw); break;
  case 7: hipLaunchKernelGGL(k_ofdm<7>, grid, blk, 0, s, d_in, d_out, a, d_tw); break;
  case 8: hipLaunchKernelGGL(k_ofdm<8>, grid, blk, 0, s, d_in, d_out, a, d_tw); break;
  case 9: hipLaunchKernelGGL(k_ofdm<9>, grid, blk, 0, s, d_in, d_out, a, d_tw); break;
  case 10: hipLaunchKernelGGL(k_ofdm<10>, grid, blk, 0, s, d_in, d_out, a, d_tw); break;
  case 11: hipLaunchKernelGGL(k_ofdm<11>, grid, blk, 0, s, d_in, d_out, a, d_tw); break;
  default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

/* Strided IDFT batch: job j transforms in[j * in_stride + in_off ...] (N words) into
 * out[j * out_stride ...] with the reference's idft decomposition (no prefix).  Used for
 * dl_ch_estimates_time (lte_dl_channel_estimation.c:704-738: idft of each estimate plane from
 * word 8, scale 1). */
template <int LOG2N>
__global__ void __launch_bounds__(128) k_idft_strided(const int32_t *__restrict__ in, int32_t *__restrict__ out,
                                                      int n_jobs, size_t in_stride, uint32_t in_off,
                                                      size_t out_stride, int scale, const uint32_t *__restrict__ tw)
{
  constexpr int N = 1 << LOG2N, T = N >> 4, UNITS = 128 / T, LDSW = idft_sel<LOG2N>::XW;
  __shared__ uint32_t lds_all[UNITS * LDSW];
  const int unit = threadIdx.x / T, t = threadIdx.x % T;
  const int j = blockIdx.x * UNITS + unit;
  const bool active = j < n_jobs;
  typename idft_sel<LOG2N>::tw_t twr;
  twr.load(tw, t);
  const size_t jj = active ? (size_t)j : 0;
  const uint32_t *src = (const uint32_t *)in + jj * in_stride + in_off;
  uint32_t *dst = (uint32_t *)out + jj * out_stride;
  idft_any<LOG2N, 1>(
      lds_all + unit * LDSW, t, active, twr, [&](s16x2 (*x)[16]) {
#pragma unroll
        for (int n = 0; n < 16; n++) x[0][n] = u2c(src[t + T * n]);
      },
      [&](int, int tt, int off, s16x2 y) { dst[tt + off] = c2u(y); }, scale);
}

hipError_t oai4g_launch_idft_strided(const int32_t *d_in, int32_t *d_out, int log2n, int n_jobs, size_t in_stride,
                                     uint32_t in_off, size_t out_stride, int scale, const uint32_t *d_tw, hipStream_t s)
{
  if (n_jobs <= 0) return hipSuccess;
  const int units = 128 / ((1 << log2n) >> 4);
  const dim3 grid((n_jobs + units - 1) / units), blk(128);
  switch (log2n) {
  case 6: hipLaunchKernelGGL(k_idft_strided<6>, grid, blk, 0, s, d_in, d_out, n_jobs, in_stride, in_off, out_stride, scale, d_tw); break;
  case 7: hipLaunchKernelGGL(k_idft_strided<7>, grid, blk, 0, s, d_in, d_out, n_jobs, in_stride, in_off, out_stride, scale, d_tw); break;
  case 8: hipLaunchKernelGGL(k_idft_strided<8>, grid, blk, 0, s, d_in, d_out, n_jobs, in_stride, in_off, out_stride, scale, d_tw); break;
  case 9: hipLaunchKernelGGL(k_idft_strided<9>, grid, blk, 0, s, d_in, d_out, n_jobs, in_stride, in_off, out_stride, scale, d_tw); break;
  case 10: hipLaunchKernelGGL(k_idft_strided<10>, grid, blk, 0, s, d_in, d_out, n_jobs, in_stride, in_off, out_stride, scale, d_tw); break;
  case 11: hipLaunchKernelGGL(k_idft_strided<11>, grid, blk, 0, s, d_in, d_out, n_jobs, in_stride, in_off, out_stride, scale, d_tw); break;
  default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

/* ======================================================================================
 * Modulation helpers shared by the fused kernel and the drop-in grid kernel.
 * ==================================================================================== */
/* PDSCH pilot class of symbol l (dlsch_modulation.c:1268-1282), normal or extended CP */
static __device__ __forceinline__ int pilots_of(uint32_t l, bool ecp)
{
  if (ecp) return (l == 3 || l == 9) ? 2 : (l == 6 ? 1 : 0);
  return (l == 4 || l == 11) ? 2 : (l == 7 ? 1 : 0);
}

/* QAM symbol from Qm bits b0..b(Qm-1) packed LSB-first in `bits` (dlsch_modulation.c:245-355). */
static __device__ __forceinline__ s16x2 qam_map(uint32_t bits, uint32_t Qm, const int16_t *tab, int16_t gain)
{
  if (Qm == 2) return (s16x2){(short)((bits & 1) ? -gain : gain), (short)((bits & 2) ? -gain : gain)};
  uint32_t ir, ii;
  if (Qm == 4) {
    ir = ((bits & 1) << 1) | ((bits >> 2) & 1);
    ii = (bits & 2) | ((bits >> 3) & 1);
  } else {
    ir = ((bits & 1) << 2) | (((bits >> 2) & 1) << 1) | ((bits >> 4) & 1);
    ii = (((bits >> 1) & 1) << 2) | (((bits >> 3) & 1) << 1) | ((bits >> 5) & 1);
  }
  return (s16x2){tab[ir], tab[ii]};
}

/* TM1 / TM3 (LARGE_CDD) precoding of one RE for antenna `ant` (dlsch_modulation.c:266-312, 733-749) */
static __device__ __forceinline__ s16x2 precode(const cfg_dev_t *__restrict__ c, uint32_t ant, uint32_t parity,
                                                s16x2 x0, s16x2 x1)
{
  if (c->mimo_mode != OAI4G_LARGE_CDD) return x0;
  if (ant == 0) return (s16x2){(short)(((int)x0.x + (int)x1.x) >> 1), (short)(((int)x0.y + (int)x1.y) >> 1)};
  int sgn = parity ? -1 : 1;
  return (s16x2){(short)(sgn * (((int)x0.x - (int)x1.x) >> 1)), (short)(sgn * (((int)x0.y - (int)x1.y) >> 1))};
}

/* LARGE_CDD on packed lanes: floor((a+b)/2) = (a&b) + ((a^b)>>1), floor((a-b)/2) = ((a^b)>>1) - (~a&b) */
[[maybe_unused]] static __device__ __forceinline__ void cdd_pair(s16x2 x0, s16x2 x1, uint32_t parity, s16x2 &y0, s16x2 &y1)
{
  const uint32_t a = c2u(x0), b = c2u(x1);
  const s16x2 h = u2c(a ^ b) >> (s16x2){1, 1};
  y0 = u2c(a & b) + h;
  s16x2 d = h - u2c(~a & b);
  y1 = parity ? (s16x2){0, 0} - d : d;
}
/* The same with the sign as a lane mask m (0 or ~0, from the RE code's parity bit): y1 = (d ^ m) - m
 * per 16-bit lane (wrapping, = -d when m = ~0).  Written as v_xor + v_pk_sub_u16 so the compiler
 * cannot turn it back into v_cmp + v_cndmask, whose SGPR mask costs an s_nop 1 hazard per RE. */
static __device__ __forceinline__ void cdd_pair_m(s16x2 x0, s16x2 x1, uint32_t m, s16x2 &y0, s16x2 &y1)
{
  const uint32_t a = c2u(x0), b = c2u(x1);
  const s16x2 h = u2c(a ^ b) >> (s16x2){1, 1};
  y0 = u2c(a & b) + h;
  const s16x2 d = h - u2c(~a & b);
  uint32_t r;
  asm("v_xor_b32_e32 %0, %1, %2\n\tv_pk_sub_u16 %0, %0, %2" : "=&v"(r) : "v"(c2u(d)), "v"(m));
  y1 = u2c(r);
}

/* ALAMOUTI levels (dlsch_modulation.c:362-546): TA = antenna 0 at RE n (x0/sqrt2), TB = antenna
 * 1 at n (-conj(x1)/sqrt2); QPSK signs are applied before the 1/sqrt2 scaling, QAM negation after */
static __device__ __forceinline__ s16x2 alm_ta(uint32_t bits, const cw_dev_t &w, uint32_t pil)
{
  if (w.Qm == 2) {
    const short p = w.alm_qpsk[pil][0], n = w.alm_qpsk[pil][1];
    return (s16x2){(bits & 1) ? n : p, (bits & 2) ? n : p};
  }
  return qam_map(bits, w.Qm, pil ? w.qam_b : w.qam_a, 0);
}
static __device__ __forceinline__ s16x2 alm_tb(uint32_t bits, const cw_dev_t &w, uint32_t pil)
{
  if (w.Qm == 2) {
    const short p = w.alm_qpsk[pil][0], n = w.alm_qpsk[pil][1];
    return (s16x2){(bits & 1) ? p : n, (bits & 2) ? n : p};
  }
  const s16x2 v = qam_map(bits, w.Qm, pil ? w.qam_b : w.qam_a, 0);
  return (s16x2){(short)-v.x, v.y};
}
/* antenna values of an ALAMOUTI RE from its pair's TA / TB: role 0 = RE n, role 1 = the partner,
 * (-TB.re, TB.im) and (TA.re, -TA.im) (:535-545) */
static __device__ __forceinline__ void alm_pair(s16x2 ta, s16x2 tb, uint32_t role, s16x2 &y0, s16x2 &y1)
{
  y0 = role ? (s16x2){(short)-tb.x, tb.y} : ta;
  y1 = role ? (s16x2){ta.x, (short)-ta.y} : tb;
}

/* 4-port large-delay CDD, rank 2 (configuration C4, a build-defined extension: 36.211 6.3.4.2.2,
 * y = W(i) D(i) U x(i), W(i) = C_k/sqrt2 over the codebook entries 12..15, k = floor(i/2) mod 4,
 * D(i) = diag(1, (-1)^i)).  Every entry of 4 W D U is +-1, so each antenna carries +-x0/2 or
 * +-x1/2 exactly: y_p = floor(c x_q / 2).  Bit (i mod 8) * 4 + p of CDD4_QSEL selects q = 1 and
 * of CDD4_NEG the sign c = -1 (tests/spec_model.py: cdd4_precode pins the tables to the
 * Householder codebook). */
__host__ __device__ constexpr uint32_t cdd4_mask(bool neg)
{
  constexpr int8_t M4[4][4][2] = {{{1, 1}, {1, 1}, {1, -1}, {-1, 1}},       /* W_12^{12} x 2 sqrt2 */
                                  {{1, -1}, {1, 1}, {-1, 1}, {1, 1}},       /* W_13^{13} */
                                  {{1, 1}, {-1, 1}, {1, 1}, {1, -1}},       /* W_14^{13} */
                                  {{1, -1}, {-1, 1}, {-1, -1}, {-1, -1}}};  /* W_15^{12} */
  uint32_t m = 0;
  for (int i8 = 0; i8 < 8; i8++)
    for (int p = 0; p < 4; p++) {
      const int a = M4[i8 >> 1][p][0], b = M4[i8 >> 1][p][1] * ((i8 & 1) ? -1 : 1);
      if (neg ? a < 0 : a != b) m |= 1u << (i8 * 4 + p);
    }
  return m;
}
static constexpr uint32_t CDD4_QSEL = cdd4_mask(false), CDD4_NEG = cdd4_mask(true);

/* floor(x/2) or floor(-x/2) per int16 lane: -x/2 rounded down = ~(x >> 1) + (~x & 1) */
static __device__ __forceinline__ s16x2 half_signed(s16x2 x, bool neg)
{
  const s16x2 h = x >> (s16x2){1, 1};
  const s16x2 nh = u2c(~c2u(h)) + u2c(~c2u(x) & 0x00010001u);
  return neg ? nh : h;
}

/* ======================================================================================
 * Fused: packed scrambled e bits -> QAM -> RE map -> precoding -> IDFT -> CP -> IQ.
 * Persistent 128-thread workgroups; a unit of T threads owns one (subframe, symbol) at a time
 * and transforms NA antenna signals (NA = 1 also serves TM1 with several antennas: the SISO
 * precoder writes the same symbol to every antenna, so one transform is stored n_ant times).
 * ==================================================================================== */
template <int LOG2N>
struct modofdm_geom {
  static constexpr int N = 1 << LOG2N, T = N >> 4, UNITS = 128 / T, LDSW = idft_sel<LOG2N>::XW;
  /* staged e-bit words per codeword: up to 12 N_RB <= 0.71 N data REs (15 PRB in 256) of 6 bits */
  static constexpr int EW = (6 * ((N * 3) / 4)) / 32 + 4;
  /* OAI4G_MOD_STAGE: per codeword one 16-bit QAM-table address per data RE (12 N_RB + 3 <= 3N/4
   * entries, host-checked), two sentinel entries at SENT; quad q = 4 REs, QPT quads per thread */
  static constexpr int SENT = (N * 3) / 4, SW = SENT + 4, QPT = 3, QROW = 64;
  /* guard band: leaf inputs t + T n with n in [ZLO, ZHI] fall between subcarrier 6 N_RB_DL and
   * first_carrier_offset = N - 6 N_RB_DL for every thread t (N_RB_DL 6/25/50/100: n = 5..10;
   * 15: n = 6..9; host-checked), where the reference's grid is zero */
  static constexpr int ZLO = LOG2N == 8 ? 6 : 5, ZHI = LOG2N == 8 ? 9 : 10;
};

/* 4 bytes from any byte address of global memory (unaligned dword load) */
typedef uint32_t __attribute__((aligned(1))) u32_a1_t;
static __device__ __forceinline__ uint32_t ld_u32_any(const uint8_t *p)
{
  return *(const __attribute__((address_space(1))) u32_a1_t *)p;
}

#ifndef OAI4G_DIAG_MODOFDM
#define OAI4G_DIAG_MODOFDM 0   /* timing diagnostics only: 1 = no IQ stores, 2 = no e-bit staging, 3 = no QAM lookups,
                                  4 = QAM table reads without bank conflicts */
#endif
#ifndef OAI4G_MOD_ENDSYNC
/* the barrier at the end of an item is not needed: the next item's LDS writes (staging, then the
 * leaves) are separated from this item's last reads (prologue, pass C) by the staging barrier */
#define OAI4G_MOD_ENDSYNC 0
#endif
#ifndef OAI4G_MOD_ZBAND
/* the guard-band leaf inputs are the constant 0: no code, LDS or QAM work for them.  1 = in every
 * kernel but the plain LARGE_CDD one (C3 without CRS / control: measured 1.7 % slower with it, while
 * the full grid gains 0.9 % and C4 4-6 %, profiles/mod_ab_r03_zband.txt); 2 = everywhere; 0 = off */
#define OAI4G_MOD_ZBAND 1
#endif
#ifndef OAI4G_MODOFDM_WAVES
/* waves per SIMD: 2048 points 4 (round 5: SGPR twiddle operands, affine LDS addresses and
 * companions rebuilt at use bring the kernel to <= 124 VGPRs, and the LDS alias to 19.0 KB per
 * workgroup: 8 workgroups per CU); smaller transforms 3 (24 KB of LDS per workgroup) */
#define OAI4G_MODOFDM_WAVES 0
#endif
#ifndef OAI4G_MOD_ALIAS
/* 2048-point symbols: the staged QAM addresses share LDS with the IDFT exchange (two more barriers
 * per item), 19.0 KB per workgroup instead of 25.0 KB */
#define OAI4G_MOD_ALIAS 1
#endif
#define MODOFDM_WAVES_OF(L) (OAI4G_MODOFDM_WAVES > 0 ? OAI4G_MODOFDM_WAVES : ((L) == 11 ? 4 : 3))
#define MODOFDM_ATTR __attribute__((amdgpu_waves_per_eu(MODOFDM_WAVES_OF(LOG2N))))
/* MODE: 0 = TM1 (one transform stored to every antenna), 1 = ALAMOUTI, 2 = LARGE_CDD, 3 = 4-port
 * LARGE_CDD (C4: two items per symbol, each transforming one antenna pair) */
/* NS: the fused ibfly4 + shr1 levels (ibfly4_shr1_ns); the host sets it only for configurations whose
 * range check passed (mod_nosat_ok) */
template <int LOG2N, int MODE, bool CRS, bool ECP, bool NS = false>
__global__ void __launch_bounds__(128) MODOFDM_ATTR k_modofdm(const cfg_dev_t *__restrict__ c, int n_items,
                                                 const uint32_t *__restrict__ ebits, int32_t *__restrict__ iq,
                                                 uint32_t sf0)
{
  using G = modofdm_geom<LOG2N>;
  constexpr int N = G::N, T = G::T, UNITS = G::UNITS, LDSW = G::LDSW, EW = G::EW;
  (void)EW;
  constexpr int NA = MODE == 0 ? 1 : 2;
  constexpr bool CW2 = MODE == 2 || MODE == 3;
  constexpr uint32_t IPS = MODE == 3 ? 2u : 1u;   /* items per (subframe, symbol) */
  __shared__ __attribute__((aligned(16))) uint32_t lds_data[UNITS * NA * LDSW];
#ifndef OAI4G_MOD_STATTM
#define OAI4G_MOD_STATTM 1   /* CRS / control kernels (staged builds): the static REs come from cfg stat_tm, ORed
                                over a data path that reads the zero sentinel there (0: per-RE code tests) */
#endif
  constexpr bool STATTM = OAI4G_MOD_STATTM && OAI4G_MOD_STAGE && CRS;
#ifndef OAI4G_MOD_STATEARLY
#define OAI4G_MOD_STATEARLY 1   /* STATTM: the static words are read before the staging barrier (0: in the prologue) */
#endif
  /* not in the two-antenna 2048-point kernels: 32 more live VGPRs there spill (20-100 bytes per lane) */
  constexpr bool SEARLY = STATTM && OAI4G_MOD_STATEARLY && (NA == 1 || LOG2N < 11);
#if OAI4G_MOD_STAGE
  /* per codeword, the qtab byte address of every data RE's QAM word: entries 4q..4q+3 staged from
   * quad q's 4 Qm bits; entries SENT, SENT + 1 address the zero word that non-data REs read */
  constexpr int SW = G::SW, SENT = G::SENT, QPT = G::QPT, QROW = G::QROW;
  constexpr uint32_t QZERO = 4u * 4u * QROW;     /* byte address of the zero word behind the 4 rows */
  constexpr bool ALIAS = OAI4G_MOD_ALIAS && LOG2N == 11;
  static_assert(!ALIAS || (UNITS == 1 && 2 * SW <= 2 * NA * LDSW), "staged addresses must fit the exchange");
  __shared__ __attribute__((aligned(16))) uint16_t lds_s_own[ALIAS ? 1 : UNITS][2][SW];
  uint16_t(*lds_s)[2][SW] = ALIAS ? (uint16_t(*)[2][SW])lds_data : lds_s_own;
  /* row cw * 2 + pilot symbol: 64 packed IQ words, 256 bytes, so a row base ORs into an entry's byte
   * offset (bits 8-9 against 2-7); then the zero word */
  __shared__ uint32_t qtab[4 * QROW + 1];
  /* OAI4G_MOD_PRE (C3's kernel): the staging step looks the QAM words of both codewords up and stores
   * their CDD sums per data RE, (y0, d) = ((x0 + x1) >> 1, (x0 - x1) >> 1) lane by lane: the RE step is
   * then one 8-byte LDS read and the sign of y1 = s d, instead of two dependent LDS round trips per
   * codeword and the sums */
  constexpr bool PRE = OAI4G_MOD_PRE && MODE == 2 && ALIAS;
  static_assert(!PRE || SW * 8 <= NA * LDSW * 4, "the precoded pairs must fit the exchange");
  u32x2_t *lds_p = (u32x2_t *)lds_data;
  /* the same for TM1 (one codeword, one transform): the staging step stores each data RE's QAM word,
   * the RE step reads it with one 4-byte LDS read (codes 4 idx) */
  constexpr bool PRE1 = OAI4G_MOD_PRE && MODE == 0 && ALIAS;
  static_assert(!PRE1 || SW * 4 <= NA * LDSW * 4, "the staged QAM words must fit the exchange");
  uint32_t *lds_w = (uint32_t *)lds_data;
#else
  __shared__ uint32_t lds_e[UNITS][2][EW];
  __shared__ uint32_t qtab[2][2][64];          /* [cw][pilot symbol][Qm bits] -> packed IQ */
#endif
  const int unit = threadIdx.x / T, t = threadIdx.x % T;
  typename idft_sel<LOG2N>::tw_t twr;
  twr.load(c->tw, t);
  /* symbols per subframe as a constant (the launch checks cfg nsymb): the item -> (subframe, symbol)
   * split is a multiply-high, not a run-time division per item */
  const uint32_t n_ant = c->n_ant;
  constexpr uint32_t nsymb = ECP ? 12u : 14u;
  constexpr uint32_t sps = ECP ? 6 : 7;
#if OAI4G_MOD_STAGE
  for (uint32_t i = threadIdx.x; i < 4 * QROW + 1; i += blockDim.x) {
    const uint32_t row = i / QROW, bits = i - row * QROW, cw = row >> 1, pil = row & 1;
    uint32_t v = 0;
    if (row < 4) {
      if constexpr (MODE == 1) {        /* one codeword: rows 0/1 = TA, rows 2/3 = TB */
        const cw_dev_t &w = c->cw[0];
        v = c2u(cw ? alm_tb(bits, w, pil) : alm_ta(bits, w, pil));
      } else {
        const cw_dev_t &w = c->cw[cw];
        v = c2u(qam_map(bits, w.Qm, pil ? w.qam_b : w.qam_a, pil ? w.qpsk_b : w.qpsk_a));
      }
    }
    qtab[i] = v;
  }
  if (!ALIAS)
    for (uint32_t i = threadIdx.x; i < UNITS * 4; i += blockDim.x) lds_s[i >> 2][(i >> 1) & 1][SENT + (i & 1)] = QZERO;
#else
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
    const uint32_t cw = i >> 7, pil = (i >> 6) & 1, bits = i & 63;
    if constexpr (MODE == 1) {          /* one codeword: [0] = TA, [1] = TB */
      const cw_dev_t &w = c->cw[0];
      qtab[cw][pil][bits] = c2u(cw ? alm_tb(bits, w, pil) : alm_ta(bits, w, pil));
    } else {
      const cw_dev_t &w = c->cw[cw];
      qtab[cw][pil][bits] = c2u(qam_map(bits, w.Qm, pil ? w.qam_b : w.qam_a, pil ? w.qpsk_b : w.qpsk_a));
    }
  }
#endif
  const uint32_t Qm0 = c->cw[0].Qm, Qm1 = c->cw[1].Qm;
  const uint32_t mask0 = (1u << Qm0) - 1u, mask1 = (1u << Qm1) - 1u;
  /* 4 Qm t: the lane part of a quad's bit offset (loop-invariant) */
  const uint32_t qt0 = 4u * Qm0 * (uint32_t)t, qt1 = 4u * Qm1 * (uint32_t)t;
  (void)qt0;
  (void)qt1;
  __syncthreads();

  /* software pipeline: the RE codes and e-bit words of a unit's next item are loaded while the
   * current item is transformed, so no item starts with an exposed HBM round trip */
#if !OAI4G_MOD_STAGE
  constexpr int EPT = (EW + T - 1) / T;          /* staged e words per thread and codeword */
#endif
  /* wave-uniform by construction: an SGPR, so the loop control never waits on the vector load of
   * the dispatch packet (a VGPR copy made every iteration wait for all the IQ stores in flight) */
  const int stride = __builtin_amdgcn_readfirstlane(gridDim.x * UNITS);
  struct pf_t {
    u32x4_t ra, rb;
#if OAI4G_MOD_STAGE
    uint32_t x0[QPT], x1[QPT];   /* quad q = t + k T: the 4 bytes holding its 4 Qm bits */
#else
    uint32_t e0[EPT], e1[EPT];
#endif
  } pf;
  /* the configuration through the constant address space: its uniform fields become scalar loads
   * (lgkmcnt) instead of vector loads the IQ stores would otherwise order behind (shared vmcnt) */
  typedef const __attribute__((address_space(4))) cfg_dev_t ccfg_t;
  const ccfg_t *cc = (const ccfg_t *)c;
  auto fetch = [&](int bse) {
    /* one unit per workgroup: unit is 0, and the item is a scalar from the start (act, nre and the
     * staging offsets become scalar too) */
    const int item = bse + (UNITS == 1 ? 0 : unit);
    const bool act = item < n_items;
    /* one unit per workgroup: the item is wave-uniform, so its table reads become scalar loads and
     * the next item's vector loads need no wait before their use */
    const uint32_t it0 = (act ? (uint32_t)item : 0u) / IPS;
    const uint32_t it = UNITS == 1 ? __builtin_amdgcn_readfirstlane(it0) : it0;
    const uint32_t sf = it / nsymb, l = it - sf * nsymb;
    const uint32_t sfi = (cc->first_sf + (sf0 + sf) * cc->sf_step) % 10;
    const uint32_t nre_u = cc->symnre[sfi][l], re0 = cc->symbase[sfi][l];   /* uniform: scalar loads */
    const uint32_t nre = act ? nre_u : 0u;
    const gu128_t *rsrc = (const gu128_t *)((CRS && !STATTM ? cc->remap_tm : cc->remap_tm0) + ((size_t)sfi * 14 + l) * N + (size_t)t * 16);
    pf.ra = rsrc[0];
    pf.rb = rsrc[1];
#if OAI4G_MOD_STAGE
    if (act && nre) {
      const uint8_t *esf = (const uint8_t *)(ebits + (size_t)(sf * cc->n_cw) * cc->ebits_words);
      const uint32_t nq = (nre + 3) >> 2;
      /* bit (re0 + 4 q) Qm of quad q = t + k T as re0 Qm + min(4 Qm t + 4 Qm T k, 4 Qm (nq - 1)): uniform
       * terms and the loop-invariant 4 Qm t, no per-lane multiply */
      const uint32_t b0 = re0 * Qm0, lim0 = 4 * Qm0 * (nq - 1), b1 = re0 * Qm1, lim1 = 4 * Qm1 * (nq - 1);
#pragma unroll
      for (int k = 0; k < QPT; k++) {   /* unconditional (quads past nq re-read the last one): no branch */
        pf.x0[k] = ld_u32_any(esf + ((b0 + min(qt0 + (uint32_t)(4 * T * k) * Qm0, lim0)) >> 3));
        if constexpr (CW2)
          pf.x1[k] = ld_u32_any(esf + (size_t)4 * cc->ebits_words + ((b1 + min(qt1 + (uint32_t)(4 * T * k) * Qm1, lim1)) >> 3));
      }
    }
#else
    if (act && nre && OAI4G_DIAG_MODOFDM != 2) {
      gu32_t *esf = (gu32_t *)(ebits + (size_t)(sf * cc->n_cw) * cc->ebits_words);
      const uint32_t wlo0 = (re0 * Qm0) >> 5, cnt0 = min((uint32_t)EW, (((re0 + nre) * Qm0 + 31) >> 5) - wlo0 + 1);
#pragma unroll
      for (int k = 0; k < EPT; k++)
        if (t + k * T < (int)cnt0) pf.e0[k] = esf[wlo0 + t + k * T];
      if constexpr (CW2) {
        const uint32_t wlo1 = (re0 * Qm1) >> 5, cnt1 = min((uint32_t)EW, (((re0 + nre) * Qm1 + 31) >> 5) - wlo1 + 1);
#pragma unroll
        for (int k = 0; k < EPT; k++)
          if (t + k * T < (int)cnt1) pf.e1[k] = esf[cc->ebits_words + wlo1 + t + k * T];
      }
    }
#endif
  };
  fetch(blockIdx.x * UNITS);
  /* no vector load crosses into the item loop: at the loop header the compiler merges the entry
   * and back-edge states, and a load pending on entry turns into a vmcnt(0) at the top of every item
   * (draining the previous item's IQ stores) */
  __builtin_amdgcn_s_waitcnt(0x0F70);

  for (int base = blockIdx.x * UNITS; base < n_items; base += stride) {
    const int item = base + (UNITS == 1 ? 0 : unit);
    const bool active = item < n_items;
    const uint32_t it0 = (active ? (uint32_t)item : 0u) / IPS, pair = (uint32_t)item % IPS;
    const uint32_t it = UNITS == 1 ? __builtin_amdgcn_readfirstlane(it0) : it0;
    const uint32_t sf = it / nsymb, l = it - sf * nsymb;
    const uint32_t sfi = (cc->first_sf + (sf0 + sf) * cc->sf_step) % 10;
    const uint32_t nre_u = cc->symnre[sfi][l], re0 = cc->symbase[sfi][l];
    const uint32_t nre = active ? nre_u : 0u;
    const bool crs_sym = (cc->pilmask >> l) & 1u;    /* CRS-bearing symbol: rho_B QAM levels */
    /* symbol with static REs: CRS (with_crs) or the control region (set_control) */
    const bool stat_sym = (cc->with_crs && crs_sym) || ((cc->ctlmask[sfi] >> l) & 1u);
    const uint32_t pil = crs_sym ? 1u : 0u;
    /* output placement: slot, symbol-in-slot i */
    const uint32_t slot = l >= sps ? 1u : 0u, si = l - slot * sps;
    const uint32_t body = slot * (cc->spt >> 1) + (si == 0 ? cc->cp0 : (N + cc->cp0) + (si - 1) * (N + cc->cp) + cc->cp);
    const int cp = (int)(si == 0 ? cc->cp0 : cc->cp);
    uint32_t *dst0 = (uint32_t *)iq + (size_t)sf * n_ant * cc->spt + body;

    if (UNITS == 1 && nre == 0 && !(CRS && stat_sym)) {
      /* control-region symbol: the transform of an all-zero grid is zero */
      fetch(base + stride);
      __builtin_amdgcn_s_waitcnt(0x0F70);   /* the prefetch lands before the stores (see idft2048_unit pass C) */
      if (active)
        for (uint32_t a = MODE == 3 ? 2 * pair : 0; a < (MODE == 3 ? 2 * pair + 2 : n_ant); a++) {
          uint32_t *d = dst0 + (size_t)a * cc->spt - cp;   /* CP start of antenna a */
          for (int f = t; f < N + cp; f += T) d[f] = 0u;
        }
      continue;
    }

    /* this thread's 16 RE codes (thread-major copy, prefetched) */
    const uint32_t rw[8] = {pf.ra.x, pf.ra.y, pf.ra.z, pf.ra.w, pf.rb.x, pf.rb.y, pf.rb.z, pf.rb.w};
    if constexpr (OAI4G_MOD_PRIO >= 1) __builtin_amdgcn_s_setprio(OAI4G_MOD_PRIO == 3 ? 3 : 2);
#if OAI4G_MOD_STAGE
    /* stage, per codeword, the QAM-table address of every data RE of this symbol: quad q's 4 Qm
     * bits from its prefetched bytes -> 4 entries (ALAMOUTI: even entries TA rows, odd TB rows) */
    if (PRE) {
      if (active && t < 2) lds_p[SENT + t] = (u32x2_t){0u, 0u};                 /* the exchange overwrote them */
    } else if (PRE1) {
      if (active && t < 2) lds_w[SENT + t] = 0u;
    } else if (ALIAS && active && t < 4) lds_s[0][t >> 1][SENT + (t & 1)] = QZERO;
    if (active && nre) {
      const uint32_t nq = (nre + 3) >> 2;
      /* quad q = t + k T starts at bit (re0 + 4 q) Qm of the codeword, (re0 Qm + 4 Qm t) mod 8 into its
       * prefetched bytes for every k (4 Qm T is a multiple of 8); x << 2 puts entry j's table offset at
       * bits j Qm + 2.., so an entry is one shift and one v_bitop3 (offset & (mask << 2)) | row base */
      const uint32_t sh0 = (re0 * Qm0 + qt0) & 7u, sh1 = (re0 * Qm1 + qt1) & 7u;
      const uint32_t m40 = mask0 << 2, m41 = mask1 << 2;
      auto ent = [&](uint32_t x4, uint32_t shift, uint32_t m4, uint32_t row) {
        uint32_t r;
        /* (a & b) | c; one SGPR operand at most (gfx9 constant bus) */
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xea" : "=v"(r) : "v"(x4 >> shift), "s"(m4), "v"(row));
        return r;
      };
      auto stage = [&](uint32_t xw, uint32_t q, uint32_t sh, uint32_t Qm, uint32_t m4, uint32_t ra, uint32_t rb, uint16_t *dst) {
        const uint32_t x4 = (xw >> sh) << 2;
        const uint32_t s0 = ent(x4, 0, m4, ra), s1 = ent(x4, Qm, m4, rb);
        const uint32_t s2 = ent(x4, 2 * Qm, m4, ra), s3 = ent(x4, 3 * Qm, m4, rb);
        *(u32x2_t *)(dst + 4 * q) = (u32x2_t){s0 | (s1 << 16), s2 | (s3 << 16)};
      };
      constexpr uint32_t RB = 4u * QROW;   /* bytes per qtab row */
      const char *qbs = (const char *)qtab;
      /* PRE: quad q's 4 QAM words of each codeword (8 independent LDS reads), their CDD sums, and the
       * 4 (y0, d) pairs as two 16-byte stores */
      auto stage_pre = [&](uint32_t xw0, uint32_t xw1, uint32_t q) {
        const uint32_t x0 = (xw0 >> sh0) << 2, x1 = (xw1 >> sh1) << 2;
        uint32_t v0[4], v1[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
          v0[j] = *(const uint32_t *)(qbs + ent(x0, j * Qm0, m40, pil * RB));
          v1[j] = *(const uint32_t *)(qbs + ent(x1, j * Qm1, m41, (2 + pil) * RB));
        }
        uint32_t o[8];
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint32_t a = v0[j], b = v1[j];
          const s16x2 h = u2c(a ^ b) >> (s16x2){1, 1};
          o[2 * j] = c2u(u2c(a & b) + h);           /* y0 = floor((x0 + x1) / 2) per int16 lane */
          /* d = floor((x0 - x1) / 2); RE 4q + j of odd index stores -d (wrapping): its CDD sign
           * (dlsch_modulation.c's per-RB alternation equals the index parity, host-checked) */
          o[2 * j + 1] = (j & 1) ? c2u(u2c(~a & b) - h) : c2u(h - u2c(~a & b));
        }
        u32x4_t *dst = (u32x4_t *)(lds_p + 4 * q);
        dst[0] = (u32x4_t){o[0], o[1], o[2], o[3]};
        dst[1] = (u32x4_t){o[4], o[5], o[6], o[7]};
      };
      /* PRE1: quad q's 4 QAM words (4 independent LDS reads) as one 16-byte store */
      auto stage_pre1 = [&](uint32_t xw0, uint32_t q) {
        const uint32_t x0 = (xw0 >> sh0) << 2;
        uint32_t v0[4];
#pragma unroll
        for (int j = 0; j < 4; j++) v0[j] = *(const uint32_t *)(qbs + ent(x0, j * Qm0, m40, pil * RB));
        *(u32x4_t *)(lds_w + 4 * q) = (u32x4_t){v0[0], v0[1], v0[2], v0[3]};
      };
#pragma unroll
      for (int k = 0; k < QPT; k++) {
        const uint32_t q = (uint32_t)t + (uint32_t)(k * T);
        if (q < nq) {
          if constexpr (PRE) {
            stage_pre(pf.x0[k], pf.x1[k], q);
          } else if constexpr (PRE1) {
            stage_pre1(pf.x0[k], q);
          } else {
            if constexpr (MODE == 1) stage(pf.x0[k], q, sh0, Qm0, m40, pil * RB, (2 + pil) * RB, lds_s[unit][0]);
            else stage(pf.x0[k], q, sh0, Qm0, m40, pil * RB, pil * RB, lds_s[unit][0]);
            if constexpr (CW2) stage(pf.x1[k], q, sh1, Qm1, m41, (2 + pil) * RB, (2 + pil) * RB, lds_s[unit][1]);
          }
        }
      }
    }
#else
    /* stage this symbol's e bits of each codeword (prefetched words, coalesced) */
    const uint32_t wlo0 = (re0 * Qm0) >> 5, wlo1 = (re0 * Qm1) >> 5;
    if (active && nre && OAI4G_DIAG_MODOFDM != 2) {
      const uint32_t cnt0 = min((uint32_t)EW, (((re0 + nre) * Qm0 + 31) >> 5) - wlo0 + 1);
#pragma unroll
      for (int k = 0; k < EPT; k++)
        if (t + k * T < (int)cnt0) lds_e[unit][0][t + k * T] = pf.e0[k];
      if constexpr (CW2) {
        const uint32_t cnt1 = min((uint32_t)EW, (((re0 + nre) * Qm1 + 31) >> 5) - wlo1 + 1);
#pragma unroll
        for (int k = 0; k < EPT; k++)
          if (t + k * T < (int)cnt1) lds_e[unit][1][t + k * T] = pf.e1[k];
      }
    }
#endif
    /* a CRS / control symbol's static words (STATTM) are read here, ahead of the staging barrier: their L2
     * round trip overlaps the barrier and the next item's prefetch instead of stalling the prologue */
    u32x4_t stw[NA][4];
    if constexpr (SEARLY) {
      if (stat_sym) {
#pragma unroll
        for (int a = 0; a < NA; a++) {
          const uint32_t ant = NA == 1 ? 0u : (uint32_t)a + 2u * pair;
          const gu128_t *sp =
              (const gu128_t *)(cc->stat_tm + ((sfi * 14u + l) * cc->stat_planes + ant) * (uint32_t)N + (uint32_t)t * 16u);
#pragma unroll
          for (int q = 0; q < 4; q++) stw[a][q] = sp[q];
        }
      }
    }
    __syncthreads();
    if constexpr (OAI4G_MOD_PRIO == 4) __builtin_amdgcn_s_setprio(0);
    fetch(base + stride);

    gu32_t *crs_tab = (gu32_t *)cc->crs_tab;
    const bool crs = CRS && stat_sym;
    gu32_t *ctl_tab = (gu32_t *)cc->ctl_tab;
#if OAI4G_MOD_STAGE
    const char *sb0 = (const char *)lds_s[unit][0], *sb1 = (const char *)lds_s[unit][1], *qb = (const char *)qtab;
#else
    const uint32_t *e0 = lds_e[unit][0], *e1 = lds_e[unit][1];
    const uint32_t *q0 = qtab[0][pil], *q1 = qtab[1][pil];
    /* bit position of data RE idx within the staged words: idx * Qm + (re0 * Qm - 32 wlo) */
    const uint32_t b0 = re0 * Qm0 - 32 * wlo0, b1 = re0 * Qm1 - 32 * wlo1;
#endif
#if OAI4G_MOD_STAGE
    constexpr bool PSYNC = ALIAS;
#else
    constexpr bool PSYNC = false;
#endif
    idft_any2<LOG2N, NA, PSYNC, NS>(
        lds_data + unit * NA * LDSW, t, active, twr,
        [&](s16x2 (*x)[16]) {
          /* branch-free and staged in groups of GR REs so each LDS round trip is issued for the
           * whole group before the first wait: codes -> bit offsets -> e words -> QAM words.  An RE
           * outside the allocation reads data RE 0 (inside the staged words), zeroed by the select */
#ifndef OAI4G_MOD_GROUP
#define OAI4G_MOD_GROUP 4   /* REs whose LDS round trips are issued together (register budget) */
#endif
          constexpr int GR = OAI4G_MOD_GROUP;
#if OAI4G_MOD_STAGE
          /* remap_tm data codes are 2 idx | parity << 15 (ALAMOUTI: 2 (2i + role)): the byte
           * offset of entry idx; any non-data code (>= 0xC000) clamps to the zero sentinel (in
           * remap_tm0 it already is the sentinel) */
          constexpr uint32_t AM = MODE == 1 ? 0x7FFCu : 0x7FFEu;
          constexpr bool ZB = OAI4G_MOD_ZBAND == 2 || (OAI4G_MOD_ZBAND == 1 && (CRS || MODE != 2));
          auto zb = [&](int n) { return ZB && n >= G::ZLO && n <= G::ZHI; };   /* constant after unrolling */
          /* the NZ leaf inputs outside the guard band, visited in groups of GZ (the i-th is act(i)) */
          constexpr int NZ = ZB ? 16 - (G::ZHI - G::ZLO + 1) : 16;
#ifndef OAI4G_MOD_GROUPZ
#define OAI4G_MOD_GROUPZ 5
#endif
          constexpr int GZ = ZB ? (NZ % OAI4G_MOD_GROUPZ == 0 ? OAI4G_MOD_GROUPZ : 4) : GR;
          auto act = [&](int i) { return (ZB && i >= G::ZLO) ? i + (G::ZHI - G::ZLO + 1) : i; };
#ifndef OAI4G_MOD_ZB_OPAQUE
#define OAI4G_MOD_ZB_OPAQUE 0   /* 1: the guard-band zeros come from a v_mov the compiler cannot fold (A/B of the leaf folding) */
#endif
#pragma unroll
          for (int n = 0; n < 16; n++)
            if (zb(n)) {
              uint32_t z = 0;
              if (OAI4G_MOD_ZB_OPAQUE) asm("v_mov_b32 %0, 0" : "=v"(z));
#pragma unroll
              for (int a = 0; a < NA; a++) x[a][n] = u2c(z);
            }
          if constexpr (PRE) {
            /* one 8-byte read per RE: the pair staged for its data index, CDD sign included (codes
             * 8 idx; every non-data code addresses the zero pair, clamped when CRS / control codes occur) */
            const char *pb = (const char *)lds_p;
#pragma unroll
            for (int g = 0; g < NZ; g += GZ) {
              uint32_t code[GZ];
              u32x2_t v[GZ];
#pragma unroll
              for (int n = 0; n < GZ; n++) {
                const int i = act(g + n);
                code[n] = (rw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
                const uint32_t a = CRS && !STATTM ? min(code[n] & 0x7FF8u, 8u * SENT) : code[n] & 0x7FF8u;
                v[n] = *(const u32x2_t *)(pb + a);
              }
#pragma unroll
              for (int n = 0; n < GZ; n++) {
                const int i = act(g + n);
                x[0][i] = u2c(v[n].x);
                x[1][i] = u2c(v[n].y);
              }
            }
          } else if constexpr (PRE1) {
            /* one 4-byte read per RE: the QAM word staged for its data index (codes 4 idx) */
            const char *pb = (const char *)lds_w;
#pragma unroll
            for (int g = 0; g < NZ; g += GZ) {
              uint32_t v[GZ];
#pragma unroll
              for (int n = 0; n < GZ; n++) {
                const int i = act(g + n);
                const uint32_t code = (rw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
                const uint32_t a = CRS && !STATTM ? min(code & 0x7FFCu, 4u * SENT) : code & 0x7FFCu;
                v[n] = *(const uint32_t *)(pb + a);
              }
#pragma unroll
              for (int n = 0; n < GZ; n++) x[0][act(g + n)] = u2c(v[n]);
            }
          } else
#pragma unroll
          for (int g = 0; g < NZ; g += GZ) {
            uint32_t code[GZ], v0[GZ], v1[GZ];
#pragma unroll
            for (int n = 0; n < GZ; n++) {
              const int i = act(g + n);
              code[n] = (rw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
              /* without CRS / control REs every non-data code is already the sentinel (remap_tm0) */
              const uint32_t a = CRS && !STATTM ? min(code[n] & AM, 2u * SENT) : code[n] & AM;
              v0[n] = *(const uint16_t *)(sb0 + a);
              if constexpr (MODE == 1) v1[n] = *(const uint16_t *)(sb0 + a + 2);
              if constexpr (CW2) v1[n] = *(const uint16_t *)(sb1 + a);
            }
#ifndef OAI4G_DIAG_QTAB
#define OAI4G_DIAG_QTAB 0    /* timing diagnostic only: 1 = QAM-table reads at lane-distinct banks (wrong values) */
#endif
#if OAI4G_DIAG_QTAB
            const uint32_t qkeep = cc->with_crs ? 0xFFFFFFFFu : 0u, qlane = ((uint32_t)threadIdx.x & 31u) << 2;
#define QADDR(x) (((x) & qkeep) | (qlane & ~qkeep))
#else
#define QADDR(x) (x)
#endif
#pragma unroll
            for (int n = 0; n < GZ; n++) {
              v0[n] = *(const uint32_t *)(qb + QADDR(v0[n]));
              if constexpr (MODE == 1 || CW2) v1[n] = *(const uint32_t *)(qb + QADDR(v1[n]));
            }
#undef QADDR
#pragma unroll
            for (int n = 0; n < GZ; n++) {
              const int i = act(g + n);
              const s16x2 x0 = u2c(v0[n]);
              if constexpr (MODE == 1) {
                alm_pair(x0, u2c(v1[n]), (code[n] >> 1) & 1u, x[0][i], x[1][i]);
              } else if constexpr (MODE == 3) {
                const s16x2 x1 = u2c(v1[n]);
                const uint32_t sel = ((re0 + ((code[n] & 0x7FFFu) >> 1)) & 7u) * 4u + 2u * pair;   /* (i mod 8, p) */
#pragma unroll
                for (int a = 0; a < 2; a++)
                  x[a][i] = half_signed(((CDD4_QSEL >> (sel + a)) & 1u) ? x1 : x0, (CDD4_NEG >> (sel + a)) & 1u);
              } else if constexpr (NA == 2) {
                /* parity bit 15 of the code -> lane mask 0 / ~0 */
                cdd_pair_m(x0, u2c(v1[n]), (uint32_t)((int32_t)(code[n] << 16) >> 31), x[0][i], x[1][i]);
              } else {
                x[0][i] = x0;                                   /* TM1: SISO precoder */
              }
            }
          }
#else
#if OAI4G_DIAG_MODOFDM == 3
#pragma unroll
          for (int n = 0; n < 16; n++)
#pragma unroll
            for (int a = 0; a < NA; a++) x[a][n] = u2c(rw[n >> 1] + (uint32_t)(a + n));
          if (0)
#endif
#pragma unroll
          for (int g = 0; g < 16; g += GR) {
            uint32_t code[GR], p[GR], lo[GR], hi[GR], v0[GR], v1[GR];
            /* ALAMOUTI codes are 2i | role: both symbols of pair i start at bit 2i Qm */
            constexpr uint32_t IDXM = MODE == 1 ? 0x7FFEu : 0x7FFFu;
#pragma unroll
            for (int n = 0; n < GR; n++) {
              code[n] = (rw[(g + n) >> 1] >> (16 * ((g + n) & 1))) & 0xFFFFu;
              p[n] = __umul24(code[n] < OAI4G_CTL_CODE ? (code[n] & IDXM) : 0u, Qm0) + b0;
            }
#pragma unroll
            for (int n = 0; n < GR; n++) { lo[n] = e0[p[n] >> 5]; hi[n] = e0[(p[n] >> 5) + 1]; }
#if OAI4G_DIAG_MODOFDM == 4   /* timing diagnostic: QAM table reads at lane-unique words (no bank conflicts) */
            const uint32_t dkeep = cc->with_crs ? 0xFFFFFFFFu : 0u, dlane = (uint32_t)threadIdx.x & 31u;
#define QIDX(x) (((x) & dkeep) | (dlane & ~dkeep))
#else
#define QIDX(x) (x)
#endif
            if constexpr (MODE == 1) {
#pragma unroll
              for (int n = 0; n < GR; n++) {
                const uint32_t wv = __builtin_amdgcn_alignbit(hi[n], lo[n], p[n] & 31);
                v0[n] = q0[wv & mask0];
                v1[n] = q1[(wv >> Qm0) & mask0];
              }
            } else {
#pragma unroll
              for (int n = 0; n < GR; n++) v0[n] = q0[QIDX(__builtin_amdgcn_alignbit(hi[n], lo[n], p[n] & 31) & mask0)];
            }
            if constexpr (CW2) {
#pragma unroll
              for (int n = 0; n < GR; n++) {
                p[n] = __umul24(code[n] < OAI4G_CTL_CODE ? (code[n] & 0x7FFFu) : 0u, Qm1) + b1;
                lo[n] = e1[p[n] >> 5];
                hi[n] = e1[(p[n] >> 5) + 1];
              }
#pragma unroll
              for (int n = 0; n < GR; n++) v1[n] = q1[QIDX(__builtin_amdgcn_alignbit(hi[n], lo[n], p[n] & 31) & mask1)];
            }
#pragma unroll
            for (int n = 0; n < GR; n++) {
              const bool valid = code[n] < OAI4G_CTL_CODE;         /* a PDSCH data RE */
              const s16x2 x0 = u2c(valid ? v0[n] : 0u);
              if constexpr (MODE == 1) {
                alm_pair(x0, u2c(valid ? v1[n] : 0u), code[n] & 1u, x[0][g + n], x[1][g + n]);
              } else if constexpr (MODE == 3) {
                const s16x2 x1 = u2c(valid ? v1[n] : 0u);
                const uint32_t sel = ((re0 + (code[n] & 0x7FFFu)) & 7u) * 4u + 2u * pair;   /* (i mod 8, p) */
#pragma unroll
                for (int a = 0; a < 2; a++)
                  x[a][g + n] = half_signed(((CDD4_QSEL >> (sel + a)) & 1u) ? x1 : x0, (CDD4_NEG >> (sel + a)) & 1u);
              } else if constexpr (NA == 2) {
                const s16x2 x1 = CW2 ? u2c(valid ? v1[n] : 0u) : (s16x2){0, 0};
                cdd_pair(x0, x1, code[n] >> 15 & 1u, x[0][g + n], x[1][g + n]);
              } else {
                x[0][g + n] = x0;                                   /* TM1: SISO precoder */
              }
            }
          }
#endif
          if constexpr (CRS && STATTM) {
            if (crs) {
              /* CRS / control symbol: the data path read the zero sentinel at every static RE (remap_tm0),
               * so the antenna's static values (0 at data REs) are ORed over it: 16 consecutive words per
               * thread and antenna, four 16-byte loads, no per-RE tests */
#pragma unroll
              for (int a = 0; a < NA; a++) {
                u32x4_t w[4];
                if constexpr (SEARLY) {
#pragma unroll
                  for (int q = 0; q < 4; q++) w[q] = stw[a][q];
                } else {
                  const uint32_t ant = NA == 1 ? 0u : (uint32_t)a + 2u * pair;
                  const gu128_t *sp = (const gu128_t *)(cc->stat_tm + ((sfi * 14u + l) * cc->stat_planes + ant) * (uint32_t)N +
                                                        (uint32_t)t * 16u);
#pragma unroll
                  for (int q = 0; q < 4; q++) w[q] = sp[q];
                }
#pragma unroll
                for (int n = 0; n < 16; n++) {
                  if (zb(n)) continue;   /* no CRS or control RE in the guard band */
                  x[a][n] = u2c(c2u(x[a][n]) | w[n >> 2][n & 3]);
                }
              }
            }
          } else if constexpr (CRS) {
            if (crs) {
              /* cell-specific RS (pilots.c:43-168): overwrite the antenna carrying port p */
#pragma unroll
              for (int n = 0; n < 16; n++) {
#if OAI4G_MOD_STAGE
                if (zb(n)) continue;   /* no CRS or control RE in the guard band */
#endif
                const uint32_t cd = (rw[n >> 1] >> (16 * (n & 1))) & 0xFFFFu;
                const bool pil_re = cd >= OAI4G_CRS_CODE && cd != 0xFFFFu;
                const uint32_t ci = (cd >> 9) & 7u, m = cd & 0xFFu, port = ((cd >> 8) & 1u) | (ci >= 4 ? 2u : 0u);
                const uint32_t pv = pil_re ? crs_tab[(sfi * 6 + ci) * 200 + m] : 0u;
#pragma unroll
                for (int a = 0; a < NA; a++)
                  if (pil_re) x[a][n] = (NA == 1 || (uint32_t)a + 2 * pair == port) ? u2c(pv) : (s16x2){0, 0};
                /* control region (generate_dci_top writes antennas 0 and 1 only, dci.c:2260-2336) */
                const bool ctl_re = (cd & 0xE000u) == OAI4G_CTL_CODE;
                if (ctl_re) {
                  const size_t cb = ((size_t)(sfi * 14 + l) * 2) * N + (uint32_t)t + (uint32_t)(N / 16) * (uint32_t)n;
#pragma unroll
                  for (int a = 0; a < NA; a++) {
                    const uint32_t ant = NA == 1 ? 0u : (uint32_t)a + 2 * pair;
                    x[a][n] = ant < 2 ? u2c(ctl_tab[cb + ant * N]) : (s16x2){0, 0};
                  }
                }
              }
            }
          }
        },
        [&](int a, int tt, int off, s16x2 y) {
          /* per-thread bases for each half of the symbol keep every store's offset within the
           * 13-bit immediate; the CP test is compiled out where no t can reach N - CP_max */
          constexpr int CPMAX = ECP ? N / 4 : (N * 160) / 2048;
          const bool hi = off >= N / 2;
          const int ro = hi ? off - N / 2 : off;
          auto store = [&](uint32_t *base) {
            uint32_t *d = base + tt + (hi ? N / 2 : 0);
#if OAI4G_DIAG_MODOFDM == 1   /* timing diagnostic: the stores (almost) never happen */
            if (c2u(y) != 0x12345678u) return;
#endif
            d[ro] = c2u(y);
            if (off + T - 1 >= N - CPMAX && tt + off >= N - cp) d[ro - N] = c2u(y);
          };
          if constexpr (NA == 2) {
            store(dst0 + (a + 2 * pair) * cc->spt);
          } else {
            for (uint32_t aa = 0; aa < n_ant; aa++) store(dst0 + aa * cc->spt);
          }
        },
        [&](int a, int tt, int off, s16x2 y0, s16x2 y1) {
          /* outputs tt + off, tt + off + 1 (even first): one 8-byte store (the symbol bodies, CP
           * lengths and slot/subframe offsets are even and iq is 8-byte aligned, host-checked); N - cp
           * is even, so both samples of a pair fall in the CP copy or neither does */
          constexpr int CPMAX = ECP ? N / 4 : (N * 160) / 2048;
          const bool hi = off >= N / 2;
          const int ro = hi ? off - N / 2 : off;
          const u32x2_t v = {c2u(y0), c2u(y1)};
          auto store = [&](uint32_t *base) {
            uint32_t *d = base + tt + (hi ? N / 2 : 0);
#if OAI4G_DIAG_MODOFDM == 1   /* timing diagnostic: the stores (almost) never happen */
            if (v.x != 0x12345678u) return;
#endif
            *(u32x2_t *)&d[ro] = v;
            if (off + 2 * T - 2 >= N - CPMAX && tt + off >= N - cp) *(u32x2_t *)&d[ro - N] = v;
          };
          if constexpr (NA == 2) {
            store(dst0 + (a + 2 * pair) * cc->spt);
          } else {
            for (uint32_t aa = 0; aa < n_ant; aa++) store(dst0 + aa * cc->spt);
          }
        },
        1, it);
    if (OAI4G_MOD_ENDSYNC || PSYNC) __syncthreads();   /* PSYNC: the next item stages into the exchange */
  }
}

template <int LOG2N, int MODE, bool CRS, bool ECP, bool NS = false>
static hipError_t launch_modofdm_t(const cfg_dev_t *d_cfg, const cfg_dev_t *h_cfg, int sf0, int n_items,
                                   const uint32_t *d_ebits, int32_t *d_iq, hipStream_t s)
{
  static int occ = 0;
  if (!occ) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_modofdm<LOG2N, MODE, CRS, ECP, NS>, 128, 0) != hipSuccess ||
        occ < 1)
      occ = 1;
    /* OAI4G_MODOFDM_OCC=n caps the persistent grid at n workgroups per CU (diagnostic: leaves
     * room for encoder workgroups of the pipelined mode) */
    if (const char *e = getenv("OAI4G_MODOFDM_OCC")) {
      const int cap = atoi(e);
      if (cap >= 1 && cap < occ) occ = cap;
    }
  }
  const int units = modofdm_geom<LOG2N>::UNITS;
  int want = (n_items + units - 1) / units, cap = occ * (int)h_cfg->n_cu;
  int grid = want < cap ? want : cap;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL((k_modofdm<LOG2N, MODE, CRS, ECP, NS>), dim3(grid), dim3(128), 0, s, d_cfg, n_items, d_ebits, d_iq,
                     (uint32_t)sf0);
  return hipGetLastError();
}

template <int LOG2N, int MODE, bool ECP>
static hipError_t launch_modofdm_c(const cfg_dev_t *d_cfg, const cfg_dev_t *h_cfg, int sf0, int n_items,
                                   const uint32_t *d_ebits, int32_t *d_iq, hipStream_t s)
{
  /* the no-saturation forms (2048 points, normal prefix) when the range check passed */
  if (h_cfg->with_crs || h_cfg->ctl_on) {
    if constexpr (LOG2N == 11 && !ECP)
      if (h_cfg->mod_nosat) return launch_modofdm_t<LOG2N, MODE, true, ECP, true>(d_cfg, h_cfg, sf0, n_items, d_ebits, d_iq, s);
    return launch_modofdm_t<LOG2N, MODE, true, ECP>(d_cfg, h_cfg, sf0, n_items, d_ebits, d_iq, s);
  }
  if constexpr (LOG2N == 11 && !ECP)
    if (h_cfg->mod_nosat) return launch_modofdm_t<LOG2N, MODE, false, ECP, true>(d_cfg, h_cfg, sf0, n_items, d_ebits, d_iq, s);
  return launch_modofdm_t<LOG2N, MODE, false, ECP>(d_cfg, h_cfg, sf0, n_items, d_ebits, d_iq, s);
}

template <int LOG2N, bool ECP>
static hipError_t launch_modofdm_m(const cfg_dev_t *d_cfg, const cfg_dev_t *h_cfg, int sf0, int n_items,
                                   const uint32_t *d_ebits, int32_t *d_iq, hipStream_t s)
{
  switch (h_cfg->mimo_mode) {
  case OAI4G_LARGE_CDD:
    return h_cfg->n_ant == 4 ? launch_modofdm_c<LOG2N, 3, ECP>(d_cfg, h_cfg, sf0, 2 * n_items, d_ebits, d_iq, s)
                             : launch_modofdm_c<LOG2N, 2, ECP>(d_cfg, h_cfg, sf0, n_items, d_ebits, d_iq, s);
  case OAI4G_ALAMOUTI: return launch_modofdm_c<LOG2N, 1, ECP>(d_cfg, h_cfg, sf0, n_items, d_ebits, d_iq, s);
  default: return launch_modofdm_c<LOG2N, 0, ECP>(d_cfg, h_cfg, sf0, n_items, d_ebits, d_iq, s);
  }
}

/* precoding mode, CRS and the prefix type are uniform per configuration and become template
 * arguments: no per-RE uniform branches in the prologue or the stores */
template <int LOG2N>
static hipError_t launch_modofdm_n(const cfg_dev_t *d_cfg, const cfg_dev_t *h_cfg, int sf0, int n_items,
                                   const uint32_t *d_ebits, int32_t *d_iq, hipStream_t s)
{
  return h_cfg->nsymb == 12 ? launch_modofdm_m<LOG2N, true>(d_cfg, h_cfg, sf0, n_items, d_ebits, d_iq, s)
                            : launch_modofdm_m<LOG2N, false>(d_cfg, h_cfg, sf0, n_items, d_ebits, d_iq, s);
}

/* subframes [sf0, sf0 + n_sf) of a batch whose e-bit words / IQ start at d_ebits / d_iq */
hipError_t oai4g_launch_modofdm(const cfg_dev_t *d_cfg, const cfg_dev_t *h_cfg, int sf0, int n_sf,
                                const uint32_t *d_ebits, int32_t *d_iq, hipStream_t s)
{
  if (n_sf <= 0) return hipSuccess;
  if (h_cfg->nsymb != 12 && h_cfg->nsymb != 14) return hipErrorInvalidValue;   /* k_modofdm: 12 <=> ECP */
  const int n_items = n_sf * (int)h_cfg->nsymb;
  d_ebits += (size_t)sf0 * h_cfg->n_cw * h_cfg->ebits_words;
  d_iq += (size_t)sf0 * h_cfg->n_ant * h_cfg->spt;
  /* two antenna transforms per unit only when they differ (LARGE_CDD, ALAMOUTI); TM1 stores one
   * n_ant times */
  if (h_cfg->mimo_mode != OAI4G_SISO && h_cfg->n_ant != 2 && !(h_cfg->mimo_mode == OAI4G_LARGE_CDD && h_cfg->n_ant == 4))
    return hipErrorInvalidValue;
  if (h_cfg->mimo_mode == OAI4G_LARGE_CDD && h_cfg->n_cw != 2) return hipErrorInvalidValue;
  if (OAI4G_MOD_ZBAND && h_cfg->log2N >= 7 && h_cfg->log2N <= 11) {
    /* the guard-band leaf inputs must be zero subcarriers: T ZLO > 6 N_RB_DL, T (ZHI + 1) <= first_carrier */
    const uint32_t T = h_cfg->N >> 4, zlo = h_cfg->log2N == 8 ? 6u : 5u, zhi = h_cfg->log2N == 8 ? 9u : 10u;
    if (h_cfg->first_carrier != h_cfg->N - 6 * h_cfg->N_RB_DL || T * zlo <= 6 * h_cfg->N_RB_DL ||
        T * (zhi + 1) > h_cfg->first_carrier)
      return hipErrorInvalidValue;
  }
  switch (h_cfg->log2N) {
  case 7: return launch_modofdm_n<7>(d_cfg, h_cfg, sf0, n_items, d_ebits, d_iq, s);
  case 8: return launch_modofdm_n<8>(d_cfg, h_cfg, sf0, n_items, d_ebits, d_iq, s);
  case 9: return launch_modofdm_n<9>(d_cfg, h_cfg, sf0, n_items, d_ebits, d_iq, s);
  case 10: return launch_modofdm_n<10>(d_cfg, h_cfg, sf0, n_items, d_ebits, d_iq, s);
  case 11: return launch_modofdm_n<11>(d_cfg, h_cfg, sf0, n_items, d_ebits, d_iq, s);
  default: return hipErrorInvalidValue;
  }
}

/* ======================================================================================
 * Drop-in dlsch_modulation: accumulate (+=, int16 wrap) QAM symbols from e BYTES into a
 * frequency grid (one subframe, all antennas).  Thread per (symbol, subcarrier).
 * ==================================================================================== */
__global__ void __launch_bounds__(256) k_modulate_bytes(const cfg_dev_t *__restrict__ c, int sfi,
                                                        const uint8_t *__restrict__ e0,
                                                        const uint8_t *__restrict__ e1, int32_t *__restrict__ grid)
{
  uint32_t N = c->N, nsymb = c->nsymb;
  uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= nsymb * N) return;
  uint32_t l = gid / N, k = gid % N;
  const uint16_t *row = c->remap + ((size_t)sfi * 14 + l) * N;
  uint32_t code = row[k];
  if (code >= OAI4G_CTL_CODE) return;                 /* no data RE (CRS / control codes included) */
  const cw_dev_t &cw0 = c->cw[0];
  const cw_dev_t &cw1 = c->cw[1];
  bool pil = pilots_of(l, nsymb == 12) != 0;
  if (c->mimo_mode == OAI4G_ALAMOUTI) {
    /* the thread of RE n writes n and its partner: the partner adds the accumulated values
     * of n (dlsch_modulation.c:535-545) */
    if (code & 1u) return;
    const uint32_t k2 = (k + 1 < N && row[k + 1] == (code | 1u)) ? k + 1 : k + 2;
    const uint32_t base = ((code & 0x7FFEu) + c->symbase[sfi][l]) * cw0.Qm;
    uint32_t ba = 0, bb = 0;
    for (uint32_t i = 0; i < cw0.Qm; i++) {
      ba |= (uint32_t)(e0[base + i] == 1) << i;
      bb |= (uint32_t)(e0[base + cw0.Qm + i] == 1) << i;
    }
    uint32_t *g0 = (uint32_t *)grid + l * N, *g1 = g0 + (size_t)nsymb * N;
    const s16x2 n0 = caddw(u2c(g0[k]), alm_ta(ba, cw0, pil)), n1 = caddw(u2c(g1[k]), alm_tb(bb, cw0, pil));
    g0[k] = c2u(n0);
    g1[k] = c2u(n1);
    s16x2 y0, y1;
    alm_pair(n0, n1, 1u, y0, y1);
    g0[k2] = c2u(caddw(u2c(g0[k2]), y0));
    g1[k2] = c2u(caddw(u2c(g1[k2]), y1));
    return;
  }
  uint32_t idx = (code & 0x7FFFu) + c->symbase[sfi][l];
  uint32_t b0 = 0, b1 = 0;
  /* the reference tests x[jj] == 1 per bit: any other byte value reads as 0 */
  for (uint32_t i = 0; i < cw0.Qm; i++) b0 |= (uint32_t)(e0[idx * cw0.Qm + i] == 1) << i;
  s16x2 x0 = qam_map(b0, cw0.Qm, pil ? cw0.qam_b : cw0.qam_a, pil ? cw0.qpsk_b : cw0.qpsk_a);
  s16x2 x1 = (s16x2){0, 0};
  if (c->n_cw > 1 && e1) {
    for (uint32_t i = 0; i < cw1.Qm; i++) b1 |= (uint32_t)(e1[idx * cw1.Qm + i] == 1) << i;
    x1 = qam_map(b1, cw1.Qm, pil ? cw1.qam_b : cw1.qam_a, pil ? cw1.qpsk_b : cw1.qpsk_a);
  }
  for (uint32_t ant = 0; ant < c->n_ant; ant++) {
    s16x2 v = precode(c, ant, code >> 15, x0, x1);
    uint32_t *p = (uint32_t *)grid + (size_t)ant * nsymb * N + l * N + k;
    *p = c2u(caddw(u2c(*p), v));
  }
}

hipError_t oai4g_launch_modulate_bytes(const cfg_dev_t *d_cfg, const cfg_dev_t *h_cfg, int sf, const uint8_t *d_e0,
                                       const uint8_t *d_e1, int32_t *d_grid, hipStream_t s)
{
  uint32_t n = h_cfg->nsymb * h_cfg->N;
  hipLaunchKernelGGL(k_modulate_bytes, dim3((n + 255) / 256), dim3(256), 0, s, d_cfg, sf, d_e0, d_e1, d_grid);
  return hipGetLastError();
}

/* ======================================================================================
 * Drop-in CRS: lte_dl_cell_spec (lte_dl_cell_spec.c:123-203) for a list of OFDM symbols.
 * Thread per (job, m); bin = first_carrier + (nu + nushift) mod 6 + 6m with the DC skip.
 * ==================================================================================== */
__global__ void __launch_bounds__(256) k_crs(int32_t *__restrict__ out, const crs_job_t *__restrict__ jobs,
                                             const uint32_t *__restrict__ gold, int16_t amp, uint32_t N,
                                             uint32_t N_RB, uint32_t nushift, uint32_t first_carrier)
{
  const crs_job_t j = jobs[blockIdx.y];
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= 2 * N_RB) return;
  const uint32_t nu = (j.p == 0) ? (j.l == 0 ? 0u : 3u) : (j.l == 0 ? 3u : 0u);
  uint32_t k = nu + nushift;
  if (k > 5) k -= 6;
  k += first_carrier + 6 * m;
  if (k >= N) k = k + 1 - N;
  const uint32_t mp = 110 - N_RB + m;
  const uint32_t idx = (gold[((uint32_t)j.Ns * 2 + j.l) * 14 + (mp >> 4)] >> (2 * (mp & 15))) & 3u;
  const short a = (short)(((int)amp * 23170) >> 15);
  out[j.off + k] = (int32_t)c2u((s16x2){(short)((idx & 1) ? -a : a), (short)((idx & 2) ? -a : a)});
}

hipError_t oai4g_launch_crs(int32_t *d_out, const crs_job_t *jobs, int n_jobs, const uint32_t *d_gold, int16_t amp,
                            uint32_t N, uint32_t N_RB, uint32_t nushift, uint32_t first_carrier, hipStream_t s)
{
  if (n_jobs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_crs, dim3((2 * N_RB + 255) / 256, n_jobs), dim3(256), 0, s, d_out, jobs, d_gold, amp, N, N_RB,
                     nushift, first_carrier);
  return hipGetLastError();
}

