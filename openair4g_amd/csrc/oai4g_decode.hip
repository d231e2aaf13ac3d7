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
 * The permuted exchanges (pi4 / pi5 of init_td16) are fused into the forward pass of the next
 * half-iteration, which gathers its systematic input and writes it back for its backward pass;
 * the hard decisions (pi6) and the CRC early stop run per block between the half-iterations.
 */
#include "oai4g_internal.h"

#include <type_traits>

typedef const __attribute__((address_space(1))) int16_t gs16_t;

static __device__ __forceinline__ short sadd(short a, short b) { return __builtin_elementwise_add_sat(a, b); }
static __device__ __forceinline__ short ssub(short a, short b) { return __builtin_elementwise_sub_sat(a, b); }

#define TD_MAXH 128    /* MAX / 2 */
#ifndef TD_FS
#define TD_FS 12             /* forward chunk (steps whose operands are loaded one chunk ahead); a multiple of 3
                                (the metric layouts rotate with period 3) */
#endif
#ifndef TD_FSG
#define TD_FSG 12            /* forward chunk of the gathered forms (two loads deep: pi, then the gather);
                                round 4, loads held unpacked: C5 3 -> 192 k, 6 -> 222 k, 9 -> 223 k, 12 -> 229 k */
#endif
#ifndef TD_FSGD
#define TD_FSGD TD_FSG       /* the same for decoder 1's deinterleave + update form (two more streams per step) */
#endif
#ifndef TD_XR
#define TD_XR 32      /* steps per round of the exchange gathers (index loads, then gathers, in flight) */
#endif
#ifndef TD_BPF
#define TD_BPF 2      /* backward pass: segments between an operand fetch and its alpha recompute (1 or 2; decoder 1's form stays at 1) */
#endif
#ifndef TD_SEG
#define TD_SEG 6      /* alpha checkpoint interval (steps), a multiple of 3 so every checkpoint holds layout EO
                         (round 2 measured 4 best of 2/4/8/16 with the fixed layout) */
#endif
static_assert(TD_FS % 3 == 0 && TD_FSG % 3 == 0 && TD_FSGD % 3 == 0, "layout period");
/* TD_SEG == 6: every checkpoint holds layout EO, and the re-run's alpha(0..5) fill exactly segment 0
 * (alpha(6) onward continue the first run); 12 spills */
static_assert(TD_SEG == 6, "checkpoint interval");

/* log_map is not inlined: explicit address spaces keep its scratch accesses global_* / ds_* (a flat
 * access counts on both vmcnt and lgkmcnt and returns out of order, so every wait on one would drain
 * all loads in flight, the one-segment-ahead operand loads included) */
#ifdef TD_NOAS
#define TD_G
#define TD_L
#else
#define TD_G __attribute__((address_space(1)))
#define TD_L __attribute__((address_space(3)))
#endif

struct td_blk_t {      /* one wave's scratch: the 8 blocks interleaved, element i of block g at
                          64 (i >> 3) + 8 g + (i & 7), so a step's loads / stores of the whole
                          wave touch one 128-byte line instead of 8 */
  short *s0, *s1, *s2, *yp1, *yp2, *ext, *ext2;
  uint4 *A;            /* alpha checkpoints: [ceil(K1/TD_SEG) + 2][8 blocks][8 lanes] x 8 states (16 B) */
};

static __device__ __forceinline__ uint32_t td_ix(uint32_t i) { return ((i >> 3) << 6) | (i & 7); }

static __device__ __forceinline__ td_blk_t td_layout(uint8_t *base, uint32_t K)
{
  td_blk_t b;
  short *p = (short *)base;
  const uint32_t n16 = (K + 8 * (TD_FS + TD_SEG) + 16 + 7) & ~7u, n128 = K + 128;   /* read-ahead slack */
  b.s0 = p; p += 8 * n16;
  b.s1 = p; p += 8 * n16;
  b.s2 = p; p += 8 * n16;
  b.yp1 = p; p += 8 * n16;
  b.yp2 = p; p += 8 * n16;
  b.ext = p; p += 8 * n128;
  b.ext2 = p; p += 8 * n128;
  b.A = (uint4 *)(((uintptr_t)p + 15) & ~(uintptr_t)15);
  return b;
}

size_t oai4g_td_block_bytes(uint32_t K)
{
  const size_t n16 = (K + 8 * (TD_FS + TD_SEG) + 16 + 7) & ~7u, n128 = K + 128;
  return (((5 * n16 + 2 * n128) * 2 + 15) & ~(size_t)15) + (size_t)(K / 8 + 1) * 8 * 16 + 256;
}

/* Trellis metrics as four packed int16 pairs: S[0] = (s0, s1), S[1] = (s2, s3), S[2] = (s4, s5),
 * S[3] = (s6, s7).  Saturating packed add/sub (v_pk_add/sub_i16 clamp) and packed max are the
 * reference's adds/subs/max_epi16 lane for lane; x - (-g) == x + g under saturation because
 * |g| <= 16384. */
typedef short s2v __attribute__((ext_vector_type(2)));
static __device__ __forceinline__ s2v adds2(s2v a, s2v b) { return __builtin_elementwise_add_sat(a, b); }
static __device__ __forceinline__ s2v subs2(s2v a, s2v b) { return __builtin_elementwise_sub_sat(a, b); }
static __device__ __forceinline__ s2v max2(s2v a, s2v b) { return __builtin_elementwise_max(a, b); }
#define SHUF2(a, b, i, j) __builtin_shufflevector((a), (b), (i), (j))

struct tm_t { s2v v[4]; };

typedef uint32_t u4v __attribute__((ext_vector_type(4)));   /* checkpoint word in log_map's global / LDS arrays */
static __device__ __forceinline__ u4v tm_packv(const tm_t &t)
{
  return (u4v){__builtin_bit_cast(uint32_t, t.v[0]), __builtin_bit_cast(uint32_t, t.v[1]),
               __builtin_bit_cast(uint32_t, t.v[2]), __builtin_bit_cast(uint32_t, t.v[3])};
}
static __device__ __forceinline__ tm_t tm_unpack(u4v u)
{
  /* the elements go through scalars: clang's __builtin_bit_cast of an ext-vector element lvalue
   * (u.y, u[1]) reads the vector's first element (measured on this toolchain) */
  const uint32_t w0 = u.x, w1 = u.y, w2 = u.z, w3 = u.w;
  tm_t t;
  t.v[0] = __builtin_bit_cast(s2v, w0); t.v[1] = __builtin_bit_cast(s2v, w1);
  t.v[2] = __builtin_bit_cast(s2v, w2); t.v[3] = __builtin_bit_cast(s2v, w3);
  return t;
}
static __device__ __forceinline__ tm_t tm_init(bool zero_first)
{
  tm_t t;
  t.v[0] = (s2v){(short)(zero_first ? 0 : -TD_MAXH), (short)-TD_MAXH};
  t.v[1] = t.v[2] = t.v[3] = (s2v){(short)-TD_MAXH, (short)-TD_MAXH};
  return t;
}

/* forward step (compute_alpha16 :286-367): r0 = max(a1+g11, a0-g11), r1 = max(a3-g10, a2+g10),
 * r2 = max(a5+g10, a4-g10), r3 = max(a7-g11, a6+g11), r4..r7 the opposite signs; minus max.
 * The reference form in the fixed layout N; log_map runs alpha_ph, its layout-rotating restatement
 * (kept as the specification alpha_ph is checked against in review; beta_step / ext_of below still
 * run the backward re-run) */
[[maybe_unused]] static __device__ __forceinline__ void alpha_step(tm_t &a, short g11, short g10)
{
  const s2v G = {g11, (short)-g10}, H = {g10, (short)-g11};
  const s2v x13 = SHUF2(a.v[0], a.v[1], 1, 3), x02 = SHUF2(a.v[0], a.v[1], 0, 2);
  const s2v x57 = SHUF2(a.v[2], a.v[3], 1, 3), x46 = SHUF2(a.v[2], a.v[3], 0, 2);
  const s2v r01 = max2(adds2(x13, G), subs2(x02, G)), r45 = max2(subs2(x13, G), adds2(x02, G));
  const s2v r23 = max2(adds2(x57, H), subs2(x46, H)), r67 = max2(subs2(x57, H), adds2(x46, H));
  const s2v m = max2(max2(r01, r23), max2(r45, r67)), mm = max2(m, SHUF2(m, m, 1, 0));
  a.v[0] = subs2(r01, mm); a.v[1] = subs2(r23, mm); a.v[2] = subs2(r45, mm); a.v[3] = subs2(r67, mm);
}

/* backward step (compute_beta16 :588-685): r0 = max(b4+g11, b0-g11), r1 = max(b4-g11, b0+g11),
 * r2 = max(b5-g10, b1+g10), r3 = max(b5+g10, b1-g10), r4 = max(b6+g10, b2-g10),
 * r5 = max(b6-g10, b2+g10), r6 = max(b7-g11, b3+g11), r7 = max(b7+g11, b3-g11); minus max */
static __device__ __forceinline__ void beta_step(tm_t &b, short g11, short g10)
{
  const s2v G = {g11, (short)-g10}, H = {g10, (short)-g11};
  const s2v r02 = max2(adds2(b.v[2], G), subs2(b.v[0], G)), r13 = max2(subs2(b.v[2], G), adds2(b.v[0], G));
  const s2v r46 = max2(adds2(b.v[3], H), subs2(b.v[1], H)), r57 = max2(subs2(b.v[3], H), adds2(b.v[1], H));
  const s2v m = max2(max2(r02, r13), max2(r46, r57)), mm = max2(m, SHUF2(m, m, 1, 0));
  const s2v n02 = subs2(r02, mm), n13 = subs2(r13, mm), n46 = subs2(r46, mm), n57 = subs2(r57, mm);
  b.v[0] = SHUF2(n02, n13, 0, 2); b.v[1] = SHUF2(n02, n13, 1, 3);
  b.v[2] = SHUF2(n46, n57, 0, 2); b.v[3] = SHUF2(n46, n57, 1, 3);
}

/* extrinsic of one step from alpha(k), beta(k+1), gamma(k) (compute_ext16 :733-875):
 * m00 = max(a0+b0, a1+b4, a6+b7, a7+b3) - g11, m11 = max(a0+b4, a1+b0, a6+b3, a7+b7) + g11,
 * m01 = max(a2+b5, a3+b1, a4+b2, a5+b6) - g10, m10 = max(a2+b1, a3+b5, a4+b6, a5+b2) + g10,
 * ext = max(m10, m11) - max(m01, m00) */
static __device__ __forceinline__ short ext_of(const tm_t &a, const tm_t &b, short g11, short g10)
{
  const s2v p04 = SHUF2(b.v[0], b.v[2], 0, 2), p40 = SHUF2(b.v[2], b.v[0], 0, 2);
  const s2v q73 = SHUF2(b.v[3], b.v[1], 1, 3), q37 = SHUF2(b.v[1], b.v[3], 1, 3);
  const s2v r51 = SHUF2(b.v[2], b.v[0], 1, 3), r15 = SHUF2(b.v[0], b.v[2], 1, 3);
  const s2v s26 = SHUF2(b.v[1], b.v[3], 0, 2), s62 = SHUF2(b.v[3], b.v[1], 0, 2);
  const s2v M00 = max2(adds2(a.v[0], p04), adds2(a.v[3], q73)), M11 = max2(adds2(a.v[0], p40), adds2(a.v[3], q37));
  const s2v M01 = max2(adds2(a.v[1], r51), adds2(a.v[2], s26)), M10 = max2(adds2(a.v[1], r15), adds2(a.v[2], s62));
  s2v T = max2(SHUF2(M00, M11, 0, 2), SHUF2(M00, M11, 1, 3));   /* (m00, m11) */
  s2v U = max2(SHUF2(M01, M10, 0, 2), SHUF2(M01, M10, 1, 3));   /* (m01, m10) */
  T = adds2(T, (s2v){(short)-g11, g11});
  U = adds2(U, (s2v){(short)-g10, g10});
  const s2v V = max2(T, U);                                      /* (max(m00, m01), max(m11, m10)) */
  return __builtin_elementwise_sub_sat(V.y, V.x);
}

template <typename P, typename Q>
static __device__ __forceinline__ void gamma_of(P sys, Q par, uint32_t e, short &g11, short &g10)
{
  const short s = sys[e], p = par[e];
  g11 = (short)(sadd(s, p) >> 1);
  g10 = (short)(ssub(s, p) >> 1);
}

/* ======================================================================================
 * Rotating metric layouts (round 4).  The 8 state metrics live in 4 packed int16 pairs; a
 * step reads its operands as pairs of one register (the same register's halves, swapped or
 * broadcast, cost nothing: VOP3P op_sel) only if the input layout matches the pairs the step
 * forms.  No single layout does for every step, but three do in rotation:
 *   EO = (0,2)(1,3)(4,6)(5,7),  N = (0,1)(2,3)(4,5)(6,7),  L2 = (0,4)(1,5)(2,6)(3,7).
 * alpha (compute_alpha16): EO -> N -> L2 -> EO; beta (compute_beta16): L2 -> N -> EO -> L2;
 * with alpha(k) in layout k mod 3 and beta(k) in layout k mod 3 (EO, N, L2) every extrinsic
 * (compute_ext16) combines alpha(k) and beta(k + 1) in one of the pairs (EO, N), (N, L2),
 * (L2, EO), each of which also has a register-local pairing.  What is left of the per-step
 * permutes are the gamma constants with mixed signs: (g11, -g10) / (g10, -g11) or
 * (g11, -g11) / (g10, -g10) on two steps of three, shared by the alpha, beta and extrinsic of
 * the step.  Every saturating add / sub / max is still the reference's own, state by state.
 * ==================================================================================== */
enum { LY_EO = 0, LY_N = 1, LY_L2 = 2 };
__host__ __device__ constexpr int ly_reg(int L, int s) { return L == LY_N ? s >> 1 : L == LY_EO ? (((s >> 2) << 1) | (s & 1)) : (s & 3); }
__host__ __device__ constexpr int ly_half(int L, int s) { return L == LY_N ? (s & 1) : L == LY_EO ? ((s >> 1) & 1) : (s >> 2); }
__host__ __device__ constexpr int ly_state(int L, int r, int h)
{
  return L == LY_N ? 2 * r + h : L == LY_EO ? (((r >> 1) << 2) | (h << 1) | (r & 1)) : r + 4 * h;
}

/* (x_I, x_J) of a metric vector held in layout L */
template <int L, int I, int J>
static __device__ __forceinline__ s2v ly_pair(const tm_t &t)
{
  constexpr int ri = ly_reg(L, I), rj = ly_reg(L, J), hi = ly_half(L, I), hj = ly_half(L, J);
  if constexpr (ri == rj) return SHUF2(t.v[ri], t.v[ri], hi, hj);
  else return SHUF2(t.v[ri], t.v[rj], hi, 2 + hj);
}

template <int LF, int LT>
static __device__ __forceinline__ tm_t ly_conv(const tm_t &t)
{
  if constexpr (LF == LT) return t;
  else {
    tm_t o;
    o.v[0] = ly_pair<LF, ly_state(LT, 0, 0), ly_state(LT, 0, 1)>(t);
    o.v[1] = ly_pair<LF, ly_state(LT, 1, 0), ly_state(LT, 1, 1)>(t);
    o.v[2] = ly_pair<LF, ly_state(LT, 2, 0), ly_state(LT, 2, 1)>(t);
    o.v[3] = ly_pair<LF, ly_state(LT, 3, 0), ly_state(LT, 3, 1)>(t);
    return o;
  }
}
/* layout change with a run-time (wave-uniform) source layout */
template <int LT>
static __device__ __forceinline__ tm_t ly_conv_from(const tm_t &t, int lf)
{
  return lf == LY_EO ? ly_conv<LY_EO, LT>(t) : lf == LY_N ? ly_conv<LY_N, LT>(t) : ly_conv<LY_L2, LT>(t);
}
template <int LF>
static __device__ __forceinline__ tm_t ly_conv_to(const tm_t &t, int lt)
{
  return lt == LY_EO ? ly_conv<LF, LY_EO>(t) : lt == LY_N ? ly_conv<LF, LY_N>(t) : ly_conv<LF, LY_L2>(t);
}

struct gk_t { s2v gg, ng; };    /* (g11, g10) and (-g11, -g10) (int16 wrap; |g| <= 16384) */
static __device__ __forceinline__ gk_t gk_of(uint32_t ggw)
{
  const s2v g = __builtin_bit_cast(s2v, ggw);
  return {g, (s2v){0, 0} - g};
}
static __device__ __forceinline__ uint32_t gg_of(short sy, short pa)   /* compute_gamma16: (s + p) >> 1, (s - p) >> 1 */
{
  const short g11 = (short)(sadd(sy, pa) >> 1), g10 = (short)(ssub(sy, pa) >> 1);
  return (uint32_t)(uint16_t)g11 | ((uint32_t)(uint16_t)g10 << 16);
}
/* the constant pair (g_A, SB g_B), A / B = 11 or 10 */
template <int GA, int GB, int SB>
static __device__ __forceinline__ s2v kpair(const gk_t &k)
{
  constexpr int ha = GA == 11 ? 0 : 1, hb = GB == 11 ? 0 : 1;
  if constexpr (SB > 0) return SHUF2(k.gg, k.gg, ha, hb);
  else return SHUF2(k.gg, k.ng, ha, 2 + hb);
}

/* the recursions as r_s = max(x[U_s] + S_s g_s, x[W_s] - S_s g_s):
 *   alpha (compute_alpha16 :286-367): U = 1 3 5 7 1 3 5 7, W = U - 1, S = + - + - - + - +, g = 11 10 10 11 11 10 10 11
 *   beta (compute_beta16 :588-685):   U = 4 4 5 5 6 6 7 7, W = U - 4, S = + - - + + - - +, g = 11 11 10 10 10 10 11 11 */
__host__ __device__ constexpr int tr_u(bool beta, int s) { return beta ? 4 + (s >> 1) : 2 * (s & 3) + 1; }
__host__ __device__ constexpr int tr_w(bool beta, int s) { return beta ? (s >> 1) : 2 * (s & 3); }
__host__ __device__ constexpr int tr_s(bool beta, int s) { return (beta ? ((s ^ (s >> 1)) & 1) : ((s & 1) ^ (s >> 2))) ? -1 : 1; }
__host__ __device__ constexpr int tr_g(bool beta, int s) { return beta ? (((s + 2) & 7) < 4 ? 11 : 10) : (((s & 3) == 0 || (s & 3) == 3) ? 11 : 10); }

/* output register O of a step: the constant is taken with a positive first lane, the adds / subs
 * swapped when S is negative there (x - c == x + (-c) under saturation for |c| <= 16384) */
template <bool BETA, int LIN, int LOUT, int O>
static __device__ __forceinline__ s2v tpair(const tm_t &x, const gk_t &k)
{
  constexpr int sa = ly_state(LOUT, O, 0), sb = ly_state(LOUT, O, 1);
  constexpr int sga = tr_s(BETA, sa), sgb = tr_s(BETA, sb);
  const s2v U = ly_pair<LIN, tr_u(BETA, sa), tr_u(BETA, sb)>(x);
  const s2v W = ly_pair<LIN, tr_w(BETA, sa), tr_w(BETA, sb)>(x);
  const s2v C = kpair<tr_g(BETA, sa), tr_g(BETA, sb), sga * sgb>(k);
  if constexpr (sga > 0) return max2(adds2(U, C), subs2(W, C));
  else return max2(subs2(U, C), adds2(W, C));
}
/* one recursion step LIN -> LOUT, normalised by the maximum (the reference's minus max) */
template <bool BETA, int LIN, int LOUT>
static __device__ __forceinline__ void tstep(tm_t &x, const gk_t &k)
{
  const s2v r0 = tpair<BETA, LIN, LOUT, 0>(x, k), r1 = tpair<BETA, LIN, LOUT, 1>(x, k);
  const s2v r2 = tpair<BETA, LIN, LOUT, 2>(x, k), r3 = tpair<BETA, LIN, LOUT, 3>(x, k);
  const s2v m = max2(max2(r0, r1), max2(r2, r3)), mm = max2(m, SHUF2(m, m, 1, 0));
  x.v[0] = subs2(r0, mm); x.v[1] = subs2(r1, mm); x.v[2] = subs2(r2, mm); x.v[3] = subs2(r3, mm);
}
template <int P> static __device__ __forceinline__ void alpha_ph(tm_t &a, const gk_t &k) { tstep<false, P, (P + 1) % 3>(a, k); }
template <int P> static __device__ __forceinline__ void beta_ph(tm_t &b, const gk_t &k) { tstep<true, P, (P + 2) % 3>(b, k); }

/* one packed term pair (a_I + b_J, a_I2 + b_J2) */
template <int LA, int LB, int I, int J, int I2, int J2>
static __device__ __forceinline__ s2v eterm(const tm_t &a, const tm_t &b)
{
  return adds2(ly_pair<LA, I, I2>(a), ly_pair<LB, J, J2>(b));
}
/* compute_ext16 (:733-875) from alpha(k) in layout P and beta(k + 1) in layout (P + 1) mod 3:
 * m00 = max(a0+b0, a1+b4, a6+b7, a7+b3) - g11, m11 = max(a0+b4, a1+b0, a6+b3, a7+b7) + g11,
 * m01 = max(a2+b5, a3+b1, a4+b2, a5+b6) - g10, m10 = max(a2+b1, a3+b5, a4+b6, a5+b2) + g10,
 * ext = max(m10, m11) - max(m01, m00); each packed term takes both its operands from one
 * register of its layout (pairings searched once for the three layout pairs) */
template <int P>
static __device__ __forceinline__ short ext_ph(const tm_t &a, const tm_t &b, const gk_t &k)
{
  constexpr int LA = P, LB = (P + 1) % 3;
  if constexpr (P == LY_EO) {             /* (m00, m10) and (m01, m11) */
    const s2v X = max2(max2(eterm<LA, LB, 0, 0, 2, 1>(a, b), eterm<LA, LB, 1, 4, 3, 5>(a, b)),
                       max2(eterm<LA, LB, 6, 7, 4, 6>(a, b), eterm<LA, LB, 7, 3, 5, 2>(a, b)));
    const s2v Y = max2(max2(eterm<LA, LB, 2, 5, 0, 4>(a, b), eterm<LA, LB, 3, 1, 1, 0>(a, b)),
                       max2(eterm<LA, LB, 4, 2, 6, 3>(a, b), eterm<LA, LB, 5, 6, 7, 7>(a, b)));
    const s2v V = max2(subs2(X, kpair<11, 10, -1>(k)), subs2(Y, kpair<10, 11, -1>(k)));   /* (max(m00, m01), max(m10, m11)) */
    return __builtin_elementwise_sub_sat(V.y, V.x);
  } else if constexpr (P == LY_N) {       /* (m00, m11) and (m01, m10) */
    const s2v X = max2(max2(eterm<LA, LB, 0, 0, 0, 4>(a, b), eterm<LA, LB, 1, 4, 1, 0>(a, b)),
                       max2(eterm<LA, LB, 6, 7, 6, 3>(a, b), eterm<LA, LB, 7, 3, 7, 7>(a, b)));
    const s2v Y = max2(max2(eterm<LA, LB, 2, 5, 2, 1>(a, b), eterm<LA, LB, 3, 1, 3, 5>(a, b)),
                       max2(eterm<LA, LB, 4, 2, 4, 6>(a, b), eterm<LA, LB, 5, 6, 5, 2>(a, b)));
    const s2v V = max2(subs2(X, kpair<11, 11, -1>(k)), subs2(Y, kpair<10, 10, -1>(k)));   /* (max(m00, m01), max(m11, m10)) */
    return __builtin_elementwise_sub_sat(V.y, V.x);
  } else {                                /* (m00, m01) and (m10, m11) */
    const s2v X = max2(max2(eterm<LA, LB, 0, 0, 4, 2>(a, b), eterm<LA, LB, 1, 4, 5, 6>(a, b)),
                       max2(eterm<LA, LB, 6, 7, 2, 5>(a, b), eterm<LA, LB, 7, 3, 3, 1>(a, b)));
    const s2v Y = max2(max2(eterm<LA, LB, 2, 1, 6, 3>(a, b), eterm<LA, LB, 3, 5, 7, 7>(a, b)),
                       max2(eterm<LA, LB, 4, 6, 0, 4>(a, b), eterm<LA, LB, 5, 2, 1, 0>(a, b)));
    const s2v Xg = subs2(X, kpair<11, 10, 1>(k)), Yg = adds2(Y, kpair<10, 11, 1>(k));
    const s2v Xm = max2(Xg, SHUF2(Xg, Xg, 1, 0)), Ym = max2(Yg, SHUF2(Yg, Yg, 1, 0));
    return __builtin_elementwise_sub_sat(Ym.x, Xm.x);
  }
}

/* compile-time loop (the layout phase of step J is J mod 3) */
template <int B, int E, class F>
static __device__ __forceinline__ void sfor(F &&f)
{
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    sfor<B + 1, E>(f);
  }
}
template <int B, int E, class F>      /* E - 1 down to B */
static __device__ __forceinline__ void sfor_down(F &&f)
{
  if constexpr (B < E) {
    f(std::integral_constant<int, E - 1>{});
    sfor_down<B, E - 1>(f);
  }
}

/*
 * log_map16 for the calling lane (window q of its block): sys / par in the reference's vector
 * layout (element 8k + q), extrinsic out likewise.  Lanes of a block exchange re-run seeds with
 * width-8 shuffles; the 8 lanes of a block are always active together.
 *
 * Alpha is not stored per step: the forward pass keeps checkpoints alpha(S c) (those with
 * S c <= 5, c = 0 included, from the re-run) plus the first run's alpha(5), and the backward
 * pass recomputes each S-step segment into registers together with its gammas, reproducing the
 * reference's mix exactly: alpha(0..5) from the re-run, alpha(6..) from the first run.  The
 * alphas of the last 6 steps, needed again by the backward re-run, wait in LDS (asave).
 */
/* Not inlined: one copy for the three call sites keeps the kernel at 2 waves per SIMD.
 * POST: the stored extrinsic is already the next half-iteration's input, ext - sys + s0
 * (the loop's update pass of phy_threegpplte_turbo_decoder16, fused into the store) */
/* SRC: where the forward pass takes the systematic input of step k (element 8k + q) from.
 *   TD_SRC_SYS:  sys[] as stored;
 *   TD_SRC_INTL: decoder 2's input, ext[pi4] gathered (the interleave exchange of the loop);
 *   TD_SRC_DINT: decoder 1's input, ext2[pi5] - ext + s0 (the deinterleave + update pass).
 * The gathered forms are written to sys[] as they are consumed, for the backward pass: the
 * exchange passes and their re-reads of the exchanged stream disappear. */
enum { TD_SRC_SYS = 0, TD_SRC_INTL = 1, TD_SRC_DINT = 2 };
/* W: the residency of the kernel that calls it (one noinline copy per kernel, so each gets its
 * caller's register budget) */
template <int WV, bool POST, int SRC>
static __device__ __attribute__((noinline)) void log_map(TD_G short *sys, TD_G const short *par, TD_G short *ext,
                                               TD_G u4v *A, uint32_t K, uint32_t q, int tf,
                                               TD_L u4v *asave /* [6][64] */, TD_G const short *s0,
                                               TD_G const short *gsrc, TD_G const uint16_t *pi)
{
  /* a noinline function receives its arguments in VGPRs: re-establish that K and tf are wave-uniform,
   * so the per-step bounds tests become scalar branches instead of exec-mask juggling */
  K = __builtin_amdgcn_readfirstlane(K);
  tf = __builtin_amdgcn_readfirstlane(tf);
  /* Every global operand of a step is loaded one chunk ahead into registers: the loads are
   * independent of the recursions, but the compiler cannot hoist them across the (possibly
   * aliasing) ext / checkpoint stores, so without this each step waits a full memory latency. */
  const uint32_t K1 = K >> 3, nseg = (K1 + TD_SEG - 1) / TD_SEG, lane = threadIdx.x & 63;
  const int pK = (int)(K1 % 3);                /* layout of alpha(K1) and beta(K1) */
  /* forward, first run, in chunks of FS steps (operands of the next chunk in flight); alpha(k) is
   * in layout k mod 3 (alpha(0) EO: tm_init puts state 0 at register 0's low half in every layout) */
  constexpr int FS = SRC == TD_SRC_SYS ? TD_FS : (SRC == TD_SRC_INTL ? TD_FSG : TD_FSGD);
  const uint32_t nfc = (K1 + FS - 1) / FS;
  tm_t a = tm_init(q == 0);
  {
    /* operands stay one 16-bit value per register until their step: packing two loads into one
     * register right after they are issued would wait on them there, a memory latency per chunk */
    short nsy[FS], npa[FS];                     /* sys, par of the next chunk */
    uint32_t nix[FS];                           /* gathered forms: pi of the chunk after next */
    short nex[FS], nzs[FS];                     /* TD_SRC_DINT: ext, s0 of the next chunk */
    auto pix = [&](uint32_t k) { return (uint32_t)pi[8 * (k < K1 ? k : K1 - 1) + q]; };
    if constexpr (SRC == TD_SRC_SYS) {
#pragma unroll
      for (int j = 0; j < FS; j++) { nsy[j] = sys[64 * j + q]; npa[j] = par[64 * j + q]; }
    } else {
      uint32_t ix0[FS];
#pragma unroll
      for (int j = 0; j < FS; j++) ix0[j] = pix(j);
#pragma unroll
      for (int j = 0; j < FS; j++) nix[j] = pix(FS + j);
#pragma unroll
      for (int j = 0; j < FS; j++) { nsy[j] = gsrc[td_ix(ix0[j])]; npa[j] = par[64 * j + q]; }
      if constexpr (SRC == TD_SRC_DINT) {
#pragma unroll
        for (int j = 0; j < FS; j++) { nex[j] = ext[64 * j + q]; nzs[j] = s0[64 * j + q]; }
      }
    }
    for (uint32_t c = 0; c < nfc; c++) {
      short csy[FS], cpa[FS], cex[FS], czs[FS];
#pragma unroll
      for (int j = 0; j < FS; j++) { csy[j] = nsy[j]; cpa[j] = npa[j]; }
      if constexpr (SRC == TD_SRC_DINT) {
#pragma unroll
        for (int j = 0; j < FS; j++) { cex[j] = nex[j]; czs[j] = nzs[j]; }
      }
      if (c + 1 < nfc) {
        const uint32_t b = 64 * FS * (c + 1) + q;
        if constexpr (SRC == TD_SRC_SYS) {
#pragma unroll
          for (int j = 0; j < FS; j++) { nsy[j] = sys[b + 64 * j]; npa[j] = par[b + 64 * j]; }
        } else {
          uint32_t ix[FS];
#pragma unroll
          for (int j = 0; j < FS; j++) ix[j] = nix[j];
#pragma unroll
          for (int j = 0; j < FS; j++) nix[j] = pix(FS * (c + 2) + j);
#pragma unroll
          for (int j = 0; j < FS; j++) { nsy[j] = gsrc[td_ix(ix[j])]; npa[j] = par[b + 64 * j]; }
          if constexpr (SRC == TD_SRC_DINT) {
#pragma unroll
            for (int j = 0; j < FS; j++) { nex[j] = ext[b + 64 * j]; nzs[j] = s0[b + 64 * j]; }
          }
        }
      }
      const bool full = c * FS + FS <= K1;     /* uniform: only the last chunk may be partial */
      sfor<0, FS>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t k = c * FS + j;
        if (full || k < K1) {
          if constexpr (SRC == TD_SRC_DINT) csy[j] = sadd(ssub(csy[j], cex[j]), czs[j]);
          if constexpr (SRC != TD_SRC_SYS) sys[64 * k + q] = csy[j];
          alpha_ph<j % 3>(a, gk_of(gg_of(csy[j], cpa[j])));
          if ((k + 1) % TD_SEG == 0) A[64 * ((k + 1) / TD_SEG) + q] = tm_packv(a);   /* layout EO */
        }
      });
    }
  }
  /* forward re-run over L/8 steps from the previous window's final alpha; its alpha(0) is
   * checkpoint 0, alpha(1..5) are recomputed from it (TD_SEG > 5: no checkpoint inside) */
  const tm_t fin = a;                          /* alpha(K1), layout pK */
  {
    const tm_t z = tm_init(true);
#pragma unroll
    for (int v = 0; v < 4; v++) {
      const uint32_t up = (uint32_t)__shfl_up((int)__builtin_bit_cast(uint32_t, a.v[v]), 1, 8);
      a.v[v] = q == 0 ? z.v[v] : __builtin_bit_cast(s2v, up);
    }
    a = ly_conv_from<LY_EO>(a, pK);            /* (z is the same in every layout) */
  }
  A[q] = tm_packv(a);
  sfor<0, 5>([&](auto J) {
    constexpr int k = decltype(J)::value;
    alpha_ph<k % 3>(a, gk_of(gg_of(sys[64 * k + q], par[64 * k + q])));
  });
  /* termination betas of the last window (compute_beta16 :467-521, int16 wrap arithmetic), layout N */
  tm_t t;
  {
    short m[3], mm[3], tv[8];
#pragma unroll
    for (int j = 0; j < 3; j++) gamma_of(sys + 64 * tf, par, 64 * K1 + j, m[j], mm[j]);   /* m_11/m_10[n + j] */
    short beta0 = (short)-m[2], beta1 = m[2];
    short b0_2 = (short)(beta0 - m[1]), b1_2 = (short)(beta0 + m[1]), b2_2 = (short)(beta1 + mm[1]),
          b3_2 = (short)(beta1 - mm[1]);
    tv[0] = (short)(b0_2 - m[0]); tv[1] = (short)(b0_2 + m[0]); tv[2] = (short)(b1_2 + mm[0]); tv[3] = (short)(b1_2 - mm[0]);
    tv[4] = (short)(b2_2 - mm[0]); tv[5] = (short)(b2_2 + mm[0]); tv[6] = (short)(b3_2 + m[0]); tv[7] = (short)(b3_2 - m[0]);
    short bm = tv[0];
#pragma unroll
    for (int s = 1; s < 8; s++) bm = bm > tv[s] ? bm : tv[s];
#pragma unroll
    for (int v = 0; v < 4; v++) t.v[v] = (s2v){(short)(tv[2 * v] - bm), (short)(tv[2 * v + 1] - bm)};
  }
  /* backward, first run: seeded with the lane's own final alpha as the reference stores it
   * after the re-run (the re-run reaches step K1 when K1 == 5); extrinsic of steps whose beta
   * the re-run does not touch.  beta(k) is in layout k mod 3, so beta(K1) shares alpha(K1)'s.
   * Segment operands (sys, par, s0, checkpoint) one segment ahead. */
  tm_t b = q == 7 ? ly_conv_to<LY_N>(t, pK) : (K1 == 5 ? a : fin);
  const int kr = (int)K1 - 6;                 /* steps >= kr take their extrinsic from the re-run */
  const int nfast = kr > 0 ? kr / TD_SEG : 0;  /* segments [0, nfast) lie wholly below kr */
  /* a segment's operands as loaded: sys, par, (POST) s0 and its alpha checkpoint, one 16-bit value
   * per register until they are taken */
  struct bundle_t {
    short sy[TD_SEG], pa[TD_SEG], zs[TD_SEG];
    u4v A;
  };
  auto fetch = [&](bundle_t &d, int seg) {
    const uint32_t b0 = 64u * (uint32_t)(seg * TD_SEG) + q;
#pragma unroll
    for (int j = 0; j < TD_SEG; j++) { d.sy[j] = sys[b0 + 64 * j]; d.pa[j] = par[b0 + 64 * j]; }
    if constexpr (POST) {
#pragma unroll
      for (int j = 0; j < TD_SEG; j++) d.zs[j] = s0[b0 + 64 * j];
    }
    d.A = A[64 * seg + q];
  };
  /* a segment's operands in registers: gammas, and (POST) its sys and s0 */
  struct segops_t {
    uint32_t gg[TD_SEG];                       /* g11 | g10 << 16 */
    s2v sz[TD_SEG];                            /* (POST) (sys, s0), packed once the loads have landed */
  };
  auto take = [&](segops_t &o, const bundle_t &d) {
#pragma unroll
    for (int j = 0; j < TD_SEG; j++) {
      o.gg[j] = gg_of(d.sy[j], d.pa[j]);
      if constexpr (POST) o.sz[j] = (s2v){d.sy[j], d.zs[j]};
    }
  };
  /* extrinsic of step k0 + j from alpha (layout j mod 3) and beta(k0 + j + 1) */
  auto emit = [&](auto J, const segops_t &o, const u4v &al, int k0) {
    constexpr int j = decltype(J)::value;
    short v = ext_ph<j % 3>(tm_unpack(al), b, gk_of(o.gg[j]));
    if constexpr (POST) {
      v = __builtin_elementwise_add_sat(__builtin_elementwise_sub_sat(v, o.sz[j].x), o.sz[j].y);
    }
    ext[64 * (k0 + j) + q] = v;
  };
  /* backward prefetch distance: decoder 1's form (POST) holds two more operand streams and has no
   * registers left for a second bundle */
  constexpr int BPF = POST ? 1 : TD_BPF;
  bundle_t bx, by;                             /* operands in flight: the next segment (and, BPF = 2, the one after) */
  fetch(bx, (int)nseg - 1);
  /* top segments (partial, or holding steps >= kr): guarded steps, alpha recompute then beta */
  for (int seg = (int)nseg - 1; seg >= nfast; seg--) {
    const int k0 = seg * TD_SEG, n = min((int)TD_SEG, (int)K1 - k0);
    /* a partial last segment reads padding past K1 (the arrays have TD_SEG steps of slack) and
     * leaves beta untouched for those steps */
    segops_t o;
    u4v al[TD_SEG];
    tm_t c = tm_unpack(bx.A);                  /* alpha(k0), layout EO */
    take(o, bx);
    if (seg > 0) fetch(bx, seg - 1);
    sfor<0, TD_SEG>([&](auto J) {
      constexpr int j = decltype(J)::value;
      al[j] = tm_packv(c);
      alpha_ph<j % 3>(c, gk_of(o.gg[j]));
    });
    sfor_down<0, TD_SEG>([&](auto J) {
      constexpr int j = decltype(J)::value;
      if (j < n) {
        const int k = k0 + j;
        if (k < kr) emit(J, o, al[j], k0);
        else asave[(k - kr) * 64 + lane] = al[j];   /* layout k mod 3 */
        beta_ph<(j + 1) % 3>(b, gk_of(o.gg[j]));      /* beta(k + 1) -> beta(k) */
      }
    });
  }
  /* full segments below kr, software-pipelined: the beta / extrinsic steps of segment seg
   * interleave with the alpha recompute of segment seg - 1 (two independent dependency chains
   * per lane); operands TD_BPF segments ahead of their alpha recompute, in alternating bundles */
  if (nfast > 0) {
    segops_t cur, nx;
    u4v alc[TD_SEG], aln[TD_SEG];
    {
      tm_t c = tm_unpack(bx.A);
      take(cur, bx);
      if (nfast > 1) fetch(bx, nfast - 2);
      if constexpr (BPF > 1) {
        if (nfast > 2) fetch(by, nfast - 3);
      }
      sfor<0, TD_SEG>([&](auto J) {
        constexpr int j = decltype(J)::value;
        alc[j] = tm_packv(c);
        alpha_ph<j % 3>(c, gk_of(cur.gg[j]));
      });
    }
    /* one segment: bt holds segment seg - 1's operands; it is refilled BPF + 1 segments down */
    auto step_seg = [&](int seg, bundle_t &bt) {
      const int k0 = seg * TD_SEG;
      tm_t c = tm_unpack(bt.A);                /* alpha((seg - 1) TD_SEG) */
      take(nx, bt);
      if (seg > BPF) fetch(bt, seg - 1 - BPF);
      sfor<0, TD_SEG>([&](auto J) {
        constexpr int j = decltype(J)::value;
        constexpr int jj = TD_SEG - 1 - j;
        aln[j] = tm_packv(c);
        alpha_ph<j % 3>(c, gk_of(nx.gg[j]));
        emit(std::integral_constant<int, jj>{}, cur, alc[jj], k0);
        beta_ph<(jj + 1) % 3>(b, gk_of(cur.gg[jj]));
      });
      cur = nx;
#pragma unroll
      for (int j = 0; j < TD_SEG; j++) alc[j] = aln[j];
    };
    int seg = nfast - 1;
    if constexpr (BPF > 1) {
      for (; seg >= 2; seg -= 2) {
        step_seg(seg, bx);
        step_seg(seg - 1, by);
      }
      if (seg == 1) step_seg(1, bx);
    } else {
      for (; seg >= 1; seg--) step_seg(seg, bx);
    }
    sfor_down<0, TD_SEG>([&](auto J) {
      constexpr int j = decltype(J)::value;
      emit(J, cur, alc[j], 0);
      beta_ph<(j + 1) % 3>(b, gk_of(cur.gg[j]));
    });
  }
  /* backward re-run over the last L/8 steps from the next window's beta[0] (layout EO), in the
   * fixed layout N (alpha_step / beta_step / ext_of): 6 steps per call */
  tm_t bn;
#pragma unroll
  for (int v = 0; v < 4; v++) {
    const uint32_t dn = (uint32_t)__shfl_down((int)__builtin_bit_cast(uint32_t, b.v[v]), 1, 8);
    bn.v[v] = __builtin_bit_cast(s2v, dn);
  }
  bn = ly_conv<LY_EO, LY_N>(bn);
  if (q == 7) bn = t;
  for (int k = (int)K1 - 1; k >= kr && k >= 0; k--) {
    const uint32_t e = 64 * k + q;
    short g11, g10;
    gamma_of(sys, par, e, g11, g10);
    const tm_t av = ly_conv_from<LY_N>(tm_unpack(asave[(k - kr) * 64 + lane]), k % 3);
    short v = ext_of(av, bn, g11, g10);
    if constexpr (POST) v = __builtin_elementwise_add_sat(__builtin_elementwise_sub_sat(v, sys[e]), s0[e]);
    ext[e] = v;
    if (k >= (int)K1 - 5) beta_step(bn, g11, g10);
  }
}

/* a * b mod P over GF(2) for the 24-bit CRC generators (P without its x^24 term) */
__device__ static __forceinline__ uint32_t td_mulmod(uint32_t a, uint32_t b, uint32_t poly)
{
  uint32_t r = 0;
  for (int i = 23; i >= 0; i--) {
    r <<= 1;
    if (r & 0x1000000u) r ^= 0x1000000u | poly;
    if ((b >> i) & 1u) r ^= a;
  }
  return r;
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

#ifndef TD16_W3_MIN_CB
/* Residency per launch size.  k_td16_w3 asks for 3 waves per SIMD (168 VGPRs; the
 * scratch of log_map's copies is its callee-saved VGPRs, saved once per call in the prologue, not
 * spills in the step loops); k_td16 leaves the choice to the compiler (2 waves, 252 VGPRs).  3 waves
 * lose at 4096-8192 subframes per launch and win from 12288 on (profiles/c5_batch_r05.txt), so the
 * 3-wave kernel runs from 12288 subframes = 98 304 blocks. */
#define TD16_W3_MIN_CB 98304
#endif

/*
 * Batch decoder: blockIdx.x decodes blocks 8 blockIdx.x .. +7 (one 64-lane wave).
 * llr: [..][llr_stride] int16 (3K + 12 each), out: [..][out_stride] bytes, iters: [..].  Block cb
 * of the launch lives at slot (cb / cg) c_per + r0 + cb % cg of those arrays: the identity for
 * cg = c_per = 1, r0 = 0; the code blocks r0 .. r0 + cg - 1 of every transport block of a
 * [tb][C] batch otherwise (one launch per block size).
 */
template <int WV>
static __device__ __forceinline__ void td16_body(int n_cb, uint32_t K, const int16_t *__restrict__ llr, size_t llr_stride,
                                                 uint8_t *__restrict__ out, size_t out_stride, uint8_t *__restrict__ iters,
                                                 uint32_t max_it, uint32_t crc_type, uint32_t F,
                                                 const uint16_t *__restrict__ pi4, const uint16_t *__restrict__ pi5,
                                                 const uint16_t *__restrict__ pi6, uint8_t *__restrict__ scratch,
                                                 size_t blk_bytes, uint32_t cg, uint32_t c_per, uint32_t r0)
{
  __shared__ uint32_t crctab[256];
  __shared__ uint8_t dec[8][6144 / 8 + 8];
  __shared__ uint32_t done_it[8];
  __shared__ uint4 asave[6 * 64];
  const uint32_t lane = threadIdx.x, g = lane >> 3, q = lane & 7;
  const int cbl = (int)(blockIdx.x * 8 + g);
  const bool valid = cbl < n_cb;
  const size_t cb = (size_t)(cbl / (int)cg) * c_per + r0 + (uint32_t)cbl % cg;   /* slot in llr / out / iters */
  const uint32_t K1 = K >> 3, Kb = K >> 3;
  td_crc_tab(crctab, crc_type == 0 ? 0x864cfbu : 0x800063u);
  /* CRC early stop split over the block's 8 lanes: chunk length, and lane q's multiplier
   * x^(8 cl (7 - q)) mod P (square and multiply, once per launch) */
  const uint32_t crc_poly = crc_type == 0 ? 0x864cfbu : 0x800063u;
  const uint32_t crc_s0 = crc_type == 0 ? (F >> 3) : 0;
  const uint32_t crc_nb = crc_type == 0 ? (K - 24 - F) >> 3 : (K - 24) >> 3;
  const uint32_t crc_cl = (crc_nb + 7) >> 3;
  uint32_t crc_mq = 1;
  {
    uint32_t base = 0x100u, n = crc_cl * (7 - (threadIdx.x & 7));
    while (n) {
      if (n & 1u) crc_mq = td_mulmod(crc_mq, base, crc_poly);
      base = td_mulmod(base, base, crc_poly);
      n >>= 1;
    }
  }
  if (lane < 8) done_it[lane] = 0;
#ifdef TD_DIAG_L2
  /* DIAGNOSTIC ONLY (wrong results): the waves of a launch share TD_DIAG_L2 scratch regions, so the
   * whole scratch working set stays in the L2s and the launch time is the kernel's no-HBM floor */
  const td_blk_t W = td_layout(scratch + (size_t)(blockIdx.x % TD_DIAG_L2) * 8 * blk_bytes, K);
#else
  const td_blk_t W = td_layout(scratch + (size_t)blockIdx.x * 8 * blk_bytes, K);
#endif
  td_blk_t B;   /* this lane's block: element i at td_ix(i) */
  B.s0 = W.s0 + 8 * g; B.s1 = W.s1 + 8 * g; B.s2 = W.s2 + 8 * g; B.yp1 = W.yp1 + 8 * g; B.yp2 = W.yp2 + 8 * g;
  B.ext = W.ext + 8 * g; B.ext2 = W.ext2 + 8 * g; B.A = W.A + 8 * g;
  if (valid) {
    /* demux (:1038-1158): bit i = window q, step v -> element 8v + q */
    gs16_t *y = (gs16_t *)(llr + cb * llr_stride);
    for (uint32_t v0 = 0; v0 < K1; v0 += 8) {   /* 8 steps per round: all loads, then all stores */
      short t0[8], t1[8], t2[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const uint32_t i = q * K1 + (v0 + u < K1 ? v0 + u : K1 - 1);
        t0[u] = y[3 * i];
        t1[u] = y[3 * i + 1];
        t2[u] = y[3 * i + 2];
      }
#pragma unroll
      for (int u = 0; u < 8; u++)
        if (v0 + u < K1) {
          const uint32_t j = 64 * (v0 + u) + q;
          B.s0[j] = t0[u];
          B.yp1[j] = t1[u];
          B.yp2[j] = t2[u];
        }
    }
    if (q == 0) {
      for (uint32_t i = 0; i < 3; i++) {   /* tails (:1164-1186) */
        const short s_a = y[3 * K + 2 * i], p_a = y[3 * K + 2 * i + 1];
        const short s_b = y[3 * K + 6 + 2 * i], p_b = y[3 * K + 6 + 2 * i + 1];
        const uint32_t ia = 64 * K1 + i, ib = 64 * (K1 + 1) + i;
        B.s0[ia] = B.s1[ia] = B.s2[ia] = s_a;
        B.yp1[ia] = p_a;
        B.s0[ib] = B.s1[ib] = B.s2[ib] = s_b;
        B.yp2[ia] = p_b;
      }
    }
  }
  __syncthreads();
  bool active = valid && max_it > 0;
  if (valid) log_map<WV, false, TD_SRC_SYS>((TD_G short *)B.s0, (TD_G short *)B.yp1, (TD_G short *)B.ext, (TD_G u4v *)B.A, K, q, 0,
                                        (TD_L u4v *)asave, (TD_G short *)B.s0, nullptr, nullptr);
  __syncthreads();
  uint32_t it = 0;
  for (it = 1; it <= max_it; it++) {
    /* decoder 2 takes ext[pi4] straight from decoder 1's output (interleave exchange fused) */
    if (active) log_map<WV, false, TD_SRC_INTL>((TD_G short *)B.s2, (TD_G short *)B.yp2, (TD_G short *)B.ext2, (TD_G u4v *)B.A, K, q,
                                                  1, (TD_L u4v *)asave, (TD_G short *)B.s0, (TD_G short *)B.ext,
                                                  (TD_G const uint16_t *)pi4);
    __syncthreads();
    if (active && it > 1) {
      for (uint32_t i0 = q; i0 < Kb; i0 += 8 * (TD_XR / 8)) {   /* hard decisions (:1267-1283), MSB first */
        uint32_t ix[TD_XR];
        short x[TD_XR];
#pragma unroll
        for (int u = 0; u < TD_XR; u++) {
          const uint32_t i = i0 + 8 * (u >> 3);
          ix[u] = i < Kb ? pi6[8 * i + (u & 7)] : 0u;
        }
#pragma unroll
        for (int u = 0; u < TD_XR; u++) x[u] = B.ext2[td_ix(ix[u])];
#pragma unroll
        for (int h = 0; h < TD_XR / 8; h++) {
          const uint32_t i = i0 + 8 * h;
          uint32_t byte = 0;
#pragma unroll
          for (int bb = 0; bb < 8; bb++) byte |= (uint32_t)(x[8 * h + bb] > 0) << (7 - bb);
          if (i < Kb) {
            dec[g][i] = (uint8_t)byte;
            out[cb * out_stride + i] = (uint8_t)byte;
          }
        }
      }
    }
    __syncthreads();
    if (active && it > 1) {                      /* CRC early stop (:1304-1351) */
      /* the block's 8 lanes each run the byte table over one chunk (chunks aligned to the end, the
       * zero bytes in front of the first leave the zero register unchanged), multiply it into
       * place by x^(8 cl (7 - q)) and XOR-reduce: a chain of nbytes / 8 table reads, not nbytes */
      const uint32_t clen = 3;
      const int st = (int)(q * crc_cl) - (int)(8 * crc_cl - crc_nb);
      uint32_t reg = 0;
      for (uint32_t i = 0; i < crc_cl; i++) {
        const int ix = st + (int)i;
        const uint32_t by = ix >= 0 ? dec[g][crc_s0 + (uint32_t)ix] : 0u;
        reg = ((reg << 8) & 0xffffffu) ^ crctab[((reg >> 16) ^ by) & 0xffu];
      }
      reg = td_mulmod(reg, crc_mq, crc_poly);
      reg ^= (uint32_t)__shfl_xor((int)reg, 1, 8);
      reg ^= (uint32_t)__shfl_xor((int)reg, 2, 8);
      reg ^= (uint32_t)__shfl_xor((int)reg, 4, 8);
      if (q == 0) {
        const uint32_t oldcrc = (uint32_t)dec[g][Kb - clen] | ((uint32_t)dec[g][Kb - clen + 1] << 8) |
                                ((uint32_t)dec[g][Kb - clen + 2] << 16);
        const uint32_t crc = ((reg & 0xffu) << 16) | (reg & 0xff00u) | ((reg >> 16) & 0xffu);
        if (crc == oldcrc && crc != 0) done_it[g] = it;
      }
    }
    __syncthreads();
    if (active && done_it[g]) active = false;
    /* decoder 1 takes ext2[pi5] - ext + s0 (deinterleave + update fused) */
    if (active && it < max_it) log_map<WV, true, TD_SRC_DINT>((TD_G short *)B.s1, (TD_G short *)B.yp1, (TD_G short *)B.ext, (TD_G u4v *)B.A,
                                                            K, q, 0, (TD_L u4v *)asave, (TD_G short *)B.s0,
                                                            (TD_G short *)B.ext2, (TD_G const uint16_t *)pi5);
    __syncthreads();
    if (!__any(active)) break;
  }
  if (valid && q == 0) iters[cb] = (uint8_t)(done_it[g] ? done_it[g] : max_it + 1);
}

#define TD16_PARAMS                                                                                                 \
  int n_cb, uint32_t K, const int16_t *__restrict__ llr, size_t llr_stride, uint8_t *__restrict__ out, size_t out_stride, \
      uint8_t *__restrict__ iters, uint32_t max_it, uint32_t crc_type, uint32_t F, const uint16_t *__restrict__ pi4,   \
      const uint16_t *__restrict__ pi5, const uint16_t *__restrict__ pi6, uint8_t *__restrict__ scratch, size_t blk_bytes, \
      uint32_t cg, uint32_t c_per, uint32_t r0
#define TD16_ARGS n_cb, K, llr, llr_stride, out, out_stride, iters, max_it, crc_type, F, pi4, pi5, pi6, scratch, blk_bytes, cg, c_per, r0
__global__ void __launch_bounds__(64) k_td16(TD16_PARAMS) { td16_body<0>(TD16_ARGS); }
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3, 3))) k_td16_w3(TD16_PARAMS)
{
  td16_body<3>(TD16_ARGS);
}

hipError_t oai4g_launch_td16(int n_cb, uint32_t K, const int16_t *d_llr, size_t llr_stride, uint8_t *d_out,
                             size_t out_stride, uint8_t *d_iters, uint32_t max_it, uint32_t crc_type, uint32_t F,
                             const uint16_t *d_pi, uint8_t *d_scratch, hipStream_t s, uint32_t cg, uint32_t c_per,
                             uint32_t r0)
{
  if (n_cb <= 0) return hipSuccess;
  if (n_cb >= TD16_W3_MIN_CB)
    hipLaunchKernelGGL(k_td16_w3, dim3((n_cb + 7) / 8), dim3(64), 0, s, n_cb, K, d_llr, llr_stride, d_out, out_stride,
                       d_iters, max_it, crc_type, F, d_pi, d_pi + K, d_pi + 2 * K, d_scratch, oai4g_td_block_bytes(K), cg,
                       c_per, r0);
  else
    hipLaunchKernelGGL(k_td16, dim3((n_cb + 7) / 8), dim3(64), 0, s, n_cb, K, d_llr, llr_stride, d_out, out_stride,
                       d_iters, max_it, crc_type, F, d_pi, d_pi + K, d_pi + 2 * K, d_scratch, oai4g_td_block_bytes(K), cg,
                       c_per, r0);
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

/* ulsch_decoding's per-block RX chain fused (ulsch_decoding.c:1208-1287), one thread per entry i of
 * code block j's deinterleaved d buffer (blockIdx.y = j: tb = j / C, r = j % C), so the stores are
 * contiguous.  sub_block_deinterleaving_turbo puts w[k] at d1[index3], w[Kpi + 2k] at
 * d1[index3 + 1] and w[Kpi + 2k + 1] at d1[index3 + 5] (index3 = 3 bitrev5(col) + 96 row,
 * k = col R + row, d1 = dfull + 96 - 3 ND); inverting that gives the w position p of entry i, whose
 * value is lte_rate_matching_turbo_rx's (clear = 1): the int16 wrap sum of the soft inputs the
 * circular selection maps to p, 0 for NULL positions.  d1[2] is never written (the reference's
 * prefix slot), d1[3 Kpi + 2] is the d[3D + 2] entry the +5 of the last column produces. */
__global__ void __launch_bounds__(256) k_ul_rm_deint(const ul_dev_t *__restrict__ c, const int16_t *__restrict__ e,
                                                     size_t e_stride, int16_t *__restrict__ dfull, size_t d_stride,
                                                     uint32_t j0)
{
  const uint32_t j = j0 + blockIdx.y, tb = j / c->C, r = j - tb * c->C;
  const ul_pat_t &P = c->pat[c->pat_of[r]];
  const uint32_t R = P.R, Kpi = R << 5, i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 3 * Kpi + 3 || i == 2) return;
  const uint32_t sft = i % 3, base = sft == 2 ? i - 5 : i, row = base / 96, cp = (base % 96) / 3;
  if (row >= R) return;
  const uint32_t k = (__builtin_bitreverse32(cp) >> 27) * R + row;
  const uint32_t p = sft == 0 ? k : Kpi + 2 * k + (sft == 2 ? 1 : 0);
  int16_t acc = 0;
  if (p < P.Ncb && P.dummy[p] != OAI4G_LTE_NULL) {
    const int16_t *soft = e + tb * e_stride + c->off[r];
    const uint32_t ci = P.cidx[p], E = c->E[r];
    for (uint32_t q = ci >= P.k0c ? ci - P.k0c : ci + P.Nnn - P.k0c; q < E; q += P.Nnn) acc = (int16_t)(acc + soft[q]);
  }
  dfull[(size_t)j * d_stride + 96 - 3 * (Kpi - P.D) + i] = acc;
}

/* k_ul_rm_deint with the block's E soft inputs staged in LDS first (one coalesced pass; the
 * deinterleaved order gathers them at stride ~R otherwise, one 128-byte line per few useful bytes):
 * one workgroup per row j = (tb, r) */
__global__ void __launch_bounds__(256) k_ul_rm_deint_lds(const ul_dev_t *__restrict__ c, const int16_t *__restrict__ e,
                                                         size_t e_stride, int16_t *__restrict__ dfull, size_t d_stride)
{
  extern __shared__ int16_t sb[];
  const uint32_t j = blockIdx.x, tb = j / c->C, r = j - tb * c->C;
  const ul_pat_t &P = c->pat[c->pat_of[r]];
  const uint32_t R = P.R, Kpi = R << 5, E = c->E[r];
  const int16_t *soft = e + tb * e_stride + c->off[r];
  for (uint32_t q = threadIdx.x; q < E; q += blockDim.x) sb[q] = soft[q];
  __syncthreads();
  int16_t *d = dfull + (size_t)j * d_stride + 96 - 3 * (Kpi - P.D);
  for (uint32_t i = threadIdx.x; i < 3 * Kpi + 3; i += blockDim.x) {
    if (i == 2) continue;
    const uint32_t sft = i % 3, base = sft == 2 ? i - 5 : i, row = base / 96, cp = (base % 96) / 3;
    if (row >= R) continue;
    const uint32_t k = (__builtin_bitreverse32(cp) >> 27) * R + row;
    const uint32_t p = sft == 0 ? k : Kpi + 2 * k + (sft == 2 ? 1 : 0);
    int16_t acc = 0;
    if (p < P.Ncb && P.dummy[p] != OAI4G_LTE_NULL) {
      const uint32_t ci = P.cidx[p];
      for (uint32_t q = ci >= P.k0c ? ci - P.k0c : ci + P.Nnn - P.k0c; q < E; q += P.Nnn) acc = (int16_t)(acc + sb[q]);
    }
    d[i] = acc;
  }
}

hipError_t oai4g_launch_ul_rm_deint(const ul_dev_t *d_cfg, const ul_dev_t *h_cfg, int n_tb, const int16_t *d_e,
                                    size_t e_stride, int16_t *d_dfull, size_t d_stride, hipStream_t s)
{
  if (n_tb <= 0) return hipSuccess;
  uint32_t emax = 0;
  for (uint32_t r = 0; r < h_cfg->C; r++) emax = h_cfg->E[r] > emax ? h_cfg->E[r] : emax;
  if (2 * (size_t)emax <= 64 * 1024) {         /* the staged form while a block's inputs fit 64 KB of LDS */
    const uint32_t rows = (uint32_t)n_tb * h_cfg->C;
    hipLaunchKernelGGL(k_ul_rm_deint_lds, dim3(rows), dim3(256), 2 * (size_t)emax, s, d_cfg, d_e, e_stride, d_dfull,
                       d_stride);
    return hipGetLastError();
  }
  /* (tb, r) rows in chunks within the 65535 limit of gridDim.y */
  const uint32_t rows = (uint32_t)n_tb * h_cfg->C, gx = (3 * (h_cfg->Rmax << 5) + 3 + 255) / 256;
  for (uint32_t j0 = 0; j0 < rows; j0 += 65535u) {
    const uint32_t n = rows - j0 < 65535u ? rows - j0 : 65535u;
    hipLaunchKernelGGL(k_ul_rm_deint, dim3(gx, n), dim3(256), 0, s, d_cfg, d_e, e_stride, d_dfull, d_stride, j0);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) return err;
  }
  return hipSuccess;
}

/* lte_rate_matching_turbo_rx (lte_rate_matching.c:688-831) of every block into its HARQ soft buffer
 * w, one thread per circular-buffer position p < Ncb (rows j = (tb, r) on blockIdx.y): clear = 1
 * (round 0) starts from 0 (the reference's memset of w[0..Ncb)), clear = 0 from the stored value;
 * the soft inputs the circular selection of this round's k0 maps to p are added with int16
 * wrap-around, in the reference's order (the sum is associative mod 2^16). */
__global__ void __launch_bounds__(256) k_ul_rm_harq(const ul_dev_t *__restrict__ c, const int16_t *__restrict__ e,
                                                    size_t e_stride, int16_t *__restrict__ w, size_t w_stride,
                                                    uint32_t rv, int clear, uint32_t j0)
{
  const uint32_t j = j0 + blockIdx.y, tb = j / c->C, r = j - tb * c->C;
  const ul_pat_t &P = c->pat[c->pat_of[r]];
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P.Ncb) return;
  int16_t *wp = w + (size_t)j * w_stride + p;
  int16_t acc = clear ? (int16_t)0 : *wp;
  if (P.dummy[p] != OAI4G_LTE_NULL) {
    const int16_t *soft = e + tb * e_stride + c->off[r];
    const uint32_t ci = P.cidx[p], E = c->E[r], k0c = P.k0cr[rv];
    for (uint32_t q = ci >= k0c ? ci - k0c : ci + P.Nnn - k0c; q < E; q += P.Nnn) acc = (int16_t)(acc + soft[q]);
  }
  *wp = acc;
}

/* sub_block_deinterleaving_turbo (lte_rate_matching.c:193-243) of every block's soft buffer into
 * its decoder row, one thread per d entry (the inverse map of k_ul_rm_deint); positions past Ncb
 * read 0, as a zero-initialised buffer the RX rate matcher never writes there gives */
__global__ void __launch_bounds__(256) k_ul_deint_w(const ul_dev_t *__restrict__ c, const int16_t *__restrict__ w,
                                                    size_t w_stride, int16_t *__restrict__ dfull, size_t d_stride,
                                                    uint32_t j0)
{
  const uint32_t j = j0 + blockIdx.y, r = j % c->C;
  const ul_pat_t &P = c->pat[c->pat_of[r]];
  const uint32_t R = P.R, Kpi = R << 5, i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 3 * Kpi + 3 || i == 2) return;
  const uint32_t sft = i % 3, base = sft == 2 ? i - 5 : i, row = base / 96, cp = (base % 96) / 3;
  if (row >= R) return;
  const uint32_t k = (__builtin_bitreverse32(cp) >> 27) * R + row;
  const uint32_t p = sft == 0 ? k : Kpi + 2 * k + (sft == 2 ? 1 : 0);
  dfull[(size_t)j * d_stride + 96 - 3 * (Kpi - P.D) + i] = p < P.Ncb ? w[(size_t)j * w_stride + p] : (int16_t)0;
}

hipError_t oai4g_launch_ul_rm_harq(const ul_dev_t *d_cfg, const ul_dev_t *h_cfg, int n_tb, const int16_t *d_e,
                                   size_t e_stride, int16_t *d_w, size_t w_stride, uint32_t rv, int clear,
                                   int16_t *d_dfull, size_t d_stride, hipStream_t s)
{
  if (n_tb <= 0) return hipSuccess;
  const uint32_t rows = (uint32_t)n_tb * h_cfg->C, gw = (3 * (h_cfg->Rmax << 5) + 255) / 256,
                 gd = (3 * (h_cfg->Rmax << 5) + 3 + 255) / 256;
  for (uint32_t j0 = 0; j0 < rows; j0 += 65535u) {
    const uint32_t n = rows - j0 < 65535u ? rows - j0 : 65535u;
    hipLaunchKernelGGL(k_ul_rm_harq, dim3(gw, n), dim3(256), 0, s, d_cfg, d_e, e_stride, d_w, w_stride, rv, clear, j0);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(k_ul_deint_w, dim3(gd, n), dim3(256), 0, s, d_cfg, d_w, w_stride, d_dfull, d_stride, j0);
    err = hipGetLastError();
    if (err != hipSuccess) return err;
  }
  return hipSuccess;
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
