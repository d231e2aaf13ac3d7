/*
 * Fixed-point complex int16 primitives shared by the inverse (oai4g_ofdm.hip) and forward
 * (oai4g_fep.hip) DFT kernels: the SSE operations of PHY/TOOLS/lte_dfts.c mapped to gfx950
 * packed-int16 VALU (v_pk_add/sub_i16 clamp, v_dot2_i32_i16, v_cvt_pk_i16_i32).
 */
#ifndef OAI4G_DFT_PRIMS_H
#define OAI4G_DFT_PRIMS_H
#include "oai4g_internal.h"

typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(1))) uint32_t gu32_t;
typedef const __attribute__((address_space(1))) uint16_t gu16_t;
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4_t gu128_t;

static __device__ __forceinline__ s16x2 u2c(uint32_t v) { return __builtin_bit_cast(s16x2, v); }
static __device__ __forceinline__ uint32_t c2u(s16x2 v) { return __builtin_bit_cast(uint32_t, v); }
static __device__ __forceinline__ s16x2 cadds(s16x2 a, s16x2 b) { return __builtin_elementwise_add_sat(a, b); }
static __device__ __forceinline__ s16x2 csubs(s16x2 a, s16x2 b) { return __builtin_elementwise_sub_sat(a, b); }
static __device__ __forceinline__ s16x2 caddw(s16x2 a, s16x2 b) { return a + b; }
/* sign_epi16(x,{-1,1}) + pair swap: -j*x with a wrapping negate (lte_dfts.c:1463-1466) */
static __device__ __forceinline__ s16x2 cflip(s16x2 a) { return (s16x2){a.y, (short)(-(int)a.x)}; }
/* The same as one v_pk_mul_lo_u16 with swapped operand halves (lo = a.hi * 1, hi = a.lo * 0xFFFF)
 * instead of the compiler's v_sub_u16 + v_alignbit pair.  Used where it measured a gain (the
 * two-antenna 2048-point kernels); elsewhere the opaque asm raised register pressure. */
static __device__ __forceinline__ s16x2 cflip_f(s16x2 a)
{
  if (__builtin_constant_p(__builtin_bit_cast(uint32_t, a)))
    return (s16x2){a.y, (short)(-(int)a.x)};
  uint32_t r;
  asm("v_pk_mul_lo_u16 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1]" : "=v"(r) : "v"(a), "s"(0xFFFF0001u));
  return __builtin_bit_cast(s16x2, r);
}
/* v_dot2_i32_i16 with an inline-zero accumulator (the compiler otherwise picks the tied
 * v_dot2c form and zeroes its accumulator with an extra v_mov per product) */
static __device__ __forceinline__ int dot2(s16x2 a, s16x2 b)
{
  int r;
  asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
/* the same with a wave-uniform second operand (twiddles from scalar loads, constants): the "s"
 * constraint keeps it in an SGPR (VOP3P reads one through the constant bus) instead of a VGPR copy.
 * Only for values that are uniform by construction. */
static __device__ __forceinline__ int dot2s(s16x2 a, s16x2 b)
{
  int r;
  asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(r) : "v"(a), "s"(b));
  return r;
}
static __device__ __forceinline__ int wadd(int a, int b) { return (int)((unsigned)a + (unsigned)b); }
static __device__ __forceinline__ int wsub(int a, int b) { return (int)((unsigned)a - (unsigned)b); }
/* cpack: srai 15 + packs_epi32 (lte_dfts.c:123-131) */
static __device__ __forceinline__ s16x2 cpack32(int re, int im)
{
  return __builtin_bit_cast(s16x2, __builtin_amdgcn_cvt_pk_i16(re >> 15, im >> 15));
}

/* a twiddle t and its rotated companion (-t.im, t.re) for the imaginary half of x*conj(t) */
struct twp_t {
  s16x2 t, tn;
};

/* x * conj(t), 32-bit (cmultc, lte_dfts.c:132-141) */
static __device__ __forceinline__ void cmulc32(s16x2 x, const twp_t &w, int &re, int &im)
{
  re = dot2(x, w.t);
  im = dot2(x, w.tn);
}
static __device__ __forceinline__ s16x2 cmulc16(s16x2 x, const twp_t &w)
{
  int re, im;
  cmulc32(x, w, re, im);
  return cpack32(re, im);
}
/* x * conj(w) with a wave-uniform twiddle pair (SGPR operands) */
static __device__ __forceinline__ s16x2 cmulc16u(s16x2 x, const twp_t &w)
{
  return cpack32(dot2s(x, w.t), dot2s(x, w.tn));
}

/* saturating inverse radix-4 (idft16 stages; ibfly4_16 lte_dfts.c:1049-1090).  NS: the caller's range
 * check guarantees no operand is -32768 and no difference saturates, so cflip(p1) - cflip(p3) =
 * cflip(p1 - p3) (one rotation instead of two) */
template <bool FF = false, bool NS = false>
static __device__ __forceinline__ void r4inv(s16x2 p0, s16x2 p1, s16x2 p2, s16x2 p3, s16x2 &o0, s16x2 &o1,
                                             s16x2 &o2, s16x2 &o3)
{
  s16x2 s02 = cadds(p0, p2), s13 = cadds(p1, p3);
  o0 = cadds(s02, s13);
  o2 = csubs(s02, s13);
  s16x2 d02 = csubs(p0, p2),
        d13 = NS ? cflip_f(csubs(p1, p3)) : FF ? csubs(cflip_f(p1), cflip_f(p3)) : csubs(cflip(p1), cflip(p3));
  o3 = cadds(d02, d13);
  o1 = csubs(d02, d13);
}

/* ibfly4 (lte_dfts.c:795-819): 32-bit products, one cpack per output, wrapping add of x0 */
static __device__ __forceinline__ void ibfly4(s16x2 x0, s16x2 x1, s16x2 x2, s16x2 x3, const twp_t &t1,
                                              const twp_t &t2, const twp_t &t3, s16x2 &y0, s16x2 &y1, s16x2 &y2,
                                              s16x2 &y3)
{
  int a1r, a1i, a2r, a2i, a3r, a3i;
  cmulc32(x1, t1, a1r, a1i);
  cmulc32(x2, t2, a2r, a2i);
  cmulc32(x3, t3, a3r, a3i);
  y0 = caddw(x0, cpack32(wadd(a1r, wadd(a2r, a3r)), wadd(a1i, wadd(a2i, a3i))));
  y3 = caddw(x0, cpack32(wsub(a1i, wadd(a2r, a3i)), wsub(wsub(a3r, a2i), a1r)));
  y2 = caddw(x0, cpack32(wsub(wsub(a2r, a3r), a1r), wsub(wsub(a2i, a3i), a1i)));
  y1 = caddw(x0, cpack32(wsub(wsub(a3i, a2r), a1i), wsub(a1r, wadd(a2i, a3r))));
}

/* v_dot2_i32_i16 with a VGPR accumulator */
static __device__ __forceinline__ int dot2acc(s16x2 a, s16x2 b, int c)
{
  int r;
  asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
/* lanes (R >> 16, I >> 16): bits 16..31 of each, one v_perm_b32 */
static __device__ __forceinline__ s16x2 hi16_pair(int R, int I)
{
  return u2c(__builtin_amdgcn_perm((uint32_t)I, (uint32_t)R, 0x07060302u));
}

/*
 * ibfly4 followed by shr1 when no value of the level can leave int16 (the caller's range check,
 * oai4g_host.cpp mod_nosat_ok): then packs_epi32 never clamps and the wrapping add of x0 never
 * wraps, and per lane
 *     (x0 + (S >> 15)) >> 1  ==  (x0 2^15 + S) >> 16          (floor division nests)
 * with S the lane's three-product sum.  So x0 2^15 joins the 32-bit sums, and the cpack, the add
 * and the shift become one v_perm of bits 16..31.  The sums share their terms pairwise:
 *   re: y0 / y2 = (X + a2r) +- (a1r + a3r),  y3 / y1 = (X - a2r) +- (a1i - a3i)
 *   im: y0 / y2 = (X + a2i) +- (a1i + a3i),  y3 / y1 = (X - a2i) +- (a3r - a1r)
 * (the terms of ibfly4 above regrouped), X + a2 from the dot2 accumulator and X - a2 = 2X - (X + a2).
 * Intermediate sums may wrap in 32 bits; each final sum is x0 2^15 + S, inside int32 under the check.
 */
static __device__ __forceinline__ void ibfly4_shr1_ns(s16x2 x0, s16x2 x1, s16x2 x2, s16x2 x3, const twp_t &t1,
                                                      const twp_t &t2, const twp_t &t3, s16x2 &y0, s16x2 &y1,
                                                      s16x2 &y2, s16x2 &y3)
{
  const uint32_t xu = c2u(x0);
  const int x2lo = (int)(xu << 16), x2hi = (int)(xu & 0xFFFF0000u);   /* 2X per lane */
  int a1r, a1i, a3r, a3i;
  cmulc32(x1, t1, a1r, a1i);
  cmulc32(x3, t3, a3r, a3i);
  const int ur = dot2acc(x2, t2.t, x2lo >> 1), ui = dot2acc(x2, t2.tn, x2hi >> 1);
  const int vr = wsub(x2lo, ur), vi = wsub(x2hi, ui);
  const int pr = wadd(a1r, a3r), pi = wadd(a1i, a3i), qr = wsub(a1i, a3i), qi = wsub(a3r, a1r);
  y0 = hi16_pair(wadd(ur, pr), wadd(ui, pi));
  y2 = hi16_pair(wsub(ur, pr), wsub(ui, pi));
  y3 = hi16_pair(wadd(vr, qr), wadd(vi, qi));
  y1 = hi16_pair(wsub(vr, qr), wsub(vi, qi));
}

/* ibfly2 (lte_dfts.c:502-527): x0 * 32767 via the same madd as the twiddled operand */
static __device__ __forceinline__ void ibfly2(s16x2 x0, s16x2 x1, const twp_t &t, s16x2 &y0, s16x2 &y1)
{
  int a0r = dot2s(x0, (s16x2){32767, 0}), a0i = dot2s(x0, (s16x2){0, 32767}), a1r, a1i;
  cmulc32(x1, t, a1r, a1i);
  y0 = cpack32(wadd(a0r, a1r), wadd(a0i, a1i));
  y1 = cpack32(wsub(a0r, a1r), wsub(a0i, a1i));
}

/* ibfly2 then mulhi2_f on both outputs when neither sum can leave int16 (the caller's range check):
 * packs_epi32 then never clamps, so each lane of y is the 32-bit sum >> 15 as it stands and the
 * x 23170 product takes it from the VGPR (v_mul_i32_i24) instead of from a packed pair (dot2): the
 * v_cvt_pk of each output disappears.  Lane extraction as mulhi2_f. */
static __device__ __forceinline__ s16x2 mulhi2_lanes(int yr, int yi)
{
  uint32_t pr, pi2, hi, r;
  /* yr, yi are int16 values in 32-bit lanes: exact 24-bit products; the imaginary one doubled (46340 =
   * 2 x 23170) is mulhi2_f's pi + pi */
  asm("v_mul_i32_i24_e32 %0, 0x5a82, %1" : "=v"(pr) : "v"(yr));
  asm("v_mul_i32_i24_e32 %0, 0xb504, %1" : "=v"(pi2) : "v"(yi));
  const uint32_t lo = pr >> 15;
  asm("v_and_b32_e32 %0, 0xfffe0000, %1" : "=v"(hi) : "v"(pi2));
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe4" : "=v"(r) : "v"(lo), "v"(hi), "s"(0x0000FFFEu));
  return u2c(r);
}
static __device__ __forceinline__ void ibfly2_mulhi_ns(s16x2 x0, s16x2 x1, const twp_t &t, s16x2 &y0, s16x2 &y1)
{
  int a0r = dot2s(x0, (s16x2){32767, 0}), a0i = dot2s(x0, (s16x2){0, 32767}), a1r, a1i;
  cmulc32(x1, t, a1r, a1i);
  y0 = mulhi2_lanes(wadd(a0r, a1r) >> 15, wadd(a0i, a1i) >> 15);
  y1 = mulhi2_lanes(wsub(a0r, a1r) >> 15, wsub(a0i, a1i) >> 15);
}

static __device__ __forceinline__ s16x2 shr3(s16x2 a) { return (s16x2){(short)(a.x >> 3), (short)(a.y >> 3)}; }
static __device__ __forceinline__ s16x2 shr1(s16x2 a) { return (s16x2){(short)(a.x >> 1), (short)(a.y >> 1)}; }
/* mulhi_int16(a, 23170) = slli(mulhi_epi16(a, 23170), 1) (lte_dfts.c:1755); |result| <= 23170 */
static __device__ __forceinline__ s16x2 mulhi2(s16x2 a)
{
  int pr = dot2s(a, (s16x2){23170, 0}), pi = dot2s(a, (s16x2){0, 23170});
  return (s16x2){(short)((pr >> 16) << 1), (short)((pi >> 16) << 1)};
}
/* The same with the packing as four fast-rate ops: lane = ((p >> 16) << 1) mod 2^16 = bits 16..30
 * of p moved up by one, so low lane (pr >> 15) & 0xFFFE, high lane (pi << 1) & 0xFFFE0000 (pi + pi
 * for << 1; the mask also clears bit 16, which holds bit 15 of pi), merged by one v_bitop3 mux
 * "c ? a : b" (0xe4, c = 0x0000FFFE).  The compiler's own form (v_perm, or v_lshlrev + v_and_or)
 * issues at the slow rate.  Used in the two-antenna 2048-point kernels; in the TM1 kernel the
 * opaque asm raised register pressure past 4 waves. */
static __device__ __forceinline__ s16x2 mulhi2_f(s16x2 a)
{
  const uint32_t pr = (uint32_t)dot2s(a, (s16x2){23170, 0}), pi = (uint32_t)dot2s(a, (s16x2){0, 23170});
  const uint32_t lo = pr >> 15;
  uint32_t hi, r;
  asm("v_add_u32_e32 %0, %1, %1\n\tv_and_b32_e32 %0, 0xfffe0000, %0" : "=&v"(hi) : "v"(pi));
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe4" : "=v"(r) : "v"(lo), "v"(hi), "s"(0x0000FFFEu));
  return u2c(r);
}

static __device__ __forceinline__ uint32_t lphys(uint32_t pos) { return pos + (pos >> 5); }

#endif
