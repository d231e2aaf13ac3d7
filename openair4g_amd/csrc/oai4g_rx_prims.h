/*
 * Per-RE demodulation arithmetic shared by k_rx_llr (oai4g_rx.hip) and the fused estimator +
 * demodulator k_rx_chest (oai4g_chest.hip): the reference's SSE lane arithmetic of
 * dlsch_channel_compensation (dlsch_demodulation.c:801-960) and dlsch_qpsk/16qam/64qam_llr
 * (dlsch_llr_computation.c:636-930) plus dlsch_unscrambling's sign (dlsch_scrambling.c:99-137).
 */
#ifndef OAI4G_RX_PRIMS_H
#define OAI4G_RX_PRIMS_H
#include "oai4g_internal.h"

/* global-qualified view of pointers read from the device configuration (generic pointers would
 * make their loads flat ops, waited for together with every LDS access) */
typedef const __attribute__((address_space(1))) uint32_t rg32_t;

static __device__ __forceinline__ int16_t rx_sat16(int32_t v) { return (int16_t)max(-32768, min(32767, v)); }
static __device__ __forceinline__ int16_t rx_abs16(int16_t v) { return v < 0 ? (int16_t)(-(int32_t)v) : v; }
static __device__ __forceinline__ int32_t rx_madd(int16_t a0, int16_t b0, int16_t a1, int16_t b1)
{
  return (int32_t)((uint32_t)((int32_t)a0 * b0) + (uint32_t)((int32_t)a1 * b1));
}

/* |h|^2 of one estimate word (dlsch_channel_level's madd, int32 wrap) */
static __device__ __forceinline__ uint32_t rx_h2(uint32_t h)
{
  return (uint32_t)rx_madd((int16_t)h, (int16_t)h, (int16_t)(h >> 16), (int16_t)(h >> 16));
}

/* unscramble (when gold != nullptr, Gold bits from stream position b) and store one RE's Qm LLRs
 * at out (one 4 / 8 / 12-byte store) */
template <int QM>
static __device__ __forceinline__ void rx_llr_store(int16_t *v, rg32_t *__restrict__ gold, uint32_t b, int16_t *out)
{
  if (gold) {                                    /* llr * (2 c - 1), int16 */
    const uint32_t w = b >> 5;
    const uint64_t win = ((uint64_t)gold[w] | ((uint64_t)gold[w + 1] << 32)) >> (b & 31);
#pragma unroll
    for (int q = 0; q < QM; q++)
      if (!((win >> q) & 1u)) v[q] = (int16_t)(-(int32_t)v[q]);
  }
  uint32_t pk[3];
#pragma unroll
  for (int q = 0; q < QM / 2; q++) pk[q] = (uint32_t)(uint16_t)v[2 * q] | ((uint32_t)(uint16_t)v[2 * q + 1] << 16);
  if (QM == 2) {
    *(uint32_t *)out = pk[0];
  } else if (QM == 4) {
    *(uint2 *)out = make_uint2(pk[0], pk[1]);
  } else {
    uint32_t *o = (uint32_t *)out;
    o[0] = pk[0];
    o[1] = pk[1];
    o[2] = pk[2];
  }
}

/* dlsch_qpsk/16qam/64qam_llr of one compensated RE (cr, ci) with magnitudes mag / magb */
template <int QM>
static __device__ __forceinline__ void rx_llr_values(int16_t cr, int16_t ci, int16_t mag, int16_t magb, int16_t *v)
{
  v[0] = cr;
  v[1] = ci;
  if (QM > 2) {
    v[2] = rx_sat16((int32_t)mag - rx_abs16(v[0]));
    v[3] = rx_sat16((int32_t)mag - rx_abs16(v[1]));
    if (QM > 4) {
      v[4] = rx_sat16((int32_t)magb - rx_abs16(v[2]));
      v[5] = rx_sat16((int32_t)magb - rx_abs16(v[3]));
    }
  }
}

/* the Qm LLRs of one RE (estimate hv, received yv), unscrambled with the Gold bits starting at
 * stream position b when gold != nullptr, stored at out (one 4 / 8 / 12-byte store) */
template <int QM>
static __device__ __forceinline__ void rx_re_llr(uint32_t hv, uint32_t yv, uint32_t sh, int16_t a1, int16_t a2,
                                                 rg32_t *__restrict__ gold, uint32_t b, int16_t *out)
{
  const int16_t hr = (int16_t)hv, hi = (int16_t)(hv >> 16), yr = (int16_t)yv, yi = (int16_t)(yv >> 16);
  const int16_t nhi = (int16_t)(-(int32_t)hi);
  int16_t v[6];
  const int16_t cr = rx_sat16(rx_madd(hr, yr, hi, yi) >> sh), ci = rx_sat16(rx_madd(nhi, yr, hr, yi) >> sh);
  int16_t mag = 0, magb = 0;
  if (QM > 2) {
    const int16_t mg = rx_sat16(rx_madd(hr, hr, hi, hi) >> sh);
    mag = (int16_t)((((int32_t)mg * a1) >> 16) << 1);
    magb = (int16_t)((((int32_t)mg * a2) >> 16) << 1);
  }
  rx_llr_values<QM>(cr, ci, mag, magb, v);
  rx_llr_store<QM>(v, gold, b, out);
}

/* prec2A_TM3_128 (dlsch_demodulation.c:1364-1396) on one RE: the stream-0 channel
 * (h0 + s h1) >> 1 per component, adds_epi16 then srai; s h1 by sign_epi16 (int16 wrap) */
static __device__ __forceinline__ uint32_t rx_prec_tm3(uint32_t h0, uint32_t h1, bool neg)
{
  const int16_t b0 = neg ? (int16_t)(-(int32_t)(int16_t)h1) : (int16_t)h1;
  const int16_t b1 = neg ? (int16_t)(-(int32_t)(int16_t)(h1 >> 16)) : (int16_t)(h1 >> 16);
  const int16_t r = (int16_t)(rx_sat16((int32_t)(int16_t)h0 + b0) >> 1);
  const int16_t i = (int16_t)(rx_sat16((int32_t)(int16_t)(h0 >> 16) + b1) >> 1);
  return (uint32_t)(uint16_t)r | ((uint32_t)(uint16_t)i << 16);
}

/* the stream-1 channel of prec2A_TM3_128: (h0 - s h1) >> 1 per component (subs_epi16, srai) */
static __device__ __forceinline__ uint32_t rx_prec_tm3_s1(uint32_t h0, uint32_t h1, bool neg)
{
  const int16_t b0 = neg ? (int16_t)(-(int32_t)(int16_t)h1) : (int16_t)h1;
  const int16_t b1 = neg ? (int16_t)(-(int32_t)(int16_t)(h1 >> 16)) : (int16_t)(h1 >> 16);
  const int16_t r = (int16_t)(rx_sat16((int32_t)(int16_t)h0 - b0) >> 1);
  const int16_t i = (int16_t)(rx_sat16((int32_t)(int16_t)(h0 >> 16) - b1) >> 1);
  return (uint32_t)(uint16_t)r | ((uint32_t)(uint16_t)i << 16);
}

/* conj(a) b >> sh, saturated per component (the madd / sign_epi16 / packs of the compensation and
 * of dlsch_dual_stream_correlation) */
static __device__ __forceinline__ void rx_conj_mul(uint32_t a, uint32_t b, uint32_t sh, int16_t &re, int16_t &im)
{
  const int16_t ar = (int16_t)a, ai = (int16_t)(a >> 16), br = (int16_t)b, bi = (int16_t)(b >> 16);
  re = rx_sat16(rx_madd(ar, br, ai, bi) >> sh);
  im = rx_sat16(rx_madd((int16_t)(-(int32_t)ai), br, ar, bi) >> sh);
}

/* qpsk_qpsk (dlsch_llr_computation.c:1041-1230) on one RE: the interference-aware max-log LLRs of
 * QPSK stream y0 with QPSK interference y1 of correlation rho (int16 saturating throughout) */
static __device__ __forceinline__ void rx_qq_llr(int16_t y0r, int16_t y0i, int16_t y1r, int16_t y1i, int16_t rr,
                                                 int16_t ri, int16_t *v)
{
  auto S = [](int32_t a, int32_t b) { return rx_sat16(a + b); };
  auto D = [](int32_t a, int32_t b) { return rx_sat16(a - b); };
  auto M = [](int16_t a, int16_t b) { return a > b ? a : b; };
  const int16_t rpi = (int16_t)(((int32_t)S(rr, ri) * 23170) >> 16), rmi = (int16_t)(((int32_t)D(rr, ri) * 23170) >> 16);
  const int16_t y0r2 = (int16_t)(y0r >> 1), y0i2 = (int16_t)(y0i >> 1), y1r2 = (int16_t)(y1r >> 1), y1i2 = (int16_t)(y1i >> 1);
  const int16_t A = rx_abs16(D(y1r2, rpi)), B = rx_abs16(D(y1i2, rmi)), C = rx_abs16(D(y1r2, rmi)), Dd = rx_abs16(S(y1i2, rpi));
  const int16_t E = rx_abs16(S(y1r2, rmi)), F = rx_abs16(D(y1i2, rpi)), G = rx_abs16(S(y1r2, rpi)), H = rx_abs16(S(y1i2, rmi));
  const int16_t num_re = M(S(B, S(A, y0i2)), S(D(C, y0i2), Dd));
  const int16_t den_re = M(S(F, S(E, y0i2)), S(D(G, y0i2), H));
  const int16_t num_im = M(S(B, S(A, y0r2)), S(D(E, y0r2), F));
  const int16_t den_im = M(S(Dd, S(C, y0r2)), S(D(G, y0r2), H));
  v[0] = D(S(y0r, num_re), den_re);
  v[1] = D(S(y0i, num_im), den_im);
}

static __device__ __forceinline__ int16_t rx_mh(int16_t a, int16_t b) { return (int16_t)(((int32_t)a * b) >> 16); }
static __device__ __forceinline__ int16_t rx_shl(int16_t a, int n) { return (int16_t)(uint16_t)((uint32_t)(uint16_t)a << n); }

/* qpsk_qam16 (dlsch_llr_computation.c:1300-1514) / qpsk_qam64 (:1584-1814) on one RE: LLRs of the QPSK
 * stream y0 with a 16 / 64-QAM interferer y1 of magnitude mag and correlation rho.  As written: y0's
 * mulhi by 1/sqrt2 is overwritten by y0 << 1, interference_abs(_64qam)_epi16 picks the interferer
 * amplitude from compare masks (OR of the masked constants), the 64-QAM psi_a is mulhi(., 23170) << 2 */
template <int QM1>
static __device__ __forceinline__ void rx_qx_llr(int16_t y0r, int16_t y0i, int16_t y1r, int16_t y1i, int16_t mag,
                                                 int16_t rr, int16_t ri, int16_t *v)
{
  auto S = [](int32_t a, int32_t b) { return rx_sat16(a + b); };
  auto D = [](int32_t a, int32_t b) { return rx_sat16(a - b); };
  auto M = [](int16_t a, int16_t b) { return a > b ? a : b; };
  const int16_t rpi = rx_shl(rx_mh(S(rr, ri), 23170), 1), rmi = rx_shl(rx_mh(D(rr, ri), 23170), 1);
  const int16_t y0a = rx_shl(y0r, 1), y0b = rx_shl(y0i, 1);
  const int16_t yp = S(y0a, y0b), ym = D(y0a, y0b);
  const int16_t psi[8] = {rx_abs16(D(y1r, rpi)), rx_abs16(D(y1i, rmi)), rx_abs16(D(y1r, rmi)), rx_abs16(S(y1i, rpi)),
                          rx_abs16(S(y1r, rmi)), rx_abs16(D(y1i, rpi)), rx_abs16(S(y1r, rpi)), rx_abs16(S(y1i, rmi))};
  const int16_t c1x = (int16_t)(mag >> 1), c3x = S(c1x, mag);
  int16_t met[4];
#pragma unroll
  for (int h = 0; h < 4; h++) {
    int16_t a[2], sq[2];
#pragma unroll
    for (int c = 0; c < 2; c++) {
      const int16_t x = psi[2 * h + c];
      if (QM1 == 4) {
        a[c] = x < mag ? (int16_t)10362 : (int16_t)31086;
      } else {
        const bool lt2 = x < mag, lt1 = x < c1x, gt3 = x > c3x;
        a[c] = (int16_t)(((lt2 != lt1) ? 10726 : 0) | (lt1 ? 3575 : 0) | ((!lt2) != gt3 ? 17876 : 0) | (gt3 ? 25027 : 0));
      }
      const int16_t t = rx_shl(rx_mh(a[c], a[c]), 1);
      sq[c] = QM1 == 4 ? rx_shl(rx_mh(rx_shl(rx_mh(t, 25905), 1), mag), 1) : rx_shl(rx_mh(rx_shl(rx_mh(t, 13272), 3), mag), 1);
    }
    int16_t pa = S(rx_shl(rx_mh(psi[2 * h], a[0]), 1), rx_shl(rx_mh(psi[2 * h + 1], a[1]), 1));
    if (QM1 == 6) pa = rx_shl(rx_mh(pa, 23170), 2);
    const int16_t d = D(pa, S(sq[0], sq[1]));
    met[h] = h == 0 ? S(d, yp) : h == 1 ? S(d, ym) : h == 2 ? D(d, ym) : D(d, yp);
  }
  v[0] = D(M(met[0], met[1]), M(met[2], met[3]));
  v[1] = D(M(met[0], met[2]), M(met[1], met[3]));
}

/* log2_approx(avg) / 2 of dlsch_channel_level (log2_approx: bits 0..30) */
static __device__ __forceinline__ uint8_t rx_shift_of(int32_t acc, uint32_t div)
{
  const int32_t avg = acc / (int32_t)div;
  const uint32_t x = avg > 0 ? (uint32_t)avg : 0u;
  const uint32_t l2 = x ? 32u - __clz(x & 0x7FFFFFFFu) : 0u;
  return (uint8_t)(l2 / 2);
}
#endif
