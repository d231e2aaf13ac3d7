/*
 * CPU ORACLE — TEST INFRASTRUCTURE ONLY.  Uplink turbo decoding chain:
 *   phy_threegpplte_turbo_decoder16  PHY/CODING/3gpplte_turbo_decoder_sse_16bit.c:945-1385
 *     compute_gamma16 :121-169, compute_alpha16 :173-440, compute_beta16 :442-693,
 *     compute_ext16 :695-880, init_td16 :898-943
 *   lte_rate_matching_turbo_rx       PHY/CODING/lte_rate_matching.c:688-831
 *   sub_block_deinterleaving_turbo   PHY/CODING/lte_rate_matching.c:193-243
 *   generate_dummy_w                 PHY/CODING/lte_rate_matching.c (NULL pattern of w)
 *
 * The SSE decoder runs 8 int16 lanes = 8 windows of K/8 bits; every __m128i operation is
 * restated here as a loop over the 8 lanes with the same saturating (adds/subs) or wrapping
 * arithmetic and the same data layout (vector v, lane q = element 8v + q), including the
 * reference's alpha/beta re-runs over L = 40 bits and its initialisation quirks.  Parity of
 * this restatement to the reference is by construction only (the reference TU needs generated
 * headers and is not built here): DESIGN.md records the decoder as "pinned to restatement".
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oai_oracle.h"
#include "../include/oai4g_qpp.h"

#define TD_MAX 256
#define TD_L 40

static inline int16_t sadd(int16_t a, int16_t b)
{
  int v = (int)a + (int)b;
  return (int16_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v));
}
static inline int16_t ssub(int16_t a, int16_t b)
{
  int v = (int)a - (int)b;
  return (int16_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v));
}
static inline int16_t smax(int16_t a, int16_t b) { return a > b ? a : b; }

/* vector helpers over 8 lanes: x[8 * v + q] */
#define V(p, v) ((p) + 8 * (v))

/* compute_gamma16 (:121-169) */
static void gamma16(int16_t *m11, int16_t *m10, const int16_t *sys, const int16_t *par, int n, int term_flag)
{
  int K1 = n >> 3, k;
  for (k = 0; k < K1; k++)
    for (int q = 0; q < 8; q++) {
      m11[8 * k + q] = (int16_t)(sadd(sys[8 * k + q], par[8 * k + q]) >> 1);
      m10[8 * k + q] = (int16_t)(ssub(sys[8 * k + q], par[8 * k + q]) >> 1);
    }
  for (int q = 0; q < 8; q++) {   /* termination vector */
    m11[8 * k + q] = (int16_t)(sadd(sys[8 * (k + term_flag) + q], par[8 * k + q]) >> 1);
    m10[8 * k + q] = (int16_t)(ssub(sys[8 * (k + term_flag) + q], par[8 * k + q]) >> 1);
  }
}

/* one forward trellis step: alpha vectors a[0..7] (each 8 lanes) -> o[0..7] (:286-367) */
static void alpha_step(const int16_t *a, const int16_t *m11, const int16_t *m10, int16_t *o)
{
  for (int q = 0; q < 8; q++) {
    int16_t g11 = m11[q], g10 = m10[q];
    int16_t mb0 = sadd(a[8 * 1 + q], g11), mb4 = ssub(a[8 * 1 + q], g11);
    int16_t mb1 = ssub(a[8 * 3 + q], g10), mb5 = sadd(a[8 * 3 + q], g10);
    int16_t mb2 = sadd(a[8 * 5 + q], g10), mb6 = ssub(a[8 * 5 + q], g10);
    int16_t mb3 = ssub(a[8 * 7 + q], g11), mb7 = sadd(a[8 * 7 + q], g11);
    int16_t n0 = ssub(a[8 * 0 + q], g11), n4 = sadd(a[8 * 0 + q], g11);
    int16_t n1 = sadd(a[8 * 2 + q], g10), n5 = ssub(a[8 * 2 + q], g10);
    int16_t n2 = ssub(a[8 * 4 + q], g10), n6 = sadd(a[8 * 4 + q], g10);
    int16_t n3 = sadd(a[8 * 6 + q], g11), n7 = ssub(a[8 * 6 + q], g11);
    int16_t r[8] = {smax(mb0, n0), smax(mb1, n1), smax(mb2, n2), smax(mb3, n3),
                    smax(mb4, n4), smax(mb5, n5), smax(mb6, n6), smax(mb7, n7)};
    int16_t mx = r[0];
    for (int s = 1; s < 8; s++) mx = smax(mx, r[s]);
    for (int s = 0; s < 8; s++) o[8 * s + q] = ssub(r[s], mx);
  }
}

/* compute_alpha16 (:173-440); alpha[(8k + s) * 8 + q] */
static void alpha16(int16_t *alpha, const int16_t *m11, const int16_t *m10, int n)
{
  const int K1 = n >> 3, l2 = TD_L >> 3;
  for (int s = 0; s < 8; s++)
    for (int q = 0; q < 8; q++) alpha[8 * s + q] = (s == 0 && q == 0) ? 0 : -TD_MAX / 2;
  for (int k = 0; k < K1; k++) alpha_step(V(alpha, 8 * k), V(m11, k), V(m10, k), V(alpha, 8 * (k + 1)));
  /* re-run: columns 1-7 start from the final alpha of columns 0-6 (slli_si128 by one lane),
   * column 0 from (0, -MAX/2, ...) */
  for (int s = 0; s < 8; s++) {
    int16_t fin[8];
    memcpy(fin, V(alpha, n + s), sizeof(fin));        /* alpha128[s + frame_length] */
    alpha[8 * s + 0] = 0;
    for (int q = 1; q < 8; q++) alpha[8 * s + q] = fin[q - 1];
  }
  for (int s = 1; s < 8; s++) alpha[8 * s] = -TD_MAX / 2;
  for (int k = 0; k < l2; k++) alpha_step(V(alpha, 8 * k), V(m11, k), V(m10, k), V(alpha, 8 * (k + 1)));
}

/* one backward step: beta vectors b[0..7] of step k+1 -> o[0..7] of step k (:588-685) */
static void beta_step(const int16_t *b, const int16_t *m11, const int16_t *m10, int16_t *o)
{
  for (int q = 0; q < 8; q++) {
    int16_t g11 = m11[q], g10 = m10[q];
    int16_t mb0 = sadd(b[8 * 4 + q], g11), mb1 = ssub(b[8 * 4 + q], g11);
    int16_t mb2 = ssub(b[8 * 5 + q], g10), mb3 = sadd(b[8 * 5 + q], g10);
    int16_t mb4 = sadd(b[8 * 6 + q], g10), mb5 = ssub(b[8 * 6 + q], g10);
    int16_t mb6 = ssub(b[8 * 7 + q], g11), mb7 = sadd(b[8 * 7 + q], g11);
    int16_t n0 = ssub(b[8 * 0 + q], g11), n1 = sadd(b[8 * 0 + q], g11);
    int16_t n2 = sadd(b[8 * 1 + q], g10), n3 = ssub(b[8 * 1 + q], g10);
    int16_t n4 = ssub(b[8 * 2 + q], g10), n5 = sadd(b[8 * 2 + q], g10);
    int16_t n6 = sadd(b[8 * 3 + q], g11), n7 = ssub(b[8 * 3 + q], g11);
    int16_t r[8] = {smax(mb0, n0), smax(mb1, n1), smax(mb2, n2), smax(mb3, n3),
                    smax(mb4, n4), smax(mb5, n5), smax(mb6, n6), smax(mb7, n7)};
    int16_t mx = r[0];
    for (int s = 1; s < 8; s++) mx = smax(mx, r[s]);
    for (int s = 0; s < 8; s++) o[8 * s + q] = ssub(r[s], mx);
  }
}

/* compute_beta16 (:442-693); beta[(8k + s) * 8 + q] */
static void beta16(const int16_t *alpha, int16_t *beta, const int16_t *m_11, const int16_t *m_10, int n)
{
  const int K1 = n >> 3;
  /* termination betas: plain int16 arithmetic (C int promotion, wrap on store) */
  int16_t m11 = m_11[2 + n], m10;
  int16_t beta0 = (int16_t)-m11, beta1 = m11;
  m11 = m_11[1 + n];
  m10 = m_10[1 + n];
  int16_t b0_2 = (int16_t)(beta0 - m11), b1_2 = (int16_t)(beta0 + m11), b2_2 = (int16_t)(beta1 + m10),
          b3_2 = (int16_t)(beta1 - m10);
  m11 = m_11[n];
  m10 = m_10[n];
  int16_t t[8] = {(int16_t)(b0_2 - m11), (int16_t)(b0_2 + m11), (int16_t)(b1_2 + m10), (int16_t)(b1_2 - m10),
                  (int16_t)(b2_2 - m10), (int16_t)(b2_2 + m10), (int16_t)(b3_2 + m11), (int16_t)(b3_2 - m11)};
  int16_t bm = t[0];
  for (int s = 1; s < 8; s++) bm = (bm > t[s]) ? bm : t[s];
  for (int s = 0; s < 8; s++) t[s] = (int16_t)(t[s] - bm);

  for (int rerun = 0; rerun < 2; rerun++) {
    int16_t *bp = V(beta, n);                          /* &beta[frame_length << 3] = step K1 */
    if (!rerun) {
      memcpy(bp, V(alpha, n), 64 * sizeof(int16_t));   /* initial beta = final alpha (alpha128[n+s]) */
    } else {
      for (int s = 0; s < 8; s++) {                    /* srli_si128 of beta at step 0: lane q <- q+1 */
        for (int q = 0; q < 7; q++) bp[8 * s + q] = beta[8 * s + q + 1];
        bp[8 * s + 7] = 0;
      }
    }
    for (int s = 0; s < 8; s++) bp[8 * s + 7] = t[s];  /* termination in the last window */
    const int stop = rerun ? ((n - TD_L) >> 3) : 0;
    for (int k = K1 - 1; k >= stop; k--) beta_step(V(beta, 8 * (k + 1)), V(m_11, k), V(m_10, k), V(beta, 8 * k));
  }
}

/* compute_ext16 (:695-880) */
static void ext16(const int16_t *alpha, const int16_t *beta, const int16_t *m_11, const int16_t *m_10, int16_t *ext,
                  int n)
{
  for (int k = 0; k < (n >> 3); k++) {
    const int16_t *a = V(alpha, 8 * k), *b = V(beta, 8 * (k + 1));
    for (int q = 0; q < 8; q++) {
#define A(s) a[8 * (s) + q]
#define B(s) b[8 * (s) + q]
      int16_t m00_4 = sadd(A(7), B(3)), m11_4 = sadd(A(7), B(7)), m00_3 = sadd(A(6), B(7)), m11_3 = sadd(A(6), B(3));
      int16_t m00_2 = sadd(A(1), B(4)), m11_2 = sadd(A(1), B(0)), m11_1 = sadd(A(0), B(4)), m00_1 = sadd(A(0), B(0));
      int16_t m01_4 = sadd(A(5), B(6)), m10_4 = sadd(A(5), B(2)), m01_3 = sadd(A(4), B(2)), m10_3 = sadd(A(4), B(6));
      int16_t m01_2 = sadd(A(3), B(1)), m10_2 = sadd(A(3), B(5)), m10_1 = sadd(A(2), B(1)), m01_1 = sadd(A(2), B(5));
#undef A
#undef B
      m01_1 = smax(smax(smax(m01_1, m01_2), m01_3), m01_4);
      m00_1 = smax(smax(smax(m00_1, m00_2), m00_3), m00_4);
      m10_1 = smax(smax(smax(m10_1, m10_2), m10_3), m10_4);
      m11_1 = smax(smax(smax(m11_1, m11_2), m11_3), m11_4);
      m01_1 = ssub(m01_1, m_10[8 * k + q]);
      m00_1 = ssub(m00_1, m_11[8 * k + q]);
      m10_1 = sadd(m10_1, m_10[8 * k + q]);
      m11_1 = sadd(m11_1, m_11[8 * k + q]);
      ext[8 * k + q] = ssub(smax(m10_1, m11_1), smax(m01_1, m00_1));
    }
  }
}

static void log_map16(const int16_t *sys, const int16_t *par, int16_t *m11, int16_t *m10, int16_t *alpha,
                      int16_t *beta, int16_t *ext, int n, int term_flag)
{
  gamma16(m11, m10, sys, par, n, term_flag);
  alpha16(alpha, m11, m10, n);
  beta16(alpha, beta, m11, m10, n);
  ext16(alpha, beta, m11, m10, ext, n);
}

/* init_td16 (:898-943) for one block size: window layout pi2 and the exchange permutations */
static void td_tables(int n, int *pi2, int *pi4, int *pi5, int *pi6)
{
  int qi = oai4g_qpp_index((uint32_t)n);
  uint64_t f1 = oai4g_qpp_table[qi].f1, f2 = oai4g_qpp_table[qi].f2;
  for (int i = 0, i2 = 0; i2 < 8; i2++)
    for (int i3 = 0, j = i2; i3 < (n >> 3); i3++, i++, j += 8) pi2[i] = j;
  for (int i = 0; i < n; i++) {
    int pi = (int)((f1 * (uint64_t)i + f2 * (uint64_t)i * (uint64_t)i) % (uint64_t)n);
    int pi3 = pi2[pi];
    pi4[pi2[i]] = pi3;
    pi5[pi3] = pi2[i];
    pi6[pi] = pi2[i];
  }
}

/* phy_threegpplte_turbo_decoder16 (:945-1385).  y: 3n+12 int16 (the d layout after &d[96]).
 * Returns the iteration count, max_iterations + 1 on CRC failure, 255 on bad arguments. */
uint8_t orc_turbo_decoder16(const int16_t *y, uint8_t *decoded_bytes, uint16_t n, uint8_t max_iterations,
                            uint8_t crc_type, uint8_t F)
{
  if (crc_type > 3 || oai4g_qpp_index(n) < 0 || (n & 7)) return 255;
  const int N16 = n + 16, N128 = n + 128;
  int16_t *s0 = calloc(N16, 2), *s1 = calloc(N16, 2), *s2 = calloc(N16, 2), *yp1 = calloc(N16, 2),
          *yp2 = calloc(N16, 2), *ext = calloc(N128, 2), *ext2 = calloc(N128, 2), *alpha = calloc((size_t)N16 * 8, 2),
          *beta = calloc((size_t)N16 * 8, 2), *m11 = calloc(N16, 2), *m10 = calloc(N16, 2);
  int *pi2 = malloc((n + 8) * sizeof(int)), *pi4 = malloc((n + 8) * sizeof(int)), *pi5 = malloc((n + 8) * sizeof(int)),
      *pi6 = malloc((n + 8) * sizeof(int));
  td_tables(n, pi2, pi4, pi5, pi6);
  const uint32_t crc_len = crc_type == 2 ? 2 : (crc_type == 3 ? 1 : 3);   /* CRC24_A 0, CRC24_B 1, CRC16 2, CRC8 3 */
  for (int i = 0; i < n; i++) {
    int j = pi2[i];
    s0[j] = y[3 * i];
    yp1[j] = y[3 * i + 1];
    yp2[j] = y[3 * i + 2];
  }
  const int16_t *yp = y + 3 * n;
  for (int i = n; i < n + 3; i++) {
    s0[i] = *yp++;
    s1[i] = s2[i] = s0[i];
    yp1[i] = *yp++;
  }
  for (int i = n + 8; i < n + 11; i++) {
    s0[i] = *yp++;
    s1[i] = s2[i] = s0[i];
    yp2[i - 8] = *yp++;
  }
  uint8_t it = 0;
  log_map16(s0, yp1, m11, m10, alpha, beta, ext, n, 0);
  uint8_t ret = 0;
  while (it++ < max_iterations) {
    for (int i = 0; i < n; i++) s2[i] = ext[pi4[i]];
    log_map16(s2, yp2, m11, m10, alpha, beta, ext2, n, 1);
    for (int i = 0; i < n; i++) s1[i] = sadd(ssub(ext2[pi5[i]], ext[i]), s0[i]);
    if (it > 1) {
      for (int i = 0; i < (n >> 3); i++) {
        uint8_t b = 0;
        for (int q = 0; q < 8; q++) b |= (uint8_t)((ext2[pi6[8 * i + q]] > 0) << (7 - q));
        decoded_bytes[i] = b;
      }
      uint32_t oldcrc = (uint32_t)decoded_bytes[(n >> 3) - crc_len] | ((uint32_t)decoded_bytes[(n >> 3) - crc_len + 1] << 8) |
                        ((uint32_t)decoded_bytes[(n >> 3) - crc_len + 2] << 16), crc;
      if (crc_type == 0 || crc_type == 1) {
        oldcrc &= 0xffffff;
        crc = crc_type == 0 ? orc_crc24a(decoded_bytes + (F >> 3), n - 24 - F) >> 8
                            : orc_crc24b(decoded_bytes, n - 24) >> 8;
        crc = ((crc & 0xff) << 16) | (crc & 0xff00) | ((crc >> 16) & 0xff);   /* swap bytes 0 and 2 */
      } else {
        ret = 255;                                  /* CRC16 / CRC8 are not on the path */
        break;
      }
      if (crc == oldcrc && crc != 0) {
        ret = it;
        break;
      }
    }
    if (it < max_iterations) {
      log_map16(s1, yp1, m11, m10, alpha, beta, ext, n, 0);
      for (int i = 0; i < n; i++) ext[i] = sadd(ssub(ext[i], s1[i]), s0[i]);
    }
  }
  if (!ret) ret = it;
  free(s0); free(s1); free(s2); free(yp1); free(yp2); free(ext); free(ext2); free(alpha); free(beta);
  free(m11); free(m10); free(pi2); free(pi4); free(pi5); free(pi6);
  return ret;
}

/* NULL pattern of w for D = K + 4 (generate_dummy_w): the sub-block interleaver applied to a d
 * whose first F systematic / first-parity entries are fillers; here F = 0 (table TBS). */
uint32_t orc_generate_dummy_w(uint32_t D, uint8_t *w)
{
  static uint8_t dbuf[96 + 3 * 6148 + 64];
  memset(dbuf, ORC_LTE_NULL, 96);
  memset(dbuf + 96, 0, sizeof(dbuf) - 96);
  return orc_subblock_interleave(D, dbuf + 96, w);
}

/* generate_dummy_w with filler bits (lte_rate_matching.c:293-382): only the NULL marks are written;
 * rows 0..2 of a column carry the ND + F NULL / filler positions of the systematic and first
 * parity streams, the second parity's ND NULLs sit one position later (index + 1 < ND) */
uint32_t orc_generate_dummy_w_F(uint32_t D, uint8_t *w, uint8_t F)
{
  static const uint8_t bitrev[32] = {0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30,
                                     1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31};
  uint32_t RTC = D >> 5;
  if (D & 0x1f) RTC++;
  const uint32_t Kpi = RTC << 5, ND = Kpi - D;
  uint8_t *wKpi = &w[Kpi], *wKpi1 = &w[Kpi + 1], *wKpi2 = &w[Kpi + 2], *wKpi4 = &w[Kpi + 4];
  uint32_t k = 0, k2 = 0;
  for (uint32_t col = 0; col < 32; col++) {
    const uint32_t index = bitrev[col];
    if (index < ND + F) { w[k] = ORC_LTE_NULL; wKpi[k2] = ORC_LTE_NULL; }
    if (index + 32 < ND + F) { w[k + 1] = ORC_LTE_NULL; wKpi2[k2] = ORC_LTE_NULL; }
    if (index + 64 < ND + F) { w[k + 2] = ORC_LTE_NULL; wKpi4[k2] = ORC_LTE_NULL; }
    if (index + 1 < ND) wKpi1[k2] = ORC_LTE_NULL;
    k += RTC;
    k2 = k << 1;
  }
  if (ND > 0) w[3 * Kpi - 1] = ORC_LTE_NULL;
  return RTC;
}

/* lte_rate_matching_turbo_rx (lte_rate_matching.c:688-831): w[ind] += soft (int16 wrap) */
int orc_rate_matching_turbo_rx(uint32_t RTC, uint32_t G, int16_t *w, const uint8_t *dummy_w, const int16_t *soft_input,
                               uint8_t C, uint32_t Nsoft, uint8_t Mdlharq, uint8_t Kmimo, uint8_t rvidx, uint8_t clear,
                               uint8_t Qm, uint8_t Nl, uint8_t r, uint32_t *E_out)
{
  if (Kmimo == 0 || Mdlharq == 0 || C == 0 || Qm == 0 || Nl == 0) return -1;
  uint32_t Nir = Nsoft / Kmimo / (Mdlharq < 8 ? Mdlharq : 8);
  uint32_t Ncb = (Nir / C < 3 * (RTC << 5)) ? Nir / C : 3 * (RTC << 5);
  uint32_t Gp = G / Nl / Qm, GpmodC = Gp % C, E;
  if (r < C - GpmodC) E = Nl * Qm * (Gp / C);
  else E = Nl * Qm * ((GpmodC == 0 ? 0 : 1) + (Gp / C));
  uint32_t Ncbmod = Ncb % (RTC << 3);
  uint32_t ind = RTC * (2 + (rvidx * (((Ncbmod == 0) ? 0 : 1) + (Ncb / (RTC << 3))) * 2));
  if (clear == 1) memset(w, 0, Ncb * sizeof(int16_t));
  uint32_t k = 0;
  for (; ind < Ncb && k < E; ind++)
    if (dummy_w[ind] != ORC_LTE_NULL) w[ind] = (int16_t)(w[ind] + soft_input[k++]);
  while (k < E)
    for (ind = 0; ind < Ncb && k < E; ind++)
      if (dummy_w[ind] != ORC_LTE_NULL) w[ind] = (int16_t)(w[ind] + soft_input[k++]);
  *E_out = E;
  return 0;
}

/* sub_block_deinterleaving_turbo (lte_rate_matching.c:193-243): d = &d_buf[96], 96 writable
 * entries before it */
void orc_sub_block_deinterleaving_turbo(uint32_t D, int16_t *d, const int16_t *w)
{
  uint32_t RTC = D >> 5;
  if (D & 0x1f) RTC++;
  const uint32_t Kpi = RTC << 5, ND = Kpi - D, ND3 = ND * 3;
  static const uint8_t bitrev[32] = {0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30,
                                     1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31};
  int16_t *d1 = d - ND3, *d2 = d1 + 1, *d3 = d1 + 5;
  uint32_t k = 0, k2 = 0;
  for (uint32_t col = 0; col < 32; col++) {
    uint32_t index3 = 3 * bitrev[col];
    for (uint32_t row = 0; row < RTC; row++) {
      d1[index3] = w[k];
      d2[index3] = w[Kpi + k2];
      d3[index3] = w[Kpi + 1 + k2];
      index3 += 96;
      k++;
      k2 += 2;
    }
  }
}
