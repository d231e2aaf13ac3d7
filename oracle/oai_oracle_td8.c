/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle of the reference's 8-bit turbo decoder
 * (PHY/CODING/3gpplte_turbo_decoder_sse_8bit.c, phy_threegpplte_turbo_decoder8 :894-1658, the x86
 * branch), restated lane for lane over its 16 int8 SSE lanes = 16 windows of n/16 trellis steps.
 * Never linked into the product library.
 *
 * Scope: n a multiple of 16 and n >= 512.  For n mod 16 = 8 the reference reads its interleaver
 * table 8 entries past the block (init_td8 :869-889, into the next size's table) and runs its
 * re-run loop over uninitialised metrics; for n < 272 the L = 16 re-run reaches past the window.
 * Neither is restated.
 *
 *   input scaling   :1001-1031  mean |y| over the first 3 (n/16) + 1 vectors of 8 (the reference
 *                               adds |w4| and |w5| twice and skips w6, w7; abs_epi16 keeps
 *                               -32768), then y >> s packed with int8 saturation, s from the mean
 *                               (0 / 1 / 2 / 3, and 3 / 4 for the two halves of each pair at >= 128)
 *   demux           :1071-1077  s[16 step + window] = y8[3 (window n/16 + step)], parities alike
 *   termination     :1300-1322, 193-207  read, but never used: the tail gammas only fed the
 *                               termination betas, which the reference replaces by 0 (:519-543)
 *   compute_gamma8  :151-191    m11 = (s + p) >> 1, m10 = (s - p) >> 1 (int16, packed to int8)
 *   compute_alpha8  :213-318    int8 saturating, re-run over L = 16 steps from the previous
 *                               window's final alpha (slli by one lane, window 0 = (0, -63 ...))
 *   compute_beta8   :412-680    seeded with the final alpha, window 15 = 0 in every state, re-run
 *                               over the last 16 steps from the next window's beta(0) (srli)
 *   compute_ext8    :682-827
 *   main loop       :1332-1656  exchanges through pi4 / pi5 (init_td8 :846-892), the hard
 *                               decisions of n mod 128 = 0 from ext2 deinterleaved (pi5), else
 *                               from ext2 + systematic2 through pi6, CRC24A / B early stop
 */
#include <stdlib.h>
#include <string.h>

#include "oai_oracle.h"
#include "../include/oai4g_qpp.h"

static int8_t s8(int v) { return (int8_t)(v > 127 ? 127 : (v < -128 ? -128 : v)); }
static int8_t adds8(int8_t a, int8_t b) { return s8((int)a + b); }
static int8_t subs8(int8_t a, int8_t b) { return s8((int)a - b); }
static int8_t max8(int8_t a, int8_t b) { return a > b ? a : b; }

#define W 16
#define L8 16
#define A(buf, k, s, w) (buf)[(((size_t)(k) * 8 + (s)) * W) + (w)]

static void gamma8(int8_t *m11, int8_t *m10, const int8_t *sys, const int8_t *par, int n)
{
  for (int e = 0; e < n; e++) {
    m11[e] = s8(((int)sys[e] + par[e]) >> 1);
    m10[e] = s8(((int)sys[e] - par[e]) >> 1);
  }
}

static void alpha8(int8_t *alpha, const int8_t *m11, const int8_t *m10, int n)
{
  const int K1 = n / W;
  for (int s = 0; s < 8; s++)
    for (int w = 0; w < W; w++) A(alpha, 0, s, w) = (s == 0 && w == 0) ? 0 : -63;
  for (int pass = 0, loopval = K1; pass < 2; pass++, loopval = L8) {
    for (int k = 0; k < loopval; k++)
      for (int w = 0; w < W; w++) {
        const int8_t g11 = m11[W * k + w], g10 = m10[W * k + w];
        int8_t a[8], r[8];
        for (int s = 0; s < 8; s++) a[s] = A(alpha, k, s, w);
        r[0] = max8(adds8(a[1], g11), subs8(a[0], g11));
        r[1] = max8(subs8(a[3], g10), adds8(a[2], g10));
        r[2] = max8(adds8(a[5], g10), subs8(a[4], g10));
        r[3] = max8(subs8(a[7], g11), adds8(a[6], g11));
        r[4] = max8(subs8(a[1], g11), adds8(a[0], g11));
        r[5] = max8(adds8(a[3], g10), subs8(a[2], g10));
        r[6] = max8(subs8(a[5], g10), adds8(a[4], g10));
        r[7] = max8(adds8(a[7], g11), subs8(a[6], g11));
        int8_t m = r[0];
        for (int s = 1; s < 8; s++) m = max8(m, r[s]);
        for (int s = 0; s < 8; s++) A(alpha, k + 1, s, w) = subs8(r[s], m);
      }
    /* slli_si128 by one lane: window w starts from window w - 1's last alpha, window 0 known */
    for (int s = 0; s < 8; s++) {
      for (int w = W - 1; w > 0; w--) A(alpha, 0, s, w) = A(alpha, K1, s, w - 1);
      A(alpha, 0, s, 0) = s == 0 ? 0 : -63;
    }
  }
}

static void beta8(const int8_t *alpha, int8_t *beta, const int8_t *m11, const int8_t *m10, int n)
{
  const int K1 = n / W;
  for (int s = 0; s < 8; s++)
    for (int w = 0; w < W; w++) A(beta, K1, s, w) = A(alpha, K1, s, w);
  for (int pass = 0, loopval = 0; pass < 2; pass++, loopval = K1 - L8) {
    for (int s = 0; s < 8; s++) A(beta, K1, s, W - 1) = 0;     /* offset8_flag = 0: "FIXME" zeros */
    for (int k = K1 - 1; k >= loopval; k--)
      for (int w = 0; w < W; w++) {
        const int8_t g11 = m11[W * k + w], g10 = m10[W * k + w];
        int8_t b[8], r[8];
        for (int s = 0; s < 8; s++) b[s] = A(beta, k + 1, s, w);
        r[0] = max8(adds8(b[4], g11), subs8(b[0], g11));
        r[1] = max8(subs8(b[4], g11), adds8(b[0], g11));
        r[2] = max8(subs8(b[5], g10), adds8(b[1], g10));
        r[3] = max8(adds8(b[5], g10), subs8(b[1], g10));
        r[4] = max8(adds8(b[6], g10), subs8(b[2], g10));
        r[5] = max8(subs8(b[6], g10), adds8(b[2], g10));
        r[6] = max8(subs8(b[7], g11), adds8(b[3], g11));
        r[7] = max8(adds8(b[7], g11), subs8(b[3], g11));
        int8_t m = r[0];
        for (int s = 1; s < 8; s++) m = max8(m, r[s]);
        for (int s = 0; s < 8; s++) A(beta, k, s, w) = subs8(r[s], m);
      }
    /* srli_si128 by one lane: window w ends at window w + 1's beta(0), window 15 at 0 */
    for (int s = 0; s < 8; s++) {
      for (int w = 0; w < W - 1; w++) A(beta, K1, s, w) = A(beta, 0, s, w + 1);
      A(beta, K1, s, W - 1) = 0;
    }
  }
}

static void ext8(const int8_t *alpha, const int8_t *beta, const int8_t *m11, const int8_t *m10, int8_t *ext, int n)
{
  const int K1 = n / W;
  for (int k = 0; k < K1; k++)
    for (int w = 0; w < W; w++) {
      int8_t a[8], b[8];
      for (int s = 0; s < 8; s++) {
        a[s] = A(alpha, k, s, w);
        b[s] = A(beta, k + 1, s, w);
      }
      const int8_t g11 = m11[W * k + w], g10 = m10[W * k + w];
      int8_t m00 = max8(max8(max8(adds8(a[0], b[0]), adds8(a[1], b[4])), adds8(a[6], b[7])), adds8(a[7], b[3]));
      int8_t m11v = max8(max8(max8(adds8(a[0], b[4]), adds8(a[1], b[0])), adds8(a[6], b[3])), adds8(a[7], b[7]));
      int8_t m01 = max8(max8(max8(adds8(a[2], b[5]), adds8(a[3], b[1])), adds8(a[4], b[2])), adds8(a[5], b[6]));
      int8_t m10v = max8(max8(max8(adds8(a[2], b[1]), adds8(a[3], b[5])), adds8(a[4], b[6])), adds8(a[5], b[2]));
      m01 = subs8(m01, g10);
      m00 = subs8(m00, g11);
      m10v = adds8(m10v, g10);
      m11v = adds8(m11v, g11);
      ext[W * k + w] = subs8(max8(m10v, m11v), max8(m01, m00));
    }
}

static void log_map8(const int8_t *sys, const int8_t *par, int8_t *m11, int8_t *m10, int8_t *alpha, int8_t *beta,
                     int8_t *ext, int n)
{
  gamma8(m11, m10, sys, par, n);
  alpha8(alpha, m11, m10, n);
  beta8(alpha, beta, m11, m10, n);
  ext8(alpha, beta, m11, m10, ext, n);
}

/* init_td8 (:846-892) for n mod 16 = 0 */
void orc_td8_tables(int n, int *pi2, int *pi4, int *pi5, int *pi6)
{
  const int qi = oai4g_qpp_index((uint32_t)n);
  const uint64_t f1 = oai4g_qpp_table[qi].f1, f2 = oai4g_qpp_table[qi].f2;
  for (int j = 0, i = 0; i < n; i++, j += W) {
    if (j >= n) j -= (n - 1);
    pi2[i] = j;
  }
  for (int i = 0; i < n; i++) {
    const int pi = (int)((f1 * (uint64_t)i + f2 * (uint64_t)i * (uint64_t)i) % (uint64_t)n), pi3 = pi2[pi];
    pi4[pi2[i]] = pi3;
    pi5[pi3] = pi2[i];
    pi6[pi] = pi2[i];
  }
}

/* the int16 -> int8 input conversion (:1001-1031): returns the shift pair used (s_lo | s_hi << 4) */
int orc_td8_input(const int16_t *y, int n, int8_t *y8)
{
  int32_t avg = 0;
  for (int i = 0; i < 3 * (n >> 4) + 1; i++) {
    const int16_t *v = y + 8 * i;
    int16_t a[8];
    for (int t = 0; t < 8; t++) a[t] = v[t] < 0 ? (int16_t)-v[t] : v[t];   /* -32768 stays */
    avg += a[0] + a[1] + a[2] + a[3] + 2 * a[4] + 2 * a[5];
  }
  const int32_t round_avg = avg / (n * 3);
  int sl, sh;
  if (round_avg < 16) sl = sh = 0;
  else if (round_avg < 32) sl = sh = 1;
  else if (round_avg < 64) sl = sh = 2;
  else if (round_avg < 128) sl = sh = 3;
  else { sl = 3; sh = 4; }
  for (int i = 0; i < 3 * (n >> 4) + 1; i++)
    for (int t = 0; t < 16; t++) y8[16 * i + t] = s8(y[16 * i + t] >> (t < 8 ? sl : sh));
  return sl | (sh << 4);
}

/* phy_threegpplte_turbo_decoder8.  y: 3n + 16 int16 readable (the reference's conversion reads 4
 * past the 3n + 12 entries; they only reach the unused tail).  Returns the iteration count,
 * max_iterations + 1 on CRC failure, 255 outside the restated scope. */
uint8_t orc_turbo_decoder8(const int16_t *y, uint8_t *decoded_bytes, uint16_t n, uint8_t max_iterations,
                           uint8_t crc_type, uint8_t F)
{
  if (crc_type > 1 || oai4g_qpp_index(n) < 0 || (n & 15) || n < 512) return 255;
  const int N = n + 32, K1 = n / W;
  int8_t *y8 = calloc(3 * (size_t)n + 64, 1);
  int8_t *s0 = calloc(N, 1), *s1 = calloc(N, 1), *s2 = calloc(N, 1), *yp1 = calloc(N, 1), *yp2 = calloc(N, 1),
         *ext = calloc(N, 1), *ext2 = calloc(N, 1), *tmp128 = calloc(N, 1), *m11 = calloc(N, 1), *m10 = calloc(N, 1);
  int8_t *alpha = calloc((size_t)(K1 + 2) * 8 * W, 1), *beta = calloc((size_t)(K1 + 2) * 8 * W, 1);
  int *pi2 = malloc(n * sizeof(int)), *pi4 = malloc(n * sizeof(int)), *pi5 = malloc(n * sizeof(int)),
      *pi6 = malloc(n * sizeof(int));
  orc_td8_tables(n, pi2, pi4, pi5, pi6);
  orc_td8_input(y, n, y8);
  for (int w = 0, t = 0; w < W; w++)
    for (int k = 0; k < K1; k++, t++) {
      s0[W * k + w] = y8[3 * t];
      yp1[W * k + w] = y8[3 * t + 1];
      yp2[W * k + w] = y8[3 * t + 2];
    }
  uint8_t it = 0, ret = 0;
  log_map8(s0, yp1, m11, m10, alpha, beta, ext, n);
  while (it++ < max_iterations) {
    for (int i = 0; i < n; i++) s2[i] = ext[pi4[i]];
    log_map8(s2, yp2, m11, m10, alpha, beta, ext2, n);
    for (int i = 0; i < n; i++) {
      const int8_t t = ext2[pi5[i]];
      if ((n & 0x7f) != 0) tmp128[i] = adds8(ext2[i], s2[i]);
      s1[i] = adds8(subs8(t, ext[i]), s0[i]);
    }
    if (it > 1) {
      /* natural bit order: window w holds bits [w n/16, (w + 1) n/16) */
      for (int b = 0; b < n; b++) {
        int bit;
        if ((n & 0x7f) == 0) {
          const int w = b / K1, k = b - w * K1;
          bit = ext2[pi5[W * k + w]] > 0;
        } else {
          bit = tmp128[pi6[b]] > 0;
        }
        if (bit) decoded_bytes[b >> 3] |= (uint8_t)(0x80 >> (b & 7));
        else decoded_bytes[b >> 3] &= (uint8_t)~(0x80 >> (b & 7));
      }
      uint32_t oldcrc = ((uint32_t)decoded_bytes[(n >> 3) - 3] | ((uint32_t)decoded_bytes[(n >> 3) - 2] << 8) |
                         ((uint32_t)decoded_bytes[(n >> 3) - 1] << 16)) & 0xffffff;
      uint32_t crc = crc_type == 0 ? orc_crc24a(decoded_bytes + (F >> 3), n - 24 - F) >> 8
                                   : orc_crc24b(decoded_bytes, n - 24) >> 8;
      crc = ((crc & 0xff) << 16) | (crc & 0xff00) | ((crc >> 16) & 0xff);
      if (crc == oldcrc && crc != 0) {
        ret = it;
        break;
      }
    }
    if (it < max_iterations) {
      log_map8(s1, yp1, m11, m10, alpha, beta, ext, n);
      for (int i = 0; i < n; i++) ext[i] = adds8(subs8(ext[i], s1[i]), s0[i]);
    }
  }
  if (!ret) ret = it;
  free(y8); free(s0); free(s1); free(s2); free(yp1); free(yp2); free(ext); free(ext2); free(tmp128); free(m11);
  free(m10); free(alpha); free(beta); free(pi2); free(pi4); free(pi5); free(pi6);
  return ret;
}
