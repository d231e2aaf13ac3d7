/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle of the UE's downlink channel estimation from the
 * cell-specific reference signals, a plain-C restatement of the reference's
 * algorithm loop for loop; never linked into the product library.
 *
 *   lte_dl_channel_estimation  PHY/LTE_ESTIMATION/lte_dl_channel_estimation.c:37-623, 629-701
 *                              (N_RB_DL 6 / 50 / 100, 25 and 15 branches; high_speed_flag = 1, dlsim.c:2057 and
 *                              lte_init.c:1212; perfect_ce = 0; eNB_offset 0; one RX antenna).
 *                              The final idft of the estimate into dl_ch_estimates_time (:704-738,
 *                              the UE timing tracker's input): orc_chest_time.
 *   lte_est_freq_offset        PHY/LTE_ESTIMATION/lte_est_freq_offset.c:45-193 (dl_channel_level, the
 *                              two half-band dot products, atan2 and the moving-average filter):
 *                              orc_fo_channel_level / orc_fo_omega / orc_fo_update
 *   dot_product                PHY/TOOLS/cdot_prod.c:40-118 (pinned to the reference TU compiled
 *                              into oracle/_ref/libref_tools.so)
 *   lte_dl_cell_spec_rx        PHY/LTE_REFSIG/lte_dl_cell_spec.c:205-260 (conjugated QPSK pilots,
 *                              amplitude ONE_OVER_SQRT2_Q15)
 *   multadd_real_vector_complex_scalar  PHY/TOOLS/cmult_sv.c:81-122 (mulhi << 2, adds)
 *   multadd_complex_vector_real_scalar  cmult_sv.c:55-80 (mulhi << 1, optional adds); both pinned to the
 *                              reference TU compiled into oracle/_ref/libref_tools.so
 *   filt24_* interpolation filters      PHY/LTE_ESTIMATION/filt96_32.h, restated by formula in
 *                              orc_chest_filters (tests/test_chest_cpu.py checks them entry by
 *                              entry against the header when the reference tree is present).
 *
 * dl_ch_estimates holds one row of ofdm_symbol_size words per OFDM symbol of the subframe
 * (high_speed_flag = 1: ch_offset = symbol * ofdm_symbol_size), subcarrier i of RB rb at
 * 5 + 12 rb + i, the layout dlsch_extract_rbs_single reads.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oai_oracle.h"

static int16_t sat16(int32_t v) { return (int16_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v)); }

/* floor(16384 v / 6): the ramp levels of every filt24 table */
static int16_t lvl(int v) { return (int16_t)((16384 * v) / 6); }

/* the six filters one pilot symbol uses, for pilot offset k = (nu + nushift) % 6
 * (lte_dl_channel_estimation.c:105-180): [0] fl (first pilot), [1] f2l2 (second pilot),
 * [2] f (even pilots), [3] f2 (odd pilots), [4] fr (last-but-one pilot), [5] f2r2 (last pilot).
 * Shapes (s = filter shift, u = tap - s):
 *   filt24_s   : triangle lvl(6 - |u - 5|) on u in [0, 10]
 *   filt24_sl  : left-edge ramp lvl(11 - u) on [0, 10]      (filt24_3l: taps 3, 4 zeroed)
 *   filt24_sl2 : triangle plus -lvl(-u - 1) on u in [-6, -1] (filt24_5l2: tap 0 zeroed)
 *   filt24_sr  : right-edge ramp lvl(u + 1) on [0, 10]
 *   filt24_sr2 : triangle plus -lvl(u - 11) on u in [11, 16] */
void orc_chest_filters(uint8_t k, int16_t out[6][24])
{
  memset(out, 0, sizeof(int16_t) * 6 * 24);
  const int s1 = k, s2 = k + 2;
  for (int t = 0; t < 24; t++) {
    const int u1 = t - s1, u2 = t - s2;
    const int16_t tri1 = (u1 >= 0 && u1 <= 10) ? lvl(6 - abs(u1 - 5)) : 0;
    const int16_t tri2 = (u2 >= 0 && u2 <= 10) ? lvl(6 - abs(u2 - 5)) : 0;
    out[2][t] = tri1;
    out[3][t] = tri2;
    if (k == 0) {                                          /* :106-119 */
      out[0][t] = tri1;
      out[1][t] = tri2;
      out[4][t] = (u1 >= 11 && u1 <= 16) ? (int16_t)-lvl(u1 - 11) : tri1;     /* filt24_0r2 */
      out[5][t] = (u2 >= 0 && u2 <= 10) ? lvl(u2 + 1) : 0;                     /* filt24_2r */
    } else {
      out[0][t] = (u1 >= 0 && u1 <= 10) ? lvl(11 - u1) : 0;                    /* filt24_kl */
      if (k == 3 && (t == 3 || t == 4)) out[0][t] = 0;
      out[1][t] = (u2 >= -6 && u2 <= -1) ? (int16_t)-lvl(-u2 - 1) : tri2;      /* filt24_(k+2)l2 */
      if (k == 3 && t == 0) out[1][t] = 0;
      out[4][t] = (u1 >= 11 && u1 <= 16) ? (int16_t)-lvl(u1 - 11) : tri1;     /* filt24_kr2 */
      out[5][t] = (u2 >= 0 && u2 <= 10) ? lvl(u2 + 1) : 0;                     /* filt24_(k+2)r */
    }
  }
}

/* The DC-pair filters of the 25-PRB interpolator (filt96_32.h:35-113), reference data (their
 * right / left slopes round irregularly, so they are kept as the table entries):
 * filt24_k_dcr for the last pilot below DC, filt24_(k+2)_dcl for the first one above it
 * (lte_dl_channel_estimation.c:116-173). */
static const int16_t dcr_tab[6][24] = {
  {2730, 5461, 8192, 10922, 13653, 16384, 14043, 11703, 9362, 7022, 4681, 0},
  {0, 2730, 5461, 8192, 10922, 13653, 16384, 14043, 11703, 9362, 7022, 4681},
  {0, 0, 2730, 5461, 8192, 10922, 13653, 16384, 14043, 11703, 9362, 4681, 2341},
  {0, 0, 0, 2730, 5461, 8192, 10922, 13653, 16384, 14043, 11703, 7022, 4681, 2341},
  {0, 0, 0, 0, 2730, 5461, 8192, 10922, 13653, 16384, 14043, 11703, 7022, 4681, 2341},
  {0, 0, 0, 0, 0, 2730, 5461, 8192, 10922, 13653, 16384, 11703, 9362, 7022, 4681, 2730}};
static const int16_t dcl_tab[6][24] = {   /* filt24_2_dcl ... filt24_7_dcl */
  {0, 0, 2341, 4681, 7022, 9362, 11703, 16384, 13653, 10922, 8192, 5461, 2730},
  {0, 0, 0, 2341, 4681, 7022, 9362, 14043, 16384, 13653, 10922, 8192, 5461, 2730},
  {0, 0, 0, 0, 2341, 7022, 9362, 11703, 14043, 16384, 13653, 10922, 8192, 5461, 2730},
  {0, 0, 0, 0, 0, 2341, 4681, 9362, 11703, 14043, 16384, 13653, 10922, 8192, 5461, 2730},
  {0, 0, 0, 0, 0, 0, 4681, 7022, 9362, 11703, 14043, 16384, 13653, 10922, 8192, 5461, 2730},
  {0, 0, 0, 0, 0, 0, 0, 4681, 7022, 9362, 11703, 14043, 16384, 13653, 10922, 8192, 5461, 2730}};

void orc_chest_dc_filters(uint8_t k, int16_t out[2][24])
{
  memcpy(out[0], dcr_tab[k % 6], sizeof(out[0]));
  memcpy(out[1], dcl_tab[k % 6], sizeof(out[1]));
}

/* the filter of pilot m (of 2 N_RB): 6 / 50 / 100 PRB fl, f2l2 at the left edge and fr, f2r2 at
 * the right edge (:212-333); 25 PRB the same plus f_dc, f2_dc on pilots 24 / 25 (:338-533);
 * 15 PRB f / f2 throughout (:535-623) */
const int16_t *orc_chest_pilot_filter(const int16_t f[6][24], const int16_t fdc[2][24], int N_RB, int m)
{
  if (N_RB != 15) {
    if (m == 0) return f[0];
    if (m == 1) return f[1];
    if (m == 2 * N_RB - 2) return f[4];
    if (m == 2 * N_RB - 1) return f[5];
    if (N_RB == 25 && m == 24) return fdc[0];
    if (N_RB == 25 && m == 25) return fdc[1];
  }
  return (m & 1) ? f[3] : f[2];
}

/* multadd_complex_vector_real_scalar (cmult_sv.c:55-80): y = mulhi(x, alpha) << 1 (zero_flag 1)
 * or y +sat= that, per int16 of N complex entries */
void orc_multadd_complex_vector_real_scalar(const int16_t *x, int16_t alpha, int16_t *y, uint8_t zero_flag, uint32_t N)
{
  for (uint32_t n = 0; n < 2 * (N & ~3u); n++) {
    const int16_t m = (int16_t)(uint16_t)((uint32_t)(((int32_t)x[n] * alpha) >> 16) << 1);
    y[n] = zero_flag == 1 ? m : sat16((int32_t)y[n] + m);
  }
}

/* multadd_real_vector_complex_scalar (cmult_sv.c:81-122): for each real x[i], y[i] +sat=
 * (mulhi(alpha.re, x[i]) << 2, mulhi(alpha.im, x[i]) << 2), N (a multiple of 8) entries */
void orc_multadd_real_vector_complex_scalar(const int16_t *x, const int16_t *alpha, int16_t *y, uint32_t N)
{
  for (uint32_t i = 0; i < (N & ~7u); i++)
    for (int c = 0; c < 2; c++) {
      const int16_t v = (int16_t)(uint16_t)((uint32_t)(((int32_t)alpha[c] * x[i]) >> 16) << 2);
      y[2 * i + c] = sat16((int32_t)y[2 * i + c] + v);
    }
}

static void multadd_row(const int32_t *x, int16_t alpha, int32_t *y, int zero_flag, int N)
{
  orc_multadd_complex_vector_real_scalar((const int16_t *)x, alpha, (int16_t *)y, (uint8_t)zero_flag, (uint32_t)N);
}

int orc_lte_dl_channel_estimation(const orc_frame_t *fp, const uint32_t gold[20][2][14], const int32_t *rxdataF,
                                  int32_t *dl_ch_estimates, uint8_t Ns, uint8_t p, uint8_t l, uint8_t symbol)
{
  const int N = fp->ofdm_symbol_size, N_RB = fp->N_RB_DL;
  const int pilot1 = fp->Ncp == 0 ? 4 : 3, pilot2 = fp->Ncp == 0 ? 7 : 6, pilot3 = fp->Ncp == 0 ? 11 : 9;
  int nu;
  if (p == 0) nu = l == 0 ? 0 : 3;                          /* :76-87 */
  else if (p == 1) nu = l == 0 ? 3 : 0;
  else return -1;
  const int k = (nu + fp->nushift) % 6;
  int16_t f[6][24], fdc[2][24];
  orc_chest_filters((uint8_t)k, f);
  orc_chest_dc_filters((uint8_t)k, fdc);
  /* lte_dl_cell_spec_rx: conjugated QPSK pilots, m' = 110 - N_RB_DL + m */
  const int16_t pamp = 23170;
  const int16_t qpsk[4][2] = {{pamp, (int16_t)-pamp}, {(int16_t)-pamp, (int16_t)-pamp}, {pamp, pamp}, {(int16_t)-pamp, pamp}};
  const int32_t *rx = rxdataF + symbol * N;
  int32_t *dl_ch = dl_ch_estimates + N * symbol;            /* ch_offset, high_speed_flag = 1 */
  memset(dl_ch, 0, sizeof(int32_t) * N);
  const int even = N_RB == 6 || N_RB == 50 || N_RB == 100;
  if (even || N_RB == 15 || N_RB == 25) {
    /* pilot m of 2 N_RB, left to right; the first N_RB sit above first_carrier_offset, the rest
     * from bin 1 (DC skipped).  15 PRB restarts the second half at 1 + nushift + 3 p instead of
     * 1 + k (:582), whatever nu is: reproduced. */
    const int off2 = N_RB == 15 ? 1 + fp->nushift + 3 * p : 1 + k;
    const int l01 = l == 0 ? 0 : 1;
    for (int m = 0; m < 2 * N_RB; m++) {
      const int mp = 110 - N_RB + m;
      const int16_t *pil = qpsk[(gold[Ns][l01][mp >> 4] >> (2 * (mp & 15))) & 3];
      const int32_t word = m < N_RB ? rx[fp->first_carrier_offset + k + 6 * m] : rx[off2 + 6 * (m - N_RB)];
      int16_t r[2];
      memcpy(r, &word, 4);
      int16_t ch[2];
      ch[0] = (int16_t)(((int32_t)pil[0] * r[0] - (int32_t)pil[1] * r[1]) >> 15);
      ch[1] = (int16_t)(((int32_t)pil[0] * r[1] + (int32_t)pil[1] * r[0]) >> 15);
      const int16_t *flt = orc_chest_pilot_filter(f, fdc, N_RB, m);
      /* dl_ch advances 4 entries after an even pilot and 8 after an odd one (also across the DC
       * pair of 15 / 25 PRB, :431-457, :573-592) */
      int32_t *y = dl_ch + 12 * (m >> 1) + 4 * (m & 1);
      orc_multadd_real_vector_complex_scalar(flt, ch, (int16_t *)y, 24);
    }
  }                                                          /* other N_RB: "not implemented", row stays 0 */
  /* temporal interpolation (high_speed_flag = 1, :639-698) */
  int32_t *E = dl_ch_estimates;
#define ROW(r) (E + (r) * N)
  if (symbol == 0) {
    multadd_row(ROW(pilot3), 21845, ROW(pilot3 + 1), 1, N);
    multadd_row(dl_ch, 10923, ROW(pilot3 + 1), 0, N);
    multadd_row(ROW(pilot3), 10923, ROW(pilot3 + 2), 1, N);
    multadd_row(dl_ch, 21845, ROW(pilot3 + 2), 0, N);
  } else if (symbol == pilot1) {
    if (fp->Ncp == 0) {
      multadd_row(ROW(0), 24576, ROW(1), 1, N);
      multadd_row(dl_ch, 8192, ROW(1), 0, N);
      multadd_row(ROW(0), 16384, ROW(2), 1, N);
      multadd_row(dl_ch, 16384, ROW(2), 0, N);
      multadd_row(ROW(0), 8192, ROW(3), 1, N);
      multadd_row(dl_ch, 24576, ROW(3), 0, N);
    } else {                                                 /* 1/3, 2/3 as the reference weights them */
      multadd_row(ROW(0), 10923, ROW(1), 1, N);
      multadd_row(dl_ch, 21845, ROW(1), 0, N);
      multadd_row(ROW(0), 21845, ROW(2), 1, N);
      multadd_row(dl_ch, 10923, ROW(2), 0, N);
    }
  } else if (symbol == pilot2) {
    multadd_row(ROW(pilot1), 21845, ROW(pilot1 + 1), 1, N);
    multadd_row(dl_ch, 10923, ROW(pilot1 + 1), 0, N);
    multadd_row(ROW(pilot1), 10923, ROW(pilot1 + 2), 1, N);
    multadd_row(dl_ch, 21845, ROW(pilot1 + 2), 0, N);
  } else {                                                   /* symbol == pilot3 */
    if (fp->Ncp == 0) {
      multadd_row(ROW(pilot2), 24576, ROW(pilot2 + 1), 1, N);
      multadd_row(dl_ch, 8192, ROW(pilot2 + 1), 0, N);
      multadd_row(ROW(pilot2), 16384, ROW(pilot2 + 2), 1, N);
      multadd_row(dl_ch, 16384, ROW(pilot2 + 2), 0, N);
      multadd_row(ROW(pilot2), 8192, ROW(pilot2 + 3), 1, N);
      multadd_row(dl_ch, 24576, ROW(pilot2 + 3), 0, N);
    } else {
      multadd_row(ROW(pilot2), 10923, ROW(pilot2 + 1), 1, N);
      multadd_row(dl_ch, 21845, ROW(pilot2 + 1), 0, N);
      multadd_row(ROW(pilot2), 21845, ROW(pilot2 + 2), 1, N);
      multadd_row(dl_ch, 10923, ROW(pilot2 + 2), 0, N);
    }
  }
#undef ROW
  return 0;
}

/* ---- frequency-offset estimation (PHY/LTE_ESTIMATION/lte_est_freq_offset.c:45-193) and the
 *      time-domain estimate (lte_dl_channel_estimation.c:704-738) ----
 * All 32-bit sums wrap (the reference's epi32 lanes); they are taken mod 2^32 here, so the
 * order of the additions does not matter. */

/* dl_channel_level (lte_est_freq_offset.c:45-102): sum of re^2 + im^2 (madd_epi16, wrapping
 * epi32 lanes) over N_RB_DL * 12 REs, divided by N_RB_DL * 12 (C int division). */
int32_t orc_fo_channel_level(const int16_t *dl_ch, int N_RB)
{
  uint32_t acc = 0;
  for (int i = 0; i < N_RB * 12; i++) {
    const int32_t re = dl_ch[2 * i], im = dl_ch[2 * i + 1];
    acc += (uint32_t)(re * re) + (uint32_t)(im * im);     /* madd_epi16: the pair sum wraps */
  }
  return (int32_t)acc / (N_RB * 12);
}

/* dot_product (PHY/TOOLS/cdot_prod.c:40-118): sum over N complex of
 *   re: (xr yr + xi yi) >> shift,  im: (xr yi - xi yr) >> shift   (each madd wraps, srai per RE)
 * then packs_pi32: both sums saturated to int16; result = re | im << 16. */
int32_t orc_dot_product(const int16_t *x, const int16_t *y, uint32_t N, uint8_t shift)
{
  uint32_t sre = 0, sim = 0;
  for (uint32_t i = 0; i < (N & ~3u); i++) {
    const int32_t xr = x[2 * i], xi = x[2 * i + 1], yr = y[2 * i], yi = y[2 * i + 1];
    /* _mm_sign_epi16(y_swapped, (1, -1)): -yr, with -(-32768) = -32768 */
    const int32_t nyr = (int16_t)(-yr);
    const int32_t re = (int32_t)((uint32_t)(xr * yr) + (uint32_t)(xi * yi));
    const int32_t im = (int32_t)((uint32_t)(xr * yi) + (uint32_t)(xi * nyr));
    sre += (uint32_t)(re >> shift);
    sim += (uint32_t)(im >> shift);
  }
  return (int32_t)(((uint32_t)(uint16_t)sat16((int32_t)sre)) | ((uint32_t)(uint16_t)sat16((int32_t)sim) << 16));
}

/* lte_est_freq_offset's integer part (:125-166), antenna 0 only (:135): dl_ch_shift from the
 * channel level of row l at offset 12, then omega from dot(row l, previous pilot row) over the
 * lower half (from RE 12) and the upper half (from RE (N_RB/2 + 1) * 12), (N_RB/2 - 1) * 12 REs
 * each.  The intended sum of the two is not what the reference computes: omega_cpx points at omega
 * itself (:152), so the upper half's dot product overwrites the lower's (:164) before
 * omega_cpx->r += omega.r (:165-166) doubles it — omega = 2 x the upper half, int16 wrap per
 * component (checked against the TU compiled here, tests/test_ref_pin_fo_cpu.py).  Returns omega
 * (re | im << 16), or -1 << 31 for an l other than 0 or 4 - Ncp (the reference prints and returns -1
 * without touching freq_offset). */
int32_t orc_fo_omega(const orc_frame_t *fp, const int32_t *dl_ch_estimates0, int l)
{
  const int N = fp->ofdm_symbol_size, N_RB = fp->N_RB_DL, lp = 4 - fp->Ncp;
  if (l != 0 && l != lp) return INT32_MIN;
  const int ch_offset = l * N;
  const int16_t *dl_ch = (const int16_t *)&dl_ch_estimates0[12 + ch_offset];
  const uint8_t shift = (uint8_t)(6 + orc_log2_approx((uint32_t)orc_fo_channel_level(dl_ch, N_RB)) / 2);
  const int16_t *prev = (const int16_t *)&dl_ch_estimates0[12 + (ch_offset == 0 ? lp * N : 0)];
  const uint32_t n = (uint32_t)((N_RB / 2 - 1) * 12);
  (void)prev;                                   /* the lower half's dot product (:150) is overwritten */
  const int hi = (N_RB / 2 + 1) * 12;
  dl_ch = (const int16_t *)&dl_ch_estimates0[hi + ch_offset];
  prev = (const int16_t *)&dl_ch_estimates0[hi + (ch_offset == 0 ? lp * N : 0)];
  const int32_t o2 = orc_dot_product(dl_ch, prev, n, shift);
  const int16_t re = (int16_t)((int16_t)o2 + (int16_t)o2), im = (int16_t)((int16_t)(o2 >> 16) + (int16_t)(o2 >> 16));
  return (int32_t)((uint32_t)(uint16_t)re | ((uint32_t)(uint16_t)im << 16));
}

/* lte_est_freq_offset's scalar tail (:168-182): phase = atan2(im, re); estimate =
 * (int)(phase / 2 pi / 285.8e-6 (normal CP) or 2.5e-4); first call (or after a reset) takes the
 * estimate, later calls filter with coef 2^10: (est * 1024 + f * 31743) >> 15.  *first_run plays
 * the reference's static first_run. */
void orc_fo_update(int Ncp, int32_t omega, int *freq_offset, int *first_run)
{
  const double phase = atan2((double)(int16_t)(omega >> 16), (double)(int16_t)omega);
  const int est = (int)(phase / (2 * M_PI) / (Ncp == 0 ? 285.8e-6 : 2.5e-4));
  if (*first_run == 1) {
    *freq_offset = est;
    *first_run = 0;
  } else
    *freq_offset = (est * (1 << 10) + *freq_offset * (32767 - (1 << 10))) >> 15;
}

/* dl_ch_estimates_time (lte_dl_channel_estimation.c:704-738): idft(log2_symbol_size; other sizes:
 * idft512) of the plane from word 8 (row 0 words 8..N-1, then row 1 words 0..7), scale 1. */
void orc_chest_time(const orc_frame_t *fp, const int32_t *dl_ch_estimates_plane, int32_t *time_out)
{
  int l2 = fp->log2_symbol_size;
  if (l2 < 7 || l2 > 11) l2 = 9;
  orc_idft(l2, (const int16_t *)(dl_ch_estimates_plane + 8), (int16_t *)time_out, 1);
}
