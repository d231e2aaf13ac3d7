/*
 * CPU ORACLE — TEST INFRASTRUCTURE ONLY (see oai_oracle.h for the pinning story).
 *
 * Scalar restatement of the reference's PDSCH transmit path.  Every function names the
 * reference lines it follows.  Written for clarity and determinism, not speed; the SIMD
 * structure of the reference is replaced by explicit index algebra, while every rounding,
 * saturation and wrap point of the reference is kept so that outputs are bit-identical.
 */
#include "oai_oracle.h"
#include "../include/oai4g_qpp.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ======================================================================================
 * CRC — crc_byte.c:53-54 (polynomials), :62-83 (crcbit), :98-153 (byte tables / crc24a,b)
 * MSB-first CRC, zero init, no final xor; the 24-bit value is returned in the top 24
 * bits of a 32-bit word exactly as the reference does.
 * ==================================================================================== */
static uint32_t crc_tab_a[256], crc_tab_b[256];
static int crc_ready;

static uint32_t crc_byte_bitwise(uint8_t byte, uint32_t poly_top)
{
  uint32_t reg = 0, in = (uint32_t)byte << 24;
  for (int i = 0; i < 8; i++) {
    uint32_t fb = (reg ^ in) & 0x80000000u;
    reg <<= 1;
    if (fb) reg ^= poly_top;
    in <<= 1;
  }
  return reg;
}

void orc_crc_init(void)
{
  if (crc_ready) return;
  for (int v = 0; v < 256; v++) {
    crc_tab_a[v] = crc_byte_bitwise((uint8_t)v, 0x864cfb00u);
    crc_tab_b[v] = crc_byte_bitwise((uint8_t)v, 0x80006300u);
  }
  crc_ready = 1;
}

static uint32_t crc_run(const uint32_t *tab, const uint8_t *in, int bitlen)
{
  uint32_t reg = 0;
  int nbytes = bitlen / 8, rem = bitlen % 8;
  for (int i = 0; i < nbytes; i++) reg = (reg << 8) ^ tab[in[i] ^ (reg >> 24)];
  if (rem > 0) reg = (reg << rem) ^ tab[(in[nbytes] >> (8 - rem)) ^ (reg >> (32 - rem))];
  return reg;
}

uint32_t orc_crc24a(const uint8_t *in, int bitlen) { orc_crc_init(); return crc_run(crc_tab_a, in, bitlen); }
uint32_t orc_crc24b(const uint8_t *in, int bitlen) { orc_crc_init(); return crc_run(crc_tab_b, in, bitlen); }

/* ======================================================================================
 * Code-block segmentation — lte_segmentation.c:39-170 (36.212 §5.1.2).
 * ==================================================================================== */
int orc_segmentation(const uint8_t *b, uint8_t **c, uint32_t B, uint32_t *C, uint32_t *Cplus,
                     uint32_t *Cminus, uint32_t *Kplus, uint32_t *Kminus, uint32_t *F)
{
  uint32_t L, Bp, per;
  if (B <= 6144) { L = 0; *C = 1; Bp = B; }
  else { L = 24; *C = (B + (6144 - L) - 1) / (6144 - L); Bp = B + *C * L; }
  if (*C > 16) return -1;
  per = Bp / *C;
  if (per <= 40) { *Kplus = 40; *Kminus = 0; }
  else if (per <= 512) { *Kplus = (per >> 3) << 3; *Kminus = per - 8; }         /* :76-79 (floor!) */
  else if (per <= 1024) { *Kplus = ((per + 15) >> 4) << 4; *Kminus = *Kplus - 16; }
  else if (per <= 2048) { *Kplus = ((per + 31) >> 5) << 5; *Kminus = *Kplus - 32; }
  else if (per <= 6144) { *Kplus = ((per + 63) >> 6) << 6; *Kminus = *Kplus - 64; }
  else return -1;
  if (*C == 1) { *Cplus = 1; *Kminus = 0; *Cminus = 0; }
  else { *Cminus = (*C * *Kplus - Bp) / (*Kplus - *Kminus); *Cplus = *C - *Cminus; }
  *F = *Cplus * *Kplus + *Cminus * *Kminus - Bp;
  if (b && c) {
    uint32_t k = 0, s = 0;
    for (; k < (*F >> 3); k++) c[0][k] = 0;                                     /* :137-139 */
    for (uint32_t r = 0; r < *C; r++) {
      uint32_t Kr = (r < *Cminus) ? *Kminus : *Kplus;
      for (; k < ((Kr - L) >> 3); k++) c[r][k] = b[s++];
      if (*C > 1) {                                                             /* :156-166 */
        uint32_t crc = orc_crc24b(c[r], (int)(Kr - 24)) >> 8;
        c[r][(Kr - 24) >> 3] = (uint8_t)(crc >> 16);
        c[r][1 + ((Kr - 24) >> 3)] = (uint8_t)(crc >> 8);
        c[r][2 + ((Kr - 24) >> 3)] = (uint8_t)crc;
      }
      k = 0;
    }
  }
  return 0;
}

/* ======================================================================================
 * Turbo encoder — 3gpplte_sse.c:96-109 (RSC step, termination), :380-476 (encoder).
 * State bits (s2 s1 s0): s2 = newest register.  out = u^s2^s1, s' = ((u^s1^s0)<<2)|(s2<<1)|s1.
 * The SSE encoder ignores F (filler bits are encoded as 0, never NULLed: quirk A6q).
 * For K/8 odd the SSE encoder leaves the last byte of its interleaved-input buffer
 * uninitialised (3gpplte_sse.c:334, n>>1 words); the oracle follows the spec there.
 * ==================================================================================== */
static inline uint8_t rsc_step(uint8_t u, uint8_t *s)
{
  uint8_t st = *s;
  uint8_t out = (u ^ (st >> 2) ^ (st >> 1)) & 1;
  *s = (uint8_t)((((u << 2) ^ (st >> 1)) ^ ((st >> 1) << 2) ^ (st << 2)) & 7);
  return out;
}

static inline void rsc_term(uint8_t *x, uint8_t *z, uint8_t *s)
{
  *z = ((*s >> 2) ^ *s) & 1;
  *x = (*s ^ (*s >> 1)) & 1;
  *s = *s >> 1;
}

void orc_turbo_encode(const uint8_t *c, uint16_t nbytes, uint8_t *d, uint16_t f1, uint16_t f2)
{
  uint32_t K = (uint32_t)nbytes * 8;
  uint8_t s0 = 0, s1 = 0;
  for (uint32_t k = 0; k < K; k++) {
    uint8_t u = (c[k >> 3] >> (7 - (k & 7))) & 1;
    uint32_t pi = (uint32_t)(((uint64_t)f1 * k + (uint64_t)f2 * k * k) % K);
    uint8_t u2 = (c[pi >> 3] >> (7 - (pi & 7))) & 1;
    d[3 * k] = u;
    d[3 * k + 1] = rsc_step(u, &s0);
    d[3 * k + 2] = rsc_step(u2, &s1);
  }
  uint8_t *x = d + 3 * K;
  rsc_term(&x[0], &x[1], &s0);
  rsc_term(&x[2], &x[3], &s0);
  rsc_term(&x[4], &x[5], &s0);
  rsc_term(&x[6], &x[7], &s1);
  rsc_term(&x[8], &x[9], &s1);
  rsc_term(&x[10], &x[11], &s1);
}

/* ======================================================================================
 * Sub-block interleaver — lte_rate_matching.c:42 (column permutation), :51-130.
 * w[0..Kpi) = v0, w[Kpi+2k] = v1, w[Kpi+2k+1] = v2.  Side effect kept: d[3D+2] = d[2].
 * ==================================================================================== */
static const uint8_t col_perm[32] = {0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30,
                                     1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31};

uint32_t orc_subblock_interleave(uint32_t D, uint8_t *d, uint8_t *w)
{
  uint32_t R = (D + 31) >> 5, Kpi = R << 5, ND = Kpi - D;
  d[3 * D + 2] = d[2];
  const uint8_t *base = d - 3 * ND;                 /* NULL prefix supplies the dummies */
  uint32_t k = 0;
  for (uint32_t col = 0; col < 32; col++) {
    for (uint32_t row = 0; row < R; row++, k++) {
      uint32_t j = col_perm[col] + 32 * row;
      w[k] = base[3 * j];
      w[Kpi + 2 * k] = base[3 * j + 1];
      w[Kpi + 2 * k + 1] = base[3 * j + 5];
    }
  }
  if (ND > 0) w[3 * Kpi - 1] = ORC_LTE_NULL;
  return R;
}

/* ======================================================================================
 * Rate matching — lte_rate_matching.c:464-634 (36.212 §5.1.4.1.2).
 * ==================================================================================== */
/* opt-in limited-buffer rate matching (the build's extension): when set, Ncb < Kw
 * selects circularly from w[0..Ncb) (36.212 5.1.4.1.2) instead of the reference's E = 0 exit */
static int g_rm_limited = 0;
void orc_set_rm_limited(int on) { g_rm_limited = on; }

uint32_t orc_rate_match(uint32_t RTC, uint32_t G, const uint8_t *w, uint8_t *e, uint8_t C,
                        uint32_t Nsoft, uint8_t Mdlharq, uint8_t Kmimo, uint8_t rvidx, uint8_t Qm,
                        uint8_t Nl, uint8_t r)
{
  uint32_t Kw = 3 * (RTC << 5);
  uint32_t Nir = Nsoft / Kmimo / (Mdlharq < 8 ? Mdlharq : 8);
  uint32_t Ncb = (Nir / C < Kw) ? Nir / C : Kw;
  if (Ncb < Kw && !g_rm_limited) {                                              /* :518-521 */
    printf("Exiting, RM condition (Nir %u, Nsoft %u, Kw %u\n", Nir, Nsoft, Kw);
    return 0;
  }
  uint32_t Gp = G / Nl / Qm, GpmodC = Gp % C, E;
  if (r < (C - GpmodC)) E = Nl * Qm * (Gp / C);
  else E = Nl * Qm * ((GpmodC == 0 ? 0 : 1) + (Gp / C));
  uint32_t ncol8 = RTC << 3;
  uint32_t k0 = RTC * (2 + rvidx * ((Ncb % ncol8 ? 1 : 0) + Ncb / ncol8) * 2);
  uint32_t k = 0, ind = k0;
  for (; ind < Ncb && k < E; ind++)
    if (w[ind] != ORC_LTE_NULL) e[k++] = w[ind];
  while (k < E)
    for (ind = 0; ind < Ncb && k < E; ind++)
      if (w[ind] != ORC_LTE_NULL) e[k++] = w[ind];
  return E;
}

/* ======================================================================================
 * Gold sequence — lte_gold.c:151-177; scrambling — dlsch_scrambling.c:51-97.
 * ==================================================================================== */
static inline void gold_step(uint32_t *x1, uint32_t *x2)
{
  *x1 = (*x1 >> 1) ^ (*x1 >> 4);
  *x1 = *x1 ^ (*x1 << 31) ^ (*x1 << 28);
  *x2 = (*x2 >> 1) ^ (*x2 >> 2) ^ (*x2 >> 3) ^ (*x2 >> 4);
  *x2 = *x2 ^ (*x2 << 31) ^ (*x2 << 30) ^ (*x2 << 29) ^ (*x2 << 28);
}

uint32_t orc_gold_generic(uint32_t *x1, uint32_t *x2, uint8_t reset)
{
  if (reset) {
    *x1 = 1u + (1u << 31);
    *x2 = *x2 ^ ((*x2 ^ (*x2 >> 1) ^ (*x2 >> 2) ^ (*x2 >> 3)) << 31);
    for (int n = 1; n < 50; n++) gold_step(x1, x2);
  }
  gold_step(x1, x2);
  return *x1 ^ *x2;
}

/* e must have room for (1 + G/32) * 32 entries: the reference overruns G (:83-92). */
void orc_scramble(uint8_t *e, int G, uint32_t c_init)
{
  uint32_t x1, x2 = c_init;
  uint32_t s = orc_gold_generic(&x1, &x2, 1);
  int k = 0;
  for (int i = 0; i < 1 + (G >> 5); i++) {
    for (int j = 0; j < 32; j++, k++) e[k] = (e[k] & 1) ^ ((s >> j) & 1);
    s = orc_gold_generic(&x1, &x2, 0);
  }
}

/* ======================================================================================
 * MCS helpers and G — lte_mcs.c:45-56 (get_Qm), :249-334 (adjust_G), :336-368 (get_G).
 * ==================================================================================== */
uint8_t orc_get_Qm(uint8_t mcs) { return mcs < 10 ? 2 : (mcs < 17 ? 4 : 6); }

static int rb_bit(const uint32_t *rb_alloc, int rb)
{
  if (rb < 32) return (rb_alloc[0] >> rb) & 1;
  if (rb < 64) return (rb_alloc[1] >> (rb - 32)) & 1;
  if (rb < 96) return (rb_alloc[2] >> (rb - 64)) & 1;
  if (rb < 100) return (rb_alloc[3] >> (rb - 96)) & 1;
  return 0;
}

static int orc_adjust_G(uint16_t N_RB_DL, uint8_t Ncp, uint8_t mode1_flag, uint8_t frame_type,
                        const uint32_t *rb_alloc, uint8_t Qm, uint8_t subframe)
{
  int re = 0;
  if (subframe != 0 && subframe != 5 && subframe != 6) return 0;
  int half = N_RB_DL >> 1;
  if (N_RB_DL & 1) {
    for (int rb = half - 3; rb <= half + 3; rb++)
      if (rb_bit(rb_alloc, rb)) re += (rb == half - 3 || rb == half + 3) ? 6 : 12;
  } else {
    for (int rb = half - 3; rb < half + 3; rb++)
      if (rb_bit(rb_alloc, rb)) re += 12;
  }
  if (subframe == 0) {
    if (frame_type == 1) return mode1_flag == 0 ? (-Ncp + 14) * re * Qm / 3 : (-Ncp + 29) * re * Qm / 6;
    return mode1_flag == 0 ? (-Ncp + 17) * re * Qm / 3 : (-Ncp + 35) * re * Qm / 6;
  }
  if (subframe == 5) return (frame_type == 0 ? 2 : 1) * re * Qm;
  if (subframe == 6 && frame_type == 1) return re * Qm;
  return 0;
}

int orc_get_G(uint16_t N_RB_DL, uint8_t Ncp, uint8_t mode1_flag, uint8_t frame_type, uint16_t nb_rb,
              const uint32_t *rb_alloc, uint8_t Qm, uint8_t Nl, uint8_t num_pdcch_symbols, uint8_t subframe)
{
  int adj = orc_adjust_G(N_RB_DL, Ncp, mode1_flag, frame_type, rb_alloc, Qm, subframe);
  int nd = (Ncp == 0) ? 11 : 9;
  if (mode1_flag == 0) return (((int)nb_rb * Qm * ((nd - num_pdcch_symbols) * 12 + 3 * 8)) - adj) * Nl;
  return ((int)nb_rb * Qm * ((nd - num_pdcch_symbols) * 12 + 3 * 10)) - adj;
}

/* ======================================================================================
 * Frame parameters — lte_parms.c:31-145 (osf = 1).
 * ==================================================================================== */
int orc_init_frame(orc_frame_t *fp, uint16_t N_RB_DL, uint16_t Nid_cell, uint8_t Ncp, uint8_t nb_antennas_tx,
                   uint8_t mode1_flag, uint8_t frame_type)
{
  memset(fp, 0, sizeof(*fp));
  fp->N_RB_DL = N_RB_DL; fp->Nid_cell = Nid_cell; fp->Ncp = Ncp; fp->nushift = Nid_cell % 6;
  fp->nb_antennas_tx = nb_antennas_tx; fp->mode1_flag = mode1_flag; fp->frame_type = frame_type;
  uint16_t cp0 = Ncp ? 512 : 160, cp = Ncp ? 512 : 144;
  fp->symbols_per_tti = Ncp ? 12 : 14;
  int sh;
  switch (N_RB_DL) {
  case 100: fp->ofdm_symbol_size = 2048; fp->log2_symbol_size = 11; sh = 0; break;
  case 50:  fp->ofdm_symbol_size = 1024; fp->log2_symbol_size = 10; sh = 1; break;
  case 25:  fp->ofdm_symbol_size = 512;  fp->log2_symbol_size = 9;  sh = 2; break;
  case 15:  fp->ofdm_symbol_size = 256;  fp->log2_symbol_size = 8;  sh = 3; break;
  case 6:   fp->ofdm_symbol_size = 128;  fp->log2_symbol_size = 7;  sh = 4; break;
  default: return -1;
  }
  fp->samples_per_tti = 30720u >> sh;
  fp->first_carrier_offset = fp->ofdm_symbol_size - 6 * N_RB_DL;
  fp->nb_prefix_samples = cp >> sh;
  fp->nb_prefix_samples0 = cp0 >> sh;
  fp->phich_resource = 6;              /* Ng = one, as dlsim.c:138 */
  fp->phich_duration = 0;
  fp->tdd_config = 3;
  fp->nb_antennas_tx_eNB = nb_antennas_tx;   /* dlsim.c:137 */
  return 0;
}

/* ======================================================================================
 * Modulation + RE mapping — dlsch_modulation.c:53-71 (is_not_pilot), :79-103 (QAM tables),
 * :139-982 (allocate_REs_in_RB: SISO, ALAMOUTI and LARGE_CDD branches), :1181-1493 (dlsch_modulation).
 * ==================================================================================== */
/* int tables, as the reference's (LTE_TRANSPORT/vars.h:72 `int qam64_table[8],qam16_table[4]`):
 * the outer 64-QAM level 20225 + 10112 + 5056 = 35393 does not fit int16 and must not wrap */
static int32_t qam16_tab[4], qam64_tab[8];

static void qam_tables(void)
{
  for (int a = -1; a <= 1; a += 2)
    for (int b = -1; b <= 1; b += 2) {
      qam16_tab[(1 + a) + (1 + b) / 2] = -a * (20724 + b * 10362);
      for (int c = -1; c <= 1; c += 2)
        qam64_tab[(1 + a) * 2 + (1 + b) + (1 + c) / 2] = -a * (20225 + b * (10112 + c * 5056));
    }
}

static int not_pilot(int pilots, int re, int nushift, int use2nd)
{
  int off = (pilots == 2) ? 3 : 0, v = nushift % 3;
  if (pilots == 0) return 1;
  if (use2nd) return (re != nushift + off) && (re != ((nushift + 6 + off) % 12));
  return (re != v) && (re != v + 6) && (re != v + 3) && (re != v + 9);
}

/* Reads Qm bits at *jj and returns the (re, im) table indices used by the reference. */
static void qam_index(const uint8_t *x, uint32_t *jj, int Qm, int *ire, int *iim)
{
  *ire = 0; *iim = 0;
  for (int b = 0; b < Qm; b += 2) {
    int wgt = 1 << ((Qm - 2 - b) >> 1);
    if (x[*jj] == 1) *ire += wgt;
    (*jj)++;
    if (x[*jj] == 1) *iim += wgt;
    (*jj)++;
  }
}

static void qam_symbol(const uint8_t *x, uint32_t *jj, int Qm, int16_t gain_qpsk, const int16_t *tab,
                       int16_t *re, int16_t *im)
{
  if (Qm == 2) {
    *re = (x[*jj] == 1) ? (int16_t)-gain_qpsk : gain_qpsk; (*jj)++;
    *im = (x[*jj] == 1) ? (int16_t)-gain_qpsk : gain_qpsk; (*jj)++;
    return;
  }
  int ir, ii;
  qam_index(x, jj, Qm, &ir, &ii);
  *re = tab[ir];
  *im = tab[ii];
}

static inline void acc16(int32_t *slot, int part, int v)
{
  int16_t *p = (int16_t *)slot;
  p[part] = (int16_t)(p[part] + v);
}

/* grid_sf: subframe index used for the grid offset (the reference uses subframe for both the
 * offset into a whole-frame txdataF and the PBCH/PSS/SSS exclusions). */
static int modulation_impl(int32_t **txdataF, int16_t amp, uint32_t subframe, uint32_t grid_sf,
                           const orc_frame_t *fp, uint8_t num_pdcch_symbols, const orc_cw_t *cw0,
                           const orc_cw_t *cw1, int16_t sqrt_rho_a, int16_t sqrt_rho_b)
{
  qam_tables();
  int nsymb = fp->Ncp == 0 ? 14 : 12;
  int Qm0 = orc_get_Qm(cw0->mcs), Qm1 = cw1 ? orc_get_Qm(cw1->mcs) : 0;
  int16_t amp_a = (int16_t)(((int32_t)amp * sqrt_rho_a) >> 13);
  int16_t amp_b = (int16_t)(((int32_t)amp * sqrt_rho_b) >> 13);
  int16_t t0a[8], t0b[8], t1a[8], t1b[8];
  const int32_t *src0 = Qm0 == 4 ? qam16_tab : qam64_tab, *src1 = Qm1 == 4 ? qam16_tab : qam64_tab;
  for (int i = 0; i < 8; i++) {
    t0a[i] = (int16_t)(((int32_t)src0[i & (Qm0 == 4 ? 3 : 7)] * amp_a) >> 15);
    t0b[i] = (int16_t)(((int32_t)src0[i & (Qm0 == 4 ? 3 : 7)] * amp_b) >> 15);
    t1a[i] = (int16_t)(((int32_t)src1[i & (Qm1 == 4 ? 3 : 7)] * amp_a) >> 15);
    t1b[i] = (int16_t)(((int32_t)src1[i & (Qm1 == 4 ? 3 : 7)] * amp_b) >> 15);
  }
  if (cw0->Nlayers > 1 || (cw1 && cw1->Nlayers > 1)) return -1;
  uint32_t jj = 0, jj2 = 0;
  int re_allocated = 0;
  int use2nd = fp->mode1_flag == 1;
  int N = fp->ofdm_symbol_size, half = fp->N_RB_DL >> 1;
  /* 4 TX antennas (configuration C4, a build-defined extension: the reference modulates 1 or 2
   * ports only): the CRS of ports 2/3 also occupy symbol 1 of each slot (36.211 6.10.1.2), with
   * the same four REs per RB as ports 0/1 (nu_shift mod 3 + {0, 3, 6, 9}) */
  const int ports4 = fp->nb_antennas_tx == 4, sps = nsymb >> 1;
  for (int l = num_pdcch_symbols; l < nsymb; l++) {
    int pilots;
    if (fp->Ncp == 0) pilots = (l == 4 || l == 11) ? 2 : (l == 7 ? 1 : 0);
    else pilots = (l == 3 || l == 9) ? 2 : (l == 6 ? 1 : 0);
    if (ports4 && l % sps == 1) pilots = 3;
    int re_offset = fp->first_carrier_offset;
    uint32_t symbol_offset = (uint32_t)N * (l + grid_sf * nsymb);
    for (int rb = 0; rb < fp->N_RB_DL; rb++) {
      int alloc = rb_bit(cw0->rb_alloc, rb);
      int skip_half = 0, skip_dc = 0;
      if (fp->N_RB_DL & 1) {                                                    /* :1303-1372 */
        skip_dc = (rb == half);
        if (subframe == 0 && rb > half - 3 && rb < half + 3 && l >= (nsymb >> 1) && l < (nsymb >> 1) + 4) alloc = 0;
        if (subframe == 0 && rb == half - 3 && l >= (nsymb >> 1) && l < (nsymb >> 1) + 4) skip_half = 1;
        else if (subframe == 0 && rb == half + 3 && l >= (nsymb >> 1) && l < (nsymb >> 1) + 4) skip_half = 2;
        if (fp->frame_type == 1) {
          if ((subframe == 0 || subframe == 5) && rb > half - 3 && rb < half + 3 && l == nsymb - 1) alloc = 0;
          if ((subframe == 0 || subframe == 5) && rb == half - 3 && l == nsymb - 1) skip_half = 1;
          else if ((subframe == 0 || subframe == 5) && rb == half + 3 && l == nsymb - 1) skip_half = 2;
          if ((subframe == 1 || subframe == 6) && rb > half - 3 && rb < half + 3 && l == 2) alloc = 0;
          if ((subframe == 1 || subframe == 6) && rb == half - 3 && l == 2) skip_half = 1;
          else if ((subframe == 1 || subframe == 6) && rb == half + 3 && l == 2) skip_half = 2;
        } else {
          int ls = (nsymb >> 1) - 1, lp = (nsymb >> 1) - 2;
          if ((subframe == 0 || subframe == 5) && rb > half - 3 && rb < half + 3 && l == ls) alloc = 0;
          if ((subframe == 0 || subframe == 5) && rb == half - 3 && l == ls) skip_half = 1;
          else if ((subframe == 0 || subframe == 5) && rb == half + 3 && l == ls) skip_half = 2;
          if ((subframe == 0 || subframe == 5) && rb > half - 3 && rb < half + 3 && l == lp) alloc = 0;
          if ((subframe == 0 || subframe == 5) && rb == half - 3 && l == lp) skip_half = 1;
          else if ((subframe == 0 || subframe == 5) && rb == half + 3 && l == lp) skip_half = 2;
        }
      } else {                                                                  /* :1373-1410 */
        if (subframe == 0 && rb >= half - 3 && rb < half + 3 && l >= (nsymb >> 1) && l < (nsymb >> 1) + 4) alloc = 0;
        if (fp->frame_type == 1) {
          if ((subframe == 0 || subframe == 5) && rb >= half - 3 && rb < half + 3 && l == nsymb - 1) alloc = 0;
          if ((subframe == 1 || subframe == 6) && rb >= half - 3 && rb < half + 3 && l == 2) alloc = 0;
        } else {
          if ((subframe == 0 || subframe == 5) && rb >= half - 3 && rb < half + 3 && l == (nsymb >> 1) - 2) alloc = 0;
          if ((subframe == 0 || subframe == 5) && rb >= half - 3 && rb < half + 3 && l == (nsymb >> 1) - 1) alloc = 0;
        }
      }
      const int16_t *tab0 = pilots ? t0b : t0a, *tab1 = pilots ? t1b : t1a;
      int16_t gain = (int16_t)(((pilots ? amp_b : amp_a) * 23170) >> 15);
      if (alloc) {                                                              /* allocate_REs_in_RB */
        int first = 0, last = 12, s = 1, re_off = re_offset;
        if (skip_half == 1) last = 6;
        else if (skip_half == 2) first = 6;
        for (int re = first; re < last; re++) {
          if (skip_dc && re == 6) re_off = re_off - N + 1;
          uint32_t tti = symbol_offset + re_off + re;
          if (!not_pilot(pilots, re, fp->nushift, use2nd)) continue;
          re_allocated++;
          if (!txdataF) continue;                                                /* count only (4-port G) */
          if (cw0->mimo_mode == 0) {                                            /* SISO :245-360 */
            int16_t vr, vi;
            qam_symbol(cw0->e, &jj, Qm0, gain, tab0, &vr, &vi);
            for (int aa = 0; aa < fp->nb_antennas_tx; aa++) {
              acc16(&txdataF[aa][tti], 0, vr);
              acc16(&txdataF[aa][tti], 1, vi);
            }
          } else if (cw0->mimo_mode == 2 && fp->nb_antennas_tx == 2) {         /* LARGE_CDD :547-749 */
            int16_t r0, i0, r1, i1;
            qam_symbol(cw0->e, &jj, Qm0, gain, tab0, &r0, &i0);
            if (cw1) qam_symbol(cw1->e, &jj2, Qm1, gain, tab1, &r1, &i1);
            else { r1 = 0; i1 = 0; }
            acc16(&txdataF[0][tti], 0, (r0 + r1) >> 1);
            acc16(&txdataF[1][tti], 0, s * ((r0 - r1) >> 1));
            acc16(&txdataF[0][tti], 1, (i0 + i1) >> 1);
            acc16(&txdataF[1][tti], 1, s * ((i0 - i1) >> 1));
            s = -s;
          } else if (cw0->mimo_mode == 2 && ports4) {
            /* 4-port large-delay CDD, rank 2 (36.211 6.3.4.2.2): y = W(i) D(i) U x(i) with
             * U = [[1, 1], [1, -1]]/sqrt2, D(i) = diag(1, (-1)^i), W(i) = C_k/sqrt2 for
             * k = floor(i/2) mod 4 over the codebook entries 12, 13, 14, 15 (Table 6.3.4.2.3-2,
             * rank-2 columns {1,2}, {1,3}, {1,3}, {1,2} of W_n = I - 2 u_n u_n^H / u_n^H u_n).
             * Every entry of 4 W D U is +-1, so y_p = (a_p (x0 + x1) + b_p s (x0 - x1)) / 4 with
             * i the layer-symbol (allocated RE) index of the subframe; rounded down (arithmetic
             * shift), accumulated into the int16 grid like the 2-port branch. */
            static const int8_t M4[4][4][2] = {{{1, 1}, {1, 1}, {1, -1}, {-1, 1}},    /* W_12^{12} */
                                               {{1, -1}, {1, 1}, {-1, 1}, {1, 1}},    /* W_13^{13} */
                                               {{1, 1}, {-1, 1}, {1, 1}, {1, -1}},    /* W_14^{13} */
                                               {{1, -1}, {-1, 1}, {-1, -1}, {-1, -1}}}; /* W_15^{12} */
            const int i = re_allocated - 1, k = (i >> 1) & 3, sg = (i & 1) ? -1 : 1;
            int16_t r0, i0, r1, i1;
            qam_symbol(cw0->e, &jj, Qm0, gain, tab0, &r0, &i0);
            if (cw1) qam_symbol(cw1->e, &jj2, Qm1, gain, tab1, &r1, &i1);
            else { r1 = 0; i1 = 0; }
            for (int p = 0; p < 4; p++) {
              const int a = M4[k][p][0], b = M4[k][p][1] * sg;
              acc16(&txdataF[p][tti], 0, (a * (r0 + r1) + b * (r0 - r1)) >> 2);
              acc16(&txdataF[p][tti], 1, (a * (i0 + i1) + b * (i0 - i1)) >> 2);
            }
          } else if (cw0->mimo_mode == 1 && fp->nb_antennas_tx == 2) {         /* ALAMOUTI :362-546 */
            /* antenna 0 at n: x0/sqrt2; antenna 1 at n: -conj(x1)/sqrt2 (both symbols from codeword 0) */
            int16_t amp2 = (int16_t)(((int32_t)(pilots ? amp_b : amp_a) * 23170) >> 15);
            int16_t v[4];
            if (Qm0 == 2) {
              const int16_t g = gain;
              int16_t t1r = (cw0->e[jj] == 1) ? (int16_t)-g : g; jj++;
              int16_t t1i = (cw0->e[jj] == 1) ? (int16_t)-g : g; jj++;
              int16_t t2r = (cw0->e[jj] == 1) ? g : (int16_t)-g; jj++;
              int16_t t2i = (cw0->e[jj] == 1) ? (int16_t)-g : g; jj++;
              v[0] = (int16_t)((t1r * 23170) >> 15); v[1] = (int16_t)((t1i * 23170) >> 15);
              v[2] = (int16_t)((t2r * 23170) >> 15); v[3] = (int16_t)((t2i * 23170) >> 15);
            } else {
              const int32_t *raw = Qm0 == 4 ? qam16_tab : qam64_tab;
              int ir, ii;
              qam_index(cw0->e, &jj, Qm0, &ir, &ii);
              v[0] = (int16_t)(((int32_t)amp2 * raw[ir]) >> 15);
              v[1] = (int16_t)(((int32_t)amp2 * raw[ii]) >> 15);
              qam_index(cw0->e, &jj, Qm0, &ir, &ii);
              v[2] = (int16_t)-(int16_t)(((int32_t)amp2 * raw[ir]) >> 15);
              v[3] = (int16_t)(((int32_t)amp2 * raw[ii]) >> 15);
            }
            acc16(&txdataF[0][tti], 0, v[0]);
            acc16(&txdataF[0][tti], 1, v[1]);
            acc16(&txdataF[1][tti], 0, v[2]);
            acc16(&txdataF[1][tti], 1, v[3]);
            /* partner RE (:535-545): the next carrier, or the one after when that is a pilot;
             * linear grid index (no DC re-offset), from the accumulated values at n */
            uint32_t t2 = tti + (not_pilot(pilots, re + 1, fp->nushift, use2nd) ? 1u : 2u);
            const int16_t *n0 = (const int16_t *)&txdataF[0][tti], *n1 = (const int16_t *)&txdataF[1][tti];
            acc16(&txdataF[0][t2], 0, -n1[0]);
            acc16(&txdataF[0][t2], 1, n1[1]);
            acc16(&txdataF[1][t2], 0, n0[0]);
            acc16(&txdataF[1][t2], 1, -n0[1]);
            /* :868-876: skip the partner (and a pilot before it), counting both */
            re++;
            re_allocated++;
            if (!not_pilot(pilots, re, fp->nushift, use2nd)) {
              re++;
              re_allocated++;
            }
          } else {
            return -1;                                                          /* mode not restated */
          }
        }
      }
      re_offset += 12;
      if (re_offset >= N) re_offset = skip_dc == 0 ? 1 : 7;
    }
  }
  return re_allocated;
}

/* PDSCH REs of a subframe (the allocation loop of dlsch_modulation without writing): G of the
 * 4-port extension, whose CRS exclusions the reference's get_G formula does not know */
int orc_count_pdsch_res(const orc_frame_t *fp, const uint32_t rb_alloc[4], uint8_t num_pdcch_symbols, uint32_t subframe)
{
  orc_cw_t c = {NULL, 0, 2, 1, {0}};
  memcpy(c.rb_alloc, rb_alloc, sizeof(c.rb_alloc));
  return modulation_impl(NULL, 512, subframe, subframe, fp, num_pdcch_symbols, &c, NULL, 8192, 8192);
}

int orc_modulation(int32_t **txdataF, int16_t amp, uint32_t subframe, const orc_frame_t *fp,
                   uint8_t num_pdcch_symbols, const orc_cw_t *cw0, const orc_cw_t *cw1,
                   int16_t sqrt_rho_a, int16_t sqrt_rho_b)
{
  return modulation_impl(txdataF, amp, subframe, subframe, fp, num_pdcch_symbols, cw0, cw1, sqrt_rho_a, sqrt_rho_b);
}

/* ======================================================================================
 * Fixed-point IDFT — lte_dfts.c.  Complex int16 pairs; every helper states the SSE op
 * sequence it reproduces.
 * ==================================================================================== */
typedef struct { int16_t r, i; } c16;

static inline int16_t sat16(int32_t v) { return (int16_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v)); }
static inline int16_t wrap16(int32_t v) { return (int16_t)(uint16_t)(uint32_t)v; }
static inline c16 cadds(c16 a, c16 b) { c16 o = {sat16(a.r + b.r), sat16(a.i + b.i)}; return o; }   /* adds_epi16 */
static inline c16 csubs(c16 a, c16 b) { c16 o = {sat16(a.r - b.r), sat16(a.i - b.i)}; return o; }   /* subs_epi16 */
static inline c16 caddw(c16 a, c16 b) { c16 o = {wrap16(a.r + b.r), wrap16(a.i + b.i)}; return o; } /* add_epi16 */
/* sign_epi16(x, {-1,1}) then swap of the int16 pair (lte_dfts.c:1463-1466): -j*x */
static inline c16 cflip(c16 a) { c16 o = {a.i, wrap16(-(int32_t)a.r)}; return o; }
static inline int32_t wadd32(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
static inline int32_t wsub32(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
/* cpack (lte_dfts.c:123-131): srai 15 then packs_epi32 */
static inline c16 cpack32(int32_t re, int32_t im) { c16 o = {sat16(re >> 15), sat16(im >> 15)}; return o; }

/* Twiddle W_N^m = exp(-2*pi*j*m/N) in Q15: (floor(32767 cos), floor(-32767 sin)).  This
 * single rule reproduces every table the path uses (tw16/64/128/256/1024/2048); the test
 * suite checks it entry-by-entry against the reference's tables in oracle/_ref. */
void orc_twiddle(int N, int m, int16_t *re, int16_t *im)
{
  double a = 2.0 * M_PI * (double)m / (double)N;
  *re = (int16_t)floor(32767.0 * cos(a));
  *im = (int16_t)floor(-32767.0 * sin(a));
}

static inline c16 tw(int N, int m) { c16 t; orc_twiddle(N, m, &t.r, &t.i); return t; }

/* x * conj(t), 32-bit, unshifted: cmultc (lte_dfts.c:132-141) */
static inline void cmulc32(c16 x, c16 t, int32_t *re, int32_t *im)
{
  *re = (int32_t)x.r * t.r + (int32_t)x.i * t.i;
  *im = (int32_t)x.r * (int32_t)wrap16(-(int32_t)t.i) + (int32_t)x.i * t.r;
}

/* packed_cmult2 with (tw, twc) (lte_dfts.c:169-176) == cpack(cmultc) */
static inline c16 cmulc16(c16 x, c16 t)
{
  int32_t re, im;
  cmulc32(x, t, &re, &im);
  return cpack32(re, im);
}

/* inverse radix-4 on saturating int16 (idft16 stages, ibfly4_16 :1049-1090) */
static inline void r4inv(c16 p0, c16 p1, c16 p2, c16 p3, c16 *o0, c16 *o1, c16 *o2, c16 *o3)
{
  c16 s02 = cadds(p0, p2), s13 = cadds(p1, p3);
  *o0 = cadds(s02, s13);
  *o2 = csubs(s02, s13);
  c16 d02 = csubs(p0, p2), d13 = csubs(cflip(p1), cflip(p3));
  *o3 = cadds(d02, d13);
  *o1 = csubs(d02, d13);
}

static void idft16_c(const c16 *x, c16 *y)                                     /* :1597-1724 */
{
  c16 S[4][4], B[4][4];
  for (int j = 0; j < 4; j++) r4inv(x[j], x[4 + j], x[8 + j], x[12 + j], &S[0][j], &S[1][j], &S[2][j], &S[3][j]);
  for (int j = 0; j < 4; j++)
    for (int k = 0; k < 4; k++) B[j][k] = (j == 0) ? S[k][j] : cmulc16(S[k][j], tw(16, j * k));
  for (int k = 0; k < 4; k++) r4inv(B[0][k], B[1][k], B[2][k], B[3][k], &y[k], &y[4 + k], &y[8 + k], &y[12 + k]);
}

static void idft64_c(const c16 *x, c16 *y, int scale)                          /* :1856-1946 */
{
  c16 blk[4][16], Y[4][16];
  for (int r = 0; r < 4; r++) {
    for (int n = 0; n < 16; n++) blk[r][n] = x[4 * n + r];
    idft16_c(blk[r], Y[r]);
  }
  for (int k = 0; k < 16; k++)
    r4inv(Y[0][k], cmulc16(Y[1][k], tw(64, k)), cmulc16(Y[2][k], tw(64, 2 * k)), cmulc16(Y[3][k], tw(64, 3 * k)),
          &y[k], &y[16 + k], &y[32 + k], &y[48 + k]);
  if (scale > 0)
    for (int k = 0; k < 64; k++) { y[k].r >>= 3; y[k].i >>= 3; }
}

/* ibfly4 (:795-819): products kept in 32 bits, one cpack per output, wrapping add of x0 */
static inline void ibfly4_c(c16 x0, c16 x1, c16 x2, c16 x3, c16 t1, c16 t2, c16 t3,
                            c16 *y0, c16 *y1, c16 *y2, c16 *y3)
{
  int32_t a1r, a1i, a2r, a2i, a3r, a3i;
  cmulc32(x1, t1, &a1r, &a1i);
  cmulc32(x2, t2, &a2r, &a2i);
  cmulc32(x3, t3, &a3r, &a3i);
  *y0 = caddw(x0, cpack32(wadd32(a1r, wadd32(a2r, a3r)), wadd32(a1i, wadd32(a2i, a3i))));
  *y3 = caddw(x0, cpack32(wsub32(a1i, wadd32(a2r, a3i)), wsub32(wsub32(a3r, a2i), a1r)));
  *y2 = caddw(x0, cpack32(wsub32(wsub32(a2r, a3r), a1r), wsub32(wsub32(a2i, a3i), a1i)));
  *y1 = caddw(x0, cpack32(wsub32(wsub32(a3i, a2r), a1i), wsub32(a1r, wadd32(a2i, a3r))));
}

/* radix-4 DIT level over four sub-transforms of size M (idft256 :2284-2338, idft1024 :2630-2684) */
static void idft_r4(const c16 *x, c16 *y, int M, void (*sub)(const c16 *, c16 *, int), int scale)
{
  int N = 4 * M;
  c16 *blk = malloc(sizeof(c16) * N), *Y = malloc(sizeof(c16) * N);
  for (int r = 0; r < 4; r++) {
    for (int n = 0; n < M; n++) blk[r * M + n] = x[4 * n + r];
    sub(blk + r * M, Y + r * M, 1);
  }
  for (int k = 0; k < M; k++)
    ibfly4_c(Y[k], Y[M + k], Y[2 * M + k], Y[3 * M + k], tw(N, k), tw(N, 2 * k), tw(N, 3 * k),
             &y[k], &y[M + k], &y[2 * M + k], &y[3 * M + k]);
  if (scale > 0)
    for (int k = 0; k < N; k++) { y[k].r >>= 1; y[k].i >>= 1; }
  free(blk);
  free(Y);
}

static void idft256_c(const c16 *x, c16 *y, int scale) { idft_r4(x, y, 64, idft64_c, scale); }
static void idft1024_c(const c16 *x, c16 *y, int scale) { idft_r4(x, y, 256, idft256_c, scale); }

/* ibfly2 (:502-527): 32767*x0 +/- x1*conj(t), >>15 (arith), packs */
static inline void ibfly2_c(c16 x0, c16 x1, c16 t, c16 *y0, c16 *y1)
{
  int32_t a0r, a0i, a1r, a1i;
  c16 w0 = {32767, 0};
  cmulc32(x0, w0, &a0r, &a0i);
  cmulc32(x1, t, &a1r, &a1i);
  *y0 = cpack32(wadd32(a0r, a1r), wadd32(a0i, a1i));
  *y1 = cpack32(wsub32(a0r, a1r), wsub32(a0i, a1i));
}

static inline int16_t mulhi_scale(int16_t v) { return wrap16((((int32_t)v * 23170) >> 16) << 1); } /* :1755 */

/* radix-2 DIT level (idft128 :2058-2154, idft2048 :2779-2866) */
static void idft_r2(const c16 *x, c16 *y, int M, void (*sub)(const c16 *, c16 *, int), int scale)
{
  int N = 2 * M;
  c16 *blk = malloc(sizeof(c16) * N), *Y = malloc(sizeof(c16) * N);
  for (int r = 0; r < 2; r++) {
    for (int n = 0; n < M; n++) blk[r * M + n] = x[2 * n + r];
    sub(blk + r * M, Y + r * M, 1);
  }
  for (int k = 0; k < M; k++) ibfly2_c(Y[k], Y[M + k], tw(N, k), &y[k], &y[M + k]);
  if (scale > 0)
    for (int k = 0; k < N; k++) { y[k].r = mulhi_scale(y[k].r); y[k].i = mulhi_scale(y[k].i); }
  free(blk);
  free(Y);
}

void orc_idft(int log2n, const int16_t *x, int16_t *y, int scale)
{
  const c16 *xc = (const c16 *)x;
  c16 *yc = (c16 *)y;
  switch (log2n) {
  case 6: idft64_c(xc, yc, scale); break;
  case 7: idft_r2(xc, yc, 64, idft64_c, scale); break;
  case 8: idft256_c(xc, yc, scale); break;
  case 9: idft_r2(xc, yc, 256, idft256_c, scale); break;                      /* idft512 :2479-2564 */
  case 10: idft1024_c(xc, yc, scale); break;
  case 11: idft_r2(xc, yc, 1024, idft1024_c, scale); break;
  default: fprintf(stderr, "orc_idft: size 2^%d not restated\n", log2n); abort();
  }
}

/* ======================================================================================
 * Forward fixed-point DFT — lte_dfts.c dft16 … dft2048 (the UE receive front end,
 * slot_fep.c:40-148).  Same DIT decomposition as the inverse, forward butterflies.
 * ==================================================================================== */
/* Forward twiddle tables.  "a"/"b" are the packed_cmult2 operand pairs (lte_dfts.c:178-188):
 * x * W = cpack(madd(x, a), madd(x, b)) with a = (Wr, -Wi), b = (Wi, Wr) where W = orc_twiddle;
 * tw256a alone rounds its second entry as floor(32767 sin) instead (lte_dfts.c:2162). */
void orc_dft_twiddle_ab(int N, int m, int16_t a[2], int16_t b[2])
{
  int16_t wr, wi;
  orc_twiddle(N, m, &wr, &wi);
  a[0] = wr;
  a[1] = (N == 256) ? (int16_t)floor(32767.0 * sin(2.0 * M_PI * (double)m / (double)N)) : (int16_t)-wi;
  b[0] = wi;
  b[1] = wr;
}

/* packed_cmult2 (:178-188) */
static inline c16 cmul2_16(c16 x, int N, int m)
{
  int16_t a[2], b[2];
  orc_dft_twiddle_ab(N, m, a, b);
  return cpack32((int32_t)x.r * a[0] + (int32_t)x.i * a[1], (int32_t)x.r * b[0] + (int32_t)x.i * b[1]);
}

/* cmult (:106-118): x * t in 32 bits, t from the plain table (tw1024 / tw2048 / W0) */
static inline void cmul32(c16 x, c16 t, int32_t *re, int32_t *im)
{
  *re = (int32_t)x.r * t.r + (int32_t)x.i * (int32_t)wrap16(-(int32_t)t.i);
  *im = (int32_t)x.r * t.i + (int32_t)x.i * t.r;
}

/* forward radix-4 on saturating int16 (bfly4_tw1 :860-889, dft16 stages :1453-1500, bfly4_16 :965-1006):
 * flip = sign(x, {-1,1}) then pair swap = -j x; y1 = x0 - x2 + (f1 - f3), y3 = x0 - x2 - (f1 - f3) */
static inline void r4fwd(c16 p0, c16 p1, c16 p2, c16 p3, c16 *o0, c16 *o1, c16 *o2, c16 *o3)
{
  c16 s02 = cadds(p0, p2), s13 = cadds(p1, p3);
  *o0 = cadds(s02, s13);
  *o2 = csubs(s02, s13);
  c16 f1 = {p1.i, wrap16(-(int32_t)p1.r)}, f3 = {p3.i, wrap16(-(int32_t)p3.r)};
  c16 d02 = csubs(p0, p2), d13 = csubs(f1, f3);
  *o1 = cadds(d02, d13);
  *o3 = csubs(d02, d13);
}

static void dft16_c(const c16 *x, c16 *y)                                      /* :1431-1500 */
{
  c16 S[4][4];
  for (int j = 0; j < 4; j++) r4fwd(x[j], x[4 + j], x[8 + j], x[12 + j], &S[0][j], &S[1][j], &S[2][j], &S[3][j]);
  /* unpack transposes: butterfly k of the second stage takes S[k][0..3], input j twiddled by W16^(j k) (tw16a/b) */
  for (int k = 0; k < 4; k++) {
    c16 in[4];
    for (int j = 0; j < 4; j++) in[j] = (j == 0) ? S[k][j] : cmul2_16(S[k][j], 16, j * k);
    r4fwd(in[0], in[1], in[2], in[3], &y[k], &y[4 + k], &y[8 + k], &y[12 + k]);
  }
}

static void dft64_c(const c16 *x, c16 *y, int scale)                           /* :1766-1854 */
{
  c16 blk[4][16], Y[4][16];
  for (int r = 0; r < 4; r++) {
    for (int n = 0; n < 16; n++) blk[r][n] = x[4 * n + r];
    dft16_c(blk[r], Y[r]);
  }
  for (int k = 0; k < 16; k++)                                                  /* bfly4_16, tw64a/b */
    r4fwd(Y[0][k], cmul2_16(Y[1][k], 64, k), cmul2_16(Y[2][k], 64, 2 * k), cmul2_16(Y[3][k], 64, 3 * k),
          &y[k], &y[16 + k], &y[32 + k], &y[48 + k]);
  if (scale > 0)
    for (int k = 0; k < 64; k++) { y[k].r >>= 3; y[k].i >>= 3; }
}

static void dft256_c(const c16 *x, c16 *y, int scale)                          /* :2172-2282 */
{
  c16 blk[4][64], Y[4][64];
  for (int r = 0; r < 4; r++) {
    for (int n = 0; n < 64; n++) blk[r][n] = x[4 * n + r];
    dft64_c(blk[r], Y[r], 1);
  }
  for (int k = 0; k < 64; k++)                                                  /* bfly4_16, tw256a/b */
    r4fwd(Y[0][k], cmul2_16(Y[1][k], 256, k), cmul2_16(Y[2][k], 256, 2 * k), cmul2_16(Y[3][k], 256, 3 * k),
          &y[k], &y[64 + k], &y[128 + k], &y[192 + k]);
  if (scale > 0)
    for (int k = 0; k < 256; k++) { y[k].r >>= 1; y[k].i >>= 1; }
}

/* bfly4 (:709-745): 32-bit products, one cpack per output, wrapping add of x0 */
static inline void bfly4_c(c16 x0, c16 x1, c16 x2, c16 x3, c16 t1, c16 t2, c16 t3,
                           c16 *y0, c16 *y1, c16 *y2, c16 *y3)
{
  int32_t a1r, a1i, a2r, a2i, a3r, a3i;
  cmul32(x1, t1, &a1r, &a1i);
  cmul32(x2, t2, &a2r, &a2i);
  cmul32(x3, t3, &a3r, &a3i);
  *y0 = caddw(x0, cpack32(wadd32(a1r, wadd32(a2r, a3r)), wadd32(a1i, wadd32(a2i, a3i))));
  *y1 = caddw(x0, cpack32(wsub32(a1i, wadd32(a2r, a3i)), wsub32(wsub32(a3r, a2i), a1r)));
  *y2 = caddw(x0, cpack32(wsub32(wsub32(a2r, a3r), a1r), wsub32(wsub32(a2i, a3i), a1i)));
  *y3 = caddw(x0, cpack32(wsub32(wsub32(a3i, a2r), a1i), wsub32(a1r, wadd32(a2i, a3r))));
}

static void dft1024_c(const c16 *x, c16 *y, int scale)                         /* :2574-2628 */
{
  c16 *blk = malloc(sizeof(c16) * 1024), *Y = malloc(sizeof(c16) * 1024);
  for (int r = 0; r < 4; r++) {
    for (int n = 0; n < 256; n++) blk[r * 256 + n] = x[4 * n + r];
    dft256_c(blk + r * 256, Y + r * 256, 1);
  }
  for (int k = 0; k < 256; k++)
    bfly4_c(Y[k], Y[256 + k], Y[512 + k], Y[768 + k], tw(1024, k), tw(1024, 2 * k), tw(1024, 3 * k),
            &y[k], &y[256 + k], &y[512 + k], &y[768 + k]);
  if (scale > 0)
    for (int k = 0; k < 1024; k++) { y[k].r >>= 1; y[k].i >>= 1; }
  free(blk);
  free(Y);
}

/* radix-2 levels: bfly2_16 (:471-483, dft128 / dft512) or bfly2 (:396-419, dft2048), then the
 * mulhi(23170) << 1 scaling (:1755) */
static void dft_r2(const c16 *x, c16 *y, int M, void (*sub)(const c16 *, c16 *, int), int scale)
{
  int N = 2 * M;
  c16 *blk = malloc(sizeof(c16) * N), *Y = malloc(sizeof(c16) * N);
  for (int r = 0; r < 2; r++) {
    for (int n = 0; n < M; n++) blk[r * M + n] = x[2 * n + r];
    sub(blk + r * M, Y + r * M, 1);
  }
  for (int k = 0; k < M; k++) {
    if (N == 2048) {
      int32_t a0r, a0i, a1r, a1i;
      c16 w0 = {32767, 0};
      cmul32(Y[k], w0, &a0r, &a0i);
      cmul32(Y[M + k], tw(N, k), &a1r, &a1i);
      y[k] = cpack32(wadd32(a0r, a1r), wadd32(a0i, a1i));
      y[M + k] = cpack32(wsub32(a0r, a1r), wsub32(a0i, a1i));
    } else {
      c16 t = cmul2_16(Y[M + k], N, k);
      y[k] = cadds(Y[k], t);
      y[M + k] = csubs(Y[k], t);
    }
  }
  if (scale > 0)
    for (int k = 0; k < N; k++) { y[k].r = mulhi_scale(y[k].r); y[k].i = mulhi_scale(y[k].i); }
  free(blk);
  free(Y);
}

void orc_dft(int log2n, const int16_t *x, int16_t *y, int scale)
{
  const c16 *xc = (const c16 *)x;
  c16 *yc = (c16 *)y;
  switch (log2n) {
  case 6: dft64_c(xc, yc, scale); break;
  case 7: dft_r2(xc, yc, 64, dft64_c, scale); break;                           /* dft128 :1957-2056 */
  case 8: dft256_c(xc, yc, scale); break;
  case 9: dft_r2(xc, yc, 256, dft256_c, scale); break;                         /* dft512 :2359-2477 */
  case 10: dft1024_c(xc, yc, scale); break;
  case 11: dft_r2(xc, yc, 1024, dft1024_c, scale); break;                      /* dft2048 :2689-2777 */
  default: fprintf(stderr, "orc_dft: size 2^%d not restated\n", log2n); abort();
  }
}

/* slot_fep (PHY/MODULATION/slot_fep.c:40-177), DFT part (channel / frequency-offset estimation of
 * the perfect_ce == 0 branch :179-222 excluded).  rxdata[aa] = frame + N words of wrap extension. */
int orc_slot_fep(int32_t **rxdata, int32_t **rxdataF, const orc_frame_t *fp, int nb_antennas_rx, uint8_t l,
                 uint8_t Ns, int sample_offset, int no_prefix)
{
  unsigned int N = fp->ofdm_symbol_size;
  unsigned char symbol = l + ((7 - fp->Ncp) * (Ns & 1));                                  /* :51 */
  unsigned int nb_prefix_samples = no_prefix ? 0 : fp->nb_prefix_samples;
  unsigned int nb_prefix_samples0 = no_prefix ? 0 : fp->nb_prefix_samples0;
  unsigned int subframe_offset, slot_offset, frame_length_samples = fp->samples_per_tti * 10, rx_offset;
  if (no_prefix) {                                                                         /* :87-93 */
    subframe_offset = N * fp->symbols_per_tti * (Ns >> 1);
    slot_offset = N * (fp->symbols_per_tti >> 1) * (Ns % 2);
  } else {
    subframe_offset = fp->samples_per_tti * (Ns >> 1);
    slot_offset = (fp->samples_per_tti >> 1) * (Ns % 2);
  }
  if (l >= 7 - fp->Ncp) { printf("slot_fep: l must be between 0 and %d\n", 7 - fp->Ncp); return -1; }
  if (Ns >= 20) { printf("slot_fep: Ns must be between 0 and 19\n"); return -1; }
  int32_t tmp[2048];
  for (int aa = 0; aa < nb_antennas_rx; aa++) {
    memset(&rxdataF[aa][N * symbol], 0, N * sizeof(int32_t));
    rx_offset = sample_offset + slot_offset + nb_prefix_samples0 + subframe_offset;       /* :111 */
    rx_offset = rx_offset - rx_offset % 4;
    if (l > 0) rx_offset += (N + nb_prefix_samples) + (N + nb_prefix_samples) * (l - 1);   /* :146 */
    if (rx_offset > (frame_length_samples - N))                                            /* :123, :153 */
      memcpy(&rxdata[aa][frame_length_samples], &rxdata[aa][0], N * sizeof(int32_t));
    if (l == 0 && (rx_offset & 3) != 0)        /* :129-133: unreachable after the alignment, restated */
      memcpy(tmp, &rxdata[aa][(rx_offset - nb_prefix_samples0) % frame_length_samples], N * sizeof(int32_t));
    else                                       /* :135-139, :163-170 (the misaligned copy reads the same words) */
      memcpy(tmp, &rxdata[aa][rx_offset % frame_length_samples], N * sizeof(int32_t));
    orc_dft(fp->log2_symbol_size, (const int16_t *)tmp, (int16_t *)&rxdataF[aa][N * symbol], 1);
  }
  return 0;
}

/* PHY_ofdm_mod, CYCLIC_PREFIX branch (ofdm_mod.c:85-171) */
void orc_ofdm_mod(const int32_t *input, int32_t *output, uint8_t log2fftsize, uint8_t nb_symbols,
                  uint16_t nb_prefix_samples)
{
  int N = 1 << log2fftsize;
  for (int i = 0; i < nb_symbols; i++) {
    int32_t *out = &output[(i << log2fftsize) + (1 + i) * nb_prefix_samples];
    orc_idft(log2fftsize, (const int16_t *)&input[i << log2fftsize], (int16_t *)out, 1);
    for (int k = 1; k <= nb_prefix_samples; k++) out[-k] = out[N - k];
  }
}

/* normal_prefix_mod (ofdm_mod.c:47-83) */
void orc_normal_prefix_mod(const int32_t *txdataF, int32_t *txdata, uint8_t nsymb, const orc_frame_t *fp)
{
  int N = fp->ofdm_symbol_size, short_offset = (2 * nsymb) < fp->symbols_per_tti;
  for (int i = 0; i < short_offset + 2 * nsymb / fp->symbols_per_tti; i++) {
    orc_ofdm_mod(txdataF + ((i * N * fp->symbols_per_tti) >> 1), txdata + ((i * fp->samples_per_tti) >> 1),
                 fp->log2_symbol_size, 1, fp->nb_prefix_samples0);
    orc_ofdm_mod(txdataF + N + i * N * (fp->symbols_per_tti >> 1),
                 txdata + (N + fp->nb_prefix_samples0) + ((i * fp->samples_per_tti) >> 1), fp->log2_symbol_size,
                 short_offset ? 1 : (fp->symbols_per_tti >> 1) - 1, fp->nb_prefix_samples);
  }
}

/* do_OFDM_mod (ofdm_mod.c:233-284): slot next_slot of every antenna's whole-frame grid.  The
 * frame parameters here carry no MBSFN configuration, so is_pmch_subframe (pmch.c:97-190) is 0
 * for every subframe and only the non-PMCH branch (:267-281) is reachable. */
void orc_do_OFDM_mod(int32_t **txdataF, int32_t **txdata, uint32_t frame, uint16_t next_slot, const orc_frame_t *fp)
{
  (void)frame;
  const uint32_t slot_offset_F = (uint32_t)next_slot * fp->ofdm_symbol_size * (fp->Ncp == 1 ? 6 : 7);
  const uint32_t slot_offset = (uint32_t)next_slot * (fp->samples_per_tti >> 1);
  for (int aa = 0; aa < fp->nb_antennas_tx; aa++) {
    if (fp->Ncp == 1)
      orc_ofdm_mod(&txdataF[aa][slot_offset_F], &txdata[aa][slot_offset], fp->log2_symbol_size, 6,
                   fp->nb_prefix_samples);
    else
      orc_normal_prefix_mod(&txdataF[aa][slot_offset_F], &txdata[aa][slot_offset], 7, fp);
  }
}

/* ======================================================================================
 * Whole subframe — dlsim.c:2567-2699 (dlsch_encoding dlsch_coding.c:254-419,
 * dlsch_scrambling, dlsch_modulation, do_OFDM_mod_l x2 slots).  DCI and pilots excluded.
 * ==================================================================================== */
/* ======================================================================================
 * Cell-specific reference signals.
 * ==================================================================================== */
/* lte_gold (lte_gold.c:52-93): c_init = 2^10 (7(ns+1) + l' + 1)(2 Nid + 1) + 2 Nid + N_CP with
 * l' = 0 or 4 (3 for extended CP); words n = 0..13 after the 1600-bit warm-up */
void orc_lte_gold_table(const orc_frame_t *fp, uint32_t table[20][2][14])
{
  uint32_t Ncp = 1 - fp->Ncp, Nid = fp->Nid_cell;
  for (uint32_t ns = 0; ns < 20; ns++)
    for (uint32_t l = 0; l < 2; l++) {
      uint32_t x1, x2 = Ncp + (Nid << 1) + (((1 + (Nid << 1)) * (1 + ((fp->Ncp == 0) ? 4 : 3) * l + 7 * (1 + ns))) << 10);
      /* lte_gold.c:82-91: 49 warm-up word steps, then 14 stored words; the first stored word is
       * the state after 50 steps, which is what orc_gold_generic(reset = 1) returns */
      table[ns][l][0] = orc_gold_generic(&x1, &x2, 1);
      for (uint32_t n = 1; n < 14; n++) table[ns][l][n] = orc_gold_generic(&x1, &x2, 0);
    }
}

/* lte_dl_cell_spec (lte_dl_cell_spec.c:123-203) */
int orc_lte_dl_cell_spec(int32_t *output, int16_t amp, const orc_frame_t *fp, const uint32_t table[20][2][14],
                         uint8_t Ns, uint8_t l, uint8_t p)
{
  int16_t a = (int16_t)((amp * 23170) >> 15);              /* ONE_OVER_SQRT2_Q15 */
  int32_t qpsk[4];
  int16_t *q = (int16_t *)qpsk;
  q[0] = a;  q[1] = a;  q[2] = -a;  q[3] = a;  q[4] = a;  q[5] = -a;  q[6] = -a;  q[7] = -a;
  uint32_t nu;
  if (p == 0) nu = l == 0 ? 0 : 3;
  else if (p == 1) nu = l == 0 ? 3 : 0;
  else return -1;
  uint32_t mprime = 110 - fp->N_RB_DL, k = nu + fp->nushift;
  if (k > 5) k -= 6;
  k += fp->first_carrier_offset;
  for (uint32_t m = 0; m < 2u * fp->N_RB_DL; m++, mprime++) {
    output[k] = qpsk[(table[Ns][l][mprime >> 4] >> (2 * (mprime & 15))) & 3];
    k += 6;
    if (k >= fp->ofdm_symbol_size) {
      k++;                                                   /* skip DC carrier */
      k -= fp->ofdm_symbol_size;
    }
  }
  return 0;
}

/* CRS of antenna ports 2/3 (4-TX extension; the reference generates ports 0/1 only): 36.211
 * 6.10.1 with l = 1 in each slot, nu = 3 (ns mod 2) for p = 2 and 3 + 3 (ns mod 2) for p = 3,
 * c_init = 2^10 (7(ns+1) + l + 1)(2 Nid + 1) + 2 Nid + N_CP as in lte_gold.c:52-93 */
void orc_cell_spec_p23(int32_t *output, int16_t amp, const orc_frame_t *fp, uint8_t Ns, uint8_t p)
{
  uint32_t Ncp = 1 - fp->Ncp, Nid = fp->Nid_cell, x1, words[14];
  uint32_t x2 = Ncp + (Nid << 1) + (((1 + (Nid << 1)) * (1 + 1 + 7 * (1 + (uint32_t)Ns))) << 10);
  words[0] = orc_gold_generic(&x1, &x2, 1);
  for (int n = 1; n < 14; n++) words[n] = orc_gold_generic(&x1, &x2, 0);
  int16_t a = (int16_t)((amp * 23170) >> 15);
  uint32_t nu = (p == 2 ? 0u : 3u) + 3u * (Ns & 1u), k = (nu + fp->nushift) % 6 + fp->first_carrier_offset;
  uint32_t mprime = 110 - fp->N_RB_DL;
  for (uint32_t m = 0; m < 2u * fp->N_RB_DL; m++, mprime++) {
    uint32_t c = (words[mprime >> 4] >> (2 * (mprime & 15))) & 3;
    int16_t *o = (int16_t *)&output[k];
    o[0] = (c & 1) ? (int16_t)-a : a;
    o[1] = (c & 2) ? (int16_t)-a : a;
    k += 6;
    if (k >= fp->ofdm_symbol_size) {
      k++;
      k -= fp->ofdm_symbol_size;
    }
  }
}

/* pilots.c:43-168 for the symbols of one subframe grid: port 0 on antenna 0; antenna 1 gets
 * port 0 too in mode1 (single-port CRS), port 1 otherwise; with 4 TX antennas ports 2/3 on
 * antennas 2/3 in symbol 1 of each slot */
static void pilots_one(int32_t **grid, int16_t amp, const orc_frame_t *fp, const uint32_t table[20][2][14],
                       uint32_t slot_offset)
{
  uint32_t N = fp->ofdm_symbol_size, Nsymb = fp->Ncp == 0 ? 14 : 12, second = fp->Ncp == 0 ? 4 : 3;
  const uint32_t sym[4] = {0, second, Nsymb >> 1, (Nsymb >> 1) + second};
  for (int i = 0; i < 4; i++) {
    uint8_t Ns = (uint8_t)(slot_offset + (i >> 1)), l = (uint8_t)(i & 1);
    orc_lte_dl_cell_spec(grid[0] + sym[i] * N, amp, fp, table, Ns, l, 0);
    if (fp->nb_antennas_tx > 1) orc_lte_dl_cell_spec(grid[1] + sym[i] * N, amp, fp, table, Ns, l, fp->mode1_flag ? 0 : 1);
  }
  if (fp->nb_antennas_tx == 4)
    for (uint32_t s = 0; s < 2; s++)
      for (uint8_t p = 2; p < 4; p++)
        orc_cell_spec_p23(grid[p] + (s * (Nsymb >> 1) + 1) * N, amp, fp, (uint8_t)(slot_offset + s), p);
}

void orc_generate_pilots(int32_t **txdataF, int16_t amp, const orc_frame_t *fp, uint16_t Ntti)
{
  static uint32_t table[20][2][14];
  orc_lte_gold_table(fp, table);
  uint32_t Nsymb = fp->Ncp == 0 ? 14 : 12;
  for (uint32_t tti = 0; tti < Ntti; tti++) {
    int32_t *g[4] = {NULL, NULL, NULL, NULL};
    for (int aa = 0; aa < fp->nb_antennas_tx && aa < 4; aa++) g[aa] = txdataF[aa] + tti * fp->ofdm_symbol_size * Nsymb;
    pilots_one(g, amp, fp, table, (tti * 2) % 20);
  }
}

void orc_generate_pilots_subframe(int32_t **txdataF, int16_t amp, const orc_frame_t *fp, uint8_t subframe)
{
  static uint32_t table[20][2][14];
  orc_lte_gold_table(fp, table);
  pilots_one(txdataF, amp, fp, table, (2u * subframe) % 20);
}

static int g_last_re_allocated = 0;
int orc_last_re_allocated(void) { return g_last_re_allocated; }

static int tx_subframe_impl(const orc_tx_cfg_t *cfg, uint8_t *payload[2], int32_t **txdataF, int32_t **txdata,
                            uint8_t *e_out[2], uint8_t n_ue_dci, uint8_t n_common_dci, const orc_dci_alloc_t *dci);

int orc_tx_subframe(const orc_tx_cfg_t *cfg, uint8_t *payload[2], int32_t **txdataF, int32_t **txdata,
                    uint8_t *e_out[2])
{
  return tx_subframe_impl(cfg, payload, txdataF, txdata, e_out, 0, 0, NULL);
}

/* dlsim's phy_proc_tx grid: generate_dci_top (dlsim.c:2553) + PDSCH + pilots, then OFDM */
int orc_tx_subframe_dci(const orc_tx_cfg_t *cfg, uint8_t *payload[2], int32_t **txdataF, int32_t **txdata,
                        uint8_t *e_out[2], uint8_t n_ue_dci, uint8_t n_common_dci, const orc_dci_alloc_t *dci)
{
  return tx_subframe_impl(cfg, payload, txdataF, txdata, e_out, n_ue_dci, n_common_dci, dci);
}

static int tx_subframe_impl(const orc_tx_cfg_t *cfg, uint8_t *payload[2], int32_t **txdataF, int32_t **txdata,
                            uint8_t *e_out[2], uint8_t n_ue_dci, uint8_t n_common_dci, const orc_dci_alloc_t *dci)
{
  const orc_frame_t *fp = &cfg->fp;
  uint8_t *e_buf[2] = {NULL, NULL};
  static uint8_t dbuf[96 + 12 + 3 + 3 * 6144 + 64], wbuf[3 * 6176 + 64], cbuf[16][8 + 3 + 768];
  for (int cw = 0; cw < cfg->n_cw; cw++) {
    uint32_t A = cfg->TBS[cw];
    uint8_t Qm = orc_get_Qm(cfg->mcs[cw]);
    int G = fp->nb_antennas_tx == 4
                ? orc_count_pdsch_res(fp, cfg->rb_alloc, cfg->num_pdcch_symbols, cfg->subframe) * Qm
                : orc_get_G(fp->N_RB_DL, fp->Ncp, fp->mode1_flag, fp->frame_type, cfg->nb_rb, cfg->rb_alloc, Qm, 1,
                            cfg->num_pdcch_symbols, cfg->subframe);
    e_buf[cw] = calloc((size_t)G + 64, 1);
    uint8_t *a = payload[cw];
    uint32_t crc = orc_crc24a(a, (int)A) >> 8;                              /* dlsch_coding.c:296-300 */
    a[A >> 3] = (uint8_t)(crc >> 16);
    a[1 + (A >> 3)] = (uint8_t)(crc >> 8);
    a[2 + (A >> 3)] = (uint8_t)crc;
    uint32_t C, Cp, Cm, Kp, Km, F;
    uint8_t *cptr[16];
    for (int r = 0; r < 16; r++) cptr[r] = cbuf[r];
    if (orc_segmentation(a, cptr, A + 24, &C, &Cp, &Cm, &Kp, &Km, &F) < 0) return -1;
    uint32_t r_off = 0;
    for (uint32_t r = 0; r < C; r++) {
      uint32_t Kr = r < Cm ? Km : Kp;
      int qi = oai4g_qpp_index(Kr);
      if (qi < 0) return -1;
      memset(dbuf, ORC_LTE_NULL, 96);
      orc_turbo_encode(cptr[r], (uint16_t)(Kr >> 3), dbuf + 96, oai4g_qpp_table[qi].f1, oai4g_qpp_table[qi].f2);
      uint32_t RTC = orc_subblock_interleave(Kr + 4, dbuf + 96, wbuf);
      r_off += orc_rate_match(RTC, (uint32_t)G, wbuf, e_buf[cw] + r_off, (uint8_t)C, ORC_NSOFT, cfg->Mdlharq,
                              cfg->Kmimo, cfg->rvidx[cw], Qm, 1, (uint8_t)r);
    }
    uint32_t c_init = ((uint32_t)cfg->rnti << 14) + ((uint32_t)cfg->q[cw] << 13) + ((uint32_t)cfg->subframe << 9) +
                      fp->Nid_cell;                          /* dlsch_scrambling.c:69; dlsim passes q = 0 */
    orc_scramble(e_buf[cw], G, c_init);
    if (e_out && e_out[cw]) memcpy(e_out[cw], e_buf[cw], (size_t)G);
  }
  orc_cw_t c0 = {e_buf[0], cfg->mcs[0], cfg->mimo_mode, 1, {0}}, c1 = {e_buf[1], cfg->mcs[1], cfg->mimo_mode, 1, {0}};
  memcpy(c0.rb_alloc, cfg->rb_alloc, sizeof(c0.rb_alloc));
  memcpy(c1.rb_alloc, cfg->rb_alloc, sizeof(c1.rb_alloc));
  int N = fp->ofdm_symbol_size, nsymb = fp->symbols_per_tti;
  for (int aa = 0; aa < fp->nb_antennas_tx; aa++) memset(txdataF[aa], 0, sizeof(int32_t) * N * nsymb);
  if (cfg->with_crs) orc_generate_pilots_subframe(txdataF, cfg->amp, fp, cfg->subframe);   /* dlsim.c:2681-2684 */
  int ret = modulation_impl(txdataF, cfg->amp, cfg->subframe, 0, fp, cfg->num_pdcch_symbols, &c0,
                            cfg->n_cw > 1 ? &c1 : NULL, cfg->sqrt_rho_a, cfg->sqrt_rho_b);
  g_last_re_allocated = ret;
  if (n_ue_dci + n_common_dci > 0) {            /* control region on a frame grid, copied back */
    int32_t *fg[4] = {0};
    for (int aa = 0; aa < fp->nb_antennas_tx; aa++) {
      fg[aa] = (int32_t *)calloc((size_t)10 * nsymb * N, sizeof(int32_t));
      memcpy(fg[aa] + (size_t)cfg->subframe * nsymb * N, txdataF[aa], sizeof(int32_t) * N * nsymb);
    }
    orc_generate_dci_top(n_ue_dci, n_common_dci, dci, 0, cfg->amp, fp, fg, cfg->subframe);
    for (int aa = 0; aa < fp->nb_antennas_tx; aa++) {
      memcpy(txdataF[aa], fg[aa] + (size_t)cfg->subframe * nsymb * N, sizeof(int32_t) * N * nsymb);
      free(fg[aa]);
    }
  }
  /* do_OFDM_mod (ofdm_mod.c:233-286): normal_prefix_mod per slot, or PHY_ofdm_mod of 6 symbols
   * with the extended prefix */
  const int sps = nsymb >> 1;
  for (int aa = 0; aa < fp->nb_antennas_tx; aa++)
    for (int slot = 0; slot < 2; slot++) {
      if (fp->Ncp == 1)
        orc_ofdm_mod(txdataF[aa] + slot * N * sps, txdata[aa] + slot * (fp->samples_per_tti >> 1),
                     (uint8_t)fp->log2_symbol_size, (uint8_t)sps, (uint16_t)fp->nb_prefix_samples);
      else
        orc_normal_prefix_mod(txdataF[aa] + slot * N * 7, txdata[aa] + slot * (fp->samples_per_tti >> 1), 7, fp);
    }
  free(e_buf[0]);
  free(e_buf[1]);
  return ret < 0 ? -1 : 0;
}

/* ======================================================================================
 * PCFICH — pcfich.c:48-228 (generate_pcfich_reg_mapping, pcfich_scrambling, generate_pcfich)
 * ==================================================================================== */
static const uint8_t orc_pcfich_b[4][32] = {                                    /* :138-142 */
  {0,1,1,0,1,1,0,1,1,0,1,1,0,1,1,0,1,1,0,1,1,0,1,1,0,1,1,0,1,1,0,1},
  {1,0,1,1,0,1,1,0,1,1,0,1,1,0,1,1,0,1,1,0,1,1,0,1,1,0,1,1,0,1,1,0},
  {1,1,0,1,1,0,1,1,0,1,1,0,1,1,0,1,1,0,1,1,0,1,1,0,1,1,0,1,1,0,1,1},
  {0}};

void orc_pcfich_reg_mapping(const orc_frame_t *fp, uint16_t reg[4], uint8_t *first_idx)  /* :48-84 */
{
  uint16_t kbar = 6 * (fp->Nid_cell % (2 * fp->N_RB_DL)), first;
  reg[0] = kbar / 6;
  first = reg[0];
  *first_idx = 0;
  reg[1] = ((kbar + (fp->N_RB_DL >> 1) * 6) % (fp->N_RB_DL * 12)) / 6;
  if (reg[1] < reg[0]) { *first_idx = 1; first = reg[1]; }
  reg[2] = ((kbar + (fp->N_RB_DL) * 6) % (fp->N_RB_DL * 12)) / 6;
  if (reg[2] < first) { *first_idx = 2; first = reg[2]; }
  reg[3] = ((kbar + ((3 * fp->N_RB_DL) >> 1) * 6) % (fp->N_RB_DL * 12)) / 6;
  if (reg[3] < first) { *first_idx = 3; first = reg[3]; }
}

int orc_generate_pcfich(uint8_t num_pdcch_symbols, int16_t amp, const orc_frame_t *fp, int32_t **txdataF,
                        uint8_t subframe)
{
  uint8_t bt[32], first_idx;
  int16_t d[2][16][2];
  uint16_t reg[4];
  if (num_pdcch_symbols < 1 || num_pdcch_symbols > 3) return -1;   /* :164 (else bt is uninitialised) */
  orc_pcfich_reg_mapping(fp, reg, &first_idx);
  uint32_t x1, x2 = ((((2 * fp->Nid_cell) + 1) * (1 + subframe)) << 9) + fp->Nid_cell, s = 0;  /* :97 */
  for (int i = 0; i < 32; i++) {                                                                /* :99-108 */
    if ((i & 0x1f) == 0) s = orc_gold_generic(&x1, &x2, 1);
    bt[i] = (orc_pcfich_b[num_pdcch_symbols - 1][i] & 1) ^ ((s >> (i & 0x1f)) & 1);
  }
  int16_t g = fp->mode1_flag == 1 ? (int16_t)((amp * 23170) >> 15) : (int16_t)(amp / 2);       /* :168-171 */
  if (fp->mode1_flag) {
    for (int i = 0; i < 16; i++) {
      d[0][i][0] = d[1][i][0] = bt[2 * i] == 1 ? -g : g;
      d[0][i][1] = d[1][i][1] = bt[2 * i + 1] == 1 ? -g : g;
    }
  } else {                                                                                      /* :182-196 */
    for (int i = 0; i < 16; i += 2) {
      d[0][i][0] = bt[2 * i] == 1 ? -g : g;
      d[0][i][1] = bt[2 * i + 1] == 1 ? -g : g;
      d[1][i][0] = bt[2 * i + 2] == 1 ? g : -g;
      d[1][i][1] = bt[2 * i + 3] == 1 ? -g : g;
      d[0][i + 1][0] = -d[1][i][0];
      d[0][i + 1][1] = d[1][i][1];
      d[1][i + 1][0] = d[0][i][0];
      d[1][i + 1][1] = -d[0][i][1];
    }
  }
  uint32_t nsymb = fp->Ncp == 0 ? 14 : 12, N = fp->ofdm_symbol_size;
  uint32_t symbol_offset = N * (subframe * nsymb), m = 0, nushiftmod3 = fp->nushift % 3;
  for (int q = 0; q < 4; q++) {                                                                 /* :209-226 */
    uint32_t reg_offset = fp->first_carrier_offset + (uint16_t)reg[q] * 6;
    if (reg_offset >= N) reg_offset = 1 + reg_offset - N;
    for (uint32_t i = 0; i < 6; i++)
      if (i != nushiftmod3 && i != nushiftmod3 + 3) {
        int16_t *t0 = (int16_t *)&txdataF[0][symbol_offset + reg_offset + i];
        t0[0] = d[0][m][0];
        t0[1] = d[0][m][1];
        if (fp->nb_antennas_tx > 1) {
          int16_t *t1 = (int16_t *)&txdataF[1][symbol_offset + reg_offset + i];
          t1[0] = d[1][m][0];
          t1[1] = d[1][m][1];
        }
        m++;
      }
  }
  return 0;
}
