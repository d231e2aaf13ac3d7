/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle of the synchronisation, broadcast and HARQ-indicator
 * channels of the downlink grid (after PCFICH and PDCCH).  A plain-C
 * restatement of the reference's algorithm, loop for loop, used by tests/ as the checker of the
 * GPU path; never linked into the product library.
 *
 *   primary_synch0/1/2       PHY/LTE_REFSIG/primary_synch.h (Zadoff-Chu roots 25/29/34, the
 *                            table's rounding: floor(32767 x), 5 zero REs either side)
 *   generate_pss             PHY/LTE_TRANSPORT/pss.c:50-103
 *   d0_sss / d5_sss          PHY/LTE_TRANSPORT/sss.h (36.211 §6.11.2.1 m-sequences)
 *   generate_sss             PHY/LTE_TRANSPORT/sss.c:47-92
 *   generate_pbch            PHY/LTE_TRANSPORT/pbch.c:161-420 (+ allocate_pbch_REs_in_RB :62-158,
 *                            pbch_scrambling :760-783)
 *   generate_phich           PHY/LTE_TRANSPORT/phich.c:401-780 (normal cyclic prefix)
 *   is_not_pilot             PHY/LTE_TRANSPORT/dlsch_modulation.c:53-71
 *
 * Pinned: the PSS and SSS tables entry by entry against the reference headers
 * (tests/test_sync_cpu.py, when /root/reference is present); the PBCH coding chain through
 * crc16 / ccodelte_encode, which are pinned to the reference's own crc_byte.c /
 * ccoding_byte_lte.c (oracle/_ref/libref_coding.so); every channel against the 36.211 / 36.212
 * spec model (tests/spec_model.py: pss_grid, sss_grid, pbch_grid, phich_grid).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oai_oracle.h"

#define ONE_OVER_SQRT2_Q15 23170   /* PHY/impl_defs_top.h */

/* ---------------------------------------------------------------- tables */
void orc_primary_synch(uint8_t Nid2, int16_t out[144])
{
  static const int u[3] = {25, 29, 34};
  memset(out, 0, 144 * sizeof(int16_t));
  for (int n = 0; n < 62; n++) {
    const int m = n < 31 ? n : n + 1;
    const double ang = -M_PI * u[Nid2 % 3] * m * (m + 1) / 63.0;
    out[10 + 2 * n] = (int16_t)floor(32767.0 * cos(ang));
    out[11 + 2 * n] = (int16_t)floor(32767.0 * sin(ang));
  }
}

static void mseq31(const int *taps, int ntaps, int8_t out[31])
{
  int x[31] = {0, 0, 0, 0, 1};
  for (int i = 0; i < 26; i++) {
    int v = 0;
    for (int t = 0; t < ntaps; t++) v += x[i + taps[t]];
    x[i + 5] = v & 1;
  }
  for (int i = 0; i < 31; i++) out[i] = (int8_t)(1 - 2 * x[i]);
}

void orc_sss_seq(uint16_t Nid_cell, int sf5, int16_t d[62])
{
  static const int ts[2] = {2, 0}, tc[2] = {3, 0}, tz[4] = {4, 2, 1, 0};
  int8_t st[31], ct[31], zt[31];
  mseq31(ts, 2, st);
  mseq31(tc, 2, ct);
  mseq31(tz, 4, zt);
  const int n1 = Nid_cell / 3, n2 = Nid_cell % 3;
  const int qp = n1 / 30, q = (n1 + qp * (qp + 1) / 2) / 30, mp = n1 + q * (q + 1) / 2;
  const int m0 = mp % 31, m1 = (m0 + mp / 31 + 1) % 31;
  for (int n = 0; n < 31; n++) {
    const int s0 = st[(n + m0) % 31], s1 = st[(n + m1) % 31];
    const int c0 = ct[(n + n2) % 31], c1 = ct[(n + n2 + 3) % 31];
    const int z0 = zt[(n + m0 % 8) % 31], z1 = zt[(n + m1 % 8) % 31];
    d[2 * n] = (int16_t)(sf5 ? s1 * c0 : s0 * c0);
    d[2 * n + 1] = (int16_t)(sf5 ? s0 * c1 * z1 : s1 * c1 * z0);
  }
}

/* ---------------------------------------------------------------- PSS / SSS (frame grids) */
int orc_generate_pss(int32_t **txdataF, int16_t amp, const orc_frame_t *fp, uint16_t symbol, uint16_t slot_offset)
{
  int16_t ps[144];
  orc_primary_synch((uint8_t)(fp->Nid_cell % 3), ps);
  const short a = (fp->nb_antennas_tx == 1) ? amp : (short)((amp * ONE_OVER_SQRT2_Q15) >> 15);
  const unsigned Nsymb = fp->Ncp == 0 ? 14 : 12, N = fp->ofdm_symbol_size;
  for (unsigned aa = 0; aa < fp->nb_antennas_tx; aa++) {
    unsigned short k = (unsigned short)(N - 3 * 12 + 5);
    for (int m = 5; m < 67; m++) {
      int16_t *p = (int16_t *)&txdataF[aa][slot_offset * Nsymb / 2 * N + symbol * N + k];
      p[0] = (int16_t)((a * ps[2 * m]) >> 15);
      p[1] = (int16_t)((a * ps[2 * m + 1]) >> 15);
      k += 1;
      if (k >= N) {
        k++;
        k -= N;
      }
    }
  }
  return 0;
}

int orc_generate_sss(int32_t **txdataF, int16_t amp, const orc_frame_t *fp, uint16_t symbol, uint16_t slot_offset)
{
  int16_t d[62];
  orc_sss_seq(fp->Nid_cell, slot_offset < 3 ? 0 : 1, d);
  const unsigned Nsymb = fp->Ncp == 0 ? 14 : 12, N = fp->ofdm_symbol_size;
  int16_t k = (int16_t)(N - 3 * 12 + 5);
  const int16_t a = (fp->nb_antennas_tx == 1) ? amp : (int16_t)((amp * ONE_OVER_SQRT2_Q15) >> 15);
  for (int i = 0; i < 62; i++) {
    for (unsigned aa = 0; aa < fp->nb_antennas_tx; aa++) {
      int16_t *p = (int16_t *)&txdataF[aa][slot_offset * Nsymb / 2 * N + symbol * N + k];
      p[0] = (int16_t)(a * d[i]);
      p[1] = 0;
    }
    k += 1;
    if (k >= (int16_t)N) {
      k++;
      k -= (int16_t)N;
    }
  }
  return 0;
}

/* ---------------------------------------------------------------- PBCH */
static uint8_t is_not_pilot(uint8_t pilots, uint8_t re, uint8_t nushift, uint8_t use2ndpilots)
{
  const uint8_t offset = (pilots == 2) ? 3 : 0;
  const int ns3 = nushift % 3;
  if (pilots == 0) return 1;
  if (use2ndpilots == 1) {
    if ((re != nushift + offset) && (re != ((nushift + 6 + offset) % 12))) return 1;
  } else {
    if ((re != ns3) && (re != ns3 + 6) && (re != ns3 + 3) && (re != ns3 + 9)) return 1;
  }
  return 0;
}

static void allocate_pbch_REs_in_RB(const orc_frame_t *fp, int32_t **txdataF, uint32_t *jj, uint16_t re_offset,
                                    uint32_t symbol_offset, const uint8_t *x0, uint8_t pilots, int16_t amp,
                                    uint32_t *re_allocated)
{
  const int siso = fp->mode1_flag == 1;
  const int16_t gain_lin_QPSK = (int16_t)((amp * ONE_OVER_SQRT2_Q15) >> 15);
  for (uint8_t re = 0; re < 12; re++) {
    const uint32_t tti_offset = symbol_offset + re_offset + re;
    if (is_not_pilot(pilots, re, fp->nushift, 0) != 1) continue;
    if (siso) {
      *re_allocated += 1;
      for (unsigned aa = 0; aa < fp->nb_antennas_tx; aa++)
        ((int16_t *)&txdataF[aa][tti_offset])[0] += (x0[*jj] == 1) ? (int16_t)-gain_lin_QPSK : gain_lin_QPSK;
      *jj += 1;
      for (unsigned aa = 0; aa < fp->nb_antennas_tx; aa++)
        ((int16_t *)&txdataF[aa][tti_offset])[1] += (x0[*jj] == 1) ? (int16_t)-gain_lin_QPSK : gain_lin_QPSK;
      *jj += 1;
    } else {
      int16_t t1[2], t2[2];
      *re_allocated += 1;
      t1[0] = (x0[*jj] == 1) ? (int16_t)-gain_lin_QPSK : gain_lin_QPSK;
      *jj += 1;
      t1[1] = (x0[*jj] == 1) ? (int16_t)-gain_lin_QPSK : gain_lin_QPSK;
      *jj += 1;
      t2[0] = (x0[*jj] == 1) ? gain_lin_QPSK : (int16_t)-gain_lin_QPSK;   /* -x1* */
      *jj += 1;
      t2[1] = (x0[*jj] == 1) ? (int16_t)-gain_lin_QPSK : gain_lin_QPSK;
      *jj += 1;
      int16_t *y0 = (int16_t *)&txdataF[0][tti_offset], *y1 = (int16_t *)&txdataF[1][tti_offset];
      y0[0] += (int16_t)((t1[0] * ONE_OVER_SQRT2_Q15) >> 15);
      y0[1] += (int16_t)((t1[1] * ONE_OVER_SQRT2_Q15) >> 15);
      y1[0] += (int16_t)((t2[0] * ONE_OVER_SQRT2_Q15) >> 15);
      y1[1] += (int16_t)((t2[1] * ONE_OVER_SQRT2_Q15) >> 15);
      const uint32_t pn = is_not_pilot(pilots, re + 1, fp->nushift, 0) == 1 ? 1 : 2;
      int16_t *z0 = (int16_t *)&txdataF[0][tti_offset + pn], *z1 = (int16_t *)&txdataF[1][tti_offset + pn];
      z0[0] += -y1[0];
      z0[1] += y1[1];
      z1[0] += y0[0];
      z1[1] += -y0[1];
      re++;
      *re_allocated += 1;
      if (is_not_pilot(pilots, re, fp->nushift, 0) == 0) {
        re++;
        *re_allocated += 1;
      }
    }
  }
}

void orc_pbch_scrambling(const orc_frame_t *fp, uint8_t *e, uint32_t length)
{
  uint32_t x1 = 0, x2 = fp->Nid_cell, s = 0;
  uint8_t reset = 1;
  for (uint32_t i = 0; i < length; i++) {
    if ((i & 0x1f) == 0) {
      s = orc_gold_generic(&x1, &x2, reset);
      reset = 0;
    }
    e[i] = (e[i] & 1) ^ ((s >> (i & 0x1f)) & 1);
  }
}

int orc_generate_pbch(orc_pbch_t *st, int32_t **txdataF, int amp, const orc_frame_t *fp, const uint8_t *pbch_pdu,
                      uint8_t frame_mod4)
{
  const uint32_t nsymb = fp->Ncp == 0 ? 14 : 12, second_pilot = fp->Ncp == 0 ? 4 : 3;
  const uint32_t pbch_D = 16 + 24, pbch_E = fp->Ncp == 0 ? 1920 : 1728;
  uint32_t jj = 0, re_allocated = 0;
  if (frame_mod4 == 0) {
    uint8_t pbch_a[3];
    uint16_t amask = 0;
    memset(st->pbch_e, 0, pbch_E);
    memset(st->pbch_d, ORC_LTE_NULL, 96);
    for (int i = 0; i < 3; i++) pbch_a[3 - i - 1] = pbch_pdu[i];
    if (fp->mode1_flag != 1) amask = fp->nb_antennas_tx_eNB == 2 ? 0xffff : (fp->nb_antennas_tx_eNB == 4 ? 0x5555 : 0);
    orc_ccodelte_encode(24, 2, pbch_a, st->pbch_d + 96, amask);
    const uint32_t RCC = orc_sub_block_interleaving_cc(pbch_D, st->pbch_d + 96, st->pbch_w);
    orc_lte_rate_matching_cc(RCC, (uint16_t)pbch_E, st->pbch_w, st->pbch_e);
    orc_pbch_scrambling(fp, st->pbch_e, pbch_E);
  }
  for (uint32_t l = nsymb >> 1; l < (nsymb >> 1) + 4; l++) {
    uint8_t pilots = 0;
    if (l == 0 || l == (nsymb >> 1)) pilots = 1;
    if (l == 1 || l == (nsymb >> 1) + 1) pilots = 1;
    if (l == second_pilot || l == second_pilot + (nsymb >> 1)) pilots = 1;
    uint32_t re_offset = fp->ofdm_symbol_size - 3 * 12;
    const uint32_t symbol_offset = (uint32_t)fp->ofdm_symbol_size * l;
    for (int rb = 0; rb < 6; rb++) {
      allocate_pbch_REs_in_RB(fp, txdataF, &jj, (uint16_t)re_offset, symbol_offset,
                              &st->pbch_e[frame_mod4 * (pbch_E >> 2)], pilots, (int16_t)amp, &re_allocated);
      re_offset += 12;
      if (re_offset >= fp->ofdm_symbol_size) re_offset = 1;
    }
  }
  return 0;
}

/* ---------------------------------------------------------------- PHICH (normal CP) */
int orc_generate_phich(const orc_frame_t *fp, int16_t amp, uint8_t nseq_PHICH, uint8_t ngroup_PHICH, uint8_t HI,
                       uint8_t subframe, int32_t **y)
{
  if (fp->Ncp != 0 || fp->phich_duration != 0) return -1;   /* restated: normal CP, normal duration */
  uint16_t reg[56][3];
  orc_phich_reg_mapping(fp, reg);
  int16_t d[24], cs[12];
  const uint32_t subframe_offset = 14u * fp->ofdm_symbol_size * subframe;
  const int16_t gain = fp->mode1_flag == 1 ? (int16_t)(((int32_t)amp * ONE_OVER_SQRT2_Q15) >> 15) : (int16_t)(amp / 2);
  memset(d, 0, sizeof(d));
  if (HI > 0) HI = 1;
  uint32_t x1 = 0, x2 = (((uint32_t)(subframe + 1) * (fp->Nid_cell + 1u)) << 9) + fp->Nid_cell;
  const uint32_t s = orc_gold_generic(&x1, &x2, 1);
  for (int i = 0; i < 12; i++) {
    cs[i] = (uint8_t)((s >> (i & 0x1f)) & 1);
    cs[i] = cs[i] == 0 ? (int16_t)(1 - (HI << 1)) : (int16_t)((HI << 1) - 1);
  }
  /* orthogonal sequence per group of 4 symbols (36.211 Table 6.9.1-2); +j entries put the
   * value in the imaginary part with the real part negated as the reference writes them */
  static const int8_t w[8][4] = {{1, 1, 1, 1},  {1, -1, 1, -1},  {1, 1, -1, -1},  {1, -1, -1, 1},
                                 {1, 1, 1, 1},  {1, -1, 1, -1},  {1, 1, -1, -1},  {1, -1, -1, 1}};
  for (int i = 0, i2 = 0, i3 = 0; i < 3; i++, i2 += 4, i3 += 8)
    for (int q = 0; q < 4; q++) {
      const int16_t v = (int16_t)(w[nseq_PHICH & 7][q] * cs[i2 + q]);
      if (nseq_PHICH < 4) {
        d[i3 + 2 * q] = v;
        d[i3 + 2 * q + 1] = v;
      } else {
        d[i3 + 2 * q] = (int16_t)-v;
        d[i3 + 2 * q + 1] = v;
      }
    }
  for (int sym = 0; sym < 3; sym++) {
    uint32_t re_offset = fp->first_carrier_offset + reg[ngroup_PHICH][sym] * 6u;
    if (re_offset > fp->ofdm_symbol_size) re_offset -= (fp->ofdm_symbol_size - 1u);   /* '>' as phich.c:560 */
    int16_t y0_16[8], y1_16[8];
    const int16_t *dd = d + 8 * sym;
    if (fp->mode1_flag == 0) {
      for (int h = 0; h < 2; h++) {
        y0_16[4 * h] = (int16_t)(dd[4 * h] * gain);
        y0_16[4 * h + 1] = (int16_t)(dd[4 * h + 1] * gain);
        y1_16[4 * h] = (int16_t)(-dd[4 * h + 2] * gain);
        y1_16[4 * h + 1] = (int16_t)(dd[4 * h + 3] * gain);
        y0_16[4 * h + 2] = (int16_t)-y1_16[4 * h];
        y0_16[4 * h + 3] = y1_16[4 * h + 1];
        y1_16[4 * h + 2] = y0_16[4 * h];
        y1_16[4 * h + 3] = (int16_t)-y0_16[4 * h + 1];
      }
      int16_t *Y0 = (int16_t *)&y[0][re_offset + subframe_offset], *Y1 = (int16_t *)&y[1][re_offset + subframe_offset];
      for (int i = 0, j = 0, m = 0; i < 6; i++, j += 2)
        if (i != fp->nushift && i != fp->nushift + 3) {
          Y0[j] += y0_16[m];
          Y1[j] += y1_16[m++];
          Y0[j + 1] += y0_16[m];
          Y1[j + 1] += y1_16[m++];
        }
    } else {
      for (int m = 0; m < 8; m++) y0_16[m] = (int16_t)(dd[m] * gain);
      int16_t *Y0 = (int16_t *)&y[0][re_offset + subframe_offset];
      for (int i = 0, j = 0, m = 0; i < 6; i++, j += 2)
        if (i != fp->nushift && i != fp->nushift + 3) {
          Y0[j] += y0_16[m++];
          Y0[j + 1] += y0_16[m++];
        }
    }
  }
  return 0;
}
