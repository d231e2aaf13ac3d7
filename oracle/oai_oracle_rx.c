/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle of the UE's PDSCH demodulation after the FEP (SURVEY.md
 * §8f item 3, second half), single transmit port (TM1), one receive antenna, even N_RB_DL.
 * A plain-C restatement of the reference's algorithm, loop for loop; never linked into the
 * product library.
 *
 *   dlsch_extract_rbs_single    PHY/LTE_TRANSPORT/dlsch_demodulation.c:3167-3300 (even N_RB_DL:
 *                               every allocated RB, pilots skipped in symbols 0 / 4-Ncp of a slot;
 *                               NB the reference applies no PBCH / PSS / SSS exclusion here)
 *   dlsch_channel_level         dlsch_demodulation.c:2777-2835 (first PDSCH symbol, int32 sums)
 *   log2_maxh                   dlsch_demodulation.c:286-300, log2_approx TOOLS/log2_approx.c:29-45
 *   dlsch_channel_compensation  dlsch_demodulation.c:801-960 (conj(h) y >> shift, packs; |h|^2 >>
 *                               shift packed, mulhi by QAM_n1 / QAM_n2, << 1)
 *   dlsch_qpsk/16qam/64qam_llr  PHY/LTE_TRANSPORT/dlsch_llr_computation.c:636-930 (len from
 *                               adjust_G2, lte_mcs.c:157-245, for 16 / 64-QAM)
 *   dlsch_unscrambling          PHY/LTE_TRANSPORT/dlsch_scrambling.c:99-137 (llr * (2 c - 1), int16)
 *
 * Channel estimates are an input (dl_ch_estimates[symbol * N + 5 + 12 rb + i], the layout the
 * reference's estimator and dlsim's perfect-CE mode write, dlsim.c:2935-2966).
 */
#include <stdlib.h>
#include <string.h>

#include "oai_oracle.h"

#define QAM16_n1 20724   /* PHY/impl_defs_top.h:215-224 */
#define QAM64_n1 20225
#define QAM64_n2 10112

static int16_t sat16(int32_t v) { return (int16_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v)); }
static int16_t abs16(int16_t v) { return (int16_t)(v < 0 ? -v : v); }      /* _mm_abs_epi16: -32768 stays */
static int16_t mulhi2(int16_t a, int16_t b) { return (int16_t)((((int32_t)a * b) >> 16) << 1); }

static int alloc_bit(const uint32_t rb_alloc[4], int rb)
{
  if (rb < 32) return (rb_alloc[0] >> rb) & 1;
  if (rb < 64) return (rb_alloc[1] >> (rb - 32)) & 1;
  if (rb < 96) return (rb_alloc[2] >> (rb - 64)) & 1;
  if (rb < 100) return (rb_alloc[3] >> (rb - 96)) & 1;
  return 0;
}

uint8_t orc_log2_approx(uint32_t x)
{
  uint8_t l2 = 0;
  for (int i = 0; i < 31; i++)
    if (x & (1u << i)) l2 = (uint8_t)(i + 1);
  return l2;
}

int orc_adjust_G2(const orc_frame_t *fp, const uint32_t rb_alloc[4], uint8_t subframe, uint8_t symbol)
{
  const int nsymb = fp->Ncp == 0 ? 14 : 12;
  int re = 0;
  if (subframe != 0 && subframe != 5 && subframe != 6) return 0;
  if (symbol < (nsymb >> 1) && fp->frame_type == 1 && subframe != 6) return 0;
  if (fp->frame_type == 1) {
    if (symbol > (nsymb >> 1) + 3 && symbol != nsymb - 1) return 0;
    if (subframe == 5 && symbol != nsymb - 1) return 0;
    if (subframe == 6 && symbol != 2) return 0;
  } else {
    if (symbol > (nsymb >> 1) + 3 || symbol < (nsymb >> 1) - 2) return 0;
    if (subframe == 5 && symbol != (nsymb >> 1) - 1 && symbol != (nsymb >> 1) - 2) return 0;
    if (subframe == 6) return 0;
  }
  if (fp->N_RB_DL & 1) {
    for (int rb = (fp->N_RB_DL >> 1) - 3; rb <= (fp->N_RB_DL >> 1) + 3; rb++)
      if (alloc_bit(rb_alloc, rb)) re += (rb == (fp->N_RB_DL >> 1) - 3 || rb == (fp->N_RB_DL >> 1) + 3) ? 6 : 12;
  } else {
    for (int rb = (fp->N_RB_DL >> 1) - 3; rb < (fp->N_RB_DL >> 1) + 3; rb++)
      if (alloc_bit(rb_alloc, rb)) re += 12;
  }
  return re;
}

/* extraction of one symbol: returns the number of extracted REs */
static int extract(const orc_frame_t *fp, const int32_t *rxF_sym, const int32_t *ch_sym, const uint32_t rb_alloc[4],
                   uint8_t symbol, int32_t *rx_ext, int32_t *ch_ext, int *nb_rb)
{
  const int symbol_mod = symbol >= 7 - fp->Ncp ? symbol - (7 - fp->Ncp) : symbol;
  const int pilots = symbol_mod == 0 || symbol_mod == 4 - fp->Ncp;
  const int poffset = symbol_mod == 4 - fp->Ncp ? 3 : 0;
  const int32_t *rxF = rxF_sym + fp->first_carrier_offset, *dl_ch0 = ch_sym + 5;
  int n = 0;
  *nb_rb = 0;
  for (int rb = 0; rb < fp->N_RB_DL; rb++) {
    if (rb == (fp->N_RB_DL >> 1)) rxF = rxF_sym + 1;
    if (alloc_bit(rb_alloc, rb)) {
      for (int i = 0; i < 12; i++)
        if (!pilots || (i != fp->nushift + poffset && i != (fp->nushift + poffset + 6) % 12)) {
          rx_ext[n] = rxF[i];
          ch_ext[n] = dl_ch0[i];
          n++;
        }
      (*nb_rb)++;
    }
    dl_ch0 += 12;
    rxF += 12;
  }
  return n;
}

int orc_rx_pdsch_siso(const orc_frame_t *fp, const int32_t *rxdataF, const int32_t *dl_ch_estimates,
                      const uint32_t rb_alloc[4], uint8_t Qm, uint8_t num_pdcch_symbols, uint8_t subframe,
                      int16_t *llr, uint8_t *log2_maxh_out)
{
  if (fp->N_RB_DL & 1) return -1;
  const int N = fp->ofdm_symbol_size, nsymb = fp->Ncp == 0 ? 14 : 12;
  int32_t *rx_ext = (int32_t *)malloc(sizeof(int32_t) * 12 * 110), *ch_ext = (int32_t *)malloc(sizeof(int32_t) * 12 * 110);
  int16_t *out = llr;
  uint8_t log2_maxh = 0;
  for (int symbol = num_pdcch_symbols; symbol < nsymb; symbol++) {
    int nb_rb;
    const int n = extract(fp, rxdataF + symbol * N, dl_ch_estimates + symbol * N, rb_alloc, (uint8_t)symbol, rx_ext,
                          ch_ext, &nb_rb);
    (void)n;
    const int symbol_mod = symbol >= 7 - fp->Ncp ? symbol - (7 - fp->Ncp) : symbol;
    const int pil = symbol_mod == 0 || symbol_mod == 4 - fp->Ncp;
    if (symbol == num_pdcch_symbols) {                       /* dlsch_channel_level, first symbol */
      int32_t acc = 0;
      const int nre = pil ? 10 : 12;                           /* mode1_flag = 1 */
      for (int j = 0; j < nb_rb * 12; j++) {                   /* 3 groups of 4 REs per RB */
        const int16_t hr = (int16_t)(ch_ext[j] & 0xFFFF), hi = (int16_t)(ch_ext[j] >> 16);
        acc = (int32_t)((uint32_t)acc + (uint32_t)((int32_t)hr * hr) + (uint32_t)((int32_t)hi * hi));
      }
      const int32_t avg = acc / (nb_rb * nre);
      log2_maxh = (uint8_t)(orc_log2_approx((uint32_t)(avg > 0 ? avg : 0)) / 2);
    }
    int len;
    if (Qm == 2) len = pil ? nb_rb * 10 : nb_rb * 12;
    else len = (pil ? nb_rb * 10 - 5 * orc_adjust_G2(fp, rb_alloc, subframe, (uint8_t)symbol) / 6
                    : nb_rb * 12 - orc_adjust_G2(fp, rb_alloc, subframe, (uint8_t)symbol));
    const int16_t a1 = Qm == 4 ? QAM16_n1 : QAM64_n1, a2 = Qm == 4 ? 0 : QAM64_n2;
    for (int j = 0; j < len; j++) {
      const int16_t hr = (int16_t)(ch_ext[j] & 0xFFFF), hi = (int16_t)(ch_ext[j] >> 16);
      const int16_t yr = (int16_t)(rx_ext[j] & 0xFFFF), yi = (int16_t)(rx_ext[j] >> 16);
      /* madd_epi16 (int32 wrap), the conjugate by sign_epi16 (int16 wrap: -(-32768) = -32768) */
      const int16_t nhi = (int16_t)-hi;
      const int16_t cr = sat16((int32_t)((uint32_t)((int32_t)hr * yr) + (uint32_t)((int32_t)hi * yi)) >> log2_maxh);
      const int16_t ci = sat16((int32_t)((uint32_t)((int32_t)nhi * yr) + (uint32_t)((int32_t)hr * yi)) >> log2_maxh);
      if (Qm == 2) {
        *out++ = cr;
        *out++ = ci;
        continue;
      }
      const int16_t m = sat16((int32_t)((uint32_t)((int32_t)hr * hr) + (uint32_t)((int32_t)hi * hi)) >> log2_maxh);
      const int16_t mag = mulhi2(m, a1), magb = mulhi2(m, a2);
      const int16_t x1r = sat16((int32_t)mag - abs16(cr)), x1i = sat16((int32_t)mag - abs16(ci));
      *out++ = cr;
      *out++ = ci;
      *out++ = x1r;
      *out++ = x1i;
      if (Qm == 6) {
        *out++ = sat16((int32_t)magb - abs16(x1r));
        *out++ = sat16((int32_t)magb - abs16(x1i));
      }
    }
  }
  free(rx_ext);
  free(ch_ext);
  if (log2_maxh_out) *log2_maxh_out = log2_maxh;
  return (int)(out - llr);
}

void orc_dlsch_unscrambling(int16_t *llr, int G, uint32_t c_init)
{
  uint32_t x1 = 0, x2 = c_init;
  uint32_t s = orc_gold_generic(&x1, &x2, 1);
  int k = 0;
  for (int i = 0; i < 1 + (G >> 5); i++) {
    for (int j = 0; j < 32; j++, k++) llr[k] = (int16_t)(((2 * ((s >> j) & 1)) - 1) * llr[k]);
    s = orc_gold_generic(&x1, &x2, 0);
  }
}
