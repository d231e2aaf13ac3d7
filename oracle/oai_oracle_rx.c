/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle of the UE's PDSCH demodulation after the FEP (SURVEY.md
 * §8f item 3, second half), single transmit port (TM1), one receive antenna.
 * A plain-C restatement of the reference's algorithm, loop for loop; never linked into the
 * product library.
 *
 *   dlsch_extract_rbs_single    PHY/LTE_TRANSPORT/dlsch_demodulation.c:3167-3681 (even N_RB_DL:
 *                               every allocated RB, pilots skipped in symbols 0 / 4-Ncp of a slot,
 *                               no PBCH / PSS / SSS exclusion; odd N_RB_DL: the RB around DC split
 *                               at bin 0, PBCH / PSS / SSS RBs dropped and the two edge RBs
 *                               halved, with the reference's pointer steps — a stream that would
 *                               read ext slots the call did not write returns -1)
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

/* one RE of dlsch_qpsk_llr / dlsch_16qam_llr / dlsch_64qam_llr (dlsch_llr_computation.c:636-930): the
 * compensated (cr, ci) pass through; 16-QAM appends mag -sat |y| (abs_epi16 keeps -32768), 64-QAM
 * also magb -sat |that|.  Returns the LLRs written. */
static int llr_qam_re(int Qm, int16_t cr, int16_t ci, int16_t mag, int16_t magb, int16_t *out)
{
  out[0] = cr;
  out[1] = ci;
  if (Qm == 2) return 2;
  const int16_t x1r = sat16((int32_t)mag - abs16(cr)), x1i = sat16((int32_t)mag - abs16(ci));
  out[2] = x1r;
  out[3] = x1i;
  if (Qm == 4) return 4;
  out[4] = sat16((int32_t)magb - abs16(x1r));
  out[5] = sat16((int32_t)magb - abs16(x1i));
  return 6;
}

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

/* one RE of dlsch_extract_rbs_single: writes slot *pos of the ext arrays (tracking the highest
 * slot written: the odd-N_RB branch can write one past the pointer it then advances) */
static void put(int32_t *rx_ext, int32_t *ch_ext, int pos, int32_t rx, int32_t ch, int *hw)
{
  rx_ext[pos] = rx;
  ch_ext[pos] = ch;
  if (pos + 1 > *hw) *hw = pos + 1;
}

/* extraction of one symbol (dlsch_extract_rbs_single, dlsch_demodulation.c:3167-3681): returns the
 * final ext pointer; *hw = the number of ext slots written (>= the pointer) */
static int extract(const orc_frame_t *fp, const int32_t *rxF_sym, const int32_t *ch_sym, const uint32_t rb_alloc[4],
                   uint8_t symbol, uint8_t subframe, int32_t *rx_ext, int32_t *ch_ext, int *nb_rb, int *hw)
{
  const int symbol_mod = symbol >= 7 - fp->Ncp ? symbol - (7 - fp->Ncp) : symbol;
  const int pilots = symbol_mod == 0 || symbol_mod == 4 - fp->Ncp;
  const int poffset = symbol_mod == 4 - fp->Ncp ? 3 : 0;
  const int nsymb = fp->Ncp == 0 ? 14 : 12, l = symbol, half = fp->N_RB_DL >> 1;
  const int sss_symb = fp->frame_type == 1 ? nsymb - 1 : (nsymb >> 1) - 2;
  const int pss_symb = fp->frame_type == 1 ? 2 : (nsymb >> 1) - 1;
  const int32_t *rxF = rxF_sym + fp->first_carrier_offset, *dl_ch0 = ch_sym + 5;
  int n = 0;
  *nb_rb = 0;
  *hw = 0;
  if ((fp->N_RB_DL & 1) == 0) {                               /* :3218-3281, no PBCH / PSS / SSS exclusion */
    for (int rb = 0; rb < fp->N_RB_DL; rb++) {
      if (rb == half) rxF = rxF_sym + 1;
      if (alloc_bit(rb_alloc, rb)) {
        for (int i = 0; i < 12; i++)
          if (!pilots || (i != fp->nushift + poffset && i != (fp->nushift + poffset + 6) % 12)) {
            put(rx_ext, ch_ext, n, rxF[i], dl_ch0[i], hw);
            n++;
          }
        (*nb_rb)++;
      }
      dl_ch0 += 12;
      rxF += 12;
    }
    return n;
  }
  /* odd N_RB_DL (:3282-3676) */
  const int pbch_l = subframe == 0 && l >= (nsymb >> 1) && l < (nsymb >> 1) + 4;
  const int sss_l = (subframe == 0 || subframe == 5) && l == sss_symb;
  const int pss_l = (fp->frame_type == 0 && (subframe == 0 || subframe == 5) && l == pss_symb) ||
                    (fp->frame_type == 1 && subframe == 6 && l == pss_symb);
  for (int rb = 0; rb < fp->N_RB_DL; rb++) {
    int ind = alloc_bit(rb_alloc, rb);
    if (rb == half) {                                         /* the RB around DC (:3434-3525) */
      if (pbch_l || sss_l || pss_l) ind = 0;
      if (ind) {
        int j = 0;
        for (int i = 0; i < 12; i++) {
          const int32_t rxv = i < 6 ? rxF[i] : rxF_sym[1 + i - 6];
          if (!pilots) put(rx_ext, ch_ext, n + i, rxv, dl_ch0[i], hw);
          else if (i < 6 ? i != (fp->nushift + poffset) % 6 : i != (fp->nushift + 6 + poffset) % 12)
            put(rx_ext, ch_ext, n + j++, rxv, dl_ch0[i], hw);
        }
        n += pilots ? 10 : 12;
        (*nb_rb)++;
      }
      rxF = rxF_sym + 7;
      dl_ch0 += 12;
      continue;
    }
    int skip_half = 0;
    if ((pbch_l || sss_l || pss_l) && rb > half - 3 && rb < half + 3) ind = 0;
    if (pbch_l || sss_l || pss_l) skip_half = rb == half - 3 ? 1 : (rb == half + 3 ? 2 : 0);
    if (ind) {
      if (skip_half) {
        const int o = skip_half == 2 ? 6 : 0;
        int j = 0;
        for (int i = 0; i < 6; i++)
          if (!pilots || i != (fp->nushift + poffset) % 6) put(rx_ext, ch_ext, n + j++, rxF[i + o], dl_ch0[i + o], hw);
        n += pilots ? 5 : 6;
      } else {
        int j = 0;
        for (int i = 0; i < 12; i++)
          if (!pilots || (i != fp->nushift + poffset && i != (fp->nushift + poffset + 6) % 12))
            put(rx_ext, ch_ext, n + j++, rxF[i], dl_ch0[i], hw);
        n += pilots ? 10 : 12;
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
  const int N = fp->ofdm_symbol_size, nsymb = fp->Ncp == 0 ? 14 : 12;
  int32_t *rx_ext = (int32_t *)malloc(sizeof(int32_t) * 12 * 110), *ch_ext = (int32_t *)malloc(sizeof(int32_t) * 12 * 110);
  int16_t *out = llr;
  uint8_t log2_maxh = 0;
  for (int symbol = num_pdcch_symbols; symbol < nsymb; symbol++) {
    int nb_rb, hw;
    extract(fp, rxdataF + symbol * N, dl_ch_estimates + symbol * N, rb_alloc, (uint8_t)symbol, subframe, rx_ext, ch_ext,
            &nb_rb, &hw);
    const int symbol_mod = symbol >= 7 - fp->Ncp ? symbol - (7 - fp->Ncp) : symbol;
    const int pil = symbol_mod == 0 || symbol_mod == 4 - fp->Ncp;
    if (symbol == num_pdcch_symbols) {                       /* dlsch_channel_level, first symbol */
      int32_t acc = 0;
      const int nre = pil ? 10 : 12;                           /* mode1_flag = 1 */
      if (nb_rb * 12 > hw) { out = NULL; break; }              /* would read stale ext slots */
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
    if (len > hw) { out = NULL; break; }                       /* would read stale ext slots */
    const int16_t a1 = Qm == 4 ? QAM16_n1 : QAM64_n1, a2 = Qm == 4 ? 0 : QAM64_n2;
    for (int j = 0; j < len; j++) {
      const int16_t hr = (int16_t)(ch_ext[j] & 0xFFFF), hi = (int16_t)(ch_ext[j] >> 16);
      const int16_t yr = (int16_t)(rx_ext[j] & 0xFFFF), yi = (int16_t)(rx_ext[j] >> 16);
      /* madd_epi16 (int32 wrap), the conjugate by sign_epi16 (int16 wrap: -(-32768) = -32768) */
      const int16_t nhi = (int16_t)-hi;
      const int16_t cr = sat16((int32_t)((uint32_t)((int32_t)hr * yr) + (uint32_t)((int32_t)hi * yi)) >> log2_maxh);
      const int16_t ci = sat16((int32_t)((uint32_t)((int32_t)nhi * yr) + (uint32_t)((int32_t)hr * yi)) >> log2_maxh);
      if (Qm == 2) {
        out += llr_qam_re(2, cr, ci, 0, 0, out);
        continue;
      }
      const int16_t m = sat16((int32_t)((uint32_t)((int32_t)hr * hr) + (uint32_t)((int32_t)hi * hi)) >> log2_maxh);
      out += llr_qam_re(Qm, cr, ci, mulhi2(m, a1), mulhi2(m, a2), out);
    }
  }
  free(rx_ext);
  free(ch_ext);
  if (!out) return -1;
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

/* ======================================================================================
 * TM3 (LARGE_CDD, 2 TX ports), nb_rx receive antennas: rx_pdsch with dual_stream_flag = 0
 * (dlsim's TM3 UE), dlsch_demodulation.c:82-800:
 *   dlsch_extract_rbs_dual      :3683-4056 (PBCH / PSS / SSS RBs dropped, 8 REs per RB in pilot
 *                               symbols; odd N_RB_DL: the RB around DC, whose non-pilot second half
 *                               is read from bins 0..5, and the skip_half = 2 pilot branch whose
 *                               pointers advance inside the RE loop — all as written)
 *   dlsch_channel_level_TM3     :2902-2981 (precoded stream-0 |h|^2 per register lane, int32 wrap,
 *                               accumulated over the receive antennas without reset, per-lane
 *                               division, max of the per-antenna values)
 *   log2_maxh                   :390-394 (log2_approx(avg) - 13 + offset_mumimo_llr_drange[mcs0]
 *                               [Qm1 / 2 - 1], >= 0; the active table :76)
 *   prec2A_TM3_128              :1364-1396 (h0' = sat(h0 + s h1) >> 1, h1' = sat(h0 - s h1) >> 1,
 *                               s = +1, -1 alternating per extracted RE, sign_epi16 wrap)
 *   dlsch_channel_compensation_TM3 :1846-2120 (magnitudes and matched filters per antenna)
 *   dlsch_detection_mrc         :2583-2718 (stream 0 and its magnitudes: (a >> 1) +sat (b >> 1))
 *   dlsch_qpsk / 16qam / 64qam_llr of stream 0 (:583-800; qpsk with Qm1 = 2 is the interference-
 *                               aware qpsk_qpsk and is not restated: refused)
 * Codeword 1 is not demodulated in this mode (the reference computes llr[1] only for Qm0 = Qm1
 * = 2).  Even N_RB_DL and odd.
 * ==================================================================================== */
static const uint8_t mumimo_off[29][3] = {{0, 6, 5}, {0, 4, 5}, {0, 4, 5}, {0, 5, 4}, {0, 5, 6}, {0, 5, 3}, {0, 4, 4},
                                          {0, 4, 4}, {0, 3, 3}, {0, 1, 2}, {1, 1, 0}, {1, 3, 2}, {3, 4, 1}, {2, 0, 0},
                                          {2, 2, 2}, {1, 1, 1}, {2, 1, 0}, {2, 1, 1}, {1, 0, 1}, {1, 0, 1}, {0, 0, 0},
                                          {1, 0, 0}, {0, 0, 0}, {0, 1, 0}, {1, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0},
                                          {0, 0, 0}};

/* one antenna's dual extraction of one symbol into ext slots (literal pointer arithmetic); returns
 * the final pointer, *hw the slots written, *nb_rb the allocated RBs counted once */
static int extract_dual(const orc_frame_t *fp, const int32_t *rxF_sym, const int32_t *ch0_sym, const int32_t *ch1_sym,
                        const uint32_t rb_alloc[4], uint8_t symbol, uint8_t subframe, int32_t *rx_ext, int32_t *c0_ext,
                        int32_t *c1_ext, int *nb_rb, int *hw)
{
  const int symbol_mod = symbol >= 7 - fp->Ncp ? symbol - (7 - fp->Ncp) : symbol;
  const int pilots = symbol_mod == 0 || symbol_mod == 4 - fp->Ncp;
  const int nsymb = fp->Ncp == 0 ? 14 : 12, l = symbol, half = fp->N_RB_DL >> 1, ns = fp->nushift;
  const int sss_symb = fp->frame_type == 1 ? nsymb - 1 : (nsymb >> 1) - 2;
  const int pss_symb = fp->frame_type == 1 ? 2 : (nsymb >> 1) - 1;
  int p = 0;                                                   /* the ext pointer (slot index) */
  int drift = 0;                                               /* dl_ch0_ext - rxF_ext, in slots */
  enum { XS = 12 * 110 + 256 };
  uint8_t wr[XS];
  int colrx[XS], colc0[XS];
  memset(wr, 0, sizeof(wr));
  for (int i = 0; i < XS; i++) colrx[i] = colc0[i] = -1;
  *nb_rb = 0;
  *hw = 0;
  /* the port-0 estimate lands `drift` slots after the others (see the odd full-RB branch below);
   * writes past the caller's ext plane (the reference overruns dl_ch_estimates_ext there) are
   * dropped, and the slots they would leave stale are refused through *hw */
#define PUT(pos, bin, col)                                                              \
  do {                                                                                  \
    rx_ext[pos] = rxF_sym[bin];                                                         \
    if ((pos) + drift < 12 * 110 + 64) c0_ext[(pos) + drift] = ch0_sym[5 + (col)];      \
    if ((pos) + drift < XS) colc0[(pos) + drift] = (col);                               \
    c1_ext[pos] = ch1_sym[5 + (col)];                                                   \
    wr[pos] = 1;                                                                        \
    colrx[pos] = (col);                                                                 \
    if ((pos) + 1 > *hw) *hw = (pos) + 1;                                               \
  } while (0)
  for (int prb = 0; prb < fp->N_RB_DL; prb++) {
    int ind = alloc_bit(rb_alloc, prb), skip_half = 0;
    if (subframe == 0 && prb > half - 3 && prb < half + 3 && l >= (nsymb >> 1) && l < (nsymb >> 1) + 4) ind = 0;
    if ((subframe == 0 || subframe == 5) && prb > half - 3 && prb < half + 3 && l == sss_symb) ind = 0;
    if (fp->frame_type == 0 && (subframe == 0 || subframe == 5) && prb > half - 3 && prb < half + 3 && l == pss_symb) ind = 0;
    if (fp->frame_type == 1 && subframe == 6 && prb >= half - 3 && prb <= half + 3 && l == pss_symb) ind = 0;
    if (!ind) continue;
    const int col0 = 12 * prb;
    if ((fp->N_RB_DL & 1) == 0) {
      const int b0 = prb < half ? fp->first_carrier_offset + 12 * prb : 1 + 12 * (prb - half);
      if (!pilots) {
        for (int i = 0; i < 12; i++) PUT(p + i, b0 + i, col0 + i);
        p += 12;
      } else {
        int j = 0;
        for (int i = 0; i < 12; i++)
          if (i != ns && i != ns + 3 && i != ns + 6 && i != (ns + 9) % 12) { PUT(p + j, b0 + i, col0 + i); j++; }
        p += 8;
      }
      (*nb_rb)++;
      continue;
    }
    /* odd N_RB_DL */
    if (subframe == 0 && prb == half - 3 && l >= (nsymb >> 1) && l < (nsymb >> 1) + 4) skip_half = 1;
    else if (subframe == 0 && prb == half + 3 && l >= (nsymb >> 1) && l < (nsymb >> 1) + 4) skip_half = 2;
    if ((subframe == 0 || subframe == 5) && prb == half - 3 && l == sss_symb) skip_half = 1;
    else if ((subframe == 0 || subframe == 5) && prb == half + 3 && l == sss_symb) skip_half = 2;
    if ((fp->frame_type == 0 && (subframe == 0 || subframe == 5)) || (fp->frame_type == 1 && (subframe == 2 || subframe == 6))) {
      if (prb == half - 3 && l == pss_symb) skip_half = 1;
      else if ((subframe == 0 || subframe == 5) && prb == half + 3 && l == pss_symb) skip_half = 2;
    }
    const int b0 = prb <= half ? fp->first_carrier_offset + 12 * prb : 7 + 12 * (prb - half - 1);
    if (prb != half) {
      if (!pilots) {
        const int o = skip_half == 2 ? 6 : 0, n = skip_half ? 6 : 12;
        for (int i = 0; i < n; i++) PUT(p + i, b0 + o + i, col0 + o + i);
        p += n;
        /* skip_half == 0 (:3929-3936): `for (i=0;i<12;i++) dl_ch0_ext+=12;` — the loop body was a
         * printf, now commented out — then dl_ch1_ext += 12, rxF_ext += 12 */
        if (!skip_half) drift += 132;
      } else if (skip_half == 1) {
        int j = 0;
        for (int i = 0; i < 6; i++)
          if (i != ns && i != (ns + 3) % 6) { PUT(p + j, b0 + i, col0 + i); j++; }
        p += 4;
      } else if (skip_half == 2) {
        int j = 0;
        for (int i = 0; i < 6; i++) {
          if (i != ns && i != (ns + 3) % 6) { PUT(p + j, b0 + i + 6, col0 + i + 6); j++; }
          p += 4;                                            /* inside the loop, as written (:3961-3963) */
        }
      } else {
        int j = 0;
        for (int i = 0; i < 12; i++)
          if (i != ns && i != ns + 3 && i != ns + 6 && i != (ns + 9) % 12) { PUT(p + j, b0 + i, col0 + i); j++; }
        p += 8;
      }
    } else {                                                   /* the RB around DC */
      if (!pilots) {
        for (int i = 0; i < 6; i++) PUT(p + i, b0 + i, col0 + i);
        for (int i = 0; i < 6; i++) PUT(p + 6 + i, i, col0 + 6 + i);   /* bins 0..5 (:4003-4007) */
        p += 12;
      } else {
        int j = 0, i = 0;
        for (; i < 6; i++)
          if (i != ns && i != (ns + 3) % 6) { PUT(p + j, b0 + i, col0 + i); j++; }
        for (; i < 12; i++)
          if (i != (ns + 6) % 12 && i != (ns + 9) % 12) { PUT(p + j, 1 + i - 6, col0 + i); j++; }
        p += 8;
      }
    }
    (*nb_rb)++;
  }
#undef PUT
  /* *hw = the written prefix (the skip_half = 2 pilot branch leaves holes that the reference fills
   * from earlier symbols' ext data: a stream reaching one is refused) */
  int n = 0;
  while (n < *hw && wr[n] && colc0[n] == colrx[n]) n++;
  *hw = n;
  return p;
}

static int16_t sgn16(int16_t x, int s) { return s < 0 ? (int16_t)(uint16_t)(0u - (uint16_t)x) : x; }   /* sign_epi16 */

int orc_rx_pdsch_tm3(const orc_frame_t *fp, int nb_rx, const int32_t *const *rxdataF, const int32_t *const *est,
                     const uint32_t rb_alloc[4], uint8_t Qm0, uint8_t Qm1, uint8_t mcs0, uint8_t num_pdcch_symbols,
                     uint8_t subframe, int16_t *llr, uint8_t *log2_maxh_out)
{
  /* rxdataF[a] = [nsymb][N] of receive antenna a; est[p * 2 + a] = dl_ch_estimates[(p << 1) + a] */
  if (Qm0 == 2)   /* codeword 0 QPSK: the interference-aware qpsk_qpsk / qpsk_qam16 / qpsk_qam64 LLRs */
    return orc_rx_pdsch_tm3_q2(fp, nb_rx, rxdataF, est, rb_alloc, Qm1, mcs0, num_pdcch_symbols, subframe, llr,
                               NULL, log2_maxh_out);
  if (nb_rx < 1 || nb_rx > 2 || (Qm0 != 4 && Qm0 != 6) || (Qm1 != 2 && Qm1 != 4 && Qm1 != 6) || mcs0 > 28) return -1;
  const int N = fp->ofdm_symbol_size, nsymb = fp->Ncp == 0 ? 14 : 12;
  const size_t X = 12 * 110 + 64;
  int32_t *rx_ext = (int32_t *)calloc(2 * X, 4), *c0 = (int32_t *)calloc(2 * X, 4), *c1 = (int32_t *)calloc(2 * X, 4);
  int16_t *comp = (int16_t *)calloc(2 * X * 2, 2), *mag = (int16_t *)calloc(2 * X, 2), *magb = (int16_t *)calloc(2 * X, 2);
  int16_t *out = llr;
  uint8_t log2_maxh = 0;
  const int16_t a1 = Qm0 == 4 ? QAM16_n1 : QAM64_n1, a2 = Qm0 == 4 ? 0 : QAM64_n2;
  for (int symbol = num_pdcch_symbols; symbol < nsymb && out; symbol++) {
    int nb_rb = 0, hw[2] = {0, 0}, ptr[2] = {0, 0};
    for (int a = 0; a < nb_rx; a++)
      ptr[a] = extract_dual(fp, rxdataF[a] + symbol * N, est[a] + symbol * N, est[2 + a] + symbol * N, rb_alloc,
                            (uint8_t)symbol, subframe, rx_ext + a * X, c0 + a * X, c1 + a * X, &nb_rb, &hw[a]);
    (void)ptr;
    const int symbol_mod = symbol >= 7 - fp->Ncp ? symbol - (7 - fp->Ncp) : symbol;
    const int pil = symbol_mod == 0 || symbol_mod == 4 - fp->Ncp;
    const int nre_rb = pil ? 8 : 12;
    if (nb_rb == 0) { out = NULL; break; }
    if (symbol == num_pdcch_symbols) {
      /* dlsch_channel_level_TM3: symbol_mod == 0 only (the 4-Ncp test is written Ncp-1) takes 8 */
      const int nre = symbol_mod == 0 ? 8 : 12;
      if (hw[0] < nb_rb * nre) { out = NULL; break; }      /* would read unwritten ext slots */
      uint32_t lane[4] = {0, 0, 0, 0};
      int32_t avg[2] = {0, 0};
      for (int a = 0; a < nb_rx; a++) {
        for (int rb = 0; rb < nb_rb; rb++)
          for (int r = 0; r < (nre == 8 ? 2 : 3); r++)
            for (int k = 0; k < 4; k++) {
              const int e = rb * nre + 4 * r + k;            /* ext slot of this register lane */
              int16_t h0[2], h1[2];
              memcpy(h0, &c0[a * X + e], 4);
              memcpy(h1, &c1[a * X + e], 4);
              const int s = (k & 1) ? -1 : 1;
              int16_t p0[2];
              for (int c = 0; c < 2; c++) p0[c] = (int16_t)(sat16((int32_t)h0[c] + sgn16(h1[c], s)) >> 1);
              lane[k] += (uint32_t)((int32_t)p0[0] * p0[0]) + (uint32_t)((int32_t)p0[1] * p0[1]);
            }
        const int div = nb_rb * nre;
        avg[a] = (int32_t)lane[0] / div + (int32_t)lane[1] / div + (int32_t)lane[2] / div + (int32_t)lane[3] / div;
      }
      const int32_t avg0 = nb_rx > 1 ? (avg[0] > avg[1] ? avg[0] : avg[1]) : (avg[0] > 0 ? avg[0] : 0);  /* cmax(avg[0], avg[1]), avg[1] = 0 with 1 RX */
      const int v = (int)orc_log2_approx((uint32_t)avg0) - 13 + mumimo_off[mcs0][(Qm1 >> 1) - 1];
      log2_maxh = (uint8_t)(v > 0 ? v : 0);
    }
    /* precoding, magnitudes, matched filter per antenna (ext slots [0, nb_rb * nre_rb)) */
    const int n = nb_rb * nre_rb;
    for (int a = 0; a < nb_rx; a++)
      for (int e = 0; e < n; e++) {
        int16_t h0[2], h1[2], y[2];
        memcpy(h0, &c0[a * X + e], 4);
        memcpy(h1, &c1[a * X + e], 4);
        memcpy(y, &rx_ext[a * X + e], 4);
        const int s = (e & 1) ? -1 : 1;
        int16_t p0[2];
        for (int c = 0; c < 2; c++) p0[c] = (int16_t)(sat16((int32_t)h0[c] + sgn16(h1[c], s)) >> 1);
        const int16_t m = sat16((int32_t)((uint32_t)((int32_t)p0[0] * p0[0]) + (uint32_t)((int32_t)p0[1] * p0[1])) >> log2_maxh);
        mag[a * X + e] = mulhi2(m, a1);
        magb[a * X + e] = mulhi2(m, a2);
        const int16_t nhi = (int16_t)-p0[1];                 /* sign_epi16 by the conjugate mask */
        comp[(a * X + e) * 2] = sat16((int32_t)((uint32_t)((int32_t)p0[0] * y[0]) + (uint32_t)((int32_t)p0[1] * y[1])) >> log2_maxh);
        comp[(a * X + e) * 2 + 1] = sat16((int32_t)((uint32_t)((int32_t)nhi * y[0]) + (uint32_t)((int32_t)p0[0] * y[1])) >> log2_maxh);
      }
    if (nb_rx > 1)                                           /* dlsch_detection_mrc, stream 0 */
      for (int e = 0; e < n; e++) {
        for (int c = 0; c < 2; c++)
          comp[e * 2 + c] = sat16((comp[e * 2 + c] >> 1) + (comp[(X + e) * 2 + c] >> 1));
        mag[e] = sat16((mag[e] >> 1) + (mag[X + e] >> 1));
        magb[e] = sat16((magb[e] >> 1) + (magb[X + e] >> 1));
      }
    const int len = pil ? nb_rb * 8 - 2 * orc_adjust_G2(fp, rb_alloc, subframe, (uint8_t)symbol) / 3
                        : nb_rb * 12 - orc_adjust_G2(fp, rb_alloc, subframe, (uint8_t)symbol);
    if (len > hw[0]) { out = NULL; break; }
    for (int j = 0; j < len; j++) out += llr_qam_re(Qm0, comp[j * 2], comp[j * 2 + 1], mag[j], magb[j], out);
  }
  free(rx_ext);
  free(c0);
  free(c1);
  free(comp);
  free(mag);
  free(magb);
  if (!out) return -1;
  if (log2_maxh_out) *log2_maxh_out = log2_maxh;
  return (int)(out - llr);
}

/* qpsk_qpsk (dlsch_llr_computation.c:1041-1230) on one RE: the interference-aware max-log LLRs of a
 * QPSK stream y0 in presence of a QPSK stream y1 with correlation rho, all int16 saturating */
static void qq_llr(const int16_t y0[2], const int16_t y1[2], const int16_t rho[2], int16_t out[2])
{
  const int16_t rpi = (int16_t)(((int32_t)sat16((int32_t)rho[0] + rho[1]) * 23170) >> 16);   /* mulhi, 1/sqrt8 */
  const int16_t rmi = (int16_t)(((int32_t)sat16((int32_t)rho[0] - rho[1]) * 23170) >> 16);
  const int16_t y0r2 = (int16_t)(y0[0] >> 1), y0i2 = (int16_t)(y0[1] >> 1);
  const int16_t y1r2 = (int16_t)(y1[0] >> 1), y1i2 = (int16_t)(y1[1] >> 1);
#define S_(a, b) sat16((int32_t)(a) + (b))
#define D_(a, b) sat16((int32_t)(a) - (b))
#define M_(a, b) ((a) > (b) ? (a) : (b))
  const int16_t A = abs16(D_(y1r2, rpi)), B = abs16(D_(y1i2, rmi)), C = abs16(D_(y1r2, rmi)), D = abs16(S_(y1i2, rpi));
  const int16_t E = abs16(S_(y1r2, rmi)), F = abs16(D_(y1i2, rpi)), G = abs16(S_(y1r2, rpi)), H = abs16(S_(y1i2, rmi));
  const int16_t num_re = M_(S_(B, S_(A, y0i2)), S_(D_(C, y0i2), D));
  const int16_t den_re = M_(S_(F, S_(E, y0i2)), S_(D_(G, y0i2), H));
  const int16_t num_im = M_(S_(B, S_(A, y0r2)), S_(D_(E, y0r2), F));
  const int16_t den_im = M_(S_(D, S_(C, y0r2)), S_(D_(G, y0r2), H));
  out[0] = D_(S_(y0[0], num_re), den_re);
  out[1] = D_(S_(y0[1], num_im), den_im);
#undef S_
#undef D_
#undef M_
}

static int16_t mh16(int16_t a, int16_t b) { return (int16_t)(((int32_t)a * b) >> 16); }   /* mulhi_epi16 */
static int16_t shl16(int16_t a, int n) { return (int16_t)(uint16_t)((uint32_t)(uint16_t)a << n); }   /* slli_epi16 */

/* interference_abs_64qam_epi16 (dlsch_llr_computation.c:616): the amplitude of the 64-QAM
 * interferer closest to psi, from the masks (psi < 2m) ^ (psi < m), psi < m, (psi >= 2m) ^ (psi > 3m),
 * psi > 3m with m = mag >> 1, 2m = mag, 3m = m +sat mag; the masked constants are OR-ed */
static int16_t ia64(int16_t psi, int16_t mag)
{
  const int16_t c1x = (int16_t)(mag >> 1), c2x = mag, c3x = sat16((int32_t)c1x + c2x);
  const int lt2 = psi < c2x, lt1 = psi < c1x, gt3 = psi > c3x;
  const int t = lt2 ^ lt1, t3 = (!lt2) ^ gt3;
  return (int16_t)((t ? 10726 : 0) | (lt1 ? 3575 : 0) | (t3 ? 17876 : 0) | (gt3 ? 25027 : 0));
}

/* qpsk_qam16 (dlsch_llr_computation.c:1300-1514) / qpsk_qam64 (:1584-1814) on one RE: the LLRs of the
 * QPSK stream y0 in presence of a 16 / 64-QAM stream y1 of magnitude mag (dl_ch_mag1) and correlation
 * rho.  Kept as written: y0's mulhi by 1/sqrt2 is overwritten by y0 << 1 (:1397-1400); the 64-QAM
 * branch scales psi_a by mulhi(., 23170) << 2 (:1761-1768) and its a^2 by sqrt(42)/4 << 3 (:622) */
static void qx_llr(int qm1, const int16_t y0[2], const int16_t y1[2], int16_t mag, const int16_t rho[2], int16_t out[2])
{
  const int16_t rpi = shl16(mh16(sat16((int32_t)rho[0] + rho[1]), 23170), 1);
  const int16_t rmi = shl16(mh16(sat16((int32_t)rho[0] - rho[1]), 23170), 1);
  const int16_t y0r = shl16(y0[0], 1), y0i = shl16(y0[1], 1);
  const int16_t yp = sat16((int32_t)y0r + y0i), ym = sat16((int32_t)y0r - y0i);
  const int16_t y1r = y1[0], y1i = y1[1];
  /* psi (r, i) for the interferer hypotheses (+1 +1), (+1 -1), (-1 +1), (-1 -1) */
  const int16_t psi[8] = {abs16(sat16((int32_t)y1r - rpi)), abs16(sat16((int32_t)y1i - rmi)),
                          abs16(sat16((int32_t)y1r - rmi)), abs16(sat16((int32_t)y1i + rpi)),
                          abs16(sat16((int32_t)y1r + rmi)), abs16(sat16((int32_t)y1i - rpi)),
                          abs16(sat16((int32_t)y1r + rpi)), abs16(sat16((int32_t)y1i + rmi))};
  int16_t met[4];
  for (int h = 0; h < 4; h++) {
    int16_t a[2], sq[2];
    for (int c = 0; c < 2; c++) {
      const int16_t x = psi[2 * h + c];
      a[c] = qm1 == 4 ? (int16_t)(x < mag ? 10362 : 31086) : ia64(x, mag);   /* interference_abs_epi16 (:612) */
      const int16_t t = shl16(mh16(a[c], a[c]), 1);                          /* square_a(_64qam)_epi16 (:619, :622) */
      sq[c] = qm1 == 4 ? shl16(mh16(shl16(mh16(t, 25905), 1), mag), 1) : shl16(mh16(shl16(mh16(t, 13272), 3), mag), 1);
    }
    int16_t pa = sat16((int32_t)shl16(mh16(psi[2 * h], a[0]), 1) + shl16(mh16(psi[2 * h + 1], a[1]), 1));   /* prodsum (:609) */
    if (qm1 == 6) pa = shl16(mh16(pa, 23170), 2);
    const int16_t d = sat16((int32_t)pa - sat16((int32_t)sq[0] + sq[1]));
    met[h] = h == 0 ? sat16((int32_t)d + yp) : h == 1 ? sat16((int32_t)d + ym) : h == 2 ? sat16((int32_t)d - ym)
                                                                                          : sat16((int32_t)d - yp);
  }
#define M_(a, b) ((a) > (b) ? (a) : (b))
  out[0] = sat16((int32_t)M_(met[0], met[1]) - M_(met[2], met[3]));
  out[1] = sat16((int32_t)M_(met[0], met[2]) - M_(met[1], met[3]));
#undef M_
}

/* The per-RE LLR stages above over flat streams of len REs, for the reference pin
 * (tests/test_ref_pin_llr_cpu.py against dlsch_llr_computation.c compiled unmodified): comp / s0 / s1 /
 * rho are (re, im) int16 pairs; mag / magb / mag1 one int16 per RE, which the reference's packed
 * magnitudes carry in both halves. */
int orc_llr_qam(int Qm, const int16_t *comp, const int16_t *mag, const int16_t *magb, int len, int16_t *llr)
{
  int16_t *o = llr;
  for (int j = 0; j < len; j++) o += llr_qam_re(Qm, comp[2 * j], comp[2 * j + 1], mag ? mag[j] : 0, magb ? magb[j] : 0, o);
  return (int)(o - llr);
}

void orc_llr_qpsk_qpsk(const int16_t *s0, const int16_t *s1, const int16_t *rho, int len, int16_t *llr)
{
  for (int j = 0; j < len; j++) qq_llr(&s0[2 * j], &s1[2 * j], &rho[2 * j], &llr[2 * j]);
}

void orc_llr_qpsk_qamx(int qm1, const int16_t *s0, const int16_t *s1, const int16_t *mag1, const int16_t *rho, int len,
                       int16_t *llr)
{
  for (int j = 0; j < len; j++) qx_llr(qm1, &s0[2 * j], &s1[2 * j], mag1[j], &rho[2 * j], &llr[2 * j]);
}

/* rx_pdsch for TM3 with both codewords QPSK (dlsch_demodulation.c:373-413, 537-552, 643-669):
 * dlsch_channel_compensation_TM3 keeps both precoded channels h0' = (h0 +sat s h1) >> 1,
 * h1' = (h0 -sat s h1) >> 1 and both matched-filter outputs; dlsch_dual_stream_correlation gives
 * rho = conj(h0') h1' and rho2 = conj(h1') h0' (>> log2_maxh, packs); dlsch_detection_mrc averages
 * stream 0 and rho over the RX antennas (with dual_stream_flag 0 stream 1 and rho2 stay antenna 0's);
 * dlsch_qpsk_qpsk_llr then gives codeword 0 from (comp0, comp1, rho) and codeword 1 from (comp1,
 * comp0, rho2).  Writes both LLR streams (same length); returns it or -1. */
/* Codeword 0 QPSK, codeword 1 of modulation order Qm1: Qm1 = 2 is the QPSK-QPSK case above (both
 * codewords); Qm1 = 4 / 6 run dlsch_qpsk_16qam_llr / dlsch_qpsk_64qam_llr (:670-690) for codeword 0
 * only, with dl_ch_mag1 = |h1'|^2 >> log2_maxh (packs) times QAM16_n1 / QAM64_n1 (mulhi << 1) of
 * antenna 0 (the MRC leaves it alone with dual_stream_flag 0); llr1 is not written. */
int orc_rx_pdsch_tm3_q2(const orc_frame_t *fp, int nb_rx, const int32_t *const *rxdataF, const int32_t *const *est,
                        const uint32_t rb_alloc[4], uint8_t Qm1, uint8_t mcs0, uint8_t num_pdcch_symbols,
                        uint8_t subframe, int16_t *llr0, int16_t *llr1, uint8_t *log2_maxh_out)
{
  if (nb_rx < 1 || nb_rx > 2 || mcs0 > 28 || (Qm1 != 2 && Qm1 != 4 && Qm1 != 6)) return -1;
  const int N = fp->ofdm_symbol_size, nsymb = fp->Ncp == 0 ? 14 : 12;
  const size_t X = 12 * 110 + 64;
  int32_t *rx_ext = (int32_t *)calloc(2 * X, 4), *c0 = (int32_t *)calloc(2 * X, 4), *c1 = (int32_t *)calloc(2 * X, 4);
  int16_t *cp0 = (int16_t *)calloc(2 * X * 2, 2), *cp1 = (int16_t *)calloc(2 * X * 2, 2);
  int16_t *rho = (int16_t *)calloc(2 * X * 2, 2), *rho2 = (int16_t *)calloc(2 * X * 2, 2);
  int16_t *mag1 = (int16_t *)calloc(2 * X, 2);
  const int16_t a1 = Qm1 == 4 ? QAM16_n1 : QAM64_n1;
  int16_t *o0 = llr0, *o1 = llr1;
  int ok = 1;
  uint8_t log2_maxh = 0;
  for (int symbol = num_pdcch_symbols; symbol < nsymb && ok; symbol++) {
    int nb_rb = 0, hw[2] = {0, 0};
    for (int a = 0; a < nb_rx; a++)
      (void)extract_dual(fp, rxdataF[a] + symbol * N, est[a] + symbol * N, est[2 + a] + symbol * N, rb_alloc,
                         (uint8_t)symbol, subframe, rx_ext + a * X, c0 + a * X, c1 + a * X, &nb_rb, &hw[a]);
    const int symbol_mod = symbol >= 7 - fp->Ncp ? symbol - (7 - fp->Ncp) : symbol;
    const int pil = symbol_mod == 0 || symbol_mod == 4 - fp->Ncp;
    if (nb_rb == 0) { ok = 0; break; }
    if (symbol == num_pdcch_symbols) {              /* dlsch_channel_level_TM3, as orc_rx_pdsch_tm3 */
      const int nre = symbol_mod == 0 ? 8 : 12;
      if (hw[0] < nb_rb * nre) { ok = 0; break; }
      uint32_t lane[4] = {0, 0, 0, 0};
      int32_t avg[2] = {0, 0};
      for (int a = 0; a < nb_rx; a++) {
        for (int rb = 0; rb < nb_rb; rb++)
          for (int r = 0; r < (nre == 8 ? 2 : 3); r++)
            for (int k = 0; k < 4; k++) {
              const int e = rb * nre + 4 * r + k;
              int16_t h0[2], h1[2];
              memcpy(h0, &c0[a * X + e], 4);
              memcpy(h1, &c1[a * X + e], 4);
              const int s = (k & 1) ? -1 : 1;
              int16_t p0[2];
              for (int c = 0; c < 2; c++) p0[c] = (int16_t)(sat16((int32_t)h0[c] + sgn16(h1[c], s)) >> 1);
              lane[k] += (uint32_t)((int32_t)p0[0] * p0[0]) + (uint32_t)((int32_t)p0[1] * p0[1]);
            }
        const int div = nb_rb * nre;
        avg[a] = (int32_t)lane[0] / div + (int32_t)lane[1] / div + (int32_t)lane[2] / div + (int32_t)lane[3] / div;
      }
      const int32_t avg0 = nb_rx > 1 ? (avg[0] > avg[1] ? avg[0] : avg[1]) : (avg[0] > 0 ? avg[0] : 0);
      const int v = (int)orc_log2_approx((uint32_t)avg0) - 13 + mumimo_off[mcs0][(Qm1 >> 1) - 1];
      log2_maxh = (uint8_t)(v > 0 ? v : 0);
    }
    const int n = nb_rb * (pil ? 8 : 12);
    for (int a = 0; a < nb_rx; a++)
      for (int e = 0; e < n; e++) {
        int16_t h0[2], h1[2], y[2], p0[2], p1[2];
        memcpy(h0, &c0[a * X + e], 4);
        memcpy(h1, &c1[a * X + e], 4);
        memcpy(y, &rx_ext[a * X + e], 4);
        const int s = (e & 1) ? -1 : 1;
        for (int c = 0; c < 2; c++) {
          const int16_t t = sgn16(h1[c], s);
          p0[c] = (int16_t)(sat16((int32_t)h0[c] + t) >> 1);
          p1[c] = (int16_t)(sat16((int32_t)h0[c] - t) >> 1);
        }
        const size_t o = (a * X + e) * 2;
        const int16_t n0 = (int16_t)-p0[1], n1 = (int16_t)-p1[1];        /* sign_epi16 by the conjugate mask */
        cp0[o] = sat16((int32_t)((uint32_t)((int32_t)p0[0] * y[0]) + (uint32_t)((int32_t)p0[1] * y[1])) >> log2_maxh);
        cp0[o + 1] = sat16((int32_t)((uint32_t)((int32_t)n0 * y[0]) + (uint32_t)((int32_t)p0[0] * y[1])) >> log2_maxh);
        cp1[o] = sat16((int32_t)((uint32_t)((int32_t)p1[0] * y[0]) + (uint32_t)((int32_t)p1[1] * y[1])) >> log2_maxh);
        cp1[o + 1] = sat16((int32_t)((uint32_t)((int32_t)n1 * y[0]) + (uint32_t)((int32_t)p1[0] * y[1])) >> log2_maxh);
        rho[o] = sat16((int32_t)((uint32_t)((int32_t)p0[0] * p1[0]) + (uint32_t)((int32_t)p0[1] * p1[1])) >> log2_maxh);
        rho[o + 1] = sat16((int32_t)((uint32_t)((int32_t)n0 * p1[0]) + (uint32_t)((int32_t)p0[0] * p1[1])) >> log2_maxh);
        rho2[o] = sat16((int32_t)((uint32_t)((int32_t)p1[0] * p0[0]) + (uint32_t)((int32_t)p1[1] * p0[1])) >> log2_maxh);
        rho2[o + 1] = sat16((int32_t)((uint32_t)((int32_t)n1 * p0[0]) + (uint32_t)((int32_t)p1[0] * p0[1])) >> log2_maxh);
        const int16_t m1 = sat16((int32_t)((uint32_t)((int32_t)p1[0] * p1[0]) + (uint32_t)((int32_t)p1[1] * p1[1])) >> log2_maxh);
        mag1[a * X + e] = mulhi2(m1, a1);
      }
    if (nb_rx > 1)                                  /* dlsch_detection_mrc: stream 0 and rho only */
      for (int e = 0; e < n; e++)
        for (int c = 0; c < 2; c++) {
          cp0[e * 2 + c] = sat16((cp0[e * 2 + c] >> 1) + (cp0[(X + e) * 2 + c] >> 1));
          rho[e * 2 + c] = sat16((rho[e * 2 + c] >> 1) + (rho[(X + e) * 2 + c] >> 1));
        }
    const int len = pil ? nb_rb * 8 - 2 * orc_adjust_G2(fp, rb_alloc, subframe, (uint8_t)symbol) / 3
                        : nb_rb * 12 - orc_adjust_G2(fp, rb_alloc, subframe, (uint8_t)symbol);
    if (len > hw[0]) { ok = 0; break; }
    for (int j = 0; j < len; j++) {
      if (Qm1 == 2) {
        qq_llr(&cp0[2 * j], &cp1[2 * j], &rho[2 * j], o0);
        if (o1) { qq_llr(&cp1[2 * j], &cp0[2 * j], &rho2[2 * j], o1); o1 += 2; }
      } else {
        qx_llr(Qm1, &cp0[2 * j], &cp1[2 * j], mag1[j], &rho[2 * j], o0);
      }
      o0 += 2;
    }
  }
  free(rx_ext); free(c0); free(c1); free(cp0); free(cp1); free(rho); free(rho2); free(mag1);
  if (!ok) return -1;
  if (log2_maxh_out) *log2_maxh_out = log2_maxh;
  return (int)(o0 - llr0);
}

int orc_rx_pdsch_tm3_qq(const orc_frame_t *fp, int nb_rx, const int32_t *const *rxdataF, const int32_t *const *est,
                        const uint32_t rb_alloc[4], uint8_t mcs0, uint8_t num_pdcch_symbols, uint8_t subframe,
                        int16_t *llr0, int16_t *llr1, uint8_t *log2_maxh_out)
{
  if (!llr1) return -1;
  return orc_rx_pdsch_tm3_q2(fp, nb_rx, rxdataF, est, rb_alloc, 2, mcs0, num_pdcch_symbols, subframe, llr0, llr1,
                             log2_maxh_out);
}

/* rx_pdsch for TM2 (ALAMOUTI, two TX ports) with dlsim's UE (dual_stream_flag 0,
 * dlsch_demodulation.c:82-800):
 *   dlsch_extract_rbs_dual      as for TM3 (extract_dual above)
 *   dlsch_channel_level         :2777-2838: per (port, RX antenna) the int32 sum of |h|^2 over the
 *                               first PDSCH symbol's nb_rb RBs (8 REs per RB where symbol_mod == 0,
 *                               its 4-Ncp test is written Ncp-1, else 12), divided by nb_rb nre;
 *                               log2_maxh = log2_approx(max(0, max avg)) / 2 (:276-285)
 *   dlsch_channel_compensation  :801-980 per (port, RX antenna): conj(h) y >> log2_maxh (madd, packs),
 *                               |h|^2 >> log2_maxh (packs) times QAM16_n1 / QAM64_n1 / QAM64_n2
 *                               (mulhi << 1); rho (:982-) only feeds the dual-stream LLRs
 *   dlsch_detection_mrc         :2583-2621 per port: (a >> 1) +sat (b >> 1), also the magnitudes
 *   dlsch_alamouti              :3067-3160 pairs of consecutive extracted REs (2k, 2k + 1):
 *                               y0 += conj-pair of port 1 (int16 wrap: C short arithmetic),
 *                               magnitudes (m0 +sat m1) >> 1, the combined symbol mulhi(., 1/sqrt2) << 1
 *   dlsch_qpsk / 16qam / 64qam_llr of the combined stream (mode1_flag 0 lengths)
 * rxdataF[a] = [nsymb][N]; est[p * 2 + a] = dl_ch_estimates[(p << 1) + a]. */
int orc_rx_pdsch_tm2(const orc_frame_t *fp, int nb_rx, const int32_t *const *rxdataF, const int32_t *const *est,
                     const uint32_t rb_alloc[4], uint8_t Qm, uint8_t num_pdcch_symbols, uint8_t subframe,
                     int16_t *llr, uint8_t *log2_maxh_out)
{
  if (nb_rx < 1 || nb_rx > 2 || (Qm != 2 && Qm != 4 && Qm != 6)) return -1;
  const int N = fp->ofdm_symbol_size, nsymb = fp->Ncp == 0 ? 14 : 12;
  const size_t X = 12 * 110 + 64;
  int32_t *rx_ext = (int32_t *)calloc(2 * X, 4), *hx = (int32_t *)calloc(4 * X, 4);   /* hx[(p * 2 + a) X + e] */
  int16_t *comp = (int16_t *)calloc(4 * X * 2, 2), *mag = (int16_t *)calloc(4 * X, 2), *magb = (int16_t *)calloc(4 * X, 2);
  int16_t *out = llr;
  uint8_t log2_maxh = 0;
  const int16_t a1 = Qm == 4 ? QAM16_n1 : (Qm == 6 ? QAM64_n1 : 0), a2 = Qm == 6 ? QAM64_n2 : 0;
  for (int symbol = num_pdcch_symbols; symbol < nsymb && out; symbol++) {
    int nb_rb = 0, hw[2] = {0, 0};
    for (int a = 0; a < nb_rx; a++)
      (void)extract_dual(fp, rxdataF[a] + symbol * N, est[a] + symbol * N, est[2 + a] + symbol * N, rb_alloc,
                         (uint8_t)symbol, subframe, rx_ext + a * X, hx + a * X, hx + (2 + a) * X, &nb_rb, &hw[a]);
    const int symbol_mod = symbol >= 7 - fp->Ncp ? symbol - (7 - fp->Ncp) : symbol;
    const int pil = symbol_mod == 0 || symbol_mod == 4 - fp->Ncp;
    const int nre_rb = pil ? 8 : 12;
    if (nb_rb == 0) { out = NULL; break; }
    if (symbol == num_pdcch_symbols) {
      const int nre = symbol_mod == 0 ? 8 : 12;
      if (hw[0] < nb_rb * nre) { out = NULL; break; }      /* would read unwritten ext slots */
      int32_t avgs = 0;
      for (int pa = 0; pa < 4; pa++) {
        if ((pa & 1) >= nb_rx) continue;
        uint32_t tot = 0;
        for (int e = 0; e < nb_rb * nre; e++) {
          int16_t h[2];
          memcpy(h, &hx[pa * X + e], 4);
          tot += (uint32_t)((int32_t)h[0] * h[0]) + (uint32_t)((int32_t)h[1] * h[1]);
        }
        const int32_t avg = (int32_t)tot / (nb_rb * nre);
        avgs = avg > avgs ? avg : avgs;                     /* cmax, starting from 0 */
      }
      log2_maxh = (uint8_t)(orc_log2_approx((uint32_t)avgs) / 2);
    }
    const int n = nb_rb * nre_rb;
    if (n > hw[0]) { out = NULL; break; }
    for (int pa = 0; pa < 4; pa++) {                        /* compensation per (port, RX antenna) */
      const int a = pa & 1;
      if (a >= nb_rx) continue;
      for (int e = 0; e < n; e++) {
        int16_t h[2], y[2];
        memcpy(h, &hx[pa * X + e], 4);
        memcpy(y, &rx_ext[a * X + e], 4);
        const int16_t m = sat16((int32_t)((uint32_t)((int32_t)h[0] * h[0]) + (uint32_t)((int32_t)h[1] * h[1])) >> log2_maxh);
        mag[pa * X + e] = mulhi2(m, a1);
        magb[pa * X + e] = mulhi2(m, a2);
        const int16_t nhi = (int16_t)-h[1];
        comp[(pa * X + e) * 2] = sat16((int32_t)((uint32_t)((int32_t)h[0] * y[0]) + (uint32_t)((int32_t)h[1] * y[1])) >> log2_maxh);
        comp[(pa * X + e) * 2 + 1] = sat16((int32_t)((uint32_t)((int32_t)nhi * y[0]) + (uint32_t)((int32_t)h[0] * y[1])) >> log2_maxh);
      }
    }
    if (nb_rx > 1)                                           /* dlsch_detection_mrc, per port */
      for (int p = 0; p < 2; p++) {
        const size_t o0 = (size_t)(2 * p) * X, o1 = o0 + X;
        for (int e = 0; e < n; e++) {
          for (int c = 0; c < 2; c++)
            comp[(o0 + e) * 2 + c] = sat16((comp[(o0 + e) * 2 + c] >> 1) + (comp[(o1 + e) * 2 + c] >> 1));
          mag[o0 + e] = sat16((mag[o0 + e] >> 1) + (mag[o1 + e] >> 1));
          magb[o0 + e] = sat16((magb[o0 + e] >> 1) + (magb[o1 + e] >> 1));
        }
      }
    /* dlsch_alamouti: rxF0 = port 0 (slot 0), rxF1 = port 1 (slot 2) */
    int16_t *c0 = comp, *c1 = comp + 2 * 2 * X;
    for (int e = 0; e + 1 < n; e += 2) {
      c0[2 * e] = (int16_t)(c0[2 * e] + c1[2 * e + 2]);
      c0[2 * e + 1] = (int16_t)(c0[2 * e + 1] - c1[2 * e + 3]);
      c0[2 * e + 2] = (int16_t)(c0[2 * e + 2] - c1[2 * e]);
      c0[2 * e + 3] = (int16_t)(c0[2 * e + 3] + c1[2 * e + 1]);
    }
    for (int e = 0; e < n; e++) {
      mag[e] = (int16_t)(sat16((int32_t)mag[e] + mag[2 * X + e]) >> 1);
      magb[e] = (int16_t)(sat16((int32_t)magb[e] + magb[2 * X + e]) >> 1);
      for (int c = 0; c < 2; c++) c0[2 * e + c] = (int16_t)(mulhi2(c0[2 * e + c], 23170));
    }
    const int adj = Qm == 2 ? 0 : orc_adjust_G2(fp, rb_alloc, subframe, (uint8_t)symbol);
    const int len = pil ? nb_rb * 8 - 2 * adj / 3 : nb_rb * 12 - adj;
    if (((len + 1) & ~1) > hw[0]) { out = NULL; break; }
    for (int j = 0; j < len; j++) out += llr_qam_re(Qm, c0[2 * j], c0[2 * j + 1], mag[j], magb[j], out);
  }
  free(rx_ext);
  free(hx);
  free(comp);
  free(mag);
  free(magb);
  if (!out) return -1;
  if (log2_maxh_out) *log2_maxh_out = log2_maxh;
  return (int)(out - llr);
}
