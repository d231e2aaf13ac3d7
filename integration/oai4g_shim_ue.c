/* oai4g_shim_ue.c — reference-side bindings that take PHY_VARS_UE / PHY_VARS_eNB.
 * Replaces: slot_fep.c:40 slot_fep, pilots.c:43 generate_pilots, lte_dl_channel_estimation.c:37,
 * dlsch_demodulation.c:82 rx_pdsch (TM1/TM2/TM3).
 * PHY_VARS_UE / PHY_VARS_eNB are defined in PHY/defs.h, whose include chain needs the asn1c-generated
 * RRC headers (PHY/INIT/defs.h:35-42), so this file compiles only inside a full reference build
 * (cmake_targets), next to oai4g_shim.c. */
#include "PHY/defs.h"
#include "PHY/extern.h"
#include "oai4g.h"
#include "oai4g_shim_fp.h"

int slot_fep(PHY_VARS_UE *ue, unsigned char l, unsigned char Ns, int sample_offset, int no_prefix,
             int reset_freq_est)
{
  oai4g_frame_parms_t fp;
  fp_to(&ue->lte_frame_parms, &fp);
  /* CP removal + DFT on the GPU (rxdata keeps its frame + ofdm_symbol_size wrap extension, as
   * allocated by lte_init.c) */
  int ret = oai4g_slot_fep((int32_t **)ue->lte_ue_common_vars.rxdata, (int32_t **)ue->lte_ue_common_vars.rxdataF,
                           &fp, ue->lte_frame_parms.nb_antennas_rx, l, Ns, sample_offset, no_prefix);
  if (ret != 0) return ret;
  /* channel estimation and the frequency-offset estimator (slot_fep.c:179-222): the GPU bindings
   * lte_dl_channel_estimation / lte_est_freq_offset below */
  if (ue->perfect_ce == 0 && (l == 0 || l == 4 - ue->lte_frame_parms.Ncp)) {
    const unsigned char symbol = l + (7 - ue->lte_frame_parms.Ncp) * (Ns & 1);
    for (int aa = 0; aa < ue->lte_frame_parms.nb_antennas_tx_eNB; aa++) {
      lte_dl_channel_estimation(ue, 0, 0, Ns, aa, l, symbol);
      for (int i = 0; i < ue->PHY_measurements.n_adj_cells; i++)
        lte_dl_channel_estimation(ue, 0, i + 1, Ns, aa, l, symbol);
    }
    if (l == 4 - ue->lte_frame_parms.Ncp)
      lte_est_freq_offset(ue->lte_ue_common_vars.dl_ch_estimates[0], &ue->lte_frame_parms, l,
                          &ue->lte_ue_common_vars.freq_offset, reset_freq_est);
  }
  return 0;
}

/* cell-specific reference signals: pilots.c:43 (all antennas of the eNB, N subframes) */
void generate_pilots(PHY_VARS_eNB *phy_vars_eNB, mod_sym_t **txdataF, int16_t amp, uint16_t N)
{
  oai4g_frame_parms_t fp;
  fp_to(&phy_vars_eNB->lte_frame_parms, &fp);
  oai4g_generate_pilots((int32_t **)txdataF, amp, &fp, N);
}

/* UE receive chain after the FFT.
 * lte_dl_channel_estimation (lte_dl_channel_estimation.c:37): the library covers eNB_offset 0 and
 * high_speed_flag 1 (dlsim's and lte_init's default); like the reference it estimates every
 * receive antenna (1 or 2) into dl_ch_estimates[eNB_offset][(p << 1) + aarx].  Anything else
 * reports -1 as the reference does for its unsupported (p, l) cases. */
int lte_dl_channel_estimation(PHY_VARS_UE *ue, uint8_t eNB_id, uint8_t eNB_offset, unsigned char Ns, unsigned char p,
                              unsigned char l, unsigned char symbol)
{
  (void)eNB_id;
  const int nrx = ue->lte_frame_parms.nb_antennas_rx;
  if (eNB_offset != 0 || ue->high_speed_flag != 1 || nrx < 1 || nrx > 2) return -1;
  oai4g_frame_parms_t fp;
  fp_to(&ue->lte_frame_parms, &fp);
  for (int a = 0; a < nrx; a++)
    if (oai4g_lte_dl_channel_estimation(&fp, (const int32_t *)ue->lte_ue_common_vars.rxdataF[a],
                                        (int32_t *)ue->lte_ue_common_vars.dl_ch_estimates[0][(p << 1) + a], Ns, p, l,
                                        symbol) != 0)
      return -1;
  /* :704-738: the idft of every (port, RX antenna) plane into dl_ch_estimates_time */
  return oai4g_dl_ch_estimates_time(&fp, nrx, (const int32_t *const *)ue->lte_ue_common_vars.dl_ch_estimates[0],
                                    (int32_t *const *)ue->lte_ue_common_vars.dl_ch_estimates_time[0]);
}

/* rx_pdsch (dlsch_demodulation.c:82) for TM1 (one TX port, one RX antenna), TM2 (ALAMOUTI) and TM3
 * (LARGE_CDD; both two TX ports, 1-2 RX antennas, dual_stream_flag 0), localized allocations (rb_alloc_even ==
 * rb_alloc_odd).  CONTRACT: the library demodulates a whole subframe, so the shim accepts dlsim's
 * call sequence only (dlsim.c:3236-3260): first_symbol_flag on symbol num_pdcch_symbols, then
 * every following symbol in order; the work runs at the last symbol, when the LLR stream and
 * log2_maxh in lte_ue_pdsch_vars[eNB_id] become the reference's.  The per-symbol intermediates
 * (rxdataF_comp, dl_ch_mag / magb) are NOT filled.  A call out of that sequence returns -1
 * (state per thread, so concurrent UE threads each keep their own sequence). */
static __thread int rx_next_symbol = -1;

int rx_pdsch(PHY_VARS_UE *ue, PDSCH_t type, unsigned char eNB_id, unsigned char eNB_id_i, uint8_t subframe,
             unsigned char symbol, unsigned char first_symbol_flag, unsigned char dual_stream_flag,
             unsigned char i_mod, unsigned char harq_pid)
{
  (void)eNB_id_i;
  (void)i_mod;
  const LTE_DL_FRAME_PARMS *f = &ue->lte_frame_parms;
  LTE_DL_UE_HARQ_t *h = ue->dlsch_ue[eNB_id][0]->harq_processes[harq_pid];
  const int tm3 = f->nb_antennas_tx_eNB == 2 && h->mimo_mode == LARGE_CDD;
  const int tm2 = f->nb_antennas_tx_eNB == 2 && h->mimo_mode == ALAMOUTI;
  if (type != PDSCH || dual_stream_flag || memcmp(h->rb_alloc_even, h->rb_alloc_odd, 16) != 0 ||
      (!tm3 && !tm2 && (f->nb_antennas_rx != 1 || f->nb_antennas_tx_eNB != 1)) ||
      ((tm3 || tm2) && f->nb_antennas_rx > 2))
    return -1;
  const int npdcch = ue->lte_ue_pdcch_vars[eNB_id]->num_pdcch_symbols;
  if (first_symbol_flag) {
    if (symbol != npdcch) { rx_next_symbol = -1; return -1; }
  } else if (symbol != rx_next_symbol) {
    rx_next_symbol = -1;
    return -1;
  }
  rx_next_symbol = symbol + 1;
  if (symbol != f->symbols_per_tti - 1) return 0;
  rx_next_symbol = -1;
  oai4g_frame_parms_t fp;
  fp_to(f, &fp);
  uint8_t log2_maxh = 0;
  int n;
  if (tm3 || tm2) {
    const int32_t *rxF[2], *est[4];
    for (int a = 0; a < f->nb_antennas_rx; a++) {
      rxF[a] = (const int32_t *)ue->lte_ue_common_vars.rxdataF[a];
      est[a] = (const int32_t *)ue->lte_ue_common_vars.dl_ch_estimates[eNB_id][a];
      est[2 + a] = (const int32_t *)ue->lte_ue_common_vars.dl_ch_estimates[eNB_id][2 + a];
    }
    if (tm2) {
      n = oai4g_rx_pdsch_tm2(&fp, f->nb_antennas_rx, rxF, est, h->rb_alloc_even, h->Qm, npdcch, subframe,
                             ue->lte_ue_pdsch_vars[eNB_id]->llr[0], &log2_maxh);
    } else {
      LTE_DL_UE_HARQ_t *h1 = ue->dlsch_ue[eNB_id][1]->harq_processes[harq_pid];
      if (h->Qm == 2 && h1->Qm == 2)   /* both QPSK: dlsch_qpsk_qpsk_llr fills llr[0] and llr[1] */
        n = oai4g_rx_pdsch_tm3_2cw(&fp, f->nb_antennas_rx, rxF, est, h->rb_alloc_even, h->mcs, npdcch, subframe,
                                   ue->lte_ue_pdsch_vars[eNB_id]->llr[0], ue->lte_ue_pdsch_vars[eNB_id]->llr[1],
                                   &log2_maxh);
      else
        n = oai4g_rx_pdsch_tm3(&fp, f->nb_antennas_rx, rxF, est, h->rb_alloc_even, h->Qm, h1->Qm,
                               h->mcs, npdcch, subframe, ue->lte_ue_pdsch_vars[eNB_id]->llr[0], &log2_maxh);
    }
  } else {
    n = oai4g_rx_pdsch_siso(&fp, (const int32_t *)ue->lte_ue_common_vars.rxdataF[0],
                            (const int32_t *)ue->lte_ue_common_vars.dl_ch_estimates[eNB_id][0], h->rb_alloc_even,
                            h->Qm, npdcch, subframe, ue->lte_ue_pdsch_vars[eNB_id]->llr[0], &log2_maxh);
  }
  if (n < 0) return -1;
  ue->lte_ue_pdsch_vars[eNB_id]->log2_maxh = log2_maxh;
  return 0;
}
