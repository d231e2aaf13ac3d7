/* oai4g_shim.c — reference-side binding of the MI355X DLSCH transmit path.
 * Replaces: dlsch_coding.c:254 dlsch_encoding, dlsch_scrambling.c:51, dlsch_modulation.c:1181,
 * ofdm_mod.c:47/85/233, lte_dfts.c idft64..idft2048, crc_byte.c:117/135, lte_segmentation.c:39,
 * 3gpplte_sse.c:380, lte_rate_matching.c:51/464, pcfich.c:48/144, dci.c:2024, pss.c:50, sss.c:47,
 * pbch.c:161, phich.c:401, lte_dl_channel_estimation.c:37, dlsch_demodulation.c:82 (rx_pdsch, TM1/TM2/TM3),
 * dlsch_scrambling.c:99 (dlsch_unscrambling), 3gpplte_turbo_decoder_sse_16bit.c:945 / _8bit.c:894,
 * lte_rate_matching.c:193 / :293 / :688 (the UL decoding chain). */
#include "PHY/defs.h"
#include "PHY/extern.h"
#include "oai4g.h"

static void fp_to(const LTE_DL_FRAME_PARMS *f, oai4g_frame_parms_t *o)
{
  memset(o, 0, sizeof(*o));
  o->N_RB_DL = f->N_RB_DL;            o->Nid_cell = f->Nid_cell;
  o->Ncp = f->Ncp;                    o->nushift = f->nushift;
  o->mode1_flag = f->mode1_flag;      o->nb_antennas_tx = f->nb_antennas_tx;
  o->frame_type = f->frame_type;      o->symbols_per_tti = f->symbols_per_tti;
  o->log2_symbol_size = f->log2_symbol_size;
  o->ofdm_symbol_size = f->ofdm_symbol_size;
  o->first_carrier_offset = f->first_carrier_offset;
  o->nb_prefix_samples = f->nb_prefix_samples;
  o->nb_prefix_samples0 = f->nb_prefix_samples0;
  o->samples_per_tti = f->samples_per_tti;
  o->phich_resource = f->phich_config_common.phich_resource;
  o->phich_duration = f->phich_config_common.phich_duration;
  o->tdd_config = f->tdd_config;      o->nb_antennas_tx_eNB = f->nb_antennas_tx_eNB;
  o->Nid_cell_mbsfn = (uint8_t)f->Nid_cell_mbsfn;   /* 0..255 (36.211 N_ID^MBSFN) */
}

/* The mirror points INTO the reference's own HARQ buffers, so every write lands in place. */
typedef struct { oai4g_dlsch_t d; oai4g_dl_harq_t h[8]; } shim_dlsch_t;

static void harq_to(LTE_DL_eNB_HARQ_t *r, oai4g_dl_harq_t *o)
{
  int i;
  o->TBS = r->TBS;  o->B = r->B;  o->b = r->b;
  for (i = 0; i < MAX_NUM_DLSCH_SEGMENTS; i++) {
    o->c[i] = r->c[i];  o->d[i] = r->d[i];  o->w[i] = r->w[i];  o->RTC[i] = r->RTC[i];
  }
  o->round = r->round;  o->mcs = r->mcs;  o->rvidx = r->rvidx;  o->mimo_mode = r->mimo_mode;
  memcpy(o->rb_alloc, r->rb_alloc, sizeof(o->rb_alloc));
  o->nb_rb = r->nb_rb;  o->e = r->e;
  o->C = r->C;  o->Cminus = r->Cminus;  o->Cplus = r->Cplus;
  o->Kminus = r->Kminus;  o->Kplus = r->Kplus;  o->F = r->F;
  o->Nl = r->Nl;  o->Nlayers = r->Nlayers;  o->first_layer = r->first_layer;
}

static void harq_from(const oai4g_dl_harq_t *o, LTE_DL_eNB_HARQ_t *r)
{
  int i;   /* scalar outputs of segmentation / sub-block interleaving */
  r->B = o->B;  r->C = o->C;  r->Cminus = o->Cminus;  r->Cplus = o->Cplus;
  r->Kminus = o->Kminus;  r->Kplus = o->Kplus;  r->F = o->F;
  for (i = 0; i < MAX_NUM_DLSCH_SEGMENTS; i++) r->RTC[i] = o->RTC[i];
}

static oai4g_dlsch_t *dlsch_to(LTE_eNB_DLSCH_t *r, shim_dlsch_t *s)
{
  int i;
  if (!r) return NULL;
  s->d.rnti = r->rnti;  s->d.current_harq_pid = r->current_harq_pid;
  s->d.Mdlharq = r->Mdlharq;  s->d.Kmimo = r->Kmimo;
  s->d.sqrt_rho_a = r->sqrt_rho_a;  s->d.sqrt_rho_b = r->sqrt_rho_b;
  for (i = 0; i < 8; i++) {
    s->d.harq_processes[i] = r->harq_processes[i] ? &s->h[i] : NULL;
    if (r->harq_processes[i]) harq_to(r->harq_processes[i], &s->h[i]);
  }
  return &s->d;
}

int32_t dlsch_encoding(uint8_t *a, LTE_DL_FRAME_PARMS *frame_parms, uint8_t num_pdcch_symbols,
                       LTE_eNB_DLSCH_t *dlsch, int frame, uint8_t subframe,
                       time_stats_t *rm_stats, time_stats_t *te_stats, time_stats_t *i_stats)
{
  oai4g_frame_parms_t fp;  shim_dlsch_t s;  int ret;
  fp_to(frame_parms, &fp);
  ret = oai4g_dlsch_encoding(a, &fp, num_pdcch_symbols, dlsch_to(dlsch, &s), frame, subframe);
  harq_from(&s.h[dlsch->current_harq_pid], dlsch->harq_processes[dlsch->current_harq_pid]);
  return ret;                          /* 0, or -1 like the reference (dlsch_coding.c:316,336) */
}

void dlsch_scrambling(LTE_DL_FRAME_PARMS *frame_parms, int mbsfn_flag, LTE_eNB_DLSCH_t *dlsch,
                      int G, uint8_t q, uint8_t Ns)
{
  oai4g_frame_parms_t fp;  shim_dlsch_t s;
  fp_to(frame_parms, &fp);
  oai4g_dlsch_scrambling(&fp, mbsfn_flag, dlsch_to(dlsch, &s), G, q, Ns);
}

int32_t dlsch_modulation(mod_sym_t **txdataF, int16_t amp, uint32_t sub_frame_offset,
                         LTE_DL_FRAME_PARMS *frame_parms, uint8_t num_pdcch_symbols,
                         LTE_eNB_DLSCH_t *dlsch0, LTE_eNB_DLSCH_t *dlsch1)
{
  oai4g_frame_parms_t fp;  shim_dlsch_t s0, s1;
  fp_to(frame_parms, &fp);
  return oai4g_dlsch_modulation((int32_t **)txdataF, amp, sub_frame_offset, &fp, num_pdcch_symbols,
                                dlsch_to(dlsch0, &s0), dlsch_to(dlsch1, &s1));
}

void PHY_ofdm_mod(int *input, int *output, unsigned char log2fftsize, unsigned char nb_symbols,
                  unsigned short nb_prefix_samples, Extension_t etype)
{
  oai4g_PHY_ofdm_mod(input, output, log2fftsize, nb_symbols, nb_prefix_samples, (int)etype);
}

void normal_prefix_mod(int32_t *txdataF, int32_t *txdata, uint8_t nsymb, LTE_DL_FRAME_PARMS *frame_parms)
{
  oai4g_frame_parms_t fp;
  fp_to(frame_parms, &fp);
  oai4g_normal_prefix_mod(txdataF, txdata, nsymb, &fp);
}

void do_OFDM_mod(mod_sym_t **txdataF, int32_t **txdata, uint32_t frame, uint16_t next_slot,
                 LTE_DL_FRAME_PARMS *frame_parms)
{
  oai4g_frame_parms_t fp;
  fp_to(frame_parms, &fp);
  oai4g_do_OFDM_mod((int32_t **)txdataF, txdata, frame, next_slot, &fp);
}

void idft2048(int16_t *x, int16_t *y, int scale) { oai4g_idft2048(x, y, scale); }
void idft1024(int16_t *x, int16_t *y, int scale) { oai4g_idft1024(x, y, scale); }
void idft512(int16_t *x, int16_t *y, int scale)  { oai4g_idft512(x, y, scale); }
void idft256(int16_t *x, int16_t *y, int scale)  { oai4g_idft256(x, y, scale); }
void idft128(int16_t *x, int16_t *y, int scale)  { oai4g_idft128(x, y, scale); }
void idft64(int16_t *x, int16_t *y, int scale)   { oai4g_idft64(x, y, scale); }

/* UE receive front end: lte_dfts.c dft64..dft2048 (TOOLS/defs.h) and slot_fep.c:40 */
void dft2048(int16_t *x, int16_t *y, int scale) { oai4g_dft2048(x, y, scale); }
void dft1024(int16_t *x, int16_t *y, int scale) { oai4g_dft1024(x, y, scale); }
void dft512(int16_t *x, int16_t *y, int scale)  { oai4g_dft512(x, y, scale); }
void dft256(int16_t *x, int16_t *y, int scale)  { oai4g_dft256(x, y, scale); }
void dft128(int16_t *x, int16_t *y, int scale)  { oai4g_dft128(x, y, scale); }
void dft64(int16_t *x, int16_t *y, int scale)   { oai4g_dft64(x, y, scale); }

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

/* control region: pcfich.c:48 / :144 (frame_parms->pcfich_reg is derived inside the library) */
void generate_pcfich_reg_mapping(LTE_DL_FRAME_PARMS *frame_parms)
{
  oai4g_frame_parms_t fp;
  fp_to(frame_parms, &fp);
  oai4g_generate_pcfich_reg_mapping(&fp, frame_parms->pcfich_reg, &frame_parms->pcfich_first_reg_idx);
}
void generate_pcfich(uint8_t num_pdcch_symbols, int16_t amp, LTE_DL_FRAME_PARMS *frame_parms,
                     mod_sym_t **txdataF, uint8_t subframe)
{
  oai4g_frame_parms_t fp;
  fp_to(frame_parms, &fp);
  oai4g_generate_pcfich(num_pdcch_symbols, amp, &fp, (int32_t **)txdataF, subframe);
}

/* synchronisation, broadcast and HARQ-indicator channels: pss.c:50, sss.c:47, pbch.c:161
 * (LTE_eNB_PBCH's pbch_e is the library's oai4g_pbch_t state, impl_defs_lte.h:959-963),
 * phich.c:401 (void in the reference; the library's -1 for its undefined cases is dropped) */
int generate_pss(mod_sym_t **txdataF, short amp, LTE_DL_FRAME_PARMS *frame_parms, unsigned short symbol,
                 unsigned short slot_offset)
{
  oai4g_frame_parms_t fp;
  fp_to(frame_parms, &fp);
  return oai4g_generate_pss((int32_t **)txdataF, amp, &fp, symbol, slot_offset);
}
int generate_sss(mod_sym_t **txdataF, int16_t amp, LTE_DL_FRAME_PARMS *frame_parms, uint16_t symbol,
                 uint16_t slot_offset)
{
  oai4g_frame_parms_t fp;
  fp_to(frame_parms, &fp);
  return oai4g_generate_sss((int32_t **)txdataF, amp, &fp, symbol, slot_offset);
}
int generate_pbch(LTE_eNB_PBCH *eNB_pbch, mod_sym_t **txdataF, int amp, LTE_DL_FRAME_PARMS *frame_parms,
                  uint8_t *pbch_pdu, uint8_t frame_mod4)
{
  oai4g_frame_parms_t fp;
  fp_to(frame_parms, &fp);
  return oai4g_generate_pbch((oai4g_pbch_t *)eNB_pbch->pbch_e, (int32_t **)txdataF, amp, &fp, pbch_pdu, frame_mod4);
}
void generate_phich(LTE_DL_FRAME_PARMS *frame_parms, int16_t amp, uint8_t nseq_PHICH, uint8_t ngroup_PHICH,
                    uint8_t HI, uint8_t subframe, mod_sym_t **y)
{
  oai4g_frame_parms_t fp;
  fp_to(frame_parms, &fp);
  (void)oai4g_generate_phich(&fp, amp, nseq_PHICH, ngroup_PHICH, HI, subframe, (int32_t **)y);
}

/* callees that dlsim / ltetest also call directly */
uint32_t crc24a(uint8_t *inPtr, int32_t bitlen) { return oai4g_crc24a(inPtr, bitlen); }   /* CODING/defs.h:375 */
uint32_t crc24b(uint8_t *inPtr, int32_t bitlen) { return oai4g_crc24b(inPtr, bitlen); }
int32_t lte_segmentation(uint8_t *input_buffer, uint8_t **output_buffers, uint32_t B, uint32_t *C,
                         uint32_t *Cplus, uint32_t *Cminus, uint32_t *Kplus, uint32_t *Kminus, uint32_t *F)
{                                                                                         /* CODING/defs.h:79 */
  return oai4g_lte_segmentation(input_buffer, output_buffers, B, C, Cplus, Cminus, Kplus, Kminus, F);
}
void threegpplte_turbo_encoder(uint8_t *input, uint16_t input_length_bytes, uint8_t *output, uint8_t F,
                               uint16_t interleaver_f1, uint16_t interleaver_f2)          /* CODING/defs.h:315 */
{
  oai4g_threegpplte_turbo_encoder(input, input_length_bytes, output, F, interleaver_f1, interleaver_f2);
}
uint32_t sub_block_interleaving_turbo(uint32_t D, uint8_t *d, uint8_t *w)
{
  return oai4g_sub_block_interleaving_turbo(D, d, w);
}
uint32_t lte_rate_matching_turbo(uint32_t RTC, uint32_t G, uint8_t *w, uint8_t *e, uint8_t C, uint32_t Nsoft,
                                 uint8_t Mdlharq, uint8_t Kmimo, uint8_t rvidx, uint8_t Qm, uint8_t Nl, uint8_t r,
                                 uint8_t nb_rb, uint8_t m)
{
  return oai4g_lte_rate_matching_turbo(RTC, G, w, e, C, Nsoft, Mdlharq, Kmimo, rvidx, Qm, Nl, r, nb_rb, m);
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

/* lte_est_freq_offset.c:104 (dot products on the GPU, atan2 + filter on the host as in the reference) */
int lte_est_freq_offset(int **dl_ch_estimates, LTE_DL_FRAME_PARMS *frame_parms, int l, int *freq_offset, int reset)
{
  oai4g_frame_parms_t fp;
  fp_to(frame_parms, &fp);
  return oai4g_lte_est_freq_offset((int32_t *const *)dl_ch_estimates, &fp, l, freq_offset, reset);
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

void dlsch_unscrambling(LTE_DL_FRAME_PARMS *frame_parms, int mbsfn_flag, LTE_UE_DLSCH_t *dlsch, int G,
                        int16_t *llr, uint8_t q, uint8_t Ns)                          /* dlsch_scrambling.c:99 */
{
  oai4g_frame_parms_t fp;
  fp_to(frame_parms, &fp);
  oai4g_dlsch_unscrambling(&fp, mbsfn_flag, dlsch->rnti, G, llr, q, Ns);
}

/* UL turbo decoding chain (CODING/defs.h:470-513, lte_rate_matching.c): the decoders, RX rate
 * matching, deinterleaving and generate_dummy_w.  The 8-bit decoder covers n % 16 == 0, n >= 512
 * (255 otherwise, as the reference returns on illegal arguments). */
uint8_t phy_threegpplte_turbo_decoder16(int16_t *y, uint8_t *decoded_bytes, uint16_t n, uint16_t interleaver_f1,
                                        uint16_t interleaver_f2, uint8_t max_iterations, uint8_t crc_type, uint8_t F,
                                        time_stats_t *init_stats, time_stats_t *alpha_stats, time_stats_t *beta_stats,
                                        time_stats_t *gamma_stats, time_stats_t *ext_stats, time_stats_t *intl1_stats,
                                        time_stats_t *intl2_stats)
{
  (void)init_stats; (void)alpha_stats; (void)beta_stats; (void)gamma_stats; (void)ext_stats; (void)intl1_stats;
  (void)intl2_stats;
  return oai4g_phy_threegpplte_turbo_decoder16(y, decoded_bytes, n, interleaver_f1, interleaver_f2, max_iterations,
                                               crc_type, F);
}
uint8_t phy_threegpplte_turbo_decoder8(int16_t *y, uint8_t *decoded_bytes, uint16_t n, uint16_t interleaver_f1,
                                       uint16_t interleaver_f2, uint8_t max_iterations, uint8_t crc_type, uint8_t F,
                                       time_stats_t *init_stats, time_stats_t *alpha_stats, time_stats_t *beta_stats,
                                       time_stats_t *gamma_stats, time_stats_t *ext_stats, time_stats_t *intl1_stats,
                                       time_stats_t *intl2_stats)
{
  (void)init_stats; (void)alpha_stats; (void)beta_stats; (void)gamma_stats; (void)ext_stats; (void)intl1_stats;
  (void)intl2_stats;
  return oai4g_phy_threegpplte_turbo_decoder8(y, decoded_bytes, n, interleaver_f1, interleaver_f2, max_iterations,
                                              crc_type, F);
}
int lte_rate_matching_turbo_rx(uint32_t RTC, uint32_t G, int16_t *w, uint8_t *dummy_w, int16_t *soft_input, uint8_t C,
                               uint32_t Nsoft, uint8_t Mdlharq, uint8_t Kmimo, uint8_t rvidx, uint8_t clear, uint8_t Qm,
                               uint8_t Nl, uint8_t r, uint32_t *E)
{
  return oai4g_lte_rate_matching_turbo_rx(RTC, G, w, dummy_w, soft_input, C, Nsoft, Mdlharq, Kmimo, rvidx, clear, Qm,
                                          Nl, r, E);
}
void sub_block_deinterleaving_turbo(uint32_t D, int16_t *d, int16_t *w) { oai4g_sub_block_deinterleaving_turbo(D, d, w); }
uint32_t generate_dummy_w(uint32_t D, uint8_t *w, uint8_t F) { return oai4g_generate_dummy_w(D, w, F); }
