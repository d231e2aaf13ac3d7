/* oai4g_shim.c — reference-side binding of the MI355X DLSCH transmit path.
 * Replaces: dlsch_coding.c:254 dlsch_encoding, dlsch_scrambling.c:51, dlsch_modulation.c:1181,
 * ofdm_mod.c:47/85/233, lte_dfts.c idft64..idft2048, crc_byte.c:117/135, lte_segmentation.c:39,
 * 3gpplte_sse.c:380, lte_rate_matching.c:51/464, pcfich.c:48/144, dci.c:2024, pss.c:50, sss.c:47,
 * pbch.c:161, phich.c:401, lte_dl_channel_estimation.c:37, dlsch_demodulation.c:82 (rx_pdsch, TM1/TM2/TM3),
 * dlsch_scrambling.c:99 (dlsch_unscrambling), 3gpplte_turbo_decoder_sse_16bit.c:945 / _8bit.c:894,
 * lte_rate_matching.c:193 / :293 / :688 (the UL decoding chain).
 *
 * The four bindings that take PHY_VARS_UE / PHY_VARS_eNB (slot_fep, generate_pilots,
 * lte_dl_channel_estimation, rx_pdsch) live in oai4g_shim_ue.c: PHY_VARS_* come from PHY/defs.h's
 * asn1c-generated chain, so that file builds only inside a full reference build.  This file builds
 * against the reference's own headers here (integration/Makefile -> liboai4g_shim.so) and is run
 * by tests/test_gpu_shim_ref.py with the reference's LTE_eNB_DLSCH_t / LTE_DL_eNB_HARQ_t. */
#include "PHY/defs.h"
#include "PHY/extern.h"
#include "oai4g.h"
#include "oai4g_shim_fp.h"

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

/* lte_est_freq_offset.c:104 (dot products on the GPU, atan2 + filter on the host as in the reference) */
int lte_est_freq_offset(int **dl_ch_estimates, LTE_DL_FRAME_PARMS *frame_parms, int l, int *freq_offset, int reset)
{
  oai4g_frame_parms_t fp;
  fp_to(frame_parms, &fp);
  return oai4g_lte_est_freq_offset((int32_t *const *)dl_ch_estimates, &fp, l, freq_offset, reset);
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
