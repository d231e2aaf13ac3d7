/* TEST INFRASTRUCTURE ONLY — linked into oracle/_ref/libref_ofdm.so next to the reference's own
 * PHY/MODULATION/ofdm_mod.c (compiled unmodified).  Not a stand-in for any reference file:
 *
 *   - ref_glue_frame() fills the reference's LTE_DL_FRAME_PARMS (PHY/impl_defs_lte.h:470-572) with
 *     the fields ofdm_mod.c reads (ofdm_symbol_size, log2_symbol_size, nb_prefix_samples{,0},
 *     symbols_per_tti, samples_per_tti, Ncp, nb_antennas_tx, and num_MBSFN_config = 0), because a
 *     ctypes test cannot build that struct itself;
 *   - is_pmch_subframe: do_OFDM_mod (ofdm_mod.c:242) calls it, and its translation unit
 *     (PHY/LTE_TRANSPORT/pmch.c:97) includes PHY/extern.h, which needs PHY_VARS_eNB/UE and the
 *     asn1c headers.  Every frame this glue builds has num_MBSFN_config = 0, for which pmch.c:106's
 *     loop runs zero times and the function returns 0; that one case is all this restates.  Any
 *     other input aborts instead of guessing.
 *
 * The remaining symbol ofdm_mod.c leaves undefined, logRecord (UTIL/LOG/log.h:157, LOG_D), is only
 * reached on the PMCH branch (ofdm_mod.c:244/260), which the case above never takes; the library is
 * therefore opened with RTLD_LAZY (tests/oracle_lib.py ref_ofdm, oracle/cpu_baseline.c), so that
 * symbol is never bound. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "PHY/impl_defs_lte.h"

void normal_prefix_mod(int32_t *txdataF, int32_t *txdata, uint8_t nsymb, LTE_DL_FRAME_PARMS *frame_parms);
void do_OFDM_mod(int32_t **txdataF, int32_t **txdata, uint32_t frame, uint16_t next_slot,
                 LTE_DL_FRAME_PARMS *frame_parms);

int is_pmch_subframe(uint32_t frame, int subframe, LTE_DL_FRAME_PARMS *frame_parms)
{
  (void)frame;
  (void)subframe;
  if (frame_parms->num_MBSFN_config != 0) abort();
  return 0;
}

static void ref_glue_frame(LTE_DL_FRAME_PARMS *fp, int N_RB_DL, int Ncp, int nb_antennas_tx, int ofdm_symbol_size,
                           int log2_symbol_size, int nb_prefix_samples, int nb_prefix_samples0, int symbols_per_tti,
                           int samples_per_tti)
{
  memset(fp, 0, sizeof(*fp));
  fp->N_RB_DL = (uint8_t)N_RB_DL;
  fp->Ncp = (lte_prefix_type_t)Ncp;
  fp->nb_antennas_tx = (uint8_t)nb_antennas_tx;
  fp->ofdm_symbol_size = (uint16_t)ofdm_symbol_size;
  fp->log2_symbol_size = (uint8_t)log2_symbol_size;
  fp->nb_prefix_samples = (uint16_t)nb_prefix_samples;
  fp->nb_prefix_samples0 = (uint16_t)nb_prefix_samples0;
  fp->symbols_per_tti = (uint16_t)symbols_per_tti;
  fp->samples_per_tti = (uint32_t)samples_per_tti;
  fp->num_MBSFN_config = 0;
}

/* geometry: {N_RB_DL, Ncp, nb_antennas_tx, ofdm_symbol_size, log2_symbol_size, nb_prefix_samples,
 *            nb_prefix_samples0, symbols_per_tti, samples_per_tti} */
void ref_glue_normal_prefix_mod(int32_t *txdataF, int32_t *txdata, uint8_t nsymb, const int32_t g[9])
{
  LTE_DL_FRAME_PARMS fp;
  ref_glue_frame(&fp, g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8]);
  normal_prefix_mod(txdataF, txdata, nsymb, &fp);
}

void ref_glue_do_OFDM_mod(int32_t **txdataF, int32_t **txdata, uint32_t frame, uint16_t next_slot, const int32_t g[9])
{
  LTE_DL_FRAME_PARMS fp;
  ref_glue_frame(&fp, g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8]);
  do_OFDM_mod(txdataF, txdata, frame, next_slot, &fp);
}
