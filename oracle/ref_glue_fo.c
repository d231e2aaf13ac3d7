/* TEST INFRASTRUCTURE ONLY — linked into oracle/_ref/libref_fo.so next to the reference's own
 * PHY/LTE_ESTIMATION/lte_est_freq_offset.c (compiled unmodified, see oracle/Makefile; its
 * dot_product / log2_approx are libref_tools.so's, PHY/TOOLS/cdot_prod.c and log2_approx.c).  Not a
 * stand-in for any reference file: ref_glue_est_freq_offset() fills the reference's
 * LTE_DL_FRAME_PARMS (PHY/impl_defs_lte.h) with the fields lte_est_freq_offset reads (N_RB_DL, Ncp,
 * ofdm_symbol_size) and calls it on antenna 0's estimate plane. */
int lte_est_freq_offset(int **dl_ch_estimates, LTE_DL_FRAME_PARMS *frame_parms, int l, int *freq_offset, int reset);

int ref_glue_est_freq_offset(int N_RB_DL, int Ncp, int ofdm_symbol_size, int32_t *plane0, int l, int *freq_offset,
                             int reset)
{
  LTE_DL_FRAME_PARMS fp;
  int *planes[1] = {(int *)plane0};
  memset(&fp, 0, sizeof(fp));
  fp.N_RB_DL = (uint8_t)N_RB_DL;
  fp.Ncp = (lte_prefix_type_t)Ncp;
  fp.ofdm_symbol_size = (uint16_t)ofdm_symbol_size;
  const int r = lte_est_freq_offset(planes, &fp, l, freq_offset, reset);
  fflush(stdout);   /* the refusal's msg (:127-130) leaves while a test's capture is on */
  return r;
}
