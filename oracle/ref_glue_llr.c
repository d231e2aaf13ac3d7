/* TEST INFRASTRUCTURE ONLY — linked into oracle/_ref/libref_llr.so next to the reference's own
 * PHY/LTE_TRANSPORT/dlsch_llr_computation.c (compiled unmodified, see oracle/Makefile).  Not a stand-in
 * for any reference file: ref_glue_qam_llr() fills the reference's LTE_DL_FRAME_PARMS
 * (PHY/impl_defs_lte.h) with the fields dlsch_qpsk_llr / dlsch_16qam_llr / dlsch_64qam_llr read
 * (N_RB_DL, Ncp, mode1_flag) and calls them for one OFDM symbol, as rx_pdsch does
 * (dlsch_demodulation.c:583-800).  The interference-aware qpsk_qpsk / qpsk_qam16 / qpsk_qam64 take
 * plain arrays and are called from the tests directly. */
void dlsch_qpsk_llr(LTE_DL_FRAME_PARMS *frame_parms, int32_t **rxdataF_comp, int16_t *dlsch_llr, uint8_t symbol,
                    uint8_t first_symbol_flag, uint16_t nb_rb, uint16_t pbch_pss_sss_adjust, int16_t **llr32p);
void dlsch_16qam_llr(LTE_DL_FRAME_PARMS *frame_parms, int32_t **rxdataF_comp, int16_t *dlsch_llr, int32_t **dl_ch_mag,
                     uint8_t symbol, uint8_t first_symbol_flag, uint16_t nb_rb, uint16_t pbch_pss_sss_adjust,
                     int16_t **llr32p);
void dlsch_64qam_llr(LTE_DL_FRAME_PARMS *frame_parms, int32_t **rxdataF_comp, int16_t *dlsch_llr, int32_t **dl_ch_mag,
                     int32_t **dl_ch_magb, uint8_t symbol, uint8_t first_symbol_flag, uint16_t nb_rb,
                     uint16_t pbch_pss_sss_adjust, int16_t **llr_save);

/* one symbol of dlsch_{qpsk,16qam,64qam}_llr: comp / mag / magb are the symbol-major arrays rx_pdsch
 * passes (symbol l at l N_RB_DL 12 words); returns the LLRs the call accounts for (its output-pointer
 * advance) */
int ref_glue_qam_llr(int Qm, int N_RB_DL, int Ncp, int mode1_flag, int32_t *comp, int32_t *mag, int32_t *magb,
                     int16_t *llr, uint8_t symbol, uint16_t nb_rb, uint16_t adjust)
{
  LTE_DL_FRAME_PARMS fp;
  int16_t *next = llr;
  memset(&fp, 0, sizeof(fp));
  fp.N_RB_DL = (uint8_t)N_RB_DL;
  fp.Ncp = (lte_prefix_type_t)Ncp;
  fp.mode1_flag = (uint8_t)mode1_flag;
  if (Qm == 2) dlsch_qpsk_llr(&fp, &comp, llr, symbol, 1, nb_rb, adjust, &next);
  else if (Qm == 4) dlsch_16qam_llr(&fp, &comp, llr, &mag, symbol, 1, nb_rb, adjust, &next);
  else {
    /* dlsch_64qam_llr advances its saved pointer by len 6 itself */
    next = llr;
    dlsch_64qam_llr(&fp, &comp, llr, &mag, &magb, symbol, 1, nb_rb, adjust, &next);
  }
  return (int)(next - llr);
}
