/*
 * CPU ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference's LTE PDSCH transmit path
 * (erlgo/openair4G openair1/PHY), used exclusively as the parity checker by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Nothing in
 * the product library (openair4g_amd/) links or calls it.
 *
 * Pinning:
 *   - IDFT/OFDM: checked bit-exactly against the reference's own lte_dfts.c,
 *     compiled unmodified from /root/reference into oracle/_ref (Makefile here).
 *   - get_G / TBS plumbing: REFERENCE_DATA/pdsch.txt known answers.
 *   - CRC-24A/B: published CRC-catalogue check values (CRC-24/LTE-A, -B).
 *   - Turbo encoder, sub-block interleaver, rate matcher, scrambling and the
 *     RE mapper: the reference TUs are unbuildable here (they include
 *     PHY/defs.h -> openair2/COMMON/platform_constants.h:40 -> asn1c-generated
 *     asn1_constants.h, and the SSE encoder needs the missing
 *     lte_interleaver.h blob).  These stages are pinned by an independent
 *     36.212 textbook model (tests/spec_model.py) plus structural properties;
 *     DESIGN.md records them as "parity pinned to spec, not to reference output".
 */
#ifndef OAI_ORACLE_H
#define OAI_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define ORC_LTE_NULL 2
#define ORC_NSOFT 1827072

/* ---- CRC (crc_byte.c:98-153) ---- */
void     orc_crc_init(void);
uint32_t orc_crc24a(const uint8_t *in, int bitlen); /* returns crc<<8 like the reference */
uint32_t orc_crc24b(const uint8_t *in, int bitlen);

/* ---- segmentation (lte_segmentation.c:39-170) ---- */
int orc_segmentation(const uint8_t *b, uint8_t **c, uint32_t B, uint32_t *C, uint32_t *Cplus,
                     uint32_t *Cminus, uint32_t *Kplus, uint32_t *Kminus, uint32_t *F);

/* ---- turbo encoder (3gpplte_sse.c:380-476 / 3gpplte.c:116-230) ---- */
void orc_turbo_encode(const uint8_t *c, uint16_t nbytes, uint8_t *d /* 3K+12 */, uint16_t f1, uint16_t f2);

/* ---- sub-block interleaver (lte_rate_matching.c:51-130); d must have 96 bytes of
 *      LTE_NULL readable in front of it ---- */
uint32_t orc_subblock_interleave(uint32_t D, uint8_t *d, uint8_t *w);

/* ---- rate matching (lte_rate_matching.c:464-634) ---- */
void orc_set_rm_limited(int on);   /* opt-in limited-buffer RM (extension, not the reference) */
uint32_t orc_rate_match(uint32_t RTC, uint32_t G, const uint8_t *w, uint8_t *e, uint8_t C,
                        uint32_t Nsoft, uint8_t Mdlharq, uint8_t Kmimo, uint8_t rvidx, uint8_t Qm,
                        uint8_t Nl, uint8_t r);

/* ---- Gold sequence / scrambling (lte_gold.c:151-177, dlsch_scrambling.c:51-97) ---- */
uint32_t orc_gold_generic(uint32_t *x1, uint32_t *x2, uint8_t reset);
void     orc_scramble(uint8_t *e, int G, uint32_t c_init);

/* ---- MCS / G (lte_mcs.c:45-368) ---- */
uint8_t orc_get_Qm(uint8_t mcs);
int     orc_get_G(uint16_t N_RB_DL, uint8_t Ncp, uint8_t mode1_flag, uint8_t frame_type, uint16_t nb_rb,
                  const uint32_t *rb_alloc, uint8_t Qm, uint8_t Nl, uint8_t num_pdcch_symbols,
                  uint8_t subframe);

/* ---- frame parameters (lte_parms.c:31-145) ---- */
typedef struct {
  uint16_t N_RB_DL;
  uint16_t Nid_cell;
  uint8_t Ncp;            /* 0 = normal */
  uint8_t nushift;
  uint8_t mode1_flag;
  uint8_t nb_antennas_tx;
  uint8_t frame_type;     /* 0 = FDD, 1 = TDD */
  uint8_t symbols_per_tti;
  uint8_t log2_symbol_size;
  uint16_t ofdm_symbol_size;
  uint16_t first_carrier_offset;
  uint16_t nb_prefix_samples;
  uint16_t nb_prefix_samples0;
  uint32_t samples_per_tti;
  /* control region (LTE_DL_FRAME_PARMS phich_config_common, tdd_config, nb_antennas_tx_eNB) */
  uint8_t phich_resource;   /* PHICH_RESOURCE_t (impl_defs_lte.h:80-85): 1, 3, 6, 12 = Ng 1/6, 1/2, 1, 2 */
  uint8_t phich_duration;   /* 0 normal, 1 extended */
  uint8_t tdd_config;
  uint8_t nb_antennas_tx_eNB;
} orc_frame_t;
int orc_init_frame(orc_frame_t *fp, uint16_t N_RB_DL, uint16_t Nid_cell, uint8_t Ncp, uint8_t nb_antennas_tx,
                   uint8_t mode1_flag, uint8_t frame_type);

/* ---- modulation + RE mapping (dlsch_modulation.c:139-1493) ----
 * mimo_mode: 0 = SISO, 1 = ALAMOUTI, 2 = LARGE_CDD */
typedef struct {
  const uint8_t *e;
  uint8_t mcs;
  uint8_t mimo_mode;
  uint8_t Nlayers;
  uint32_t rb_alloc[4];
} orc_cw_t;
/* 4-TX extension (configuration C4): PDSCH RE count with the port-2/3 CRS exclusions (G = count x Qm) */
int orc_count_pdsch_res(const orc_frame_t *fp, const uint32_t rb_alloc[4], uint8_t num_pdcch_symbols, uint32_t subframe);
void orc_cell_spec_p23(int32_t *output, int16_t amp, const orc_frame_t *fp, uint8_t Ns, uint8_t p);
int orc_modulation(int32_t **txdataF, int16_t amp, uint32_t subframe, const orc_frame_t *fp,
                   uint8_t num_pdcch_symbols, const orc_cw_t *cw0, const orc_cw_t *cw1,
                   int16_t sqrt_rho_a, int16_t sqrt_rho_b);

/* ---- fixed-point IDFT (lte_dfts.c:1597-2866) and OFDM modulation (ofdm_mod.c:47-229) ---- */
void orc_idft(int log2n, const int16_t *x, int16_t *y, int scale);
void orc_twiddle(int N, int m, int16_t *re, int16_t *im);
void orc_dft(int log2n, const int16_t *x, int16_t *y, int scale);           /* forward dft64 … dft2048 */
void orc_dft_twiddle_ab(int N, int m, int16_t a[2], int16_t b[2]);
/* PCFICH (pcfich.c:48-228) into symbol 0 of `subframe` of frame grids txdataF[ant] */
void orc_pcfich_reg_mapping(const orc_frame_t *fp, uint16_t reg[4], uint8_t *first_idx);
int orc_generate_pcfich(uint8_t num_pdcch_symbols, int16_t amp, const orc_frame_t *fp, int32_t **txdataF,
                        uint8_t subframe);
/* slot_fep DFT part (slot_fep.c:40-177); rxdata[aa] = 10 subframes + N words of wrap extension */
int orc_slot_fep(int32_t **rxdata, int32_t **rxdataF, const orc_frame_t *fp, int nb_antennas_rx, uint8_t l,
                 uint8_t Ns, int sample_offset, int no_prefix);
void orc_ofdm_mod(const int32_t *input, int32_t *output, uint8_t log2fftsize, uint8_t nb_symbols,
                  uint16_t nb_prefix_samples);
void orc_normal_prefix_mod(const int32_t *txdataF, int32_t *txdata, uint8_t nsymb, const orc_frame_t *fp);
void orc_do_OFDM_mod(int32_t **txdataF, int32_t **txdata, uint32_t frame, uint16_t next_slot, const orc_frame_t *fp);

/* ---- cell-specific reference signals (LTE_REFSIG/lte_gold.c:52-93, lte_dl_cell_spec.c:123-203,
 *      LTE_TRANSPORT/pilots.c:43-168) ---- */
void orc_lte_gold_table(const orc_frame_t *fp, uint32_t table[20][2][14]);
int  orc_lte_dl_cell_spec(int32_t *output, int16_t amp, const orc_frame_t *fp, const uint32_t table[20][2][14],
                          uint8_t Ns, uint8_t l, uint8_t p);
/* txdataF[ant] spans Ntti subframes of nsymb * ofdm_symbol_size REs (the reference's frame grid) */
void orc_generate_pilots(int32_t **txdataF, int16_t amp, const orc_frame_t *fp, uint16_t Ntti);
/* the same for one subframe grid (txdataF[ant] = 14 * N REs of subframe `subframe`) */
void orc_generate_pilots_subframe(int32_t **txdataF, int16_t amp, const orc_frame_t *fp, uint8_t subframe);

/* ---- whole-subframe TX (dlsim.c:2567-2699 minus DCI; pilots when cfg->with_crs) ----
 * payload[cw] holds TBS/8 bytes (+3 bytes of room; the CRC is appended in place as in the
 * reference).  txdata[ant] receives samples_per_tti int32 samples.  Returns 0 on success. */
typedef struct {
  orc_frame_t fp;
  uint8_t n_cw;
  uint8_t mimo_mode;
  uint8_t num_pdcch_symbols;
  uint8_t subframe;
  uint16_t rnti;
  int16_t amp;
  int16_t sqrt_rho_a, sqrt_rho_b;
  uint8_t Kmimo, Mdlharq;
  uint32_t rb_alloc[4];
  uint16_t nb_rb;
  uint8_t mcs[2];
  uint8_t rvidx[2];
  uint8_t q[2];            /* scrambling codeword index (dlsim.c:2646 passes 0) */
  uint32_t TBS[2];
  uint8_t with_crs;        /* 1: cell-specific reference signals in the grid (generate_pilots) */
} orc_tx_cfg_t;
int orc_tx_subframe(const orc_tx_cfg_t *cfg, uint8_t *payload[2], int32_t **txdataF, int32_t **txdata,
                    uint8_t *e_out[2] /* optional: scrambled e bytes per cw */);
int orc_last_re_allocated(void);   /* dlsch_modulation's return value of the last orc_tx_subframe */

/* ---- uplink turbo decoding (oai_oracle_td.c; 3gpplte_turbo_decoder_sse_16bit.c:945-1385,
 *      lte_rate_matching.c:193-243, 688-831) ---- */
enum { ORC_CRC24_A = 0, ORC_CRC24_B = 1, ORC_CRC16 = 2, ORC_CRC8 = 3 };
uint8_t orc_turbo_decoder16(const int16_t *y, uint8_t *decoded_bytes, uint16_t n, uint8_t max_iterations,
                            uint8_t crc_type, uint8_t F);
uint32_t orc_generate_dummy_w(uint32_t D, uint8_t *w);
uint32_t orc_generate_dummy_w_F(uint32_t D, uint8_t *w, uint8_t F);
int orc_rate_matching_turbo_rx(uint32_t RTC, uint32_t G, int16_t *w, const uint8_t *dummy_w, const int16_t *soft_input,
                               uint8_t C, uint32_t Nsoft, uint8_t Mdlharq, uint8_t Kmimo, uint8_t rvidx, uint8_t clear,
                               uint8_t Qm, uint8_t Nl, uint8_t r, uint32_t *E_out);
void orc_sub_block_deinterleaving_turbo(uint32_t D, int16_t *d, const int16_t *w);

/* ---- control region: PDCCH / DCI (oai_oracle_ctrl.c; dci.c:62-341, 1905-2346, 2494-2538,
 *      phich.c:59-118, 280-386, ccoding_byte_lte.c:55-230, lte_rate_matching.c:133-190, 637-680,
 *      crc_byte.c:155-171, phy_procedures_lte_eNb.c:308-391) ---- */
typedef struct {           /* DCI_ALLOC_t (LTE_TRANSPORT/defs.h:734-749) */
  uint8_t dci_length;      /* bits */
  uint8_t L;               /* log2 aggregation level */
  int32_t nCCE;            /* first CCE, < 0: not transmitted */
  uint8_t ra_flag;
  uint16_t rnti;
  uint32_t format;
  uint8_t dci_pdu[8];
} orc_dci_alloc_t;
uint32_t orc_crc16(const uint8_t *in, int bitlen);
void orc_ccodelte_encode(int32_t numbits, uint8_t add_crc, const uint8_t *in, uint8_t *out, uint16_t rnti);
uint32_t orc_sub_block_interleaving_cc(uint32_t D, const uint8_t *d, uint8_t *w);
uint32_t orc_lte_rate_matching_cc(uint32_t RCC, uint16_t E, const uint8_t *w, uint8_t *e);
uint8_t orc_get_mi(const orc_frame_t *fp, uint8_t subframe);
uint16_t orc_get_nquad(uint8_t num_pdcch_symbols, const orc_frame_t *fp, uint8_t mi);
uint16_t orc_get_nCCE(uint8_t num_pdcch_symbols, const orc_frame_t *fp, uint8_t mi);
uint8_t orc_get_num_pdcch_symbols(uint8_t num_dci, const orc_dci_alloc_t *dci_alloc, const orc_frame_t *fp,
                                  uint8_t subframe);
/* phich_reg[56][3] (normal PHICH duration); returns the number of groups written */
int orc_phich_reg_mapping(const orc_frame_t *fp, uint16_t phich_reg[56][3]);
/* get_nCCE_offset over a caller-owned CCE_table[800] */
int orc_get_nCCE_offset(int *CCE_table, uint8_t L, int nCCE, int common_dci, uint16_t rnti, uint8_t subframe);
/* generate_dci_top into the frame grids txdataF[ant]; returns num_pdcch_symbols */
uint8_t orc_generate_dci_top(uint8_t num_ue_spec_dci, uint8_t num_common_dci, const orc_dci_alloc_t *dci_alloc,
                             uint32_t n_rnti, int16_t amp, const orc_frame_t *fp, int32_t **txdataF,
                             uint32_t subframe);
/* the scrambled PDCCH bits e[] of the last orc_generate_dci_top (values 0/1/2 = NIL), for tests */
const uint8_t *orc_last_dci_e(uint32_t *len);
/* ---- synchronisation / broadcast / HARQ-indicator channels (oai_oracle_sync.c; pss.c:50-103,
 *      sss.c:47-92, pbch.c:62-420, 760-783, phich.c:401-780, primary_synch.h, sss.h) ---- */
typedef struct {           /* LTE_eNB_PBCH (LTE_TRANSPORT/defs.h): state kept across frame_mod4 */
  uint8_t pbch_d[96 + 3 * (16 + 24)];
  uint8_t pbch_w[3 * 3 * (16 + 24)];
  uint8_t pbch_e[1920];
} orc_pbch_t;
void orc_primary_synch(uint8_t Nid2, int16_t out[144]);
void orc_sss_seq(uint16_t Nid_cell, int sf5, int16_t d[62]);
int orc_generate_pss(int32_t **txdataF, int16_t amp, const orc_frame_t *fp, uint16_t symbol, uint16_t slot_offset);
int orc_generate_sss(int32_t **txdataF, int16_t amp, const orc_frame_t *fp, uint16_t symbol, uint16_t slot_offset);
void orc_pbch_scrambling(const orc_frame_t *fp, uint8_t *e, uint32_t length);
int orc_generate_pbch(orc_pbch_t *st, int32_t **txdataF, int amp, const orc_frame_t *fp, const uint8_t *pbch_pdu,
                      uint8_t frame_mod4);
int orc_generate_phich(const orc_frame_t *fp, int16_t amp, uint8_t nseq_PHICH, uint8_t ngroup_PHICH, uint8_t HI,
                       uint8_t subframe, int32_t **y);
/* ---- UE PDSCH demodulation after the FEP, TM1 / one RX antenna / even N_RB_DL (oai_oracle_rx.c;
 *      dlsch_demodulation.c:82-700, 801-960, 2777-2835, 3167-3300, dlsch_llr_computation.c:636-930,
 *      lte_mcs.c:157-245, dlsch_scrambling.c:99-137, log2_approx.c:29-45) ----
 * rxdataF: one subframe [nsymb][N]; dl_ch_estimates: [nsymb][N] per-symbol estimates (entry
 * 5 + 12 rb + i = subcarrier 12 rb + i).  Writes the LLR stream of every PDSCH symbol; returns
 * its length or -1. */
uint8_t orc_log2_approx(uint32_t x);
int orc_adjust_G2(const orc_frame_t *fp, const uint32_t rb_alloc[4], uint8_t subframe, uint8_t symbol);
int orc_rx_pdsch_siso(const orc_frame_t *fp, const int32_t *rxdataF, const int32_t *dl_ch_estimates,
                      const uint32_t rb_alloc[4], uint8_t Qm, uint8_t num_pdcch_symbols, uint8_t subframe,
                      int16_t *llr, uint8_t *log2_maxh_out);
void orc_dlsch_unscrambling(int16_t *llr, int G, uint32_t c_init);
/* the LLR stages alone over flat streams (dlsch_llr_computation.c: dlsch_qpsk / 16qam / 64qam_llr :636-930,
 * qpsk_qpsk :1041, qpsk_qam16 :1300, qpsk_qam64 :1584), as the receivers above use them per RE */
int orc_llr_qam(int Qm, const int16_t *comp, const int16_t *mag, const int16_t *magb, int len, int16_t *llr);
void orc_llr_qpsk_qpsk(const int16_t *s0, const int16_t *s1, const int16_t *rho, int len, int16_t *llr);
void orc_llr_qpsk_qamx(int qm1, const int16_t *s0, const int16_t *s1, const int16_t *mag1, const int16_t *rho, int len,
                       int16_t *llr);
/* rx_pdsch for TM3 (LARGE_CDD, 2 ports), dual_stream_flag = 0: codeword 0's LLRs (Qm0 4 / 6; Qm0 2
 * runs orc_rx_pdsch_tm3_q2 for codeword 0).
 * rxdataF[a] = [nsymb][N] per receive antenna, est[p * 2 + a] = [nsymb][N] estimates of port p. */
int orc_rx_pdsch_tm3(const orc_frame_t *fp, int nb_rx, const int32_t *const *rxdataF, const int32_t *const *est,
                     const uint32_t rb_alloc[4], uint8_t Qm0, uint8_t Qm1, uint8_t mcs0, uint8_t num_pdcch_symbols,
                     uint8_t subframe, int16_t *llr, uint8_t *log2_maxh_out);
/* TM3 with codeword 0 QPSK: Qm1 = 2 both codewords (qpsk_qpsk; llr1 may be NULL), Qm1 = 4 / 6 codeword 0
 * (qpsk_qam16 / qpsk_qam64) */
int orc_rx_pdsch_tm3_q2(const orc_frame_t *fp, int nb_rx, const int32_t *const *rxdataF, const int32_t *const *est,
                        const uint32_t rb_alloc[4], uint8_t Qm1, uint8_t mcs0, uint8_t num_pdcch_symbols,
                        uint8_t subframe, int16_t *llr0, int16_t *llr1, uint8_t *log2_maxh_out);
int orc_rx_pdsch_tm3_qq(const orc_frame_t *fp, int nb_rx, const int32_t *const *rxdataF, const int32_t *const *est,
                        const uint32_t rb_alloc[4], uint8_t mcs0, uint8_t num_pdcch_symbols, uint8_t subframe,
                        int16_t *llr0, int16_t *llr1, uint8_t *log2_maxh_out);
int orc_rx_pdsch_tm2(const orc_frame_t *fp, int nb_rx, const int32_t *const *rxdataF, const int32_t *const *est,
                     const uint32_t rb_alloc[4], uint8_t Qm, uint8_t num_pdcch_symbols, uint8_t subframe,
                     int16_t *llr, uint8_t *log2_maxh_out);
/* orc_tx_subframe plus generate_dci_top's PCFICH + PDCCH before the OFDM step (dlsim.c:2553) */
int orc_tx_subframe_dci(const orc_tx_cfg_t *cfg, uint8_t *payload[2], int32_t **txdataF, int32_t **txdata,
                        uint8_t *e_out[2], uint8_t n_ue_dci, uint8_t n_common_dci, const orc_dci_alloc_t *dci);

#ifdef __cplusplus
}
#endif
/* ---- downlink channel estimation (LTE_ESTIMATION/lte_dl_channel_estimation.c:37-701, high_speed_flag 1) ---- */
void orc_chest_filters(uint8_t k, int16_t out[6][24]);
void orc_chest_dc_filters(uint8_t k, int16_t out[2][24]);      /* filt24_k_dcr, filt24_(k+2)_dcl */
const int16_t *orc_chest_pilot_filter(const int16_t f[6][24], const int16_t fdc[2][24], int N_RB, int m);
int  orc_lte_dl_channel_estimation(const orc_frame_t *fp, const uint32_t gold[20][2][14], const int32_t *rxdataF,
                                   int32_t *dl_ch_estimates, uint8_t Ns, uint8_t p, uint8_t l, uint8_t symbol);
/* lte_est_freq_offset.c:45-193, cdot_prod.c:40-118, lte_dl_channel_estimation.c:704-738 */
void    orc_multadd_complex_vector_real_scalar(const int16_t *x, int16_t alpha, int16_t *y, uint8_t zero_flag, uint32_t N);
void    orc_multadd_real_vector_complex_scalar(const int16_t *x, const int16_t *alpha, int16_t *y, uint32_t N);
int32_t orc_fo_channel_level(const int16_t *dl_ch, int N_RB);
int32_t orc_dot_product(const int16_t *x, const int16_t *y, uint32_t N, uint8_t shift);
int32_t orc_fo_omega(const orc_frame_t *fp, const int32_t *dl_ch_estimates0, int l);
void    orc_fo_update(int Ncp, int32_t omega, int *freq_offset, int *first_run);
void    orc_chest_time(const orc_frame_t *fp, const int32_t *dl_ch_estimates_plane, int32_t *time_out);

/* ---- dlsim's channel stage (PHY/TOOLS/signal_energy.c:66-110, SIMULATION/TOOLS/rangen_double.c:47-118,
 *      SIMULATION/LTE_PHY/dlsim.c:2852-2866) ---- */
int32_t orc_signal_energy(const int32_t *input, uint32_t length);
void    orc_randominit(uint32_t seed_init);
double  orc_uniformrandom(void);
double  orc_gaussdouble(double mean, double variance);
double  orc_awgn_sigma2(int32_t tx_lev, double offset_db);
void    orc_awgn(const int32_t *tx, int32_t *rx, uint32_t n, double sigma2);

/* ---- 8-bit turbo decoder (CODING/3gpplte_turbo_decoder_sse_8bit.c:846-1658), n % 16 == 0, n >= 512 ---- */
void    orc_td8_tables(int n, int *pi2, int *pi4, int *pi5, int *pi6);
int     orc_td8_input(const int16_t *y, int n, int8_t *y8);
uint8_t orc_turbo_decoder8(const int16_t *y, uint8_t *decoded_bytes, uint16_t n, uint8_t max_iterations,
                           uint8_t crc_type, uint8_t F);

#endif
