/*
 * openair4g_amd — MI355X-native LTE PDSCH transmit path, C ABI.
 *
 * Two surfaces:
 *
 *  1. Drop-in entry points mirroring the reference call surface of the DLSCH transmit path
 *     (erlgo/openair4G openair1/PHY).  Same argument meaning, same in-place side effects on
 *     caller-owned buffers, same return conventions; host buffers in, host buffers out, the
 *     arithmetic runs on the GPU.  The reference passes its own LTE_DL_FRAME_PARMS /
 *     LTE_eNB_DLSCH_t; here the fields the path touches are mirrored in oai4g_frame_parms_t /
 *     oai4g_dlsch_t (the reference-side shim that fills them is in INTEGRATION.md).
 *
 *  2. A batched, device-resident API (oai4g_tx_*) that runs whole subframes
 *     (encode -> rate-match -> scramble -> modulate/map -> IDFT + CP) for many subframes per
 *     launch, with payloads already in HBM.  This is the throughput path.
 *
 * Every entry point that computes returns/records an error if the HIP runtime or a gfx950
 * device is unavailable: there is no CPU fallback.  oai4g_last_error() gives the message.
 */
#ifndef OAI4G_H
#define OAI4G_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OAI4G_LTE_NULL 2                    /* PHY/CODING/defs.h:53 */
#define OAI4G_NSOFT 1827072                 /* PHY/LTE_TRANSPORT/defs.h:62 */
#define OAI4G_MAX_SEGMENTS 16               /* PHY/LTE_TRANSPORT/defs.h:67 */
#define OAI4G_MAX_CHANNEL_BITS (14 * 1200 * 6)
#define OAI4G_D_BYTES (96 + 12 + 3 + 3 * 6144)
#define OAI4G_W_BYTES (3 * 6144 + 96)

/* MIMO_mode_t subset (PHY/impl_defs_lte.h) */
enum { OAI4G_SISO = 0, OAI4G_ALAMOUTI = 1, OAI4G_LARGE_CDD = 2 };
/* Extension_t (PHY/MODULATION/defs.h) */
enum { OAI4G_CYCLIC_PREFIX = 0, OAI4G_CYCLIC_SUFFIX = 1, OAI4G_ZEROS = 2, OAI4G_NONE = 3 };

/* Fields of LTE_DL_FRAME_PARMS (PHY/impl_defs_lte.h:470-572) used on this path. */
typedef struct {
  uint16_t N_RB_DL;
  uint16_t Nid_cell;
  uint8_t Ncp;              /* 0 = normal CP, 1 = extended */
  uint8_t nushift;          /* Nid_cell % 6 */
  uint8_t mode1_flag;       /* 1 = single-port CRS (TM1) */
  uint8_t nb_antennas_tx;
  uint8_t frame_type;       /* 0 = FDD, 1 = TDD */
  uint8_t symbols_per_tti;
  uint8_t log2_symbol_size;
  uint8_t Nid_cell_mbsfn;   /* MBSFN area id (impl_defs_lte.h:482; 36.211 N_ID^MBSFN is 0..255) */
  uint16_t ofdm_symbol_size;
  uint16_t first_carrier_offset;
  uint16_t nb_prefix_samples;
  uint16_t nb_prefix_samples0;
  uint32_t samples_per_tti;
  /* control region (phich_config_common, tdd_config, nb_antennas_tx_eNB of LTE_DL_FRAME_PARMS) */
  uint8_t phich_resource;   /* PHICH_RESOURCE_t (impl_defs_lte.h:80-85): 1, 3, 6, 12 = Ng 1/6, 1/2, 1, 2 */
  uint8_t phich_duration;   /* 0 normal (extended is not supported by the PDCCH path) */
  uint8_t tdd_config;
  uint8_t nb_antennas_tx_eNB;
} oai4g_frame_parms_t;

/* DCI_ALLOC_t (PHY/LTE_TRANSPORT/defs.h:734-749) */
typedef struct {
  uint8_t dci_length;       /* bits */
  uint8_t L;                /* log2 aggregation level 0..3 */
  int32_t nCCE;             /* first CCE; < 0: not transmitted */
  uint8_t ra_flag;
  uint16_t rnti;
  uint32_t format;          /* DCI_format_t (not used by the encoder) */
  uint8_t dci_pdu[8];
} oai4g_dci_alloc_t;

/* LTE_DL_eNB_HARQ_t (PHY/LTE_TRANSPORT/defs.h:104-169), path fields only. */
typedef struct {
  uint32_t TBS;
  uint32_t B;
  uint8_t *b;
  uint8_t *c[OAI4G_MAX_SEGMENTS];
  uint32_t RTC[OAI4G_MAX_SEGMENTS];
  uint8_t round;
  uint8_t mcs;
  uint8_t rvidx;
  uint8_t mimo_mode;
  uint32_t rb_alloc[4];
  uint16_t nb_rb;
  uint8_t *e;                              /* OAI4G_MAX_CHANNEL_BITS bytes */
  uint8_t *d[OAI4G_MAX_SEGMENTS];          /* OAI4G_D_BYTES; first 96 = LTE_NULL */
  uint8_t *w[OAI4G_MAX_SEGMENTS];          /* OAI4G_W_BYTES */
  uint32_t C, Cminus, Cplus, Kminus, Kplus, F;
  uint8_t Nl;
  uint8_t Nlayers;
  uint8_t first_layer;
} oai4g_dl_harq_t;

/* LTE_eNB_DLSCH_t (PHY/LTE_TRANSPORT/defs.h:240-274), path fields only. */
typedef struct {
  uint16_t rnti;
  uint8_t current_harq_pid;
  uint8_t Mdlharq;
  uint8_t Kmimo;
  int16_t sqrt_rho_a;
  int16_t sqrt_rho_b;
  oai4g_dl_harq_t *harq_processes[8];
} oai4g_dlsch_t;

/* ---------------- library / device ----------------
 * The library runs on one device (oai4g_set_device before oai4g_init, else the current one).  Every
 * compute call makes that device the calling thread's current HIP device and leaves it so. */
int oai4g_init(void);                       /* idempotent; 0 on success, <0 if no usable GPU */
const char *oai4g_last_error(void);
int oai4g_device_name(char *buf, int len);

/* ---------------- parameter helpers (host-side, scalar) ---------------- */
/* init_frame_parms (PHY/INIT/lte_parms.c:31), osf = 1 */
int oai4g_init_frame_parms(oai4g_frame_parms_t *fp, uint16_t N_RB_DL, uint16_t Nid_cell, uint8_t Ncp,
                           uint8_t nb_antennas_tx, uint8_t mode1_flag, uint8_t frame_type);
/* get_Qm (lte_mcs.c:45), get_G (lte_mcs.c:336) */
uint8_t oai4g_get_Qm(uint8_t mcs);
int oai4g_get_G(const oai4g_frame_parms_t *fp, uint16_t nb_rb, const uint32_t *rb_alloc, uint8_t mod_order,
                uint8_t Nl, uint8_t num_pdcch_symbols, int frame, uint8_t subframe);
/* get_Qm_ul (lte_mcs.c:57), get_I_TBS (:69), get_I_TBS_UL (:84) */
uint8_t oai4g_get_Qm_ul(uint8_t mcs);
uint8_t oai4g_get_I_TBS(uint8_t mcs);
uint8_t oai4g_get_I_TBS_UL(uint8_t mcs);
/* TBStable[I_TBS][nb_rb-1] (LTE_TRANSPORT/dlsch_tbs_full.h:34, 36.213 Table 7.1.7.2.1-1) in bits,
 * 0 outside 0..26 x 1..110.  The reference's entry for I_TBS 6, 1 PRB is 328 (the spec's is 88);
 * the table keeps the reference's value. */
uint32_t oai4g_tbs_bits(uint8_t I_TBS, uint16_t nb_rb);
/* get_TBS_DL (lte_mcs.c:118) / get_TBS_UL (:137): TBS in BYTES, as the reference returns it;
 * 0 when nb_rb == 0 or mcs >= 29 */
uint32_t oai4g_get_TBS_DL(uint8_t mcs, uint16_t nb_rb);
uint32_t oai4g_get_TBS_UL(uint8_t mcs, uint16_t nb_rb);
/* new_eNB_dlsch / free_eNB_dlsch (dlsch_coding.c:120 / :85) */
oai4g_dlsch_t *oai4g_new_dlsch(uint8_t Kmimo, uint8_t Mdlharq, uint8_t N_RB_DL);
void oai4g_free_dlsch(oai4g_dlsch_t *dlsch);
/* lte_gold_generic (PHY/LTE_REFSIG/lte_gold.c:151): scalar 32-bit LFSR helper, host-side */
uint32_t oai4g_lte_gold_generic(uint32_t *x1, uint32_t *x2, uint8_t reset);

/* ---------------- drop-in entry points (GPU compute on host buffers) ---------------- */
/* crc24a / crc24b (PHY/CODING/crc_byte.c:117 / :135): returns crc << 8 */
uint32_t oai4g_crc24a(const uint8_t *in, int bitlen);
uint32_t oai4g_crc24b(const uint8_t *in, int bitlen);
/* lte_segmentation (PHY/CODING/lte_segmentation.c:39) */
int oai4g_lte_segmentation(const uint8_t *input_buffer, uint8_t **output_buffers, uint32_t B, uint32_t *C,
                           uint32_t *Cplus, uint32_t *Cminus, uint32_t *Kplus, uint32_t *Kminus, uint32_t *F);
/* threegpplte_turbo_encoder (PHY/CODING/3gpplte_sse.c:380, decl CODING/defs.h:315) */
void oai4g_threegpplte_turbo_encoder(const uint8_t *input, uint16_t input_length_bytes, uint8_t *output,
                                     uint8_t F, uint16_t interleaver_f1, uint16_t interleaver_f2);
/* sub_block_interleaving_turbo (lte_rate_matching.c:51, decl CODING/defs.h:112).
 * d points at &d[96] of a buffer whose 96 preceding bytes are readable (LTE_NULL). */
uint32_t oai4g_sub_block_interleaving_turbo(uint32_t D, uint8_t *d, uint8_t *w);
/* lte_rate_matching_turbo (lte_rate_matching.c:464, decl CODING/defs.h:191) */
uint32_t oai4g_lte_rate_matching_turbo(uint32_t RTC, uint32_t G, const uint8_t *w, uint8_t *e, uint8_t C,
                                       uint32_t Nsoft, uint8_t Mdlharq, uint8_t Kmimo, uint8_t rvidx,
                                       uint8_t Qm, uint8_t Nl, uint8_t r, uint8_t nb_rb, uint8_t m);
/* dlsch_encoding (PHY/LTE_TRANSPORT/dlsch_coding.c:254, decl proto.h:110) */
int oai4g_dlsch_encoding(uint8_t *a, const oai4g_frame_parms_t *frame_parms, uint8_t num_pdcch_symbols,
                         oai4g_dlsch_t *dlsch, int frame, uint8_t subframe);
/* dlsch_scrambling (PHY/LTE_TRANSPORT/dlsch_scrambling.c:51, decl proto.h:1600) */
void oai4g_dlsch_scrambling(const oai4g_frame_parms_t *frame_parms, int mbsfn_flag, oai4g_dlsch_t *dlsch, int G,
                            uint8_t q, uint8_t Ns);
/* dlsch_modulation (PHY/LTE_TRANSPORT/dlsch_modulation.c:1181, decl proto.h:197).
 * txdataF[aa] is the caller's whole-frame grid as in the reference (indexed by
 * ofdm_symbol_size*(l + subframe_offset*nsymb)).  Returns REs allocated, or -1. */
int oai4g_dlsch_modulation(int32_t **txdataF, int16_t amp, uint32_t subframe_offset,
                           const oai4g_frame_parms_t *frame_parms, uint8_t num_pdcch_symbols,
                           oai4g_dlsch_t *dlsch0, oai4g_dlsch_t *dlsch1);
/* PHY_ofdm_mod (PHY/MODULATION/ofdm_mod.c:85, decl MODULATION/defs.h:48); CYCLIC_PREFIX only */
void oai4g_PHY_ofdm_mod(const int32_t *input, int32_t *output, uint8_t log2fftsize, uint8_t nb_symbols,
                        uint16_t nb_prefix_samples, int etype);
/* normal_prefix_mod (ofdm_mod.c:47, decl MODULATION/defs.h:88) */
void oai4g_normal_prefix_mod(const int32_t *txdataF, int32_t *txdata, uint8_t nsymb,
                             const oai4g_frame_parms_t *frame_parms);
/* do_OFDM_mod (ofdm_mod.c:233, decl MODULATION/defs.h:90); PMCH subframes not supported */
void oai4g_do_OFDM_mod(int32_t **txdataF, int32_t **txdata, uint32_t frame, uint16_t next_slot,
                       const oai4g_frame_parms_t *frame_parms);
/* generate_pilots (PHY/LTE_TRANSPORT/pilots.c:43, decl proto.h): CRS into txdataF[ant] for
 * Ntti subframes (the reference's frame grid; overwrites the pilot REs).  The reference passes
 * PHY_VARS_eNB for its frame parameters and Gold table; here the table is derived from fp. */
void oai4g_generate_pilots(int32_t **txdataF, int16_t amp, const oai4g_frame_parms_t *frame_parms, uint16_t Ntti);
/* lte_dl_cell_spec (PHY/LTE_REFSIG/lte_dl_cell_spec.c:123): CRS of port p, pilot l (0/1) of slot
 * Ns into one OFDM symbol `output` (ofdm_symbol_size REs).  Returns 0, or -1 for a bad port. */
int oai4g_lte_dl_cell_spec(int32_t *output, int16_t amp, const oai4g_frame_parms_t *frame_parms, uint8_t Ns,
                           uint8_t l, uint8_t p);
/* idft64..idft2048 (PHY/TOOLS/lte_dfts.c:1856-2866 incl. idft512 :2479, decl TOOLS/defs.h:555): y = IDFT(x) */
int oai4g_idft(int log2n, const int16_t *x, int16_t *y, int scale);
void oai4g_idft2048(const int16_t *x, int16_t *y, int scale);
void oai4g_idft1024(const int16_t *x, int16_t *y, int scale);
void oai4g_idft512(const int16_t *x, int16_t *y, int scale);   /* lte_dfts.c:2479 */
void oai4g_idft256(const int16_t *x, int16_t *y, int scale);
void oai4g_idft128(const int16_t *x, int16_t *y, int scale);
void oai4g_idft64(const int16_t *x, int16_t *y, int scale);

/* ---------------- control region of the transmit grid ---------------- */
/* generate_pcfich_reg_mapping (PHY/LTE_TRANSPORT/pcfich.c:48): REG indices (units of 6 REs) and
 * the index of the lowest; prints them as the reference does. */
void oai4g_generate_pcfich_reg_mapping(const oai4g_frame_parms_t *frame_parms, uint16_t pcfich_reg[4],
                                       uint8_t *pcfich_first_reg_idx);
/* generate_pcfich (pcfich.c:144, decl LTE_TRANSPORT/proto.h:1432): CFI codeword, scrambling, QPSK
 * (SISO / ALAMOUTI) and REG mapping into symbol 0 of `subframe` of the frame grids txdataF[ant]
 * (overwrites 16 REs per antenna).  Returns 0, or -1 (num_pdcch_symbols outside 1..3). */
int oai4g_generate_pcfich(uint8_t num_pdcch_symbols, int16_t amp, const oai4g_frame_parms_t *frame_parms,
                          int32_t **txdataF, uint8_t subframe);

/* PDCCH geometry (host-side scalar helpers): get_mi (phich.c:59), get_nquad / get_nCCE
 * (dci.c:2494-2538), get_num_pdcch_symbols (dci.c:1964), generate_phich_reg_mapping
 * (phich.c:280; normal duration: returns the number of groups written into phich_reg[56][3]),
 * get_nCCE_offset (SCHED/phy_procedures_lte_eNb.c:308, over the library's CCE table, cleared by
 * oai4g_init_nCCE_table as init_nCCE_table :302 does; not thread-safe, like the reference) */
uint8_t oai4g_get_mi(const oai4g_frame_parms_t *frame_parms, uint8_t subframe);
uint16_t oai4g_get_nquad(uint8_t num_pdcch_symbols, const oai4g_frame_parms_t *frame_parms, uint8_t mi);
uint16_t oai4g_get_nCCE(uint8_t num_pdcch_symbols, const oai4g_frame_parms_t *frame_parms, uint8_t mi);
uint8_t oai4g_get_num_pdcch_symbols(uint8_t num_dci, const oai4g_dci_alloc_t *dci_alloc,
                                    const oai4g_frame_parms_t *frame_parms, uint8_t subframe);
int oai4g_generate_phich_reg_mapping(const oai4g_frame_parms_t *frame_parms, uint16_t phich_reg[56][3]);
void oai4g_init_nCCE_table(void);
int oai4g_get_nCCE_offset(uint8_t L, int nCCE, int common_dci, uint16_t rnti, uint8_t subframe);
/* generate_dci_top (PHY/LTE_TRANSPORT/dci.c:2024, decl LTE_TRANSPORT/proto.h): PCFICH + every
 * DCI (CRC16 with the RNTI mask, tail-biting convolutional code, rate matching to 72 * 2^L bits
 * at CCE nCCE), <NIL> filling, scrambling, QPSK (SISO / ALAMOUTI), quadruplet interleaving with
 * the cell-id cyclic shift and the REG mapping around the PCFICH / PHICH REGs, into the control
 * symbols of `subframe` of the frame grids txdataF[0..1] (overwrites).  Returns
 * num_pdcch_symbols; when that is outside 1..3 (too many CCEs, or an N_RB_DL without a PDCCH
 * geometry in get_nquad: 15 / 75) nothing is written (the reference maps an undefined CFI
 * codeword there) and oai4g_last_error() says why. */
uint8_t oai4g_generate_dci_top(uint8_t num_ue_spec_dci, uint8_t num_common_dci, const oai4g_dci_alloc_t *dci_alloc,
                               uint32_t n_rnti, int16_t amp, const oai4g_frame_parms_t *frame_parms,
                               int32_t **txdataF, uint32_t subframe);

/* ---------------- UE PDSCH demodulation (second half) ---------------- */
/* rx_pdsch (PHY/LTE_TRANSPORT/dlsch_demodulation.c:82) over the PDSCH symbols of one subframe as
 * dlsim runs it (dlsim.c:3188-3260): dlsch_extract_rbs_single (:3167), dlsch_channel_level (:2777)
 * -> log2_maxh, dlsch_channel_compensation (:801) and dlsch_qpsk / 16qam / 64qam_llr
 * (dlsch_llr_computation.c:636, 688, 810).  Transmission mode 1 (one TX port), one receive
 * antenna, every N_RB_DL (the odd 15 / 25 PRB extraction around the DC carrier included; a
 * subframe whose extraction would read slots the reference leaves unwritten returns -1), the
 * first PDSCH symbol without pilots.  rxdataF and dl_ch_estimates are one subframe, [nsymb][N]
 * each (estimate of subcarrier 12 rb + i at entry 5 + 12 rb + i of its symbol, the layout of the
 * reference's estimator and of dlsim's perfect-CE mode, dlsim.c:2935-2966).  Writes the LLR
 * stream (not unscrambled) and log2_maxh; returns its length or -1. */
int oai4g_rx_pdsch_siso(const oai4g_frame_parms_t *frame_parms, const int32_t *rxdataF, const int32_t *dl_ch_estimates,
                        const uint32_t rb_alloc[4], uint8_t Qm, uint8_t num_pdcch_symbols, uint8_t subframe,
                        int16_t *llr, uint8_t *log2_maxh);
/* dlsch_unscrambling (dlsch_scrambling.c:99, decl LTE_TRANSPORT/proto.h): llr[k] *= 2 c(k) - 1
 * for k < 32 (1 + G / 32) with c_init = rnti 2^14 + q 2^13 + (Ns / 2) 2^9 + Nid_cell, or with
 * mbsfn_flag != 0 (PMCH) c_init = (Ns / 2) 2^9 + Nid_cell_mbsfn (:115-118).  The reference reads
 * rnti from its LTE_UE_DLSCH_t. */
void oai4g_dlsch_unscrambling(const oai4g_frame_parms_t *frame_parms, int mbsfn_flag, uint16_t rnti, int G,
                              int16_t *llr, uint8_t q, uint8_t Ns);
/* Batched demodulation: n_sf subframes (subframe index first_subframe + i * subframe_step mod 10)
 * of rxdataF and per-symbol channel estimates ([n_sf][nsymb][N] int32 each, device) -> LLR
 * streams [n_sf][oai4g_rx_llr_stride] int16 (device), unscrambled (q = 0, Ns = 2 subframe) when
 * unscramble != 0.  The demodulator is elementwise per RE after the per-subframe channel level. */
typedef struct oai4g_rx_config oai4g_rx_config_t;
oai4g_rx_config_t *oai4g_rx_config_create(const oai4g_frame_parms_t *frame_parms, const uint32_t rb_alloc[4], uint8_t Qm,
                                          uint8_t num_pdcch_symbols, uint16_t rnti, uint8_t first_subframe,
                                          uint8_t subframe_step);
void oai4g_rx_config_destroy(oai4g_rx_config_t *cfg);
int oai4g_rx_llr_count(const oai4g_rx_config_t *cfg, int subframe_index);
size_t oai4g_rx_llr_stride(const oai4g_rx_config_t *cfg);
int oai4g_rx_batch(oai4g_rx_config_t *cfg, int n_sf, const int32_t *d_rxdataF, const int32_t *d_dl_ch_estimates,
                   int16_t *d_llr, int unscramble, void *stream);

/* TM3 (LARGE_CDD, two TX ports) with dlsim's UE (rx_pdsch with dual_stream_flag = 0,
 * dlsch_demodulation.c:82-800): dlsch_extract_rbs_dual, dlsch_channel_level_TM3 + log2_maxh,
 * dlsch_channel_compensation_TM3 (prec2A_TM3), dlsch_detection_mrc over nb_rx (1-2) receive
 * antennas, then codeword 0's LLRs: the single-stream 16 / 64-QAM LLRs for Qm0 4 / 6 (the reference
 * computes no codeword-1 LLRs there); for Qm0 = 2 the interference-aware dlsch_qpsk_qpsk_llr /
 * dlsch_qpsk_16qam_llr / dlsch_qpsk_64qam_llr against codeword 1 of modulation order Qm1
 * (dlsch_demodulation.c:643-690, dlsch_llr_computation.c:983, :1232, :1516).  Drop-in on host
 * buffers: rxdataF[a] = [nsymb][N] per receive
 * antenna, dl_ch_estimates[p * 2 + a] = [nsymb][N] (the reference's dl_ch_estimates[(p << 1) + a]).
 * Returns the LLR count (not unscrambled) or -1. */
int oai4g_rx_pdsch_tm3(const oai4g_frame_parms_t *frame_parms, int nb_rx, const int32_t *const *rxdataF,
                       const int32_t *const *dl_ch_estimates, const uint32_t rb_alloc[4], uint8_t Qm0, uint8_t Qm1,
                       uint8_t mcs0, uint8_t num_pdcch_symbols, uint8_t subframe, int16_t *llr, uint8_t *log2_maxh);
/* Batched TM3 demodulation: d_rxdataF = [n_sf][nb_rx][nsymb][N] (the FEP batch output),
 * d_est = four planes [p * 2 + a][n_sf][nsymb][N] (channel estimation batches of ports 0 / 1 per
 * receive antenna) -> codeword 0's LLR streams [n_sf][oai4g_rx_llr_stride] (unscrambled when asked). */
oai4g_rx_config_t *oai4g_rx_config_create_tm3(const oai4g_frame_parms_t *frame_parms, const uint32_t rb_alloc[4],
                                              uint8_t Qm0, uint8_t Qm1, uint8_t mcs0, uint8_t num_pdcch_symbols,
                                              uint16_t rnti, uint8_t first_subframe, uint8_t subframe_step, uint8_t nb_rx);
int oai4g_rx_batch_tm3(oai4g_rx_config_t *cfg, int n_sf, const int32_t *d_rxdataF, const int32_t *d_est, int16_t *d_llr,
                       int unscramble, void *stream);

/* TM3 with both codewords QPSK (rx_pdsch, dlsch_demodulation.c:643-669): both precoded streams'
 * matched filters, dlsch_dual_stream_correlation (rho, rho2), the MRC of stream 0 and rho, and the
 * interference-aware dlsch_qpsk_qpsk_llr of each stream: codeword 0's LLRs in llr0, codeword 1's in
 * llr1 (same length, returned; -1 on error). */
int oai4g_rx_pdsch_tm3_2cw(const oai4g_frame_parms_t *frame_parms, int nb_rx, const int32_t *const *rxdataF,
                           const int32_t *const *dl_ch_estimates, const uint32_t rb_alloc[4], uint8_t mcs0,
                           uint8_t num_pdcch_symbols, uint8_t subframe, int16_t *llr0, int16_t *llr1,
                           uint8_t *log2_maxh);
/* batch of the same (configuration from oai4g_rx_config_create_tm3 with Qm0 = Qm1 = 2) */
int oai4g_rx_batch_tm3_2cw(oai4g_rx_config_t *cfg, int n_sf, const int32_t *d_rxdataF, const int32_t *d_est,
                           int16_t *d_llr0, int16_t *d_llr1, int unscramble, void *stream);
/* The same two TM3 batches from the pilot rows only: d_pil = four planes [p * 2 + a][n_sf][4][N][2]
 * written by oai4g_chest_batch_pilots (plane p * 2 + a from a port-p configuration over receive
 * antenna a). Every other estimate row is formed in the demodulator with
 * lte_dl_channel_estimation's temporal interpolation (lte_dl_channel_estimation.c:639-698), so the
 * 14-row estimate planes never reach memory. The LLRs are bit-identical. */
int oai4g_rx_batch_tm3_pilots(oai4g_rx_config_t *cfg, int n_sf, const int32_t *d_rxdataF, const int32_t *d_pil,
                              int16_t *d_llr, int unscramble, void *stream);
int oai4g_rx_batch_tm3_2cw_pilots(oai4g_rx_config_t *cfg, int n_sf, const int32_t *d_rxdataF, const int32_t *d_pil,
                                  int16_t *d_llr0, int16_t *d_llr1, int unscramble, void *stream);

/* TM2 (ALAMOUTI, two TX ports, mode1_flag 0) with dlsim's UE (rx_pdsch, dlsch_demodulation.c:82-800):
 * dlsch_extract_rbs_dual, dlsch_channel_level over both ports (log2_maxh = log2_approx(max avg) / 2),
 * dlsch_channel_compensation per (port, RX antenna), dlsch_detection_mrc over nb_rx (1-2),
 * dlsch_alamouti over pairs of extracted REs, dlsch_qpsk / 16qam / 64qam_llr.  Same buffers as the
 * TM3 entry points (estimate planes [p * 2 + a]).  Returns the LLR count (not unscrambled) or -1. */
int oai4g_rx_pdsch_tm2(const oai4g_frame_parms_t *frame_parms, int nb_rx, const int32_t *const *rxdataF,
                       const int32_t *const *dl_ch_estimates, const uint32_t rb_alloc[4], uint8_t Qm,
                       uint8_t num_pdcch_symbols, uint8_t subframe, int16_t *llr, uint8_t *log2_maxh);
oai4g_rx_config_t *oai4g_rx_config_create_tm2(const oai4g_frame_parms_t *frame_parms, const uint32_t rb_alloc[4],
                                              uint8_t Qm, uint8_t num_pdcch_symbols, uint16_t rnti,
                                              uint8_t first_subframe, uint8_t subframe_step, uint8_t nb_rx);
int oai4g_rx_batch_tm2(oai4g_rx_config_t *cfg, int n_sf, const int32_t *d_rxdataF, const int32_t *d_est, int16_t *d_llr,
                       int unscramble, void *stream);

/* lte_dl_channel_estimation (PHY/LTE_ESTIMATION/lte_dl_channel_estimation.c:37, decl
 * LTE_ESTIMATION/defs.h; called by slot_fep.c:188 for the pilot symbols of every slot) with the
 * reference's defaults high_speed_flag = 1 (dlsim.c:2057), eNB_offset 0, one RX antenna: the
 * frequency interpolation of the conjugate-pilot products of port p (filt96_32.h filters) into row
 * `symbol` of dl_ch_estimates (subcarrier i of RB rb at 5 + 12 rb + i), then the temporal
 * interpolation of the rows between this pilot symbol and the previous one (symbol 0 closes rows
 * 12 / 13 of the previous subframe's pilot 11).  rxdataF / dl_ch_estimates = [nsymb][N] host
 * buffers of the subframe; N_RB_DL 6 / 15 / 25 / 50 / 100 (other sizes: the reference's "not
 * implemented" row of zeros; 15 PRB with its second-half start 1 + nushift + 3 p, :582).  The idft of the estimate into
 * dl_ch_estimates_time (:704-738) is the separate entry oai4g_dl_ch_estimates_time below, which the
 * shim calls after this one.  Returns 0 / -1. */
int oai4g_lte_dl_channel_estimation(const oai4g_frame_parms_t *frame_parms, const int32_t *rxdataF,
                                    int32_t *dl_ch_estimates, uint8_t Ns, uint8_t p, uint8_t l, uint8_t symbol);
/* The tail of lte_dl_channel_estimation (lte_dl_channel_estimation.c:704-738): for every RX antenna
 * aarx < nb_antennas_rx and port p < nb_antennas_tx_eNB (nb_antennas_tx when 0) whose plane
 * dl_ch_estimates[(p << 1) + aarx] is not NULL, dl_ch_estimates_time[(p << 1) + aarx] =
 * idft_N(plane from word 8, scale 1): words 8 .. N + 7 (row 0 then the first 8 words of row 1),
 * N = ofdm_symbol_size (log2_symbol_size outside 7..11: idft512, the switch's default).  The
 * input of the UE timing tracker (lte_adjust_sync.c:60-70).  Returns 0 / -1. */
int oai4g_dl_ch_estimates_time(const oai4g_frame_parms_t *frame_parms, int nb_antennas_rx,
                               const int32_t *const *dl_ch_estimates, int32_t *const *dl_ch_estimates_time);
/* Batched form: job j transforms d_est[j * est_stride + 8 ...] into d_time[j * time_stride ...]
 * (est_stride >= N + 8, time_stride >= N words); device pointers, async on `stream`. */
int oai4g_chest_time_batch(const oai4g_frame_parms_t *frame_parms, int n_jobs, const int32_t *d_est,
                           size_t est_stride, int32_t *d_time, size_t time_stride, void *stream);

/* lte_est_freq_offset (PHY/LTE_ESTIMATION/lte_est_freq_offset.c:104-193, called by slot_fep.c:211-217
 * at l = 4 - Ncp): antenna 0's plane dl_ch_estimates[0]; dl_ch_shift = 6 + log2_approx(
 * dl_channel_level(row l from RE 12)) / 2; omega as the reference computes it: its dot_product
 * (cdot_prod.c:40) of row l against the other pilot row (row 4 - Ncp when l = 0, else row 0) over
 * (N_RB_DL / 2 - 1) * 12 REs from RE (N_RB_DL / 2 + 1) * 12, doubled (int16 wrap per component) — the
 * lower-half product from RE 12 is overwritten through the omega_cpx alias (:150-166) and never
 * counts; freq_offset_est = (int)(atan2(omega) / 2 pi / 285.8 us
 * (normal CP) or 250 us); the first call (or one with reset != 0) stores it, later calls filter
 * (est * 2^10 + f * (32767 - 2^10)) >> 15.  The filter state is process-wide, as the reference's
 * static first_run.  The dot products run on the GPU; atan2 and the filter are the host's scalar
 * tail, as in the reference.  Returns 0, or -1 for l other than 0 / 4 - Ncp (freq_offset untouched). */
int oai4g_lte_est_freq_offset(int32_t *const *dl_ch_estimates, const oai4g_frame_parms_t *frame_parms, int l,
                              int *freq_offset, int reset);
/* Batched integer part: omega (re | im << 16) of n_jobs estimate planes d_est[j * est_stride ...]
 * (rows 0 .. 4 - Ncp present) into d_omega[j]; then oai4g_freq_offset_update applies the scalar
 * tail of one call per omega with a caller-held first_run (1 = the reference's first run). */
int oai4g_freq_offset_omega_batch(const oai4g_frame_parms_t *frame_parms, int n_jobs, const int32_t *d_est,
                                  size_t est_stride, int l, int32_t *d_omega, void *stream);
int oai4g_freq_offset_update(const oai4g_frame_parms_t *frame_parms, int32_t omega, int *freq_offset, int *first_run);
/* The six interpolation filters of pilot offset k = (nu + nushift) % 6 as the estimator uses them
 * (lte_dl_channel_estimation.c:105-180): fl, f2l2, f, f2, fr, f2r2 (filt96_32.h by formula). */
void oai4g_chest_filters(uint8_t k, int16_t out[6][24]);
/* The 25-PRB branch's DC pair (lte_dl_channel_estimation.c:116-173): filt24_k_dcr, filt24_(k+2)_dcl
 * (filt96_32.h table data). */
void oai4g_chest_dc_filters(uint8_t k, int16_t out[2][24]);
/* Batched estimation of every symbol of n_sf consecutive subframes (subframe index first_subframe
 * + i * subframe_step mod 10) in dlsim's order (dlsim.c:2907-2931): d_rxdataF = [n_sf][nsymb][N]
 * followed by the symbol 0 of the subframe after the batch (N more words), d_est = [n_sf][nsymb][N]
 * -- the rows rx_pdsch reads for each subframe (row 0 that subframe's own estimate). */
typedef struct oai4g_chest_config oai4g_chest_config_t;
oai4g_chest_config_t *oai4g_chest_config_create(const oai4g_frame_parms_t *frame_parms, uint8_t p,
                                                uint8_t first_subframe, uint8_t subframe_step);
void oai4g_chest_config_destroy(oai4g_chest_config_t *cfg);
/* Batch elements `subframes_per_element` subframes apart in d_rxdataF, the symbol 0 that closes rows
 * 12 / 13 `next_subframes` subframes after each element's start (default 1 / 1).  dlsim's BLER loop:
 * 2 / 1 (each trial's subframe followed by the next one); a receive antenna of an n-antenna FEP
 * batch: n / n (pass d_rxdataF + a nsymb N). */
int oai4g_chest_config_set_stride(oai4g_chest_config_t *cfg, uint32_t subframes_per_element, uint32_t next_subframes);
int oai4g_chest_batch(oai4g_chest_config_t *cfg, int n_sf, const int32_t *d_rxdataF, int32_t *d_est, void *stream);
/* The pilot rows only: per subframe the 5 frequency-interpolated rows P0..P4 of symbols 0, p1, p2,
 * p3 and the next subframe's symbol 0, stored as the pairs of consecutive rows: d_pil =
 * [n_sf][4][N][2] words, pair k at column j = (P_k[j], P_k+1[j]); columns below 12 N_RB + 16 (the
 * others are not written). They feed oai4g_rx_batch_tm3_pilots. */
int oai4g_chest_batch_pilots(oai4g_chest_config_t *cfg, int n_sf, const int32_t *d_rxdataF, int32_t *d_pil,
                             void *stream);
/* The batch chain without the estimate buffer: oai4g_chest_batch followed by oai4g_rx_batch, fused
 * (the estimate of each PDSCH RE is formed in LDS from the pilot rows), same LLRs; d_rxdataF as
 * for oai4g_chest_batch (n_sf subframes + the next symbol 0).  rx and ce describe the same frame
 * and subframe sequence (port 0). */
int oai4g_rx_batch_estimated(oai4g_rx_config_t *rx, oai4g_chest_config_t *ce, int n_sf, const int32_t *d_rxdataF,
                             int16_t *d_llr, int unscramble, void *stream);

/* ---------------- synchronisation, broadcast and HARQ-indicator channels ---------------- */
/* generate_pss (PHY/LTE_TRANSPORT/pss.c:50, decl LTE_TRANSPORT/proto.h): the Zadoff-Chu sequence
 * of root 25 / 29 / 34 (Nid_cell % 3, the Q15 table of PHY/LTE_REFSIG/primary_synch.h, here
 * generated as floor(32767 x)) scaled (a v) >> 15, a = amp or (amp 23170) >> 15 with two antennas,
 * on the 62 subcarriers around DC of symbol `symbol` of slot `slot_offset` of every frame grid
 * txdataF[ant] (overwrites).  Returns 0. */
int oai4g_generate_pss(int32_t **txdataF, int16_t amp, const oai4g_frame_parms_t *frame_parms, uint16_t symbol,
                       uint16_t slot_offset);
/* generate_sss (sss.c:47): d0_sss / d5_sss (PHY/LTE_TRANSPORT/sss.h, 36.211 6.11.2.1 m-sequences,
 * slot_offset < 3 selects d0) as (a d, 0) on the same 62 subcarriers.  Returns 0. */
int oai4g_generate_sss(int32_t **txdataF, int16_t amp, const oai4g_frame_parms_t *frame_parms, uint16_t symbol,
                       uint16_t slot_offset);
/* LTE_eNB_PBCH (LTE_TRANSPORT/defs.h): the scrambled coded bits, one byte per bit, computed when
 * frame_mod4 == 0 and mapped a quarter per frame */
typedef struct {
  uint8_t pbch_e[1920];
} oai4g_pbch_t;
/* generate_pbch (pbch.c:161): MIB (pbch_pdu[0..2]), CRC16 with the antenna mask, tail-biting
 * convolutional code, rate matching to 1920 (1728) bits and scrambling (frame_mod4 == 0), then
 * quarter frame_mod4 in QPSK (SISO / ALAMOUTI) on slot 1 symbols 0..3 of the subframe-0 grids
 * txdataF[ant] ('+='), around the RS positions.  Returns 0. */
int oai4g_generate_pbch(oai4g_pbch_t *eNB_pbch, int32_t **txdataF, int amp, const oai4g_frame_parms_t *frame_parms,
                        const uint8_t *pbch_pdu, uint8_t frame_mod4);
/* generate_phich (phich.c:401, normal cyclic prefix): HI -> BPSK x3, orthogonal sequence nseq,
 * scrambling, SISO / ALAMOUTI, onto the three REGs of group ngroup in symbol 0 of `subframe` of the
 * frame grids y[ant] ('+=').  The reference returns void; here 0, or -1 for what it does not
 * define (extended CP, extended PHICH duration, nushift >= 3 where phich.c:563-569 reads past its
 * 8-entry arrays, ngroup / nseq out of range). */
int oai4g_generate_phich(const oai4g_frame_parms_t *frame_parms, int16_t amp, uint8_t nseq_PHICH, uint8_t ngroup_PHICH,
                         uint8_t HI, uint8_t subframe, int32_t **y);
/* generate_phich_top's group / sequence of an uplink allocation (phich.c:1449-1465, FDD):
 * ngroup = (first_rb + n_DMRS) mod Ngroup, nseq = (first_rb / Ngroup + n_DMRS) mod 2 NSF. */
int oai4g_phich_group_seq(const oai4g_frame_parms_t *frame_parms, uint16_t first_rb, uint8_t n_DMRS, uint8_t *ngroup_PHICH,
                          uint8_t *nseq_PHICH);

/* ---------------- UE receive front end ---------------- */
/* dft64..dft2048 (PHY/TOOLS/lte_dfts.c:1766, 1957, 2172, 2359, 2574, 2689; decl TOOLS/defs.h):
 * y = DFT(x), bit-exact fixed point.  oai4g_dft returns 0 or -1. */
int oai4g_dft(int log2n, const int16_t *x, int16_t *y, int scale);
void oai4g_dft2048(const int16_t *x, int16_t *y, int scale);
void oai4g_dft1024(const int16_t *x, int16_t *y, int scale);
void oai4g_dft512(const int16_t *x, int16_t *y, int scale);
void oai4g_dft256(const int16_t *x, int16_t *y, int scale);
void oai4g_dft128(const int16_t *x, int16_t *y, int scale);
void oai4g_dft64(const int16_t *x, int16_t *y, int scale);
/* slot_fep's DFT window start (slot_fep.c:55-150) before the % frame_length; -1 for bad l / Ns */
int64_t oai4g_slot_fep_offset(const oai4g_frame_parms_t *frame_parms, uint8_t l, uint8_t Ns, int sample_offset,
                              int no_prefix);
/* slot_fep (PHY/MODULATION/slot_fep.c:40, decl MODULATION/defs.h): the reference passes
 * PHY_VARS_UE; here its rxdata / rxdataF / frame parameters / antenna count are explicit.
 * rxdata[aa]: 10 * samples_per_tti + ofdm_symbol_size words (wrap extension, written as the
 * reference does); rxdataF[aa]: symbols_per_tti * ofdm_symbol_size words.  Returns 0 or -1.
 * Channel estimation (perfect_ce == 0 branch, :179-222) is not included. */
int oai4g_slot_fep(int32_t *const *rxdata, int32_t *const *rxdataF, const oai4g_frame_parms_t *frame_parms,
                   uint8_t nb_antennas_rx, uint8_t l, uint8_t Ns, int sample_offset, int no_prefix);
/* Batched FEP, device pointers: d_rx [n_sf][n_ant][samples_per_tti] -> d_rxF
 * [n_sf][n_ant][symbols_per_tti][ofdm_symbol_size] (every symbol of both slots, sample_offset 0).
 * Asynchronous on `stream` (a hipStream_t, NULL = default). */
int oai4g_fep_batch(const oai4g_frame_parms_t *frame_parms, int n_sf, int n_ant, const int32_t *d_rx,
                    int32_t *d_rxF, void *stream);

/* ---------------- dlsim's channel stage (SIMULATION/LTE_PHY/dlsim.c:2714-2866) ---------------- */
/* signal_energy (PHY/TOOLS/signal_energy.c:66, decl TOOLS/defs.h): mean of (re^2 + im^2) >> 4 over
 * `length` complex int16 samples minus the squared DC, with the SSE code's integer wraps; >= 1. */
int32_t oai4g_signal_energy(const int32_t *input, uint32_t length);
/* Batched, device pointers: d_energy[i] = signal_energy(d_x + i * stride, length) — dlsim's tx_lev
 * of one transmit antenna (:2714-2719).  Asynchronous on `stream`. */
int oai4g_signal_energy_batch(const int32_t *d_x, int n, size_t stride, uint32_t length, int32_t *d_energy,
                              void *stream);
/* dlsim's AWGN (:2852-2866), device pointers, n <= 65535 vectors: vector i is the tx_len samples at
 * d_tx + i * tx_stride followed by the tail_len samples of the common d_tail (dlsim adds the noise
 * over two subframes, the second carrying only the next subframe's CRS); d_rx + i * rx_stride gets
 * (short)(s + sqrt(sigma2_i / 2) g) per I / Q component with sigma2_i in dB = 10 log10(d_tx_lev[i])
 * + offset_db (offset_db = 10 log10(N / (12 NB_RB)) - SNR - pa_dB) and g ~ N(0, 1) from a counter-
 * based stream keyed by (seed, first_vector + i, sample).  Asynchronous on `stream`. */
int oai4g_awgn_batch(const int32_t *d_tx, size_t tx_stride, uint32_t tx_len, const int32_t *d_tail, uint32_t tail_len,
                     int32_t *d_rx, size_t rx_stride, int n, const int32_t *d_tx_lev, double offset_db, uint64_t seed,
                     uint32_t first_vector, void *stream);

/* ---------------- uplink turbo decoding ---------------- */
enum { OAI4G_CRC24_A = 0, OAI4G_CRC24_B = 1 };
/* phy_threegpplte_turbo_decoder16 (PHY/CODING/3gpplte_turbo_decoder_sse_16bit.c:945, decl
 * CODING/defs.h): y = 3n+12 int16 LLRs (&d[96]), positive = bit 1.  Returns the iteration count,
 * max_iterations+1 when no CRC check passes, 255 on bad arguments (CRC16 / CRC8 unsupported). */
uint8_t oai4g_phy_threegpplte_turbo_decoder16(const int16_t *y, uint8_t *decoded_bytes, uint16_t n, uint16_t f1,
                                              uint16_t f2, uint8_t max_iterations, uint8_t crc_type, uint8_t F);
/* lte_rate_matching_turbo_rx (PHY/CODING/lte_rate_matching.c:688, decl CODING/defs.h) */
int oai4g_lte_rate_matching_turbo_rx(uint32_t RTC, uint32_t G, int16_t *w, const uint8_t *dummy_w,
                                     const int16_t *soft_input, uint8_t C, uint32_t Nsoft, uint8_t Mdlharq,
                                     uint8_t Kmimo, uint8_t rvidx, uint8_t clear, uint8_t Qm, uint8_t Nl, uint8_t r,
                                     uint32_t *E_out);
/* sub_block_deinterleaving_turbo (lte_rate_matching.c:193): d points at &d[96] (96 writable
 * entries before it), w holds 3*Kpi entries */
void oai4g_sub_block_deinterleaving_turbo(uint32_t D, int16_t *d, const int16_t *w);
/* Batched decoder, device pointers: n_cb blocks of size K, llr [n_cb][llr_stride] int16
 * (3K+12 each), out [n_cb][out_stride] bytes (K/8 each), iters [n_cb]; scratch of
 * oai4g_td_scratch_bytes(K, n_cb) bytes.  Asynchronous on `stream`.  As the reference's
 * decoded_bytes, a block's out row is written only by hard decisions (iteration >= 2): with
 * max_iterations = 1 it keeps the caller's previous contents. */
size_t oai4g_td_scratch_bytes(uint16_t K, int n_cb);
int oai4g_td_batch(int n_cb, uint16_t K, const int16_t *d_llr, size_t llr_stride, uint8_t *d_out, size_t out_stride,
                   uint8_t *d_iters, uint8_t max_iterations, uint8_t crc_type, uint8_t F, void *d_scratch,
                   void *stream);

/* phy_threegpplte_turbo_decoder8 (PHY/CODING/3gpplte_turbo_decoder_sse_8bit.c:894, decl CODING/defs.h):
 * the 8-bit decoder (16 windows of int8 lanes, inputs scaled by their |LLR| mean).  Restated for
 * n % 16 == 0 and n >= 512 (other sizes: the reference reads past its interleaver tables) and
 * CRC24_A / CRC24_B; returns 255 outside that scope.  f1 / f2 are implied by n. */
uint8_t oai4g_phy_threegpplte_turbo_decoder8(const int16_t *y, uint8_t *decoded_bytes, uint16_t n, uint16_t f1,
                                             uint16_t f2, uint8_t max_iterations, uint8_t crc_type, uint8_t F);
/* Batched 8-bit decoder, device pointers as oai4g_td_batch; llr rows of >= 3K + 16 int16 (the
 * last 4 are read by the input scaling only); scratch of oai4g_td8_scratch_bytes(K, n_cb). */
size_t oai4g_td8_scratch_bytes(uint16_t K, int n_cb);
int oai4g_td8_batch(int n_cb, uint16_t K, const int16_t *d_llr, size_t llr_stride, uint8_t *d_out, size_t out_stride,
                    uint8_t *d_iters, uint8_t max_iterations, uint8_t crc_type, uint8_t F, void *d_scratch,
                    void *stream);

/* generate_dummy_w (PHY/CODING/lte_rate_matching.c:293, decl CODING/defs.h): marks LTE_NULL in w at
 * the NULL / filler positions of the 3 Kpi circular buffer of a block of D = K + 4 bits with F
 * filler bits (other entries untouched, as the reference); returns R = ceil(D / 32). */
uint32_t oai4g_generate_dummy_w(uint32_t D, uint8_t *w, uint8_t F);

/* Batched UL receive chain of ulsch_decoding (PHY/LTE_TRANSPORT/ulsch_decoding.c:1208-1350) for
 * n_tb transport blocks of one configuration (B = TBS + 24 bits, G soft bits, Qm, rvidx, first
 * round: clear = 1, Nl = 1, Kmimo = 1; later rounds: oai4g_ul_decode_batch_harq below): per code block r, lte_rate_matching_turbo_rx of the
 * E_r soft bits at offset r_offset(r) of the TB's e stream, sub_block_deinterleaving_turbo and
 * phy_threegpplte_turbo_decoder16 (CRC24_B when C > 1, else CRC24_A with the filler F).  Device
 * pointers: d_e [n_tb][e_stride] int16, d_c [n_tb][C][c_stride] bytes (the reference's c[r],
 * K_r / 8 each), d_iters [n_tb][C] (iterations, or max_iterations + 1 on a CRC failure). */
typedef struct oai4g_ul_config oai4g_ul_config_t;
oai4g_ul_config_t *oai4g_ul_config_create(uint32_t B, uint32_t G, uint8_t Qm, uint8_t rvidx, uint8_t Mdlharq,
                                          uint32_t Nsoft, uint8_t max_iterations);
void oai4g_ul_config_destroy(oai4g_ul_config_t *cfg);
int oai4g_ul_config_C(const oai4g_ul_config_t *cfg);
/* Decoder of the chain: 16 (default, phy_threegpplte_turbo_decoder16) or 8 (the 8-bit decoder, as
 * dlsch_decoding with llr8_flag = 1, dlsim -L; one block size K % 16 == 0, K >= 512).  0 / -1. */
int oai4g_ul_config_set_decoder(oai4g_ul_config_t *cfg, int bits);
uint32_t oai4g_ul_config_E(const oai4g_ul_config_t *cfg, int r);
uint32_t oai4g_ul_config_G_offset(const oai4g_ul_config_t *cfg, int r);
int oai4g_ul_decode_batch(oai4g_ul_config_t *cfg, int n_tb, const int16_t *d_e, size_t e_stride, uint8_t *d_c,
                          size_t c_stride, uint8_t *d_iters, void *stream);
/* The same chain with HARQ soft combining across rounds, as dlsch_decoding / ulsch_decoding run it
 * (dlsch_decoding.c:348-383: lte_rate_matching_turbo_rx with clear = (round == 0), the round's
 * rvidx; dlsim's round loop, dlsim.c:2141): d_w [n_tb][C][w_stride] int16 device soft buffers, the
 * reference's harq->w[r], updated in place (w_stride >= oai4g_ul_config_w_entries(cfg)).  clear = 1
 * writes every entry below Ncb (NULL positions 0, as the reference's memset); entries at or past
 * Ncb are never read, so no initialisation of d_w is needed.  rvidx 0..3 overrides the
 * configuration's.  The configuration's soft-buffer split is Kmimo = 1 (the uplink; dlsch_decoding
 * with one codeword per TB, TM1 / TM2): a DL TM3 transport block (Kmimo = 2) has another Ncb and k0
 * and is outside this API. */
size_t oai4g_ul_config_w_entries(const oai4g_ul_config_t *cfg);
int oai4g_ul_decode_batch_harq(oai4g_ul_config_t *cfg, int n_tb, const int16_t *d_e, size_t e_stride, int16_t *d_w,
                               size_t w_stride, uint8_t rvidx, uint8_t clear, uint8_t *d_c, size_t c_stride,
                               uint8_t *d_iters, void *stream);

/* ---------------- batched device-resident transmit path ---------------- */
/* Plain-old-data parameter block: what rank 0 broadcasts (RCCL) to the other ranks. */
typedef struct {
  uint16_t N_RB_DL;
  uint16_t Nid_cell;
  uint8_t Ncp;
  uint8_t nb_antennas_tx;
  uint8_t mode1_flag;
  uint8_t frame_type;
  uint8_t n_cw;               /* 1 (TM1) or 2 (TM3) */
  uint8_t mimo_mode;          /* OAI4G_SISO or OAI4G_LARGE_CDD */
  uint8_t num_pdcch_symbols;
  uint8_t Kmimo;
  uint8_t Mdlharq;
  uint8_t first_subframe;     /* subframe index of batch element 0 */
  uint8_t subframe_step;      /* 0: every element uses first_subframe; 1: consecutive subframes */
  uint8_t with_crs;           /* 1: cell-specific reference signals in the grid (pilots.c:43) */
  uint16_t rnti;
  int16_t amp;
  int16_t sqrt_rho_a;
  int16_t sqrt_rho_b;
  uint32_t rb_alloc[4];
  uint16_t nb_rb;
  uint8_t mcs[2];
  uint8_t rvidx[2];
  uint8_t q[2];               /* scrambling codeword index q (dlsim passes 0) */
  uint32_t TBS[2];
  uint32_t payload_stride;    /* bytes between consecutive transport blocks in the payload buffer */
  uint32_t rm_limited_buffer; /* opt-in extension: 36.212 5.1.4.1.2 limited-buffer
                                 rate matching when Ncb < Kw, where the reference prints "RM condition"
                                 and emits E = 0 (lte_rate_matching.c:518-521); unlocks TM3 MCS >= 20.
                                 0 (default) keeps the reference's behaviour (config_create fails). */
  uint32_t reserved[7];
} oai4g_tx_params_t;

typedef struct oai4g_tx_config oai4g_tx_config_t;

/* Derive every per-configuration table (segmentation, rate-matching geometry, RE maps,
 * QAM/twiddle/Gold tables) and upload it to the current device.  NULL on error. */
oai4g_tx_config_t *oai4g_tx_config_create(const oai4g_tx_params_t *p);
void oai4g_tx_config_destroy(oai4g_tx_config_t *cfg);
/* Derived sizes */
uint32_t oai4g_tx_G(const oai4g_tx_config_t *cfg, int cw, int subframe);
uint32_t oai4g_tx_ebits_words(const oai4g_tx_config_t *cfg);        /* per codeword per subframe */
uint32_t oai4g_tx_iq_samples(const oai4g_tx_config_t *cfg);         /* per antenna per subframe */
size_t oai4g_tx_workspace_bytes(const oai4g_tx_config_t *cfg, int n_sf);

/* Run n_sf subframes.  All pointers are device pointers:
 *   d_payload : [n_sf][n_cw][payload_stride] bytes, TBS/8 valid bytes each (not modified)
 *   d_work    : oai4g_tx_workspace_bytes() bytes (packed scrambled e bits)
 *   d_iq      : [n_sf][nb_antennas_tx][samples_per_tti] int32 (int16 I, int16 Q)
 *               (8-byte aligned: sample pairs leave as 8-byte stores; -1 otherwise)
 * stream is a hipStream_t (NULL = default stream).  Asynchronous. */
int oai4g_tx_batch(const oai4g_tx_config_t *cfg, int n_sf, const uint8_t *d_payload, void *d_work,
                   int32_t *d_iq, void *stream);
/* Same, but records HIP events around each kernel on `stream`, synchronizes, and returns the
 * two kernel durations in ms (kernel_ms[0] = encode/RM/scramble, [1] = modulate/IDFT/CP). */
int oai4g_tx_batch_timed(const oai4g_tx_config_t *cfg, int n_sf, const uint8_t *d_payload, void *d_work,
                         int32_t *d_iq, void *stream, float *kernel_ms);
/* Control region in the batched grid: every batch element of subframe index
 * sf also carries generate_dci_top's PCFICH + PDCCH for this DCI set (the same DCIs in every
 * subframe, as dlsim transmits them), merged by the modulator; n_dci = 0 switches it off.
 * The control values are computed on the GPU once here, per subframe index.  Returns 0 / -1. */
int oai4g_tx_config_set_control(oai4g_tx_config_t *cfg, uint8_t num_ue_spec_dci, uint8_t num_common_dci,
                                const oai4g_dci_alloc_t *dci_alloc);
/* Common signals in the batched grid (the eNB's common signal procedures,
 * phy_procedures_lte_eNb.c:1529-1760, and generate_phich_top :2585): PSS + SSS in subframe
 * indices 0 and 5, the PBCH quarter frame_mod4 of pbch_pdu in subframe index 0, and the listed
 * PHICHs; merged with the PCFICH / PDCCH of oai4g_tx_config_set_control, so with with_crs = 1 the
 * GPU grid is the eNB's complete txdataF.  NULL switches them off.  Returns 0 / -1. */
#define OAI4G_MAX_PHICH_ITEMS 64
typedef struct {
  uint8_t subframe, ngroup, nseq, hi;
} oai4g_phich_item_t;
typedef struct {
  uint8_t pss_sss;
  uint8_t pbch;
  uint8_t pbch_pdu[3];
  uint8_t frame_mod4;
  uint8_t n_phich;
  oai4g_phich_item_t phich[OAI4G_MAX_PHICH_ITEMS];
} oai4g_common_sig_t;
int oai4g_tx_config_set_common(oai4g_tx_config_t *cfg, const oai4g_common_sig_t *common);
/* Stage entry for parity tests: run only the encoder kernel (payload -> packed e bits). */
int oai4g_tx_encode(const oai4g_tx_config_t *cfg, int n_sf, const uint8_t *d_payload, void *d_work, void *stream);
/* Stage entry: run only the modulator kernel (packed scrambled e bits in d_work, as oai4g_tx_encode
 * leaves them -> QAM / RE map / precoding / IDFT / CP -> d_iq). */
int oai4g_tx_modulate(const oai4g_tx_config_t *cfg, int n_sf, const void *d_work, int32_t *d_iq, void *stream);
/* 1 when the configuration's range check admits the modulator's fused IDFT levels (2048-point
 * two-antenna LARGE_CDD whose largest QAM level keeps every 256- / 1024-level value inside int16;
 * DESIGN.md), 0 otherwise. */
int oai4g_tx_mod_nosat(const oai4g_tx_config_t *cfg);

/* Diagnostics: average ms of the encoder kernel stopped after phase `stop_phase`
 * (0 load+Gold, 1 CRC, 2 segmentation, 3 turbo, 4 w build, 99 = complete).  Outputs invalid. */
int oai4g_diag_encode_phase_ms(const oai4g_tx_config_t *cfg, int n_sf, const uint8_t *d_payload, void *d_work,
                               int stop_phase, int reps, float *ms);
/* Diagnostics: resident k_encode workgroups per CU and the dynamic LDS bytes per workgroup. */
int oai4g_diag_encode_occupancy(const oai4g_tx_config_t *cfg, int *blocks_per_cu, size_t *lds_bytes);
/* PMC calibration: stream `bytes` through HBM at 4 B per lane (mode 0 read, 1 write) */
int oai4g_diag_stream(const void *d_src, void *d_dst, size_t bytes, int mode, void *stream);

/* ---------------- multi-GPU: one process per GPU, RCCL over xGMI ---------------- */
/* The device this process drives (its local rank); call before any other oai4g_ call.  0 / -1. */
int oai4g_set_device(int device);
#define OAI4G_DIST_ID_BYTES 128
/* rank 0: a fresh RCCL unique id (ncclGetUniqueId) for every rank, passed out of band.  0 / -1. */
int oai4g_dist_unique_id(uint8_t id[OAI4G_DIST_ID_BYTES]);
/* join the RCCL communicator as `rank` of `world` (ncclCommInitRank, on the oai4g_set_device
 * device).  0 / -1. */
int oai4g_dist_init(int rank, int world, const uint8_t id[OAI4G_DIST_ID_BYTES]);
/* the parameter block of rank `root` into *p on every rank (ncclBroadcast of its bytes): the one
 * collective the transmit path needs.  0 / -1. */
int oai4g_dist_broadcast_params(oai4g_tx_params_t *p, int root);
/* in-place sum of n counters / checksums, max of n doubles (timings) over the ranks.  0 / -1. */
int oai4g_dist_allreduce_sum_u64(uint64_t *v, int n);
int oai4g_dist_allreduce_max_f64(double *v, int n);
int oai4g_dist_barrier(void);
int oai4g_dist_rank(void);             /* -1 before oai4g_dist_init */
int oai4g_dist_world(void);            /* 0 before oai4g_dist_init */
int oai4g_dist_finalize(void);
/* the contiguous shard [*first, *first + *count) of n_total units owned by rank of world (sizes
 * differ by at most one) */
void oai4g_shard_range(int n_total, int rank, int world, int *first, int *count);
/* the oai4g_fill_payload seed that makes a rank's buffer of global subframes [first_subframe, ...)
 * equal to that slice of the global payload stream of `seed` (payloads derive from (seed, global
 * subframe index), whatever the world size) */
uint64_t oai4g_payload_seed(uint64_t seed, uint64_t first_subframe, uint32_t n_cw, uint32_t payload_stride);

/* ---------------- device memory helpers (for hosts without another allocator) ---------------- */
void *oai4g_dev_alloc(size_t bytes);
void oai4g_dev_free(void *p);
int oai4g_memcpy_h2d(void *dst, const void *src, size_t bytes);
int oai4g_memcpy_d2h(void *dst, const void *src, size_t bytes);
int oai4g_memset_d(void *dst, int value, size_t bytes);
int oai4g_sync(void);
/* Deterministic device-side payload generator: 8-byte word w = splitmix64 output for the counter
 * seed + 0x9e3779b97f4a7c15 (w + 1) (little-endian bytes). */
int oai4g_fill_payload(uint8_t *d_payload, size_t bytes, uint64_t seed, void *stream);

#ifdef __cplusplus
}
#endif
#endif
