/*
 * Internal definitions shared by the host layer (oai4g_host.cpp) and the gfx950 kernels.
 *
 * Device-resident configuration ("cfg_dev_t") holds everything that depends only on the
 * cell / DLSCH parameters and the subframe index: code-block geometry, rate-matching
 * geometry, per-symbol RE maps, QAM tables, Gold jump tables and IDFT twiddles.  It is built
 * once per configuration on the host (the same derivations the reference re-does on every
 * call) and read by every workgroup through scalar loads.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/oai4g.h"

#define OAI4G_MAX_CB 16
#define OAI4G_MAX_NULLS 104
#define OAI4G_MAX_CHUNKS 192                /* 6144 / 32 */
#define OAI4G_MAX_TASKS (OAI4G_MAX_CB * 20)  /* ceil(R/32) + ceil(R/16) tiles per block, R <= 193 */
#define OAI4G_RM_TILES 20                     /* ceil(R/32) + ceil(R/16) for R <= 193 */
#define OAI4G_RM_SRC_LAST (1u << 20)
#define OAI4G_RM_DST_WRAP (1u << 27)
#define OAI4G_PIPE_MAX_CHUNKS 16
#define OAI4G_CRS_CODE 0xE000u               /* remap codes >= this (and != 0xFFFF) are CRS REs:
                                                CRS_CODE | pilot entry i << 9 | port & 1 << 8 | m */
#define OAI4G_CTL_CODE 0xC000u               /* remap code of a control-region RE (generate_dci_top) */
#ifndef OAI4G_MOD_STAGE
#define OAI4G_MOD_STAGE 1   /* k_modofdm stages a QAM-table address per data RE (remap_tm data codes
                               2 idx | parity << 15); 0 = per-RE bit extraction from staged e words */
#endif
#ifndef OAI4G_MOD_PRE
#define OAI4G_MOD_PRE 1     /* 2048-point LARGE_CDD (C3): the staging step also does the QAM lookups and the
                               CDD sums of both codewords, one (y0, d) pair of words per data RE; the RE
                               codes of that kernel are 8 idx | parity << 15 (oai4g_mod_pre) */
#endif
#define OAI4G_ENC_CRC_TABLE_WORDS (256 + 256) /* byte tables A/B (the combine multipliers stay in global memory;
                                                  slice-by-4 tables, 2048 words, cost one workgroup per CU: slower) */
#define OAI4G_GOLD_LANES 256
#define OAI4G_GOLD_STRIDE 17   /* odd: lanes 17l + k hit distinct LDS banks */
#define OAI4G_MAX_GOLD_WORDS (OAI4G_GOLD_LANES * OAI4G_GOLD_STRIDE) /* >= (14*1200*6)/32 */
#define OAI4G_TW_TOTAL (16 + 64 + 128 + 256 + 512 + 1024 + 2048)

/* twiddle table offsets (packed int16 pairs), indexed by log2 of the level size */
static inline __host__ __device__ uint32_t oai4g_tw_offset(int log2s)
{
  /* 16:0, 64:16, 128:80, 256:208, 512:464, 1024:976, 2048:2000 */
  switch (log2s) {
  case 4: return 0;
  case 6: return 16;
  case 7: return 80;
  case 8: return 208;
  case 9: return 464;
  case 10: return 976;
  case 11: return 2000;
  default: return 0;
  }
}

struct cw_dev_t {
  uint32_t TBS;            /* bits */
  uint32_t A_bytes;        /* TBS/8 */
  uint32_t C, Cminus, Kplus, Kminus, F, L;
  uint32_t Qm;
  uint32_t q;              /* scrambling codeword index */
  /* per code block (segmentation, lte_segmentation.c:39-170) */
  uint32_t K[OAI4G_MAX_CB];
  uint32_t f1[OAI4G_MAX_CB], f2[OAI4G_MAX_CB];
  uint32_t src[OAI4G_MAX_CB];   /* byte offset in b (= TB||CRC24A) of the first copied byte */
  uint32_t fill[OAI4G_MAX_CB];  /* zero filler bytes at the start of the block */
  uint32_t ncopy[OAI4G_MAX_CB]; /* bytes copied from b */
  uint32_t crc_off[OAI4G_MAX_CB]; /* word offset of the block's streams in LDS */
  /* per code block rate-matching geometry (lte_rate_matching.c:51-130, 464-566) */
  uint32_t R[OAI4G_MAX_CB], Kpi[OAI4G_MAX_CB], ND[OAI4G_MAX_CB], Ncb[OAI4G_MAX_CB];
  uint32_t Nnn[OAI4G_MAX_CB];   /* non-NULL entries of w[0..Ncb) */
  uint32_t k0c[OAI4G_MAX_CB];   /* non-NULL entries of w[0..k0): compacted start */
  uint32_t kidx[OAI4G_MAX_CB];  /* which null list (0: Kminus, 1: Kplus) */
  uint32_t wpk_off[OAI4G_MAX_CB + 1]; /* LDS word offset of block r's packed w (3R words + 2 pad) */
  uint32_t ntask;                     /* sub-block interleaver tiles of all blocks */
  uint16_t tasks[OAI4G_MAX_TASKS];    /* block | kind << 4 (0: v0 rows, 1: v1/v2 rows) | tile << 5 */
  uint32_t ilv_off[OAI4G_MAX_CB + 1]; /* LDS word offset of block r's QPP-interleaved input words */
  /* QPP interleaver walk per 8-step unit j of the quarter fold (kidx list): Pi(8j) | (Pi(8j+1) -
   * Pi(8j) mod K) << 16, j < K/32, and the second difference 2 f2 mod K (3gpplte.c:50-74 restated
   * incrementally) */
  uint32_t qpp0[2][OAI4G_MAX_CHUNKS];
  /* the quarter fold's walk as a table: entry k < K/4 (two uint16 per word) = word index of
   * x' = Pi(k) mod K/4 in the byte-interleaved planes (x' >> 3) | shift (8 (Pi(k) div K/4) +
   * (x' & 7)) << 11 */
  alignas(16) uint32_t qpp_tab[2][OAI4G_MAX_CHUNKS * 4];
  uint32_t qpp_d2[2];
  /* quarter folding: Pi(k + K/4) = Pi(k) + c4 mod K with c4 = f1 K/4 mod K in {K/4, 3K/4}
   * (f2 even, 8 | K); qpp_s3 = (c4 == 3K/4) */
  uint32_t qpp_s3[2];
  /* closed-form unit -> (block, word) map of the ilv word space: n0 blocks of size kk[0] first
   * (u0 = n0 kw[0] words), then blocks of kk[1]; kmag[i] = ceil(2^20 / kw[i]) */
  uint32_t n0, u0, kk[2], kw[2], kmag[2];
  /* per block size (index as kk): sub-block interleaver / rate-matching geometry, so the encoder
   * derives block metadata from wave-uniform scalars instead of per-lane table loads */
  uint32_t Rk[2], NDk[2], Ncbk[2], Nnnk[2], k0ck[2];
  uint32_t ntk[2], t0k[2], ntmag[2];   /* tiles per block, v0 tiles per block, ceil(2^20 / ntk) */
  uint32_t rm_wrapt[2];                /* the tile whose run straddles the circular buffer's end (RM_DST_WRAP), or ~0 */
  /* NULL columns of w per block size: bit w' of [0] = row 0 of v0 / v1 column w' is NULL
   * (bitrev5(w') < ND), of [1] = row 0 of v2 column w' is NULL (bitrev5(w') + 1 < ND) */
  uint32_t nullcol[2][2];
  /* per subframe index: blocks r < esplit have E = E[sf][0], the rest E[sf][C-1]; ew = words of
   * each, emag = ceil(2^32 / ew) */
  uint32_t esplit[10], ew[10][2], emag[10][2];
  uint32_t nnull[2];
  uint16_t nullpos[2][OAI4G_MAX_NULLS]; /* sorted NULL positions of w for K = Kminus / Kplus */
  /* per subframe index */
  uint32_t G[10];
  uint32_t E[10][OAI4G_MAX_CB];
  uint32_t roff[10][OAI4G_MAX_CB + 1];
  int16_t qam_a[8], qam_b[8];   /* amp_rho-scaled QAM levels (dlsch_modulation.c:1223-1246) */
  int16_t qpsk_a, qpsk_b;
  /* ALAMOUTI (dlsch_modulation.c:362-546): qam_a/qam_b hold the 1/sqrt2-scaled levels
   * (amp/sqrt2 * table >> 15) and the QPSK symbol is scaled after its sign: [pilot][+g, -g] */
  int16_t alm_qpsk[2][2];
  uint32_t stream_words;        /* LDS words per stream per block (padded) */
  /* CRC tree combine (x^(8*per*2^d) mod P as 6 nibble tables of 16 entries per level) */
  uint32_t crc_per_tb;          /* bytes per lane, 256 lanes, CRC-24A over the TB (C == 1) */
  uint32_t crc_per_cb;          /* C > 1: bytes per lane, crc_lpb lanes per block, CRC-24A and -24B together */
  uint32_t crc_lpb;             /* lanes per block (16, 32 or 64) */
  uint32_t crcmul_tb[8][6][16];
  /* C > 1: block r's CRC-24A contribution to the TB's, x^(8 (A_bytes - end_r)) mod P_A (end_r = the
   * block's last TB byte + 1), as 6 nibble tables */
  uint32_t crcmul_blk[OAI4G_MAX_CB][96];
  /* two-level in-wave combine: lane l's chunk CRC times x^(8 per (7 - l mod 8)) ([0][j] = power
   * j), XOR over the 8 lanes of its group, times x^(64 per (g - 1 - l / 8)) ([1][j], g groups of 8),
   * XOR over the g groups */
  uint32_t crc2_tb[2][8][96];
  uint32_t crc2_cb[2][2][8][96];   /* [P_A, P_B] at crc_per_cb */
  /* sub-block interleaver + rate matcher plan per block size (k_encode phase 4), tile t of a
   * block (v0 tiles of 32 rows, then interlaced tiles of 16 y1 / y2 row pairs), half-wave lane L:
   *   rm_src: before the 32x32 transpose, the stream bits lane L loads: bit shift (0..4) and LDS
   *           word (5..19) relative to the block's streams minus one word (s sw + (pos >> 5) + 1),
   *           RM_SRC_LAST (stream-2 row R-1: bit 31 is y2_0, not a stream bit);
   *   rm_dst: after it, the run of column lane L: circular offset o = (compact index - k0c) mod
   *           Nnn, leading NULLs z << 16, run length m << 21 (0: nothing), RM_DST_WRAP when
   *           o + m > Nnn. */
  uint32_t rm_src[2][OAI4G_RM_TILES + 1][32];   /* + one idle tile: a pair's second tile may be past nt */
  uint32_t rm_dst[2][OAI4G_RM_TILES + 1][32];
};

struct cfg_dev_t {
  uint32_t N_RB_DL, N, log2N, cp0, cp, spt, nsymb, n_ant, first_carrier;
  uint32_t n_cw, mimo_mode, num_pdcch, rnti, Nid_cell, first_sf, sf_step;
  uint32_t payload_stride;
  uint32_t ebits_words;         /* per codeword per subframe */
  uint32_t lds_tb_words;        /* LDS words for TB || CRC */
  uint32_t lds_stream_words;    /* LDS words for all block streams of one codeword */
  uint32_t lds_gold_words;      /* = e-bit staging words (Gold-prefilled) */
  uint32_t lds_w_words;         /* packed sub-block interleaver output of every block */
  uint32_t lds_a_words;         /* region A: TB + CRC tables (0-2) | interleaved words (3) | packed w (4) */
  uint32_t lds_b_words;         /* region B: constituent streams */
  uint32_t mod_nosat;            /* 1: k_modofdm may take the fused IDFT levels (oai4g_host.cpp mod_nosat_ok) */
  uint32_t pad;
  uint32_t crctab[2][256];      /* CRC byte tables (crc_byte.c:98-105): [0] CRC-24A, [1] CRC-24B */
  cw_dev_t cw[2];
  uint32_t symbase[10][14];     /* data REs before symbol l */
  uint32_t symnre[10][14];      /* data REs in symbol l (32-bit: the modulator reads it with a scalar load) */
  uint32_t n_cu;                /* compute units of the device (persistent grids) */
  const uint16_t *remap;        /* [10][14][N] data-RE index | parity<<15; OAI4G_CRS_CODE | pilot
                                   symbol<<9 | port<<8 | m for a CRS RE; 0xFFFF = none */
  const uint16_t *remap_tm;     /* the same codes thread-major: per (sf, l), [t][n] = remap[t + (N/16) n],
                                   so each modofdm thread fetches its 16 codes with two 16-B loads */
  const uint16_t *remap_tm0;    /* remap_tm with every non-data code replaced by the staged zero
                                   sentinel's byte offset (2 * 3N/4): the kernels without CRS or control
                                   REs then address the sentinel without a clamp */
  uint32_t with_crs;
  uint32_t pilmask;             /* bit l: symbol l carries CRS (QAM levels scaled by rho_B) */
  const uint32_t *crs_tab;      /* [10][6][200] packed CRS IQ of pilot symbol i (l = 0, 4, 7, 11; 1, 8 for
                                   ports 2/3 with 4 TX antennas), index m */
  const uint32_t *ctl_tab;      /* [10][14][2][N] packed IQ of the static REs (PCFICH, PDCCH, PHICH, PSS, SSS, PBCH; antennas
                                   0 / 1) per subframe index; REs with code OAI4G_CTL_CODE take it */
  uint32_t ctlmask[10];         /* bit l: symbol l of subframe index sf carries control REs */
  uint32_t ctl_on;
  const uint32_t *gold_tab;     /* [10][n_cw][ebits_words] scrambling words (dlsch_scrambling.c:51-97) per
                                   subframe index and codeword: c_init depends on nothing else */
  const uint32_t *gold_x1;      /* [256]     x1 state after 50+16l word steps */
  const uint32_t *gold_x2j;     /* [256][32] columns of M2^(50+16l) */
  const uint32_t *tw;           /* 2 x OAI4G_TW_TOTAL packed twiddles t, then (-t.im, t.re) */
  const uint32_t *stat_tm;      /* [10][14][stat_planes][N] thread-major like remap_tm: the packed IQ each
                                   kernel antenna takes at a CRS or control RE, 0 elsewhere (CRS / control
                                   configurations; k_modofdm ORs it over the data path, which reads the
                                   zero sentinel there) */
  uint32_t stat_planes;         /* 1 (TM1: one transform) or the TX antennas */
  uint32_t pad2;
};

/* ---------------- launch helpers implemented in the .hip files ---------------- */
/* encoder path */
hipError_t oai4g_launch_encode(const cfg_dev_t *d_cfg, const cfg_dev_t *h_cfg, int sf0, int n_sf,
                               const uint8_t *d_payload, uint32_t *d_ebits, hipStream_t s);
hipError_t oai4g_encode_occupancy(const cfg_dev_t *h_cfg, int *blocks_per_cu, size_t *lds_bytes);
hipError_t oai4g_launch_encode_phase(const cfg_dev_t *d_cfg, const cfg_dev_t *h_cfg, int n_sf,
                                     const uint8_t *d_payload, uint32_t *d_ebits, int stop_phase, hipStream_t s);
struct enc_debug_t {
  uint8_t *c;      /* [C][8+3+768]                         */
  uint8_t *d;      /* [C][OAI4G_D_BYTES] (offset 96 = d[r][96]) */
  uint8_t *w;      /* [C][OAI4G_W_BYTES]                   */
  uint8_t *e;      /* [G] pre-scrambling rate-matcher output */
  uint8_t *b;      /* [A/8+4] TB with CRC appended          */
};
hipError_t oai4g_launch_encode_debug(const cfg_dev_t *d_cfg, const cfg_dev_t *h_cfg, int cw, int sf,
                                     const uint8_t *d_payload, enc_debug_t dbg, hipStream_t s);
hipError_t oai4g_launch_crc24(const uint8_t *d_in, int bitlen, uint32_t poly_top, uint32_t *d_out, hipStream_t s);
hipError_t oai4g_launch_turbo_bytes(const uint8_t *d_c, int nbytes, uint8_t *d_out, uint32_t f1, uint32_t f2,
                                    hipStream_t s);
hipError_t oai4g_launch_subblock_bytes(uint32_t D, const uint8_t *d_dfull, uint8_t *d_w, hipStream_t s);
hipError_t oai4g_launch_rm_bytes(const uint8_t *d_w, uint32_t Ncb, uint32_t k0, uint32_t E, uint8_t *d_e,
                                 uint32_t *d_status, hipStream_t s);
hipError_t oai4g_launch_scramble_bytes(uint8_t *d_e, int n_entries, uint32_t c_init, const uint32_t *d_gold_x1,
                                       const uint32_t *d_gold_x2j, hipStream_t s);
hipError_t oai4g_launch_fill(uint8_t *d, size_t bytes, uint64_t seed, hipStream_t s);
/* CRS into nsym_grids OFDM-symbol grids: job j writes grid `out + jobs[j].off` (N REs) with port
 * jobs[j].p, pilot l of slot Ns from gold[Ns][l][14] */
struct crs_job_t {
  uint32_t off;
  uint8_t Ns, l, p, pad;
};
hipError_t oai4g_launch_crs(int32_t *d_out, const crs_job_t *jobs, int n_jobs, const uint32_t *d_gold, int16_t amp,
                            uint32_t N, uint32_t N_RB, uint32_t nushift, uint32_t first_carrier, hipStream_t s);
hipError_t oai4g_launch_diag_stream(const void *src, void *dst, size_t bytes, int mode, hipStream_t s);

/* uplink turbo decoding (oai4g_decode.hip) */
size_t oai4g_td_block_bytes(uint32_t K);
hipError_t oai4g_launch_td16(int n_cb, uint32_t K, const int16_t *d_llr, size_t llr_stride, uint8_t *d_out,
                             size_t out_stride, uint8_t *d_iters, uint32_t max_it, uint32_t crc_type, uint32_t F,
                             const uint16_t *d_pi /* pi4 | pi5 | pi6, K each */, uint8_t *d_scratch, hipStream_t s,
                             uint32_t cg = 1, uint32_t c_per = 1, uint32_t r0 = 0);
/* 8-bit turbo decoder (oai4g_decode8.hip) */
size_t oai4g_td8_wave_bytes(uint32_t K);
hipError_t oai4g_launch_td8(int n_cb, uint32_t K, const int16_t *d_llr, size_t llr_stride, uint8_t *d_out,
                            size_t out_stride, uint8_t *d_iters, uint32_t max_it, uint32_t crc_type, uint32_t F,
                            const uint16_t *d_pi, uint8_t *d_scratch, hipStream_t s);
/* batched UL receive chain (ulsch_decoding.c:1208-1350): per code-block pattern (block size,
 * filler) the NULL map and compact indices of the rate-matching circular buffer */
#define OAI4G_UL_MAX_C 16
struct ul_pat_t {
  uint32_t D, R, Ncb, Nnn, k0c;
  uint32_t k0cr[4];                /* k0c of rvidx 0..3 (the HARQ rounds) */
  const uint8_t *dummy;            /* [3 R 32] LTE_NULL marks */
  const uint32_t *cidx;            /* [Ncb] compact index */
};
struct ul_dev_t {
  uint32_t C, Rmax;
  uint32_t E[OAI4G_UL_MAX_C], off[OAI4G_UL_MAX_C], pat_of[OAI4G_UL_MAX_C];
  ul_pat_t pat[3];
};
hipError_t oai4g_launch_ul_rm_deint(const ul_dev_t *d_cfg, const ul_dev_t *h_cfg, int n_tb, const int16_t *d_e,
                                    size_t e_stride, int16_t *d_dfull, size_t d_stride, hipStream_t s);
/* HARQ form: w [rows][w_stride] int16 circular soft buffers kept across rounds; the round's rv and
 * clear (round 0) select k0 and the reset; then w -> the decoder's d buffers */
hipError_t oai4g_launch_ul_rm_harq(const ul_dev_t *d_cfg, const ul_dev_t *h_cfg, int n_tb, const int16_t *d_e,
                                   size_t e_stride, int16_t *d_w, size_t w_stride, uint32_t rv, int clear,
                                   int16_t *d_dfull, size_t d_stride, hipStream_t s);
hipError_t oai4g_launch_rm_rx(const int16_t *d_soft, uint32_t E, int16_t *d_w, const uint8_t *d_dummy,
                              const uint32_t *d_cidx, uint32_t Ncb, uint32_t Nnn, uint32_t k0c, int clear, hipStream_t s);
hipError_t oai4g_launch_subblock_deint(uint32_t D, int16_t *d_dfull, const int16_t *d_w, hipStream_t s);

/* OFDM path */
hipError_t oai4g_launch_modofdm(const cfg_dev_t *d_cfg, const cfg_dev_t *h_cfg, int sf0, int n_sf,
                                const uint32_t *d_ebits, int32_t *d_iq, hipStream_t s);
struct ofdm_sym_t {
  uint32_t in_off;   /* int32 index of the symbol's frequency-domain input */
  uint32_t out_off;  /* int32 index of the symbol's time-domain body (after the CP) */
  uint32_t cp;       /* cyclic-prefix length written in front of the body */
};
hipError_t oai4g_launch_ofdm(const int32_t *d_in, int32_t *d_out, int log2n, int nsym, const ofdm_sym_t *syms,
                             int scale, const uint32_t *d_tw, hipStream_t s);
hipError_t oai4g_launch_idft_strided(const int32_t *d_in, int32_t *d_out, int log2n, int n_jobs, size_t in_stride,
                                     uint32_t in_off, size_t out_stride, int scale, const uint32_t *d_tw, hipStream_t s);
/* lte_est_freq_offset's integer part (oai4g_chest.hip) */
hipError_t oai4g_launch_freq_offset(const int32_t *d_est, size_t est_stride, int n_jobs, int N_RB, uint32_t row_off,
                                    uint32_t prev_off, int32_t *d_omega, hipStream_t s);
/* control region (oai4g_ctrl.hip): PCFICH */
struct pcfich_args_t {
  uint32_t c_init;      /* pcfich_scrambling x2 (pcfich.c:97) */
  uint32_t cfi;         /* num_pdcch_symbols, 1..3 */
  int16_t gain;         /* QPSK amplitude (pcfich.c:168-171) */
  uint8_t mode1;        /* 1 = SISO mapping, 0 = ALAMOUTI */
  uint8_t nushift3;     /* nushift % 3 */
  uint32_t reg_off[4];  /* first RE of each REG in the symbol, DC-skip applied (pcfich.c:210-213) */
  uint32_t n_ant;
};
hipError_t oai4g_launch_pcfich(int32_t *d_g0, int32_t *d_g1, const pcfich_args_t &a, hipStream_t s);

/* PDCCH (generate_dci_top, dci.c:2024-2346) */
#define OAI4G_MAX_DCI 32
struct dci_dev_t {
  uint8_t flip[8];      /* the pdu bytes in generate_dci0's order (dci.c:233-251) */
  uint32_t A;           /* DCI bits */
  uint32_t L;           /* log2 aggregation level */
  int32_t nCCE;
  uint32_t rnti;
};
struct dci_args_t {
  uint32_t n_dci;
  dci_dev_t dci[OAI4G_MAX_DCI];
  uint32_t nbits;       /* scrambled PDCCH bits, 8 * nquad (pdcch_scrambling length) */
  uint32_t c_init;      /* (subframe << 9) + Nid_cell */
  uint32_t n_re;        /* REs mapped */
  int16_t gain;         /* QPSK amplitude (dci.c:2170-2174) */
  uint8_t mode1;        /* 1: SISO (<NIL> -> 0), 0: ALAMOUTI (<NIL> -> +gain) */
  uint8_t n_ant;        /* antennas written (nb_antennas_tx_eNB > 1 ? 2 : 1) */
};
/* map[r] = grid offset of mapped RE r (symbol * N + subcarrier), src[r] = its QPSK symbol index
 * after quadruplet interleaving and the cyclic shift.  One workgroup. */
hipError_t oai4g_launch_dci(const dci_args_t &a, const uint32_t *d_map, const uint16_t *d_src, int32_t *d_g0,
                            int32_t *d_g1, uint32_t g1_stride, hipStream_t s);

/* synchronisation / broadcast / HARQ-indicator channels (oai4g_ctrl.hip) */
struct sync_args_t {    /* generate_pss (pss.c:50-103) / generate_sss (sss.c:47-92) */
  int16_t val[62][2];   /* PSS: the Zadoff-Chu table entries (primary_synch.h); SSS: (d(n), 0), d = +-1 */
  int16_t a;            /* amp or (amp ONE_OVER_SQRT2_Q15) >> 15 */
  uint8_t pss;          /* 1: (a v) >> 15 per component; 0: (int16)(a v), imaginary 0 */
  uint8_t n_ant;
  uint32_t N;           /* ofdm_symbol_size: k starts at N - 31 and skips DC */
};
hipError_t oai4g_launch_sync(int32_t *const *d_sym /* per antenna: the symbol's N REs */, const sync_args_t &a,
                             hipStream_t s);
struct pbch_args_t {    /* generate_pbch (pbch.c:161-420) */
  uint8_t a[3];         /* pbch_a: the pdu bytes reversed (pbch.c:214-215) */
  uint8_t encode;       /* frame_mod4 == 0: encode and scramble into e; else map the stored e */
  uint16_t amask;       /* CRC16 antenna mask (pbch.c:223-238) */
  uint16_t E;           /* 1920 (normal CP) / 1728 */
  uint32_t Nid;         /* scrambling c_init (pbch.c:770) */
  uint32_t quarter;     /* frame_mod4 */
  uint32_t N;           /* ofdm_symbol_size */
  uint32_t pil_mask;    /* bit l (0..3): symbol nsymb/2 + l is a pilot symbol for the PBCH (pbch.c:345-362) */
  uint32_t nushift3;
  int16_t gain;         /* (amp ONE_OVER_SQRT2_Q15) >> 15 */
  uint8_t mode1;
  uint8_t n_ant;
};
/* d_g[a]: 4 consecutive symbols (nsymb/2 .. +3) of antenna a; d_e: the 1920-bit state (bytes) */
hipError_t oai4g_launch_pbch(int32_t *const *d_g, uint8_t *d_e, const pbch_args_t &a, hipStream_t s);
#define OAI4G_MAX_PHICH 64
struct phich_item_t {
  uint32_t c_init;      /* ((subframe + 1)(Nid + 1)) << 9 + Nid (phich.c:440) */
  uint32_t reg_off[3];  /* first RE of each REG relative to the subframe's symbol 0 (phich.c:556-561) */
  uint8_t nseq, hi;
};
struct phich_args_t {   /* generate_phich (phich.c:401-780), normal CP */
  uint32_t n;
  phich_item_t it[OAI4G_MAX_PHICH];
  int16_t gain;         /* SISO (amp 23170) >> 15, ALAMOUTI amp / 2 */
  uint8_t mode1;
  uint8_t n_ant;
  uint32_t nushift;     /* < 3 */
  uint32_t win;         /* REs of the window the offsets index (2 symbols) */
};
/* d_g[a]: window of symbols 0..1 of the subframe, antenna a; d_acc: 4 * win int32 scratch */
hipError_t oai4g_launch_phich(int32_t *const *d_g, int32_t *d_acc, const phich_args_t &a, hipStream_t s);

/* UE receive front end (oai4g_fep.hip): per-symbol CP removal + forward DFT */
#define OAI4G_FEP_MAX_SYM 14
struct fep_args_t {
  int n_units;        /* items x nsym */
  int nsym;           /* symbols per item */
  uint32_t in_stride, in_len, out_stride;   /* int32 samples */
  uint32_t in_off[OAI4G_FEP_MAX_SYM];       /* DFT window start of each symbol (< in_len) */
  uint32_t out_off[OAI4G_FEP_MAX_SYM];      /* output offset of each symbol */
  int scale;
};
hipError_t oai4g_launch_fep(const int32_t *d_in, int32_t *d_out, int log2n, const fep_args_t &a,
                            const uint32_t *d_twf, int n_cu, hipStream_t s);
hipError_t oai4g_launch_modulate_bytes(const cfg_dev_t *d_cfg, const cfg_dev_t *h_cfg, int sf,
                                       const uint8_t *d_e0, const uint8_t *d_e1, int32_t *d_grid, hipStream_t s);

/* UE PDSCH demodulation (oai4g_rx.hip): TM1, one receive antenna, even N_RB_DL */
/* downlink channel estimation (lte_dl_channel_estimation, high_speed_flag = 1, one RX antenna) */
struct chest_dev_t {
  uint32_t N, N_RB, nsymb, Ncp, fco, p;
  uint32_t first_sf, sf_step;
  uint32_t branch;                /* 1: the 6 / 15 / 25 / 50 / 100 PRB interpolators; 0: "not implemented" (rows of 0) */
  uint32_t k[2];                  /* pilot offset (nu + nushift) % 6 for pilot symbols l = 0 / l > 0 */
  uint32_t off2[2];               /* first bin of the pilots above DC: 1 + k, or 1 + nushift + 3 p at 15 PRB */
  uint32_t elem_syms;             /* symbols between batch elements in rxdataF (nsymb; 2 nsymb in dlsim's BLER
                                     loop, where each trial's subframe is followed by the next one) */
  uint32_t next_syms;             /* symbols from an element's start to the symbol 0 closing its rows 12 / 13 */
  int16_t filt[2][8][24];         /* fl, f2l2, f, f2, fr, f2r2, f_dc, f2_dc (filt96_32.h) for k[0] / k[1] */
  uint32_t gold[20][2][14];       /* lte_gold_table */
};
void oai4g_set_error(const char *fmt, ...);
/* binds the calling thread to the device the library was initialised on (hipSetDevice is per thread) */
int oai4g_bind_thread(void);
hipError_t oai4g_launch_signal_energy(const int32_t *d_x, int n, size_t stride, uint32_t length, int32_t *d_out,
                                      hipStream_t s);
hipError_t oai4g_launch_awgn(const int32_t *d_tx, size_t tx_stride, uint32_t tx_len, const int32_t *d_tail,
                             uint32_t tail_len, int32_t *d_rx, size_t rx_stride, int n, const int32_t *d_tx_lev,
                             double offset_db, uint64_t seed, uint32_t vec0, hipStream_t s);
hipError_t oai4g_launch_unscramble(int16_t *d_llr, const uint32_t *d_c, int n, hipStream_t s);
hipError_t oai4g_launch_chest(const chest_dev_t *d_cfg, const chest_dev_t *h_cfg, int n_sf, const int32_t *d_rxF,
                              int32_t *d_est, hipStream_t s);
/* the 5 pilot rows per subframe only ([n_sf][5][N], columns < 12 N_RB + 16) */
hipError_t oai4g_launch_chest_pilots(const chest_dev_t *d_cfg, const chest_dev_t *h_cfg, int n_sf, const int32_t *d_rxF,
                                     int32_t *d_pil, hipStream_t s);
hipError_t oai4g_launch_chest_symbol(const chest_dev_t *d_cfg, const chest_dev_t *h_cfg, const int32_t *d_rxF_sym,
                                     int32_t *d_est, int Ns, int l, int symbol, hipStream_t s);

struct rx_dev_t {
  uint32_t N, nsymb, Qm, npdcch;
  uint32_t llr_stride;            /* LLRs per batch element */
  uint32_t n_sym;                 /* PDSCH symbols per subframe (nsymb - npdcch) */
  /* per subframe index and PDSCH symbol: extraction map offset, extracted REs, demodulated REs,
   * LLR offset; level REs and divisor for the first symbol */
  uint32_t map_off[10][14], n_ext[10][14], len[10][14], llr_off[10][14];
  uint32_t lvl_n[10], lvl_div[10];
  uint32_t gold_words;            /* scrambling words per subframe index */
  uint32_t first_sf, sf_step;
  int16_t a1, a2;                 /* QAM_n1 / QAM_n2 of the channel magnitude (0 for QPSK) */
  const uint32_t *map;            /* extracted RE j: FFT bin | (estimate index within the symbol) << 16 */
  const uint32_t *gold;           /* [10][gold_words] */
  /* TM3 (LARGE_CDD, dual extraction; rx_pdsch with dual_stream_flag = 0): receive antennas, the
   * channel_level_TM3 RE count per RB of the first PDSCH symbol, offset_mumimo_llr_drange */
  uint32_t tm3, nb_rx, lvl_nre;
  int32_t mu_off;
  /* TM2 (ALAMOUTI, dual extraction): dlsch_channel_level over both ports, dlsch_alamouti */
  uint32_t tm2;
  uint32_t qm1;                   /* TM3: codeword 1's modulation order (Qm = 2 picks qpsk_qpsk / _qam16 / _qam64) */
  /* estimate row l from the 5 pilot rows (lte_dl_channel_estimation.c:639-698): pilot row ea[l]
   * when ewa[l] == 0, else mulhi(P[ea], ewa) << 1 +sat mulhi(P[eb], ewb) << 1 */
  uint8_t ea[14], eb[14];
  int16_t ewa[14], ewb[14];
};
hipError_t oai4g_launch_rx_chest(const chest_dev_t *d_ce, const rx_dev_t *d_rx, const rx_dev_t *h_rx, int n_sf,
                                 const int32_t *d_rxF, int16_t *d_llr, uint8_t *d_shift, int unscramble, hipStream_t s);
hipError_t oai4g_launch_rx_tm3(const rx_dev_t *d_cfg, const rx_dev_t *h_cfg, int n_sf, const int32_t *d_rxF,
                               const int32_t *d_est, size_t plane, int16_t *d_llr, uint8_t *d_shift, int unscramble,
                               hipStream_t s, int pil = 0);
/* TM3 with codeword 0 QPSK: Qm1 = 2 both codewords (d_llr1 may be null), Qm1 = 4 / 6 codeword 0 */
hipError_t oai4g_launch_rx_tm3qq(const rx_dev_t *d_cfg, const rx_dev_t *h_cfg, int n_sf, const int32_t *d_rxF,
                                 const int32_t *d_est, size_t plane, int16_t *d_llr0, int16_t *d_llr1,
                                 uint8_t *d_shift, int unscramble, hipStream_t s, int pil = 0);
hipError_t oai4g_launch_rx_tm2(const rx_dev_t *d_cfg, const rx_dev_t *h_cfg, int n_sf, const int32_t *d_rxF,
                               const int32_t *d_est, size_t plane, int16_t *d_llr, uint8_t *d_shift, int unscramble,
                               hipStream_t s);
hipError_t oai4g_launch_rx(const rx_dev_t *d_cfg, const rx_dev_t *h_cfg, int n_sf, const int32_t *d_rxF,
                           const int32_t *d_ch, int16_t *d_llr, uint8_t *d_shift, int unscramble, hipStream_t s);
