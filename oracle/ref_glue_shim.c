/* TEST INFRASTRUCTURE ONLY — built into oracle/_ref/libref_shimglue.so against the reference's own
 * headers (PHY/impl_defs_lte.h, PHY/LTE_TRANSPORT/defs.h, same recipe as ref_glue_mod.c).  It is the
 * caller a ctypes test needs to drive the reference-side boundary integration/liboai4g_shim.so with
 * the reference's own types, because Python cannot lay out LTE_DL_FRAME_PARMS, LTE_eNB_DLSCH_t or
 * LTE_DL_eNB_HARQ_t itself:
 *
 *   - ref_shim_frame fills an LTE_DL_FRAME_PARMS (impl_defs_lte.h:470-572) with the fields the
 *     shim's fp_to reads, from the values init_frame_parms (lte_parms.c:31-145) derives -- the test
 *     passes them in (they equal the library's oai4g_init_frame_parms, pinned in test_abi_cpu.py);
 *   - ref_shim_new_dlsch allocates the tree as new_eNB_dlsch does (dlsch_coding.c:120-220: malloc16 +
 *     bzero of the struct and of each HARQ process, b of MAX_DLSCH_PAYLOAD_BYTES / bw_scaling bytes,
 *     c[r] of (r == 0 ? 8 : 0) + 3 + 768 bytes and d[r] of 96 + 12 + 3 + 3 * 6144 bytes for
 *     r < MAX_NUM_DLSCH_SEGMENTS / bw_scaling, d[r][0..95] = LTE_NULL, round = 0).  new_eNB_dlsch's
 *     own TU (dlsch_coding.c) also defines dlsch_encoding, the function under test, and needs the
 *     missing lte_interleaver.h tables through threegpplte_turbo_encoder, so it is not linked here;
 *   - ref_shim_set / ref_shim_get / ref_shim_buf set the DCI-derived fields dlsim sets
 *     (generate_eNB_dlsch_params_from_dci, dci_tools.c:1869-1910) and read back what the shim wrote. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* f: N_RB_DL, Nid_cell, Ncp, nushift, mode1_flag, nb_antennas_tx, nb_antennas_tx_eNB, frame_type,
 *    tdd_config, symbols_per_tti, log2_symbol_size, ofdm_symbol_size, first_carrier_offset,
 *    nb_prefix_samples, nb_prefix_samples0, samples_per_tti, phich_resource, phich_duration,
 *    Nid_cell_mbsfn, nb_antennas_rx */
LTE_DL_FRAME_PARMS *ref_shim_frame(const int32_t f[20])
{
  LTE_DL_FRAME_PARMS *fp = (LTE_DL_FRAME_PARMS *)calloc(1, sizeof(LTE_DL_FRAME_PARMS));
  if (!fp) return NULL;
  fp->N_RB_DL = (uint8_t)f[0];
  fp->Nid_cell = (uint16_t)f[1];
  fp->Ncp = (lte_prefix_type_t)f[2];
  fp->nushift = (uint8_t)f[3];
  fp->mode1_flag = (uint8_t)f[4];
  fp->nb_antennas_tx = (uint8_t)f[5];
  fp->nb_antennas_tx_eNB = (uint8_t)f[6];
  fp->frame_type = (lte_frame_type_t)f[7];
  fp->tdd_config = (uint8_t)f[8];
  fp->symbols_per_tti = (uint8_t)f[9];
  fp->log2_symbol_size = (uint8_t)f[10];
  fp->ofdm_symbol_size = (uint16_t)f[11];
  fp->first_carrier_offset = (uint16_t)f[12];
  fp->nb_prefix_samples = (uint16_t)f[13];
  fp->nb_prefix_samples0 = (uint16_t)f[14];
  fp->samples_per_tti = (uint32_t)f[15];
  fp->phich_config_common.phich_resource = (PHICH_RESOURCE_t)f[16];
  fp->phich_config_common.phich_duration = (PHICH_DURATION_t)f[17];
  fp->Nid_cell_mbsfn = (uint16_t)f[18];
  fp->nb_antennas_rx = (uint8_t)f[19];
  return fp;
}

void ref_shim_free(void *p) { free(p); }

static int bw_scaling(uint8_t N_RB_DL)
{
  return N_RB_DL == 6 ? 16 : N_RB_DL == 25 ? 4 : N_RB_DL == 50 ? 2 : 1;   /* dlsch_coding.c:127-142 */
}

static void *zalloc16(size_t n)
{
  void *p = NULL;
  if (posix_memalign(&p, 16, n ? n : 16) != 0) abort();
  memset(p, 0, n);
  return p;
}

LTE_eNB_DLSCH_t *ref_shim_new_dlsch(uint8_t Kmimo, uint8_t Mdlharq, uint8_t N_RB_DL)
{
  const int bw = bw_scaling(N_RB_DL);
  LTE_eNB_DLSCH_t *d = (LTE_eNB_DLSCH_t *)zalloc16(sizeof(LTE_eNB_DLSCH_t));
  d->Kmimo = Kmimo;
  d->Mdlharq = Mdlharq;
  for (int i = 0; i < 10; i++) d->harq_ids[i] = Mdlharq;
  for (int i = 0; i < Mdlharq; i++) {
    LTE_DL_eNB_HARQ_t *h = (LTE_DL_eNB_HARQ_t *)zalloc16(sizeof(LTE_DL_eNB_HARQ_t));
    d->harq_processes[i] = h;
    h->b = (uint8_t *)zalloc16(MAX_DLSCH_PAYLOAD_BYTES / bw);
    for (int r = 0; r < MAX_NUM_DLSCH_SEGMENTS / bw; r++) {
      h->c[r] = (uint8_t *)zalloc16((r == 0 ? 8 : 0) + 3 + 768);
      h->d[r] = (uint8_t *)zalloc16(96 + 12 + 3 + 3 * 6144);
      memset(h->d[r], LTE_NULL, 96);
    }
    h->round = 0;
  }
  return d;
}

void ref_shim_free_dlsch(LTE_eNB_DLSCH_t *d)
{
  if (!d) return;
  for (int i = 0; i < 8; i++) {
    LTE_DL_eNB_HARQ_t *h = d->harq_processes[i];
    if (!h) continue;
    for (int r = 0; r < MAX_NUM_DLSCH_SEGMENTS; r++) { free(h->c[r]); free(h->d[r]); }
    free(h->b);
    free(h);
  }
  free(d);
}

/* v: rnti, TBS, mcs, rvidx, round, mimo_mode, Nl, nb_rb, rb_alloc[0..3], sqrt_rho_a, sqrt_rho_b,
 *    Nlayers, first_layer (HARQ process current_harq_pid = 0) */
void ref_shim_set(LTE_eNB_DLSCH_t *d, const int32_t v[16])
{
  LTE_DL_eNB_HARQ_t *h = d->harq_processes[0];
  d->rnti = (uint16_t)v[0];
  d->current_harq_pid = 0;
  h->TBS = (uint32_t)v[1];
  h->mcs = (uint8_t)v[2];
  h->rvidx = (uint8_t)v[3];
  h->round = (uint8_t)v[4];
  h->mimo_mode = (MIMO_mode_t)v[5];
  h->Nl = (uint8_t)v[6];
  h->nb_rb = (uint16_t)v[7];
  for (int i = 0; i < 4; i++) h->rb_alloc[i] = (uint32_t)v[8 + i];
  d->sqrt_rho_a = (int16_t)v[12];
  d->sqrt_rho_b = (int16_t)v[13];
  h->Nlayers = (uint8_t)v[14];
  h->first_layer = (uint8_t)v[15];
}

/* out: B, C, Cplus, Cminus, Kplus, Kminus, F, RTC[0..15] of HARQ process 0 */
void ref_shim_get(const LTE_eNB_DLSCH_t *d, uint32_t out[23])
{
  const LTE_DL_eNB_HARQ_t *h = d->harq_processes[0];
  out[0] = h->B; out[1] = h->C; out[2] = h->Cplus; out[3] = h->Cminus;
  out[4] = h->Kplus; out[5] = h->Kminus; out[6] = h->F;
  for (int r = 0; r < 16; r++) out[7 + r] = r < MAX_NUM_DLSCH_SEGMENTS ? h->RTC[r] : 0;
}

/* which: 0 = b, 1 = c[r], 2 = d[r], 3 = w[r], 4 = e (HARQ process 0) */
uint8_t *ref_shim_buf(LTE_eNB_DLSCH_t *d, int which, int r)
{
  LTE_DL_eNB_HARQ_t *h = d->harq_processes[0];
  switch (which) {
  case 0: return h->b;
  case 1: return h->c[r];
  case 2: return h->d[r];
  case 3: return h->w[r];
  default: return h->e;
  }
}

/* sizeof checks the test compares against the reference layout it was built with */
uint32_t ref_shim_sizes(int which)
{
  return which == 0 ? (uint32_t)sizeof(LTE_DL_FRAME_PARMS) : which == 1 ? (uint32_t)sizeof(LTE_eNB_DLSCH_t)
                                                                          : (uint32_t)sizeof(LTE_DL_eNB_HARQ_t);
}
