/* TEST INFRASTRUCTURE ONLY — linked into oracle/_ref/libref_mod.so next to the reference's own
 * PHY/LTE_TRANSPORT/dlsch_modulation.c and dlsch_scrambling.c (both compiled unmodified, see
 * oracle/Makefile) and the reference's variable definitions PHY/LTE_TRANSPORT/vars.h (included
 * below, unmodified).  Not a stand-in for any reference file:
 *
 *   - ref_glue_dlsch_modulation() / ref_glue_dlsch_scrambling() fill the reference's own
 *     LTE_DL_FRAME_PARMS (PHY/impl_defs_lte.h), LTE_eNB_DLSCH_t and LTE_DL_eNB_HARQ_t
 *     (PHY/LTE_TRANSPORT/defs.h:104-274) with the fields those two functions read, because a ctypes
 *     test cannot build those structs itself, and call the reference functions;
 *   - get_Qm: dlsch_modulation.c:1200 calls it, and its translation unit (PHY/LTE_TRANSPORT/lte_mcs.c)
 *     includes proto.h, which needs PHY_VARS_eNB / PHY_VARS_UE from PHY/defs.h and through it the
 *     asn1c-generated headers.  It is restated here from lte_mcs.c:45-55 (three comparisons); the
 *     modulation order it returns is also what the tests pass explicitly to the oracle.
 *
 * PHY/LTE_TRANSPORT/pcfich.c is in the same library, also unmodified (its MAC_INTERFACE/extern.h, which
 * reaches the asn1c chain too, skipped by its guard: the TU uses nothing from it); ref_glue_pcfich()
 * fills the frame for generate_pcfich_reg_mapping / generate_pcfich.
 *
 * The other symbol the two TUs leave undefined, logRecord (UTIL/LOG/log.h, LOG_E / LOG_W), is only
 * reached on their error branches (an unsupported MIMO mode or layer count), which no test case
 * takes; the library is opened with RTLD_LAZY (tests/oracle_lib.py ref_mod, oracle/cpu_baseline.c),
 * so that symbol is never bound. */
#include "PHY/LTE_TRANSPORT/vars.h"

int dlsch_modulation(mod_sym_t **txdataF, int16_t amp, uint32_t subframe_offset, LTE_DL_FRAME_PARMS *frame_parms,
                     uint8_t num_pdcch_symbols, LTE_eNB_DLSCH_t *dlsch0, LTE_eNB_DLSCH_t *dlsch1);
void dlsch_scrambling(LTE_DL_FRAME_PARMS *frame_parms, int mbsfn_flag, LTE_eNB_DLSCH_t *dlsch, int G, uint8_t q,
                      uint8_t Ns);
void generate_64qam_table(void);
void generate_16qam_table(void);
void generate_pcfich_reg_mapping(LTE_DL_FRAME_PARMS *frame_parms);
void generate_pcfich(uint8_t num_pdcch_symbols, int16_t amp, LTE_DL_FRAME_PARMS *frame_parms, mod_sym_t **txdataF,
                     uint8_t subframe);

unsigned char get_Qm(unsigned char I_MCS)
{
  return I_MCS < 10 ? 2 : (I_MCS < 17 ? 4 : 6);
}

/* one codeword as the tests describe it (mirrors the oracle's orc_cw_t) */
typedef struct {
  const uint8_t *e;      /* G entries 0/1 */
  int32_t G;
  uint8_t mcs;
  uint8_t mimo_mode;     /* MIMO_mode_t: 0 SISO, 1 ALAMOUTI, 2 LARGE_CDD */
  uint8_t Nlayers;
  uint8_t first_layer;
  uint32_t rb_alloc[4];
  uint16_t nb_rb;
  uint16_t pmi_alloc;
} ref_cw_t;

/* frame: {N_RB_DL, Ncp, nb_antennas_tx, ofdm_symbol_size, first_carrier_offset, nushift, mode1_flag,
 *         frame_type, Nid_cell} */
static void ref_glue_frame(LTE_DL_FRAME_PARMS *fp, const int32_t f[9])
{
  memset(fp, 0, sizeof(*fp));
  fp->N_RB_DL = (uint8_t)f[0];
  fp->Ncp = (lte_prefix_type_t)f[1];
  fp->nb_antennas_tx = (uint8_t)f[2];
  fp->ofdm_symbol_size = (uint16_t)f[3];
  fp->first_carrier_offset = (uint16_t)f[4];
  fp->nushift = (uint8_t)f[5];
  fp->mode1_flag = (uint8_t)f[6];
  fp->frame_type = (lte_frame_type_t)f[7];
  fp->Nid_cell = (uint16_t)f[8];
}

static LTE_DL_eNB_HARQ_t *g_harq[2];
static LTE_eNB_DLSCH_t g_dlsch[2];
static int g_tables;

static void ref_glue_init(void)
{
  if (!g_tables) {
    generate_64qam_table();
    generate_16qam_table();
    g_tables = 1;
  }
  for (int i = 0; i < 2; i++)
    if (!g_harq[i]) {
      g_harq[i] = (LTE_DL_eNB_HARQ_t *)calloc(1, sizeof(LTE_DL_eNB_HARQ_t));
      if (!g_harq[i]) abort();
    }
}

static void ref_glue_dlsch(int i, const ref_cw_t *cw, uint16_t rnti, int16_t sqrt_rho_a, int16_t sqrt_rho_b)
{
  LTE_eNB_DLSCH_t *d = &g_dlsch[i];
  LTE_DL_eNB_HARQ_t *h = g_harq[i];
  memset(d, 0, sizeof(*d));
  d->rnti = rnti;
  d->current_harq_pid = 0;
  d->harq_processes[0] = h;
  d->sqrt_rho_a = sqrt_rho_a;
  d->sqrt_rho_b = sqrt_rho_b;
  if (!cw) return;
  h->mcs = cw->mcs;
  h->mimo_mode = (MIMO_mode_t)cw->mimo_mode;
  h->Nl = 1;
  h->Nlayers = cw->Nlayers;
  h->first_layer = cw->first_layer;
  memcpy(h->rb_alloc, cw->rb_alloc, sizeof(h->rb_alloc));
  h->nb_rb = cw->nb_rb;
  h->pmi_alloc = cw->pmi_alloc;
  if (cw->G < 0 || cw->G > MAX_NUM_CHANNEL_BITS) abort();
  memset(h->e, 0, sizeof(h->e));
  if (cw->e) memcpy(h->e, cw->e, (size_t)cw->G);
}

/* dlsch_modulation (dlsch_modulation.c:1181-1493) into txdataF[ant] (frame grids, subframe_offset as
 * the reference takes it); returns its value (re_allocated or -1) */
int ref_glue_dlsch_modulation(int32_t **txdataF, int16_t amp, uint32_t subframe_offset, const int32_t f[9],
                              uint8_t num_pdcch_symbols, const ref_cw_t *cw0, const ref_cw_t *cw1,
                              int16_t sqrt_rho_a, int16_t sqrt_rho_b)
{
  LTE_DL_FRAME_PARMS fp;
  ref_glue_init();
  ref_glue_frame(&fp, f);
  ref_glue_dlsch(0, cw0, 0, sqrt_rho_a, sqrt_rho_b);
  ref_glue_dlsch(1, cw1, 0, sqrt_rho_a, sqrt_rho_b);
  return dlsch_modulation((mod_sym_t **)txdataF, amp, subframe_offset, &fp, num_pdcch_symbols, &g_dlsch[0],
                          cw1 ? &g_dlsch[1] : NULL);
}

/* dlsch_scrambling (dlsch_scrambling.c:51-97) of e[0 .. G) in place; `e` must hold 32 (1 + G / 32)
 * entries: the reference writes whole 32-entry words past G, and those land in e too */
void ref_glue_dlsch_scrambling(uint8_t *e, int G, uint16_t rnti, uint16_t Nid_cell, uint8_t q, uint8_t Ns)
{
  LTE_DL_FRAME_PARMS fp;
  ref_cw_t cw;
  const int n = 32 * (1 + (G >> 5));
  ref_glue_init();
  memset(&fp, 0, sizeof(fp));
  fp.Nid_cell = Nid_cell;
  memset(&cw, 0, sizeof(cw));
  cw.G = n;
  cw.e = e;
  ref_glue_dlsch(0, &cw, rnti, 0, 0);
  dlsch_scrambling(&fp, 0, &g_dlsch[0], G, q, Ns);
  memcpy(e, g_harq[0]->e, (size_t)n);
}

/* The same two calls on persistent structures, for oracle/cpu_baseline.c: the caller writes the
 * rate-matched bits straight into HARQ process 0's e of codeword cw (as dlsch_encoding does) and
 * times the reference functions alone, without the copies of the functions above. */
uint8_t *ref_glue_harq_e(int cw)
{
  ref_glue_init();
  return g_harq[cw & 1]->e;
}

void ref_glue_set_cw(int cw, const ref_cw_t *c, uint16_t rnti, int16_t sqrt_rho_a, int16_t sqrt_rho_b)
{
  LTE_DL_eNB_HARQ_t *h;
  ref_glue_init();
  h = g_harq[cw & 1];
  memset(&g_dlsch[cw & 1], 0, sizeof(g_dlsch[0]));
  g_dlsch[cw & 1].rnti = rnti;
  g_dlsch[cw & 1].harq_processes[0] = h;
  g_dlsch[cw & 1].sqrt_rho_a = sqrt_rho_a;
  g_dlsch[cw & 1].sqrt_rho_b = sqrt_rho_b;
  h->mcs = c->mcs;
  h->mimo_mode = (MIMO_mode_t)c->mimo_mode;
  h->Nl = 1;
  h->Nlayers = c->Nlayers;
  h->first_layer = c->first_layer;
  memcpy(h->rb_alloc, c->rb_alloc, sizeof(h->rb_alloc));
  h->nb_rb = c->nb_rb;
  h->pmi_alloc = c->pmi_alloc;
}

void ref_glue_scramble_cw(int cw, const int32_t f[9], int G, uint8_t q, uint8_t Ns)
{
  LTE_DL_FRAME_PARMS fp;
  ref_glue_frame(&fp, f);
  dlsch_scrambling(&fp, 0, &g_dlsch[cw & 1], G, q, Ns);
}

int ref_glue_modulate(int32_t **txdataF, int16_t amp, uint32_t subframe_offset, const int32_t f[9],
                      uint8_t num_pdcch_symbols, int n_cw)
{
  LTE_DL_FRAME_PARMS fp;
  ref_glue_frame(&fp, f);
  return dlsch_modulation((mod_sym_t **)txdataF, amp, subframe_offset, &fp, num_pdcch_symbols, &g_dlsch[0],
                          n_cw > 1 ? &g_dlsch[1] : NULL);
}

/* the reference's qam tables after generate_*qam_table (dlsch_modulation.c:79-103) */
void ref_glue_qam_tables(int32_t q16[4], int32_t q64[8])
{
  ref_glue_init();
  for (int i = 0; i < 4; i++) q16[i] = qam16_table[i];
  for (int i = 0; i < 8; i++) q64[i] = qam64_table[i];
}

/* generate_pcfich_reg_mapping then generate_pcfich (pcfich.c:48-84, 144-228) into txdataF[ant] (frame
 * grids); nb_antennas_tx_eNB (the field generate_pcfich tests) = f[2].  reg / first_idx: the mapping. */
void ref_glue_pcfich(uint8_t num_pdcch_symbols, int16_t amp, const int32_t f[9], int32_t **txdataF, uint8_t subframe,
                     uint16_t reg[4], uint8_t *first_idx)
{
  LTE_DL_FRAME_PARMS fp;
  ref_glue_frame(&fp, f);
  fp.nb_antennas_tx_eNB = (uint8_t)f[2];
  generate_pcfich_reg_mapping(&fp);
  for (int i = 0; i < 4; i++) reg[i] = fp.pcfich_reg[i];
  *first_idx = fp.pcfich_first_reg_idx;
  generate_pcfich(num_pdcch_symbols, amp, &fp, (mod_sym_t **)txdataF, subframe);
  fflush(stdout);   /* the mapping's own printf (pcfich.c:80-82) leaves while a test's capture is on */
}
