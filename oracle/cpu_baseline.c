/* cpu_baseline — TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).
 *
 * Times the transmit path of one configuration on the host CPU, one subframe after another, the
 * way dlsim's phy_proc_tx timer covers it (dlsim.c:2167-2699, generate_dci_top / generate_pilots
 * excluded), with every stage that has a buildable reference translation unit running the
 * REFERENCE's own code, compiled unmodified into oracle/_ref (oracle/Makefile), and the others the
 * oracle's restatement (oracle/liboracle.so):
 *
 *   stage                  runs                                   reference
 *   crc24a                 ref  crc24a                           crc_byte.c:117 (libref_coding.so)
 *   segmentation           ref  lte_segmentation (+ its crc24b)  lte_segmentation.c:39 (libref_seg.so)
 *   turbo_encoder          port orc_turbo_encode                 3gpplte_sse.c:380 (lte_interleaver.h blob missing)
 *   subblock_interleaving  ref  sub_block_interleaving_turbo     lte_rate_matching.c:51 (libref_rm.so)
 *   rate_matching          ref  lte_rate_matching_turbo          lte_rate_matching.c:464 (libref_rm.so)
 *   scrambling             ref  dlsch_scrambling                 dlsch_scrambling.c:51 (libref_mod.so, over
 *                                                                lte_gold.c's lte_gold_generic, libref_gold.so)
 *   modulation             ref  dlsch_modulation                 dlsch_modulation.c:1181 (libref_mod.so)
 *   ofdm_mod               ref  do_OFDM_mod x 2 slots            ofdm_mod.c:233 -> normal_prefix_mod :47 ->
 *                               (IDFT + CP + slot layout)        PHY_ofdm_mod :85 -> idft2048 (libref_ofdm.so,
 *                                                                libref_dfts.so)
 *
 * A stage whose reference library is absent falls back to the port and says so.  The first
 * subframe's IQ is checked bit-exactly against orc_tx_subframe (the oracle's whole chain), so the
 * composition does the same work.  Output: one JSON line with the per-stage microseconds per
 * subframe, the subframes done and the rate from the stage-time sum.
 *
 *   cpu_baseline SECONDS SEED N_RB n_ant mode1 n_cw mimo_mode npdcch subframe Kmimo mcs0 mcs1 TBS0 TBS1
 *                ra0 ra1 ra2 ra3 nb_rb rnti
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <libgen.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "../include/oai4g_qpp.h"
#include "oai_oracle.h"

enum { S_CRC, S_SEG, S_TURBO, S_SBI, S_RM, S_SCR, S_MOD, S_OFDM, S_N };
static const char *S_NAME[S_N] = {"crc24a", "segmentation", "turbo_encoder", "subblock_interleaving",
                                  "rate_matching", "scrambling", "modulation", "ofdm_mod"};

static uint32_t (*ref_crc24a)(uint8_t *, uint32_t);
static void (*ref_crcTableInit)(void);
static uint32_t (*ref_sbi)(uint32_t, uint8_t *, uint8_t *);
static uint32_t (*ref_rm)(uint32_t, uint32_t, uint8_t *, uint8_t *, uint8_t, uint32_t, uint8_t, uint8_t, uint8_t,
                          uint8_t, uint8_t, uint8_t, uint8_t, uint8_t);
static uint32_t (*ref_gold)(uint32_t *, uint32_t *, uint8_t);
static int (*ref_seg)(uint8_t *, uint8_t **, unsigned, unsigned *, unsigned *, unsigned *, unsigned *, unsigned *,
                      unsigned *);
static void (*ref_do_ofdm)(int32_t **, int32_t **, uint32_t, uint16_t, const int32_t *);
/* oracle/ref_glue_mod.c over dlsch_modulation.c / dlsch_scrambling.c (libref_mod.so) */
typedef struct {
  const uint8_t *e;
  int32_t G;
  uint8_t mcs, mimo_mode, Nlayers, first_layer;
  uint32_t rb_alloc[4];
  uint16_t nb_rb, pmi_alloc;
} ref_cw_t;
static uint8_t *(*ref_harq_e)(int);
static void (*ref_set_cw)(int, const ref_cw_t *, uint16_t, int16_t, int16_t);
static void (*ref_scramble_cw)(int, const int32_t *, int, uint8_t, uint8_t);
static int (*ref_modulate)(int32_t **, int16_t, uint32_t, const int32_t *, uint8_t, int);

static double now(void)
{
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

static void *ref_open(const char *dir, const char *name, int mode)
{
  char p[4096];
  snprintf(p, sizeof(p), "%s/_ref/%s", dir, name);
  return dlopen(p, mode | RTLD_LOCAL);
}

static uint64_t splitmix64(uint64_t *s)
{
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int main(int argc, char **argv)
{
  if (argc < 21) {
    fprintf(stderr, "usage: see the header of oracle/cpu_baseline.c\n");
    return 2;
  }
  char exe[4096];
  ssize_t n_exe = readlink("/proc/self/exe", exe, sizeof(exe) - 1);
  if (n_exe <= 0) return 2;
  exe[n_exe] = 0;
  const char *dir = dirname(exe);

  const double seconds = atof(argv[1]);
  uint64_t seed = strtoull(argv[2], NULL, 0);
  orc_tx_cfg_t cfg;
  memset(&cfg, 0, sizeof(cfg));
  const int N_RB = atoi(argv[3]), n_ant = atoi(argv[4]), mode1 = atoi(argv[5]);
  cfg.n_cw = (uint8_t)atoi(argv[6]);
  cfg.mimo_mode = (uint8_t)atoi(argv[7]);
  cfg.num_pdcch_symbols = (uint8_t)atoi(argv[8]);
  cfg.subframe = (uint8_t)atoi(argv[9]);
  cfg.Kmimo = (uint8_t)atoi(argv[10]);
  cfg.mcs[0] = (uint8_t)atoi(argv[11]);
  cfg.mcs[1] = (uint8_t)atoi(argv[12]);
  cfg.TBS[0] = (uint32_t)atoi(argv[13]);
  cfg.TBS[1] = (uint32_t)atoi(argv[14]);
  for (int i = 0; i < 4; i++) cfg.rb_alloc[i] = (uint32_t)strtoul(argv[15 + i], NULL, 0);
  cfg.nb_rb = (uint16_t)atoi(argv[19]);
  cfg.rnti = (uint16_t)atoi(argv[20]);
  cfg.amp = 512;
  cfg.sqrt_rho_a = cfg.sqrt_rho_b = 8192;
  cfg.Mdlharq = 8;
  if (orc_init_frame(&cfg.fp, (uint16_t)N_RB, 0, 0, (uint8_t)n_ant, (uint8_t)mode1, 0) != 0) return 2;
  const orc_frame_t *fp = &cfg.fp;
  const int N = fp->ofdm_symbol_size, nsymb = fp->symbols_per_tti, spt = (int)fp->samples_per_tti;

  /* the reference's own code where it builds (oracle/_ref); the port otherwise */
  void *hc = ref_open(dir, "libref_coding.so", RTLD_NOW), *hr = ref_open(dir, "libref_rm.so", RTLD_NOW);
  void *hg = ref_open(dir, "libref_gold.so", RTLD_NOW), *hs = ref_open(dir, "libref_seg.so", RTLD_NOW);
  /* RTLD_LAZY: ofdm_mod.c's LOG_D (logRecord) sits on the PMCH branch only (oracle/ref_glue_ofdm.c) */
  void *ho = ref_open(dir, "libref_ofdm.so", RTLD_LAZY);
  /* RTLD_LAZY: logRecord (LOG_E / LOG_W) sits on dlsch_modulation's unsupported-mode branches only */
  void *hm = ref_open(dir, "libref_mod.so", RTLD_LAZY);
  if (hc) {
    ref_crc24a = (uint32_t(*)(uint8_t *, uint32_t))dlsym(hc, "crc24a");
    ref_crcTableInit = (void (*)(void))dlsym(hc, "crcTableInit");
    if (ref_crcTableInit) ref_crcTableInit();
    if (!ref_crcTableInit) ref_crc24a = NULL;
  }
  if (hr) {
    ref_sbi = (uint32_t(*)(uint32_t, uint8_t *, uint8_t *))dlsym(hr, "sub_block_interleaving_turbo");
    ref_rm = (uint32_t(*)(uint32_t, uint32_t, uint8_t *, uint8_t *, uint8_t, uint32_t, uint8_t, uint8_t, uint8_t, uint8_t,
                          uint8_t, uint8_t, uint8_t, uint8_t))dlsym(hr, "lte_rate_matching_turbo");
  }
  if (hg) ref_gold = (uint32_t(*)(uint32_t *, uint32_t *, uint8_t))dlsym(hg, "lte_gold_generic");
  /* lte_segmentation's crc24b is libref_coding.so's (the same loaded object: DT_NEEDED via $ORIGIN),
   * whose table crcTableInit filled above */
  if (hs && ref_crc24a)
    ref_seg = (int (*)(uint8_t *, uint8_t **, unsigned, unsigned *, unsigned *, unsigned *, unsigned *, unsigned *,
                       unsigned *))dlsym(hs, "lte_segmentation");
  if (ho) ref_do_ofdm = (void (*)(int32_t **, int32_t **, uint32_t, uint16_t, const int32_t *))dlsym(ho, "ref_glue_do_OFDM_mod");
  if (hm) {
    ref_harq_e = (uint8_t * (*)(int)) dlsym(hm, "ref_glue_harq_e");
    ref_set_cw = (void (*)(int, const ref_cw_t *, uint16_t, int16_t, int16_t))dlsym(hm, "ref_glue_set_cw");
    ref_scramble_cw = (void (*)(int, const int32_t *, int, uint8_t, uint8_t))dlsym(hm, "ref_glue_scramble_cw");
    ref_modulate = (int (*)(int32_t **, int16_t, uint32_t, const int32_t *, uint8_t, int))dlsym(hm, "ref_glue_modulate");
    if (!ref_harq_e || !ref_set_cw || !ref_scramble_cw || !ref_modulate) ref_modulate = NULL;
  }
  /* the reference modulation reads the e bits from its own HARQ structure, which the reference
   * scrambling writes: both or neither */
  const int ref_mod_ok = ref_modulate != NULL && n_ant <= 2;
  const int use_ref[S_N] = {ref_crc24a != NULL, ref_seg != NULL, 0, ref_sbi != NULL, ref_rm != NULL,
                            ref_mod_ok || ref_gold != NULL, ref_mod_ok, ref_do_ofdm != NULL};
  const int32_t geom[9] = {fp->N_RB_DL, fp->Ncp, fp->nb_antennas_tx, N, fp->log2_symbol_size, fp->nb_prefix_samples,
                           fp->nb_prefix_samples0, nsymb, spt};
  const int32_t fmod[9] = {fp->N_RB_DL, fp->Ncp, fp->nb_antennas_tx, N, fp->first_carrier_offset, fp->nushift,
                           fp->mode1_flag, fp->frame_type, fp->Nid_cell};

  int G[2] = {0, 0};
  uint8_t Qm[2];
  for (int cw = 0; cw < cfg.n_cw; cw++) {
    Qm[cw] = orc_get_Qm(cfg.mcs[cw]);
    G[cw] = n_ant == 4 ? orc_count_pdsch_res(fp, cfg.rb_alloc, cfg.num_pdcch_symbols, cfg.subframe) * Qm[cw]
                       : orc_get_G(fp->N_RB_DL, fp->Ncp, fp->mode1_flag, fp->frame_type, cfg.nb_rb, cfg.rb_alloc, Qm[cw],
                                   1, cfg.num_pdcch_symbols, cfg.subframe);
  }
  /* buffers: 16-byte aligned as the reference's malloc16 gives them, sized from the TBS (+ CRC) */
  for (int cw = 0; cw < cfg.n_cw; cw++)
    if (cfg.TBS[cw] == 0 || cfg.TBS[cw] > 16 * 6120 - 24) {
      fprintf(stderr, "cpu_baseline: TBS %u outside 1..%d (16 code blocks)\n", cfg.TBS[cw], 16 * 6120 - 24);
      return 2;
    }
  const size_t abytes = (((cfg.TBS[0] > cfg.TBS[1] ? cfg.TBS[0] : cfg.TBS[1]) / 8 + 3 + 63) / 64 + 1) * 64;
  uint8_t *pay[2], *a[2], *e[2];
  for (int cw = 0; cw < 2; cw++) {
    pay[cw] = aligned_alloc(64, abytes);
    a[cw] = aligned_alloc(64, abytes);
    e[cw] = aligned_alloc(64, (size_t)((1 + (G[cw] >> 5)) * 32 + 128));
    if (cw < cfg.n_cw && ref_mod_ok) {
      /* rate matching writes into the reference HARQ structure's e, as dlsch_encoding does */
      free(e[cw]);
      e[cw] = ref_harq_e(cw);
      ref_cw_t rc;
      memset(&rc, 0, sizeof(rc));
      rc.mcs = cfg.mcs[cw];
      rc.mimo_mode = cfg.mimo_mode;
      rc.Nlayers = 1;
      memcpy(rc.rb_alloc, cfg.rb_alloc, sizeof(rc.rb_alloc));
      rc.nb_rb = cfg.nb_rb;
      ref_set_cw(cw, &rc, cfg.rnti, cfg.sqrt_rho_a, cfg.sqrt_rho_b);
    }
    for (size_t i = 0; i < abytes; i++) pay[cw][i] = (uint8_t)splitmix64(&seed);
  }
  static uint8_t cbuf[16][8 + 3 + 768];
  uint8_t *dbuf = aligned_alloc(64, 96 + 12 + 3 + 3 * 6144 + 128), *wbuf = aligned_alloc(64, 3 * 6176 + 128);
  int32_t *txF[4], *txd[4], *chk[4], *chkF[4];
  for (int aa = 0; aa < n_ant; aa++) {
    txF[aa] = aligned_alloc(64, (size_t)10 * nsymb * N * 4);
    txd[aa] = aligned_alloc(64, (size_t)10 * spt * 4 + 64);      /* the frame, as do_OFDM_mod indexes it */
    chk[aa] = aligned_alloc(64, (size_t)spt * 4 + 64);
    chkF[aa] = aligned_alloc(64, (size_t)nsymb * N * 4);
    memset(txF[aa], 0, (size_t)10 * nsymb * N * 4);
  }

  double st[S_N];
  memset(st, 0, sizeof(st));
  long done = 0;
  const double t_start = now();
  for (;;) {
    double t0, t1;
    for (int cw = 0; cw < cfg.n_cw; cw++) {
      const uint32_t A = cfg.TBS[cw];
      memcpy(a[cw], pay[cw], A / 8);
      t0 = now();
      uint32_t crc = (use_ref[S_CRC] ? ref_crc24a(a[cw], A) : orc_crc24a(a[cw], (int)A)) >> 8;   /* dlsch_coding.c:296 */
      a[cw][A >> 3] = (uint8_t)(crc >> 16);
      a[cw][1 + (A >> 3)] = (uint8_t)(crc >> 8);
      a[cw][2 + (A >> 3)] = (uint8_t)crc;
      t1 = now(); st[S_CRC] += t1 - t0; t0 = t1;
      uint32_t C, Cp, Cm, Kp, Km, F;
      uint8_t *cptr[16];
      for (int r = 0; r < 16; r++) cptr[r] = cbuf[r];
      if ((use_ref[S_SEG] ? ref_seg(a[cw], cptr, A + 24, &C, &Cp, &Cm, &Kp, &Km, &F)
                          : orc_segmentation(a[cw], cptr, A + 24, &C, &Cp, &Cm, &Kp, &Km, &F)) < 0)
        return 3;
      t1 = now(); st[S_SEG] += t1 - t0;
      uint32_t r_off = 0;
      for (uint32_t r = 0; r < C; r++) {
        const uint32_t Kr = r < Cm ? Km : Kp;
        const int qi = oai4g_qpp_index(Kr);
        t0 = now();
        memset(dbuf, ORC_LTE_NULL, 96);
        orc_turbo_encode(cptr[r], (uint16_t)(Kr >> 3), dbuf + 96, oai4g_qpp_table[qi].f1, oai4g_qpp_table[qi].f2);
        t1 = now(); st[S_TURBO] += t1 - t0; t0 = t1;
        uint32_t RTC = use_ref[S_SBI] ? ref_sbi(Kr + 4, dbuf + 96, wbuf) : orc_subblock_interleave(Kr + 4, dbuf + 96, wbuf);
        t1 = now(); st[S_SBI] += t1 - t0; t0 = t1;
        r_off += use_ref[S_RM] ? ref_rm(RTC, (uint32_t)G[cw], wbuf, e[cw] + r_off, (uint8_t)C, ORC_NSOFT, cfg.Mdlharq,
                                        cfg.Kmimo, 0, Qm[cw], 1, (uint8_t)r, 0, 0)
                               : orc_rate_match(RTC, (uint32_t)G[cw], wbuf, e[cw] + r_off, (uint8_t)C, ORC_NSOFT,
                                                cfg.Mdlharq, cfg.Kmimo, 0, Qm[cw], 1, (uint8_t)r);
        t1 = now(); st[S_RM] += t1 - t0;
      }
      /* dlsch_scrambling (dlsch_scrambling.c:51-97; dlsim passes q = 0, Ns = 2 subframe) */
      t0 = now();
      if (ref_mod_ok) {
        ref_scramble_cw(cw, fmod, G[cw], 0, (uint8_t)(2 * cfg.subframe));
      } else {       /* the loop restated around the reference's (or the oracle's) Gold generator */
        uint32_t x1 = 0, x2 = ((uint32_t)cfg.rnti << 14) + ((uint32_t)cfg.subframe << 9) + fp->Nid_cell;
        uint32_t (*gold)(uint32_t *, uint32_t *, uint8_t) = ref_gold ? ref_gold : orc_gold_generic;
        uint32_t s = gold(&x1, &x2, 1);
        uint8_t *ep = e[cw];
        for (int i = 0, k = 0; i < 1 + (G[cw] >> 5); i++) {
          for (int j = 0; j < 32; j++, k++) ep[k] = (ep[k] & 1) ^ ((s >> j) & 1);
          s = gold(&x1, &x2, 0);
        }
      }
      t1 = now(); st[S_SCR] += t1 - t0;
    }
    /* dlsch_modulation into the frame grid (dlsim zeroes txdataF before its timer, dlsim.c:2161) */
    for (int aa = 0; aa < n_ant; aa++) memset(txF[aa] + (size_t)cfg.subframe * nsymb * N, 0, (size_t)nsymb * N * 4);
    t0 = now();
    if (ref_mod_ok) {
      if (ref_modulate(txF, cfg.amp, cfg.subframe, fmod, cfg.num_pdcch_symbols, cfg.n_cw) < 0) return 3;
    } else {
      orc_cw_t c0 = {e[0], cfg.mcs[0], cfg.mimo_mode, 1, {0}}, c1 = {e[1], cfg.mcs[1], cfg.mimo_mode, 1, {0}};
      memcpy(c0.rb_alloc, cfg.rb_alloc, sizeof(c0.rb_alloc));
      memcpy(c1.rb_alloc, cfg.rb_alloc, sizeof(c1.rb_alloc));
      if (orc_modulation(txF, cfg.amp, cfg.subframe, fp, cfg.num_pdcch_symbols, &c0, cfg.n_cw > 1 ? &c1 : NULL,
                         cfg.sqrt_rho_a, cfg.sqrt_rho_b) < 0)
        return 3;
    }
    t1 = now(); st[S_MOD] += t1 - t0;
    /* do_OFDM_mod_l x 2 slots (dlsim.c:2680-2699) -> normal_prefix_mod -> PHY_ofdm_mod, normal CP */
    t0 = now();
    for (int slot = 2 * cfg.subframe; slot < 2 * cfg.subframe + 2; slot++) {
      if (use_ref[S_OFDM]) ref_do_ofdm(txF, txd, 0, (uint16_t)slot, geom);
      else orc_do_OFDM_mod(txF, txd, 0, (uint16_t)slot, fp);
    }
    t1 = now(); st[S_OFDM] += t1 - t0;
    if (done == 0) {
      /* the composition against the oracle's whole chain, bit for bit */
      uint8_t *pp[2] = {a[0], a[1]};
      for (int cw = 0; cw < cfg.n_cw; cw++) memcpy(a[cw], pay[cw], cfg.TBS[cw] / 8);
      if (orc_tx_subframe(&cfg, pp, chkF, chk, NULL) != 0) return 4;
      for (int aa = 0; aa < n_ant; aa++)
        if (memcmp(chk[aa], txd[aa] + (size_t)cfg.subframe * spt, (size_t)spt * 4) != 0) {
          fprintf(stderr, "cpu_baseline: composed IQ differs from orc_tx_subframe (antenna %d)\n", aa);
          return 5;
        }
    }
    done++;
    if (now() - t_start >= seconds) break;
  }
  double tot = 0, port = 0;
  for (int k = 0; k < S_N; k++) {
    tot += st[k];
    if (!use_ref[k] || (k == S_SCR && !ref_mod_ok)) port += st[k];   /* a restated loop around the ref generator is a port */
  }
  printf("{\"subframes\": %ld, \"wall_s\": %.6f, \"stage_s\": %.6f, \"rate\": %.3f, \"validated\": true, "
         "\"port_share\": %.4f, \"stage_us\": {",
         done, now() - t_start, tot, done / tot, port / tot);
  for (int k = 0; k < S_N; k++) printf("%s\"%s\": %.3f", k ? ", " : "", S_NAME[k], 1e6 * st[k] / done);
  printf("}, \"impl\": {");
  for (int k = 0; k < S_N; k++)
    printf("%s\"%s\": \"%s\"", k ? ", " : "", S_NAME[k],
           use_ref[k] ? (k == S_SCR && !ref_mod_ok ? "reference generator + port loop" : "reference") : "port");
  printf("}}\n");
  return 0;
}
