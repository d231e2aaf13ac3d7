/*
 * dlsim_tx — C host driver of the MI355X DLSCH transmit path (north_star:
 * "host code stays in C and calls into a thin C-ABI HIP layer").  Plain C (gcc), linked
 * against openair4g_amd/lib/libopenair4g_amd.so, no Python.
 *
 * It runs dlsim's transmit loop (openair1/SIMULATION/LTE_PHY/dlsim.c:2567-2699) two ways:
 *
 *   drop-in : per subframe, per codeword dlsch_encoding (dlsim.c:2613) -> get_G ->
 *             dlsch_scrambling(fp, 0, dlsch, G, 0, subframe << 1) (:2642-2647), then
 *             dlsch_modulation into the pre-zeroed frame grid (:2666, :2161-2163) and
 *             do_OFDM_mod of both slots (:2688-2696), through the oai4g_ drop-in entry points
 *             on host buffers (what a dlsim linked with INTEGRATION.md's shim executes);
 *   batch   : the device-resident oai4g_tx_batch over -B subframes per launch.
 *
 * and prints dlsim -P style timing ("Total PHY proc tx" = mean over the trials).  Options:
 *   -c C1|C2|C3|C4|TM2   configuration (bench.py / openair4g_amd CONFIGS)
 *   -s subframe          subframe index (default 7, dlsim's default, :304)
 *   -n trials            drop-in subframes to time (default 10)
 *   -B batch             subframes per batched launch (default 1024; 0 = skip the batch path)
 *   -i payload.bin       n_cw transport blocks of TBS/8 bytes (default: splitmix64 bytes)
 *   -o iq_dropin.bin     IQ of the drop-in subframe [n_ant][samples_per_tti] int32
 *   -O iq_batch.bin      IQ of batch element 0
 *   -P                   print the timing lines
 *   -g N                 multi-GPU: fork N ranks before any HIP call, one per GPU; rank 0
 *                        builds the parameter block and oai4g_dist_broadcast_params (RCCL over xGMI)
 *                        hands it to the others; each rank runs the batch path over its shard
 *                        (oai4g_shard_range) of N x B global subframes with payloads derived from
 *                        (seed, global subframe index) (oai4g_payload_seed); the per-rank IQ checksums
 *                        are summed and the step times max-reduced over the ranks (RCCL); rank 0
 *                        prints "world N checksum 0x..." and the aggregate rate.  The checksum does
 *                        not depend on N.  No drop-in path in this mode.
 * Exit code 0 when both paths ran and (with -B) their IQ agree, 1 otherwise.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include "oai4g.h"

typedef struct {
  const char *name;
  uint16_t N_RB_DL;
  uint8_t n_ant, mode1, n_cw, mimo_mode, npdcch, Kmimo, mcs0, mcs1;
} cfg_t;

static const cfg_t CFGS[] = {
    {"C1", 6, 1, 1, 1, OAI4G_SISO, 3, 1, 9, 0},
    {"C2", 100, 1, 1, 1, OAI4G_SISO, 1, 1, 16, 0},
    {"C3", 100, 2, 0, 2, OAI4G_LARGE_CDD, 1, 2, 19, 19},
    {"C4", 100, 4, 0, 2, OAI4G_LARGE_CDD, 1, 2, 19, 19},
    {"TM2", 100, 2, 0, 1, OAI4G_ALAMOUTI, 1, 1, 16, 0},
};

static double now_us(void)
{
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static void full_alloc(uint16_t nrb, uint32_t ra[4])
{
  memset(ra, 0, 4 * sizeof(uint32_t));
  for (int i = 0; i < nrb; i++) ra[i >> 5] |= 1u << (i & 31);
}

static uint64_t splitmix64(uint64_t *s)
{
  uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

#define CHECK(x, msg)                                                                    \
  do {                                                                                   \
    if (!(x)) {                                                                          \
      fprintf(stderr, "dlsim_tx: %s (%s)\n", msg, oai4g_last_error());                  \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

/* the batch path of one rank of -g N: parameters broadcast from rank 0, this rank's shard of the
 * N x batch global subframes, checksum and timing reduced over the ranks */
static int dist_batch(const cfg_t *c, int subframe, int batch, int rank, int world, int print_timing)
{
  oai4g_tx_params_t p;
  memset(&p, 0, sizeof(p));
  if (rank == 0) {
    uint32_t ra[4];
    full_alloc(c->N_RB_DL, ra);
    p.N_RB_DL = c->N_RB_DL;
    p.nb_antennas_tx = c->n_ant;
    p.mode1_flag = c->mode1;
    p.n_cw = c->n_cw;
    p.mimo_mode = c->mimo_mode;
    p.num_pdcch_symbols = c->npdcch;
    p.Kmimo = c->Kmimo;
    p.Mdlharq = 8;
    p.first_subframe = (uint8_t)subframe;
    p.rnti = 0x1234;
    p.amp = 512;
    p.sqrt_rho_a = p.sqrt_rho_b = 8192;
    memcpy(p.rb_alloc, ra, sizeof(ra));
    p.nb_rb = c->N_RB_DL;
    const uint8_t mcs[2] = {c->mcs0, c->mcs1};
    uint32_t maxA = 0;
    for (int cw = 0; cw < c->n_cw; cw++) {
      p.mcs[cw] = mcs[cw];
      p.TBS[cw] = oai4g_get_TBS_DL(mcs[cw], c->N_RB_DL) << 3;
      if (p.TBS[cw] / 8 > maxA) maxA = p.TBS[cw] / 8;
    }
    p.payload_stride = (maxA + 3 + 15) & ~15u;
  }
  CHECK(oai4g_dist_broadcast_params(&p, 0) == 0, "dist_broadcast_params");
  int first = 0, count = 0;
  oai4g_shard_range(world * batch, rank, world, &first, &count);
  oai4g_tx_config_t *cfg = oai4g_tx_config_create(&p);
  CHECK(cfg, "tx_config_create (broadcast parameters)");
  const size_t spt = oai4g_tx_iq_samples(cfg);
  const size_t pbytes = (size_t)count * p.n_cw * p.payload_stride, iqn = (size_t)count * p.nb_antennas_tx * spt;
  uint8_t *d_pay = (uint8_t *)oai4g_dev_alloc(pbytes);
  void *d_work = oai4g_dev_alloc(oai4g_tx_workspace_bytes(cfg, count));
  int32_t *d_iq = (int32_t *)oai4g_dev_alloc(iqn * 4);
  CHECK(d_pay && d_work && d_iq, "device allocation");
  CHECK(oai4g_fill_payload(d_pay, pbytes, oai4g_payload_seed(0x5EED, (uint64_t)first, p.n_cw, p.payload_stride),
                           NULL) == 0, "fill_payload");
  CHECK(oai4g_tx_batch(cfg, count, d_pay, d_work, d_iq, NULL) == 0 && oai4g_sync() == 0, "tx_batch (warm-up)");
  CHECK(oai4g_dist_barrier() == 0, "barrier");
  const int reps = 10;
  const double b0 = now_us();
  for (int r = 0; r < reps; r++) CHECK(oai4g_tx_batch(cfg, count, d_pay, d_work, d_iq, NULL) == 0, "tx_batch");
  CHECK(oai4g_sync() == 0, "sync");
  double dt = (now_us() - b0) / reps;
  CHECK(oai4g_dist_allreduce_max_f64(&dt, 1) == 0, "allreduce max");
  /* position-weighted IQ checksum of this shard: additive over ranks, independent of N */
  uint32_t *iq = (uint32_t *)malloc(iqn * 4);
  CHECK(iq && oai4g_memcpy_d2h(iq, d_iq, iqn * 4) == 0, "IQ download");
  uint64_t sums[2] = {0, (uint64_t)count};
  const size_t per_sf = (size_t)p.nb_antennas_tx * spt;
  for (size_t i = 0; i < iqn; i++) {
    const uint64_t g = (uint64_t)first * per_sf + i;
    sums[0] += (uint64_t)iq[i] * (g * 0x9E3779B97F4A7C15ull + 1);
  }
  free(iq);
  CHECK(oai4g_dist_allreduce_sum_u64(sums, 2) == 0, "allreduce sum");
  if (rank == 0) {
    printf("dlsim_tx %s world %d checksum 0x%016llx subframes %llu\n", c->name, world, (unsigned long long)sums[0],
           (unsigned long long)sums[1]);
    if (print_timing)
      printf("[batch x%d] %.0f subframes/s aggregate (%d subframes per GPU per launch, max over ranks %.1f us)\n",
             world, 1e6 * (double)sums[1] / dt, batch, dt);
  }
  oai4g_dev_free(d_pay);
  oai4g_dev_free(d_work);
  oai4g_dev_free(d_iq);
  oai4g_tx_config_destroy(cfg);
  CHECK(oai4g_dist_finalize() == 0, "dist_finalize");
  return 0;
}

int main(int argc, char **argv)
{
  const char *cname = "C3", *pay_file = NULL, *out_drop = NULL, *out_batch = NULL;
  int subframe = 7, trials = 10, batch = 1024, print_timing = 0, opt, world = 0, rank = 0;
  while ((opt = getopt(argc, argv, "c:s:n:B:i:o:O:Pg:")) != -1) {
    switch (opt) {
    case 'c': cname = optarg; break;
    case 's': subframe = atoi(optarg); break;
    case 'n': trials = atoi(optarg); break;
    case 'B': batch = atoi(optarg); break;
    case 'i': pay_file = optarg; break;
    case 'o': out_drop = optarg; break;
    case 'O': out_batch = optarg; break;
    case 'P': print_timing = 1; break;
    case 'g': world = atoi(optarg); break;
    default:
      fprintf(stderr, "usage: %s [-c C1|C2|C3|C4|TM2] [-s sf] [-n trials] [-B batch] [-i pay] [-o iq] [-O iq] [-P]\n",
              argv[0]);
      return 2;
    }
  }
  const cfg_t *c = NULL;
  for (size_t i = 0; i < sizeof(CFGS) / sizeof(CFGS[0]); i++)
    if (!strcmp(CFGS[i].name, cname)) c = &CFGS[i];
  if (!c || subframe < 0 || subframe > 9 || trials < 1) {
    fprintf(stderr, "dlsim_tx: bad configuration / subframe / trials\n");
    return 2;
  }
  if (world > 0) {
    /* one process per GPU: fork the ranks before anything touches HIP; rank 0's RCCL unique id
     * reaches the others through pipes */
    if (batch < 1 || world > 64) {
      fprintf(stderr, "dlsim_tx: -g needs -B >= 1 and at most 64 ranks\n");
      return 2;
    }
    int fds[64][2];
    for (int r = 1; r < world; r++) CHECK(pipe(fds[r]) == 0, "pipe");
    pid_t pids[64];
    for (int r = 0; r < world; r++) {
      pids[r] = fork();
      CHECK(pids[r] >= 0, "fork");
      if (pids[r] == 0) {
        /* keep only this rank's end of the id pipes: a rank 0 that fails before writing the id
         * then closes the last write end, and the other ranks read EOF and exit non-zero */
        rank = r;
        for (int q = 1; q < world; q++) {
          if (r != 0) close(fds[q][1]);
          if (q != r) close(fds[q][0]);
        }
        goto rank_main;
      }
    }
    for (int q = 1; q < world; q++) {
      close(fds[q][0]);
      close(fds[q][1]);
    }
    int rc_all = 0;
    for (int r = 0; r < world; r++) {
      int st = 0;
      waitpid(pids[r], &st, 0);
      if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) rc_all = 1;
    }
    return rc_all;
  rank_main:
    CHECK(oai4g_set_device(rank) == 0, "set_device");
    CHECK(oai4g_init() == 0, "no usable gfx950 device");
    uint8_t id[OAI4G_DIST_ID_BYTES];
    if (rank == 0) {
      CHECK(oai4g_dist_unique_id(id) == 0, "dist_unique_id");
      for (int r = 1; r < world; r++) CHECK(write(fds[r][1], id, sizeof(id)) == (ssize_t)sizeof(id), "id pipe write");
    } else {
      CHECK(read(fds[rank][0], id, sizeof(id)) == (ssize_t)sizeof(id), "id pipe read");
    }
    CHECK(oai4g_dist_init(rank, world, id) == 0, "dist_init");
    return dist_batch(c, subframe, batch, rank, world, print_timing);
  }
  CHECK(oai4g_init() == 0, "no usable gfx950 device");

  oai4g_frame_parms_t fp;
  CHECK(oai4g_init_frame_parms(&fp, c->N_RB_DL, 0, 0, c->n_ant, c->mode1, 0) == 0, "init_frame_parms");
  uint32_t ra[4];
  full_alloc(c->N_RB_DL, ra);
  const uint8_t mcs[2] = {c->mcs0, c->mcs1};
  uint32_t TBS[2] = {0, 0};
  uint8_t *pay[2] = {NULL, NULL};
  uint64_t seed = 0x5EED;
  FILE *pf = pay_file ? fopen(pay_file, "rb") : NULL;
  CHECK(!pay_file || pf, "cannot open the payload file");
  for (int cw = 0; cw < c->n_cw; cw++) {
    TBS[cw] = oai4g_get_TBS_DL(mcs[cw], c->N_RB_DL) << 3;     /* dlsim: get_TBS_DL << 3 */
    pay[cw] = (uint8_t *)calloc(TBS[cw] / 8 + 8, 1);
    if (pf) {
      CHECK(fread(pay[cw], 1, TBS[cw] / 8, pf) == TBS[cw] / 8, "short payload file");
    } else {
      for (uint32_t i = 0; i < TBS[cw] / 8; i++) pay[cw][i] = (uint8_t)splitmix64(&seed);
    }
  }
  if (pf) fclose(pf);

  /* ---------------- drop-in path: dlsim's per-subframe loop ---------------- */
  const int N = fp.ofdm_symbol_size, nsymb = fp.symbols_per_tti;
  const size_t spt = fp.samples_per_tti;
  int32_t *txdataF[4], *txdata[4];
  for (int aa = 0; aa < c->n_ant; aa++) {
    txdataF[aa] = (int32_t *)aligned_alloc(64, (size_t)10 * nsymb * N * 4);
    txdata[aa] = (int32_t *)aligned_alloc(64, 10 * spt * 4);
    memset(txdataF[aa], 0, (size_t)10 * nsymb * N * 4);
    memset(txdata[aa], 0, 10 * spt * 4);
  }
  oai4g_dlsch_t *dl[2] = {NULL, NULL};
  for (int cw = 0; cw < c->n_cw; cw++) {
    dl[cw] = oai4g_new_dlsch(c->Kmimo, 8, c->N_RB_DL);
    CHECK(dl[cw], "new_dlsch");
    dl[cw]->rnti = 0x1234;                                 /* dlsim.c:258 */
    dl[cw]->current_harq_pid = 0;
    oai4g_dl_harq_t *h = dl[cw]->harq_processes[0];
    h->TBS = TBS[cw];
    h->mcs = mcs[cw];
    h->rvidx = 0;
    h->round = 0;
    h->mimo_mode = c->mimo_mode;
    memcpy(h->rb_alloc, ra, sizeof(ra));
    h->nb_rb = c->N_RB_DL;
    h->Nl = 1;
  }
  const int drop_ok = c->n_ant <= 2;                      /* the drop-in modulation covers 1-2 ports */
  double t_enc = 0, t_scr = 0, t_mod = 0, t_ofdm = 0, t_tot = 0;
  uint8_t *a[2];
  for (int cw = 0; cw < c->n_cw; cw++) a[cw] = (uint8_t *)calloc(TBS[cw] / 8 + 8, 1);
  for (int t = 0; drop_ok && t < trials; t++) {
    const double t0 = now_us();
    for (int cw = 0; cw < c->n_cw; cw++) {
      memcpy(a[cw], pay[cw], TBS[cw] / 8);
      const double e0 = now_us();
      CHECK(oai4g_dlsch_encoding(a[cw], &fp, c->npdcch, dl[cw], 0, (uint8_t)subframe) == 0, "dlsch_encoding");
      const double e1 = now_us();
      const int G = oai4g_get_G(&fp, c->N_RB_DL, ra, oai4g_get_Qm(mcs[cw]), 1, c->npdcch, 0, (uint8_t)subframe);
      oai4g_dlsch_scrambling(&fp, 0, dl[cw], G, 0, (uint8_t)(subframe << 1));
      t_enc += e1 - e0;
      t_scr += now_us() - e1;
    }
    for (int aa = 0; aa < c->n_ant; aa++) memset(txdataF[aa] + (size_t)subframe * nsymb * N, 0, (size_t)nsymb * N * 4);
    const double m0 = now_us();
    CHECK(oai4g_dlsch_modulation(txdataF, 512, subframe, &fp, c->npdcch, dl[0], dl[1]) > 0, "dlsch_modulation");
    const double m1 = now_us();
    oai4g_do_OFDM_mod(txdataF, txdata, 0, (uint16_t)(subframe << 1), &fp);
    oai4g_do_OFDM_mod(txdataF, txdata, 0, (uint16_t)((subframe << 1) + 1), &fp);
    const double m2 = now_us();
    t_mod += m1 - m0;
    t_ofdm += m2 - m1;
    t_tot += m2 - t0;
  }
  if (print_timing && drop_ok) {
    printf("[drop-in] DLSCH encoding time      : %10.1f us (%d trials)\n", t_enc / trials, trials);
    printf("[drop-in] DLSCH scrambling time    : %10.1f us\n", t_scr / trials);
    printf("[drop-in] DLSCH modulation time    : %10.1f us\n", t_mod / trials);
    printf("[drop-in] OFDM_mod time            : %10.1f us\n", t_ofdm / trials);
    printf("[drop-in] Total PHY proc tx        : %10.1f us per subframe (%.0f subframes/s, host buffers, PCIe "
           "included)\n", t_tot / trials, 1e6 * trials / t_tot);
  }
  if (out_drop && drop_ok) {
    FILE *f = fopen(out_drop, "wb");
    CHECK(f, "cannot write the drop-in IQ");
    for (int aa = 0; aa < c->n_ant; aa++) fwrite(txdata[aa] + (size_t)subframe * spt, 4, spt, f);
    fclose(f);
  }

  /* ---------------- batched device-resident path ---------------- */
  int rc = 0;
  if (batch > 0) {
    oai4g_tx_params_t p;
    memset(&p, 0, sizeof(p));
    p.N_RB_DL = c->N_RB_DL;
    p.nb_antennas_tx = c->n_ant;
    p.mode1_flag = c->mode1;
    p.n_cw = c->n_cw;
    p.mimo_mode = c->mimo_mode;
    p.num_pdcch_symbols = c->npdcch;
    p.Kmimo = c->Kmimo;
    p.Mdlharq = 8;
    p.first_subframe = (uint8_t)subframe;
    p.rnti = 0x1234;
    p.amp = 512;
    p.sqrt_rho_a = p.sqrt_rho_b = 8192;
    memcpy(p.rb_alloc, ra, sizeof(ra));
    p.nb_rb = c->N_RB_DL;
    uint32_t maxA = 0;
    for (int cw = 0; cw < c->n_cw; cw++) {
      p.mcs[cw] = mcs[cw];
      p.TBS[cw] = TBS[cw];
      if (TBS[cw] / 8 > maxA) maxA = TBS[cw] / 8;
    }
    p.payload_stride = (maxA + 3 + 15) & ~15u;
    oai4g_tx_config_t *cfg = oai4g_tx_config_create(&p);
    CHECK(cfg, "tx_config_create");
    const size_t pbytes = (size_t)batch * c->n_cw * p.payload_stride, iqn = (size_t)batch * c->n_ant * spt;
    uint8_t *hp = (uint8_t *)calloc(pbytes, 1);
    for (int i = 0; i < batch; i++)
      for (int cw = 0; cw < c->n_cw; cw++) memcpy(hp + ((size_t)i * c->n_cw + cw) * p.payload_stride, pay[cw], TBS[cw] / 8);
    uint8_t *d_pay = (uint8_t *)oai4g_dev_alloc(pbytes);
    void *d_work = oai4g_dev_alloc(oai4g_tx_workspace_bytes(cfg, batch));
    int32_t *d_iq = (int32_t *)oai4g_dev_alloc(iqn * 4);
    CHECK(d_pay && d_work && d_iq, "device allocation");
    CHECK(oai4g_memcpy_h2d(d_pay, hp, pbytes) == 0, "payload upload");
    CHECK(oai4g_tx_batch(cfg, batch, d_pay, d_work, d_iq, NULL) == 0 && oai4g_sync() == 0, "tx_batch (warm-up)");
    const int reps = 10;
    const double b0 = now_us();
    for (int r = 0; r < reps; r++) CHECK(oai4g_tx_batch(cfg, batch, d_pay, d_work, d_iq, NULL) == 0, "tx_batch");
    CHECK(oai4g_sync() == 0, "sync");
    const double dt = (now_us() - b0) / reps;
    if (print_timing)
      printf("[batch]   Total PHY proc tx        : %10.3f us per subframe (%d subframes per launch, %.0f subframes/s, "
             "inputs resident in HBM)\n", dt / batch, batch, 1e6 * batch / dt);
    int32_t *iq0 = (int32_t *)malloc((size_t)c->n_ant * spt * 4);
    CHECK(oai4g_memcpy_d2h(iq0, d_iq, (size_t)c->n_ant * spt * 4) == 0, "IQ download");
    if (out_batch) {
      FILE *f = fopen(out_batch, "wb");
      CHECK(f, "cannot write the batch IQ");
      fwrite(iq0, 4, (size_t)c->n_ant * spt, f);
      fclose(f);
    }
    if (drop_ok)
      for (int aa = 0; aa < c->n_ant; aa++)
        if (memcmp(iq0 + (size_t)aa * spt, txdata[aa] + (size_t)subframe * spt, spt * 4)) {
          fprintf(stderr, "dlsim_tx: antenna %d: batch IQ differs from the drop-in IQ\n", aa);
          rc = 1;
        }
    free(iq0);
    free(hp);
    oai4g_dev_free(d_pay);
    oai4g_dev_free(d_work);
    oai4g_dev_free(d_iq);
    oai4g_tx_config_destroy(cfg);
  }
  for (int cw = 0; cw < c->n_cw; cw++) {
    oai4g_free_dlsch(dl[cw]);
    free(pay[cw]);
    free(a[cw]);
  }
  for (int aa = 0; aa < c->n_ant; aa++) {
    free(txdataF[aa]);
    free(txdata[aa]);
  }
  if (rc == 0 && print_timing) printf("dlsim_tx %s subframe %d: OK\n", c->name, subframe);
  return rc;
}
