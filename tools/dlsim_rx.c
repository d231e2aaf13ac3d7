/*
 * dlsim_rx — C host driver of dlsim's whole downlink loop on the GPU (north_star: "host code stays in
 * C and calls into a thin C-ABI HIP layer").  Plain C (gcc), linked against
 * openair4g_amd/lib/libopenair4g_amd.so, no Python.  Device-resident from payload to decoded bits:
 *
 *   eNB   oai4g_tx_batch            dlsch_encoding .. do_OFDM_mod with CRS (dlsim.c:2567-2699)
 *   UE    oai4g_fep_batch           slot_fep of every symbol (dlsim.c:2907-2931, slot_fep.c:40-177)
 *         oai4g_chest_batch         lte_dl_channel_estimation in dlsim's call order (perfect_ce = 0)
 *         oai4g_freq_offset_omega_batch + oai4g_freq_offset_update
 *                                   lte_est_freq_offset at l = 4 - Ncp, twice per subframe (slot_fep.c:211)
 *         oai4g_chest_time_batch    dl_ch_estimates_time (lte_dl_channel_estimation.c:704-738)
 *         oai4g_rx_batch            rx_pdsch TM1 + dlsch_unscrambling (dlsim.c:3236-3360)
 *         oai4g_ul_decode_batch     dlsch_decoding's per-block chain: RX rate matching, sub-block
 *                                   deinterleaving, the 16-bit turbo decoder with CRC24B / CRC24A
 *
 * over -n consecutive subframes starting at -s (the channel is the identity, as dlsim's AWGN at
 * infinite SNR).  The transport blocks are rebuilt from the decoded code blocks (lte_segmentation's
 * geometry: filler bits of block 0, CRC24B of each block when C > 1) and compared with the payload.
 * Options:
 *   -r N_RB_DL  (6 / 15 / 25 / 50 / 100, default 100)   -m mcs (default 16)
 *   -p num_pdcch_symbols (default 1)   -s first subframe (default 1)   -n subframes (default 4)
 *   -P          print the per-stage timing of one pass
 * Subframes 0 and 5 are refused: with even N_RB_DL the reference's receiver extracts the PBCH /
 * PSS / SSS REs as PDSCH, so those subframes do not close the loop in the reference either.
 * Exit code 0 when every transport block comes back bit-exact, 1 otherwise.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "oai4g.h"

#define CHECK(x, msg)                                                                    \
  do {                                                                                   \
    if (!(x)) {                                                                          \
      fprintf(stderr, "dlsim_rx: %s (%s)\n", msg, oai4g_last_error());                  \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

static double now_us(void)
{
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static int get_bit(const uint8_t *b, uint32_t i) { return (b[i >> 3] >> (7 - (i & 7))) & 1; }

int main(int argc, char **argv)
{
  int nrb = 100, mcs = 16, npdcch = 1, sf0 = 1, n_sf = 4, timing = 0, opt;
  while ((opt = getopt(argc, argv, "r:m:p:s:n:P")) != -1) {
    switch (opt) {
    case 'r': nrb = atoi(optarg); break;
    case 'm': mcs = atoi(optarg); break;
    case 'p': npdcch = atoi(optarg); break;
    case 's': sf0 = atoi(optarg); break;
    case 'n': n_sf = atoi(optarg); break;
    case 'P': timing = 1; break;
    default: fprintf(stderr, "usage: dlsim_rx [-r N_RB] [-m mcs] [-p npdcch] [-s subframe] [-n count] [-P]\n"); return 2;
    }
  }
  if (n_sf < 1 || n_sf > 9 || sf0 < 0 || sf0 > 9 || mcs < 0 || mcs > 28) { fprintf(stderr, "dlsim_rx: bad arguments\n"); return 2; }
  for (int i = 0; i < n_sf; i++)
    if ((sf0 + i) % 10 == 0 || (sf0 + i) % 10 == 5) {
      fprintf(stderr, "dlsim_rx: subframes 0 / 5 do not close the loop (PBCH / sync REs extracted as PDSCH)\n");
      return 2;
    }
  CHECK(oai4g_init() == 0, "init");
  oai4g_frame_parms_t fp;
  CHECK(oai4g_init_frame_parms(&fp, (uint16_t)nrb, 0, 0, 1, 1, 0) == 0, "init_frame_parms");
  const uint8_t Qm = mcs < 10 ? 2 : mcs < 17 ? 4 : 6;

  /* eNB: n_sf + 1 consecutive subframes (the last one's symbol 0 closes rows 12 / 13) */
  oai4g_tx_params_t p;
  memset(&p, 0, sizeof(p));
  p.N_RB_DL = (uint16_t)nrb;
  p.nb_antennas_tx = 1;
  p.mode1_flag = 1;
  p.n_cw = 1;
  p.mimo_mode = OAI4G_SISO;
  p.num_pdcch_symbols = (uint8_t)npdcch;
  p.Kmimo = 1;
  p.Mdlharq = 8;
  p.first_subframe = (uint8_t)sf0;
  p.subframe_step = 1;
  p.with_crs = 1;
  p.rnti = 0x1234;
  p.amp = 512;
  p.sqrt_rho_a = p.sqrt_rho_b = 8192;
  for (int i = 0; i < nrb; i++) p.rb_alloc[i >> 5] |= 1u << (i & 31);
  p.nb_rb = (uint16_t)nrb;
  p.mcs[0] = (uint8_t)mcs;
  p.TBS[0] = oai4g_get_TBS_DL((uint8_t)mcs, (uint16_t)nrb) << 3;
  p.payload_stride = (p.TBS[0] / 8 + 3 + 15) & ~15u;
  oai4g_tx_config_t *tx = oai4g_tx_config_create(&p);
  CHECK(tx, "tx_config_create");
  const int n_tx = n_sf + 1;
  const size_t spt = oai4g_tx_iq_samples(tx), N = fp.ofdm_symbol_size, grid = (size_t)fp.symbols_per_tti * N;
  uint8_t *d_pay = (uint8_t *)oai4g_dev_alloc((size_t)n_tx * p.payload_stride);
  void *d_work = oai4g_dev_alloc(oai4g_tx_workspace_bytes(tx, n_tx));
  int32_t *d_iq = (int32_t *)oai4g_dev_alloc((size_t)n_tx * spt * 4);
  int32_t *d_rxF = (int32_t *)oai4g_dev_alloc((size_t)n_tx * grid * 4);
  int32_t *d_est = (int32_t *)oai4g_dev_alloc((size_t)n_sf * grid * 4);
  int32_t *d_time = (int32_t *)oai4g_dev_alloc((size_t)n_sf * N * 4);
  int32_t *d_om = (int32_t *)oai4g_dev_alloc((size_t)n_sf * 4);
  CHECK(d_pay && d_work && d_iq && d_rxF && d_est && d_time && d_om, "device allocation");
  CHECK(oai4g_fill_payload(d_pay, (size_t)n_tx * p.payload_stride, 0xD15C0ull, NULL) == 0, "fill_payload");

  oai4g_chest_config_t *ce = oai4g_chest_config_create(&fp, 0, (uint8_t)sf0, 1);
  oai4g_rx_config_t *rx = oai4g_rx_config_create(&fp, p.rb_alloc, Qm, (uint8_t)npdcch, p.rnti, (uint8_t)sf0, 1);
  CHECK(ce && rx, "chest / rx config");
  const size_t llr_stride = oai4g_rx_llr_stride(rx);
  int16_t *d_llr = (int16_t *)oai4g_dev_alloc((size_t)n_sf * llr_stride * 2);
  CHECK(d_llr, "device allocation (LLR)");

  double t[8];
  t[0] = now_us();
  CHECK(oai4g_tx_batch(tx, n_tx, d_pay, d_work, d_iq, NULL) == 0 && oai4g_sync() == 0, "tx_batch");
  t[1] = now_us();
  CHECK(oai4g_fep_batch(&fp, n_tx, 1, d_iq, d_rxF, NULL) == 0 && oai4g_sync() == 0, "fep_batch");
  t[2] = now_us();
  CHECK(oai4g_chest_batch(ce, n_sf, d_rxF, d_est, NULL) == 0 && oai4g_sync() == 0, "chest_batch");
  t[3] = now_us();
  CHECK(oai4g_freq_offset_omega_batch(&fp, n_sf, d_est, grid, 4 - fp.Ncp, d_om, NULL) == 0 &&
            oai4g_chest_time_batch(&fp, n_sf, d_est, grid, d_time, N, NULL) == 0 && oai4g_sync() == 0,
        "freq_offset / time estimates");
  t[4] = now_us();
  CHECK(oai4g_rx_batch(rx, n_sf, d_rxF, d_est, d_llr, 1, NULL) == 0 && oai4g_sync() == 0, "rx_batch");
  t[5] = now_us();

  /* UE scalar tails: the frequency-offset filter over the calls (two per subframe) and the timing
   * tracker's peak of the time-domain estimate (lte_adjust_sync.c:60-76's |h|^2 maximum) */
  int32_t *om = (int32_t *)malloc((size_t)n_sf * 4);
  int32_t *tim = (int32_t *)malloc((size_t)n_sf * N * 4);
  CHECK(om && tim, "host allocation");
  CHECK(oai4g_memcpy_d2h(om, d_om, (size_t)n_sf * 4) == 0 && oai4g_memcpy_d2h(tim, d_time, (size_t)n_sf * N * 4) == 0,
        "copy back");
  int freq_offset = 0, first_run = 1;
  for (int i = 0; i < n_sf; i++)
    for (int k = 0; k < 2; k++) CHECK(oai4g_freq_offset_update(&fp, om[i], &freq_offset, &first_run) == 0, "freq_offset_update");
  int peak = 0;
  int64_t best = -1;
  for (size_t j = 0; j < fp.nb_prefix_samples; j++) {
    const int16_t re = (int16_t)(tim[j] & 0xFFFF), im = (int16_t)(tim[j] >> 16);
    const int64_t e = (int64_t)re * re / 2 + (int64_t)im * im / 2;
    if (e > best) { best = e; peak = (int)j; }
  }

  /* dlsch_decoding: one oai4g_ul_decode_batch per run of consecutive subframes with the same G
   * (G differs between subframe indices with the control / CRS REs) */
  uint32_t C, Cp, Cm, Kp, Km, F;
  const uint32_t B = p.TBS[0] + 24;
  CHECK(oai4g_lte_segmentation(NULL, NULL, B, &C, &Cp, &Cm, &Kp, &Km, &F) == 0, "lte_segmentation");
  uint8_t *pay = (uint8_t *)malloc((size_t)n_tx * p.payload_stride);
  const size_t c_stride = 6144 / 8 + 8;
  uint8_t *cb = (uint8_t *)malloc((size_t)n_sf * C * c_stride), *its = (uint8_t *)malloc((size_t)n_sf * C);
  uint8_t *d_c = (uint8_t *)oai4g_dev_alloc((size_t)n_sf * C * c_stride), *d_it = (uint8_t *)oai4g_dev_alloc(256 + (size_t)n_sf * C);
  CHECK(pay && cb && its && d_c && d_it, "allocation (decoder)");
  CHECK(oai4g_memcpy_d2h(pay, d_pay, (size_t)n_tx * p.payload_stride) == 0, "copy payload");
  int ok = 1, max_it = 0, launches = 0;
  double t_dec = 0;
  for (int i0 = 0; i0 < n_sf;) {
    const int G = oai4g_rx_llr_count(rx, (sf0 + i0) % 10);
    CHECK(G > 0, "rx_llr_count");
    int n = 1;
    while (i0 + n < n_sf && oai4g_rx_llr_count(rx, (sf0 + i0 + n) % 10) == G) n++;
    oai4g_ul_config_t *ul = oai4g_ul_config_create(B, (uint32_t)G, Qm, 0, 8, OAI4G_NSOFT, 4);
    CHECK(ul && oai4g_ul_config_C(ul) == (int)C, "ul_config_create");
    const double d0 = now_us();
    CHECK(oai4g_ul_decode_batch(ul, n, d_llr + (size_t)i0 * llr_stride, llr_stride, d_c + (size_t)i0 * C * c_stride,
                                c_stride, d_it + (size_t)i0 * C, NULL) == 0 && oai4g_sync() == 0, "ul_decode_batch");
    t_dec += now_us() - d0;
    launches++;
    oai4g_ul_config_destroy(ul);
    i0 += n;
  }
  CHECK(oai4g_memcpy_d2h(cb, d_c, (size_t)n_sf * C * c_stride) == 0 && oai4g_memcpy_d2h(its, d_it, (size_t)n_sf * C) == 0,
        "copy blocks");
  for (int i = 0; i < n_sf; i++) {
    const int sf = (sf0 + i) % 10;
    /* the TB from the blocks: skip block 0's F fillers, drop each block's CRC24B when C > 1 */
    uint32_t pos = 0;
    int tb_ok = 1;
    for (uint32_t r = 0; r < C; r++) {
      const uint32_t K = r < Cm ? Km : Kp, lo = r == 0 ? F : 0, hi = K - (C > 1 ? 24 : 0);
      const uint8_t it = its[(size_t)i * C + r], *blk = cb + ((size_t)i * C + r) * c_stride;
      if (it > max_it) max_it = it;
      if (it > 4) tb_ok = 0;
      for (uint32_t k = lo; k < hi && pos < p.TBS[0]; k++, pos++)
        if (get_bit(blk, k) != get_bit(pay + (size_t)i * p.payload_stride, pos)) tb_ok = 0;
    }
    if (pos != p.TBS[0]) tb_ok = 0;
    printf("subframe %d: G %d, %u blocks, TB %s\n", sf, oai4g_rx_llr_count(rx, sf), C, tb_ok ? "ok" : "FAILED");
    ok &= tb_ok;
  }
  oai4g_dev_free(d_c);
  oai4g_dev_free(d_it);
  printf("N_RB %d mcs %d TBS %u: %d subframes, %s; max turbo iterations %d; freq_offset %d Hz; timing peak %d\n", nrb,
         mcs, p.TBS[0], n_sf, ok ? "all transport blocks recovered" : "DECODING FAILED", max_it, freq_offset, peak);
  if (timing)
    printf("tx %.1f us, fep %.1f us, chest %.1f us, freq/time %.1f us, rx %.1f us, decode %.1f us in %d launch(es) "
           "(first pass, includes launch setup)\n",
           t[1] - t[0], t[2] - t[1], t[3] - t[2], t[4] - t[3], t[5] - t[4], t_dec, launches);
  free(om);
  free(tim);
  free(pay);
  free(cb);
  free(its);
  return ok ? 0 : 1;
}
