/*
 * gfx950 kernels for the UE's PDSCH demodulation after the FEP (second
 * half): TM1 (one transmit port), one receive antenna; any N_RB_DL (the extraction map carries the
 * odd-N_RB split around DC).
 *   dlsch_extract_rbs_single    PHY/LTE_TRANSPORT/dlsch_demodulation.c:3167-3300
 *   dlsch_channel_level         dlsch_demodulation.c:2777-2835, log2_maxh :286-300
 *   dlsch_channel_compensation  dlsch_demodulation.c:801-960
 *   dlsch_qpsk/16qam/64qam_llr  PHY/LTE_TRANSPORT/dlsch_llr_computation.c:636-930
 *   dlsch_unscrambling          PHY/LTE_TRANSPORT/dlsch_scrambling.c:99-137
 * Every step after the channel level is elementwise per extracted RE, so the demodulator is one
 * thread per RE of a (subframe, symbol): the host's extraction map gives the FFT bin and the
 * channel-estimate index, the RE's Qm LLRs go to their place in the subframe's LLR stream with the
 * scrambling sign applied.  Integer arithmetic is the reference's SSE arithmetic lane for lane:
 * madd_epi16 (int32 wrap) with the conjugate by sign_epi16 (int16 wrap), srai + packs_epi32
 * (saturation), mulhi_epi16 << 1, abs_epi16 (-32768 stays), subs_epi16.
 */
#include "oai4g_rx_prims.h"

/* estimate entry of plane pa (= p * 2 + a), subframe sf, symbol l, estimate column col: from the
 * estimate planes [pa][n_sf][nsymb][N] (plane words each), or (PIL) from the pilot-row pairs
 * [pa][n_sf][4][N] x (P_k, P_k+1) with lte_dl_channel_estimation's temporal interpolation
 * (:639-698: mulhi(P_a, w_a) << 1 +sat mulhi(P_a+1, w_b) << 1, per component; one 8-byte load) */
template <bool PIL>
static __device__ __forceinline__ uint32_t rx_est(const rx_dev_t *__restrict__ c, const int32_t *__restrict__ est,
                                                  size_t plane, uint32_t pa, uint32_t sf, uint32_t l, uint32_t col)
{
  if constexpr (!PIL) {
    return (uint32_t)est[pa * plane + ((size_t)sf * c->nsymb + l) * c->N + col];
  } else {
    typedef uint32_t u32x2p_t __attribute__((ext_vector_type(2)));
    const u32x2p_t v = *((const u32x2p_t *)(est + pa * plane) + ((size_t)sf * 4 + c->ea[l]) * c->N + col);
    const int16_t wa = c->ewa[l];
    const uint32_t x = v.x, y = v.y;                              /* P_a, P_a+1 (eb = ea + 1) */
    if (wa == 0) return x;
    const int16_t wb = c->ewb[l];
    const int16_t r = rx_sat16((int32_t)rx_shl(rx_mh((int16_t)x, wa), 1) + rx_shl(rx_mh((int16_t)y, wb), 1));
    const int16_t i = rx_sat16((int32_t)rx_shl(rx_mh((int16_t)(x >> 16), wa), 1) + rx_shl(rx_mh((int16_t)(y >> 16), wb), 1));
    return (uint32_t)(uint16_t)r | ((uint32_t)(uint16_t)i << 16);
  }
}

/* dlsch_channel_level over the first PDSCH symbol -> log2_maxh = log2_approx(avg) / 2, per subframe */
__global__ void __launch_bounds__(256) k_rx_level(const rx_dev_t *__restrict__ c, const int32_t *__restrict__ ch,
                                                  uint8_t *__restrict__ shift)
{
  __shared__ uint32_t acc;
  const uint32_t sf = blockIdx.x, sfi = (c->first_sf + sf * c->sf_step) % 10, l = c->npdcch;
  if (threadIdx.x == 0) acc = 0;
  __syncthreads();
  rg32_t *map = (rg32_t *)(c->map + c->map_off[sfi][0]);
  const int32_t *chs = ch + ((size_t)sf * c->nsymb + l) * c->N;
  uint32_t part = 0;
  for (uint32_t j = threadIdx.x; j < c->lvl_n[sfi]; j += blockDim.x) part += rx_h2((uint32_t)chs[map[j] >> 16]);
  atomicAdd(&acc, part);                       /* int32 wrap-add commutes (the reference's epi32 lanes) */
  __syncthreads();
  if (threadIdx.x == 0) shift[sf] = rx_shift_of((int32_t)acc, c->lvl_div[sfi]);
}

/* A 256-thread workgroup per (subframe, PDSCH symbol); thread t takes REs t + 256 r, r < 5 (>= the
 * 1200 REs of 100 PRB).  All map words, then all estimate / received words are loaded before any
 * arithmetic, so each thread waits for two memory round trips rather than two per RE.  An RE's Qm
 * LLRs leave as one 4 / 8 / 12-byte store (a symbol's stream offset is a multiple of Qm entries);
 * the scrambling signs of all Qm come from one 64-bit window of the Gold words (gold_words carries
 * one word of slack). */
constexpr int RX_R = 5;

template <int QM>
__global__ void __launch_bounds__(256) k_rx_llr(const rx_dev_t *__restrict__ c, const int32_t *__restrict__ rxF,
                                                const int32_t *__restrict__ ch, int16_t *__restrict__ llr,
                                                const uint8_t *__restrict__ shift, int unscramble)
{
  const uint32_t sf = blockIdx.y, k = blockIdx.x, sfi = (c->first_sf + sf * c->sf_step) % 10;
  const uint32_t l = c->npdcch + k, len = c->len[sfi][k];
  rg32_t *map = (rg32_t *)(c->map + c->map_off[sfi][k]);
  const size_t so = ((size_t)sf * c->nsymb + l) * c->N;
  const int32_t *y = rxF + so, *h = ch + so;
  int16_t *out = llr + (size_t)sf * c->llr_stride + c->llr_off[sfi][k];
  const uint32_t sh = shift[sf], base = c->llr_off[sfi][k];
  rg32_t *gold = (rg32_t *)(c->gold + (size_t)sfi * c->gold_words);
  const int16_t a1 = c->a1, a2 = c->a2;
  uint32_t mw[RX_R], hv[RX_R], yv[RX_R];
#pragma unroll
  for (int r = 0; r < RX_R; r++) {
    const uint32_t j = threadIdx.x + 256 * r;
    mw[r] = j < len ? map[j] : 0u;
  }
#pragma unroll
  for (int r = 0; r < RX_R; r++) {
    hv[r] = (uint32_t)h[mw[r] >> 16];
    yv[r] = (uint32_t)y[mw[r] & 0xFFFFu];
  }
#pragma unroll
  for (int r = 0; r < RX_R; r++) {
    const uint32_t j = threadIdx.x + 256 * r;
    if (j >= len) break;
    rx_re_llr<QM>(hv[r], yv[r], sh, a1, a2, unscramble ? gold : nullptr, base + j * QM, out + QM * j);
  }
}

/* ======================================================================================
 * TM3 (LARGE_CDD, two ports), nb_rx receive antennas, rx_pdsch with dual_stream_flag = 0:
 *   dlsch_extract_rbs_dual      dlsch_demodulation.c:3683-4056 (the host's map; ports 0 / 1 and
 *                               every receive antenna share the slots)
 *   dlsch_channel_level_TM3     :2902-2981 (stream-0 |h|^2 per register lane e mod 4, int32 wrap,
 *                               accumulated over the antennas without reset, per-lane division)
 *   log2_maxh                   :390-394 (log2_approx(avg) - 13 + offset_mumimo_llr_drange, >= 0)
 *   dlsch_channel_compensation_TM3 :1846-2120 with prec2A_TM3_128 (s alternates per slot)
 *   dlsch_detection_mrc         :2583-2718 (stream 0: (a >> 1) +sat (b >> 1))
 *   dlsch_16qam / 64qam_llr     of stream 0, unscrambled
 * d_est holds the estimate planes [p * 2 + a][n_sf][nsymb][N] (plane = n_sf nsymb N words), or with
 * PIL the pilot rows [p * 2 + a][n_sf][5][N] (plane = n_sf 5 N words); d_rxF the FEP output
 * [n_sf][nb_rx][nsymb][N].
 * ==================================================================================== */
template <bool PIL>
__global__ void __launch_bounds__(256) k_rx_level_tm3(const rx_dev_t *__restrict__ c, const int32_t *__restrict__ est,
                                                      size_t plane, uint8_t *__restrict__ shift)
{
  __shared__ uint32_t lane[2][4];
  const uint32_t sf = blockIdx.x, sfi = (c->first_sf + sf * c->sf_step) % 10, l = c->npdcch;
  if (threadIdx.x < 8) lane[threadIdx.x >> 2][threadIdx.x & 3] = 0;
  __syncthreads();
  rg32_t *map = (rg32_t *)(c->map + c->map_off[sfi][0]);
  uint32_t part[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  for (uint32_t j = threadIdx.x; j < c->lvl_n[sfi]; j += blockDim.x) {
    const uint32_t col = map[j] >> 16;
    for (uint32_t a = 0; a < c->nb_rx; a++) {
      const uint32_t h0 = rx_est<PIL>(c, est, plane, a, sf, l, col), h1 = rx_est<PIL>(c, est, plane, 2 + a, sf, l, col);
      const uint32_t v = rx_h2(rx_prec_tm3(h0, h1, (j & 1u) != 0));
#pragma unroll
      for (int q = 0; q < 4; q++)
        if ((j & 3u) == (uint32_t)q) part[a][q] += v;
    }
  }
#pragma unroll
  for (int a = 0; a < 2; a++)
#pragma unroll
    for (int q = 0; q < 4; q++)
      if (part[a][q]) atomicAdd(&lane[a][q], part[a][q]);
  __syncthreads();
  if (threadIdx.x == 0) {
    const int32_t div = (int32_t)c->lvl_div[sfi];
    int32_t avg[2] = {0, 0};
    uint32_t cum[4] = {0, 0, 0, 0};
    for (uint32_t a = 0; a < c->nb_rx; a++) {
      for (int q = 0; q < 4; q++) cum[q] += lane[a][q];      /* avg128D is not reset per antenna */
      avg[a] = (int32_t)cum[0] / div + (int32_t)cum[1] / div + (int32_t)cum[2] / div + (int32_t)cum[3] / div;
    }
    const int32_t m = avg[0] > avg[1] ? avg[0] : avg[1];     /* cmax(avg[0], avg[1]); avg[1] = 0 with one antenna */
    const uint32_t x = (uint32_t)m;
    const int32_t l2 = x ? 32 - (int32_t)__clz(x & 0x7FFFFFFFu) : 0;   /* log2_approx (bits 0..30) */
    const int32_t v = l2 - 13 + c->mu_off;
    shift[sf] = (uint8_t)(v > 0 ? v : 0);
  }
}

template <int QM, bool PIL>
__global__ void __launch_bounds__(256) k_rx_llr_tm3(const rx_dev_t *__restrict__ c, const int32_t *__restrict__ rxF,
                                                    const int32_t *__restrict__ est, size_t plane,
                                                    int16_t *__restrict__ llr, const uint8_t *__restrict__ shift,
                                                    int unscramble)
{
  const uint32_t sf = blockIdx.y, k = blockIdx.x, sfi = (c->first_sf + sf * c->sf_step) % 10;
  const uint32_t l = c->npdcch + k, len = c->len[sfi][k], nb_rx = c->nb_rx, NS = c->nsymb * c->N;
  rg32_t *map = (rg32_t *)(c->map + c->map_off[sfi][k]);
  int16_t *out = llr + (size_t)sf * c->llr_stride + c->llr_off[sfi][k];
  const uint32_t sh = shift[sf], base = c->llr_off[sfi][k];
  rg32_t *gold = (rg32_t *)(c->gold + (size_t)sfi * c->gold_words);
  const int16_t a1 = c->a1, a2 = c->a2;
  uint32_t mw[RX_R];
#pragma unroll
  for (int r = 0; r < RX_R; r++) {
    const uint32_t j = threadIdx.x + 256 * r;
    mw[r] = j < len ? map[j] : 0u;
  }
  uint32_t yv[2][RX_R], h0[2][RX_R], h1[2][RX_R];
#pragma unroll
  for (uint32_t a = 0; a < 2; a++)
#pragma unroll
    for (int r = 0; r < RX_R; r++) {
      const uint32_t aa = a < nb_rx ? a : 0u;
      const size_t yo = ((size_t)sf * nb_rx + aa) * NS + (size_t)l * c->N;
      yv[a][r] = (uint32_t)rxF[yo + (mw[r] & 0xFFFFu)];
      h0[a][r] = rx_est<PIL>(c, est, plane, aa, sf, l, mw[r] >> 16);
      h1[a][r] = rx_est<PIL>(c, est, plane, 2 + aa, sf, l, mw[r] >> 16);
    }
#pragma unroll
  for (int r = 0; r < RX_R; r++) {
    const uint32_t j = threadIdx.x + 256 * r;
    if (j >= len) break;
    int16_t cr[2], ci[2], mg[2], mgb[2];
#pragma unroll
    for (uint32_t a = 0; a < 2; a++) {
      const uint32_t p = rx_prec_tm3(h0[a][r], h1[a][r], (j & 1u) != 0);
      const int16_t hr = (int16_t)p, hi = (int16_t)(p >> 16), yr = (int16_t)yv[a][r], yi = (int16_t)(yv[a][r] >> 16);
      const int16_t nhi = (int16_t)(-(int32_t)hi);
      cr[a] = rx_sat16(rx_madd(hr, yr, hi, yi) >> sh);
      ci[a] = rx_sat16(rx_madd(nhi, yr, hr, yi) >> sh);
      const int16_t m = rx_sat16(rx_madd(hr, hr, hi, hi) >> sh);
      mg[a] = (int16_t)((((int32_t)m * a1) >> 16) << 1);
      mgb[a] = (int16_t)((((int32_t)m * a2) >> 16) << 1);
    }
    if (nb_rx > 1) {                                          /* dlsch_detection_mrc */
      cr[0] = rx_sat16((cr[0] >> 1) + (cr[1] >> 1));
      ci[0] = rx_sat16((ci[0] >> 1) + (ci[1] >> 1));
      mg[0] = rx_sat16((mg[0] >> 1) + (mg[1] >> 1));
      mgb[0] = rx_sat16((mgb[0] >> 1) + (mgb[1] >> 1));
    }
    int16_t v[6];
    rx_llr_values<QM>(cr[0], ci[0], mg[0], mgb[0], v);
    rx_llr_store<QM>(v, unscramble ? gold : nullptr, base + j * QM, out + QM * j);
  }
}

/* TM3 with codeword 0 QPSK (dlsch_demodulation.c:643-690): the compensation keeps both precoded
 * streams, dlsch_dual_stream_correlation gives rho = conj(h0') h1' and rho2 = conj(h1') h0', the MRC
 * averages stream 0 and rho over the RX antennas (stream 1, rho2 and dl_ch_mag1 stay antenna 0's with
 * dual_stream_flag 0).  QM1 = 2: dlsch_qpsk_qpsk_llr yields codeword 0 (comp0, comp1, rho) and, when
 * llr1 is given, codeword 1 (comp1, comp0, rho2), both scrambled with q = 0 as dlsim transmits them;
 * QM1 = 4 / 6: dlsch_qpsk_16qam_llr / dlsch_qpsk_64qam_llr yield codeword 0 from (comp0, comp1,
 * dl_ch_mag1, rho) */
template <int QM1, bool PIL>
__global__ void __launch_bounds__(256) k_rx_llr_tm3qq(const rx_dev_t *__restrict__ c, const int32_t *__restrict__ rxF,
                                                      const int32_t *__restrict__ est, size_t plane,
                                                      int16_t *__restrict__ llr0, int16_t *__restrict__ llr1,
                                                      const uint8_t *__restrict__ shift, int unscramble)
{
  const uint32_t sf = blockIdx.y, k = blockIdx.x, sfi = (c->first_sf + sf * c->sf_step) % 10;
  const uint32_t l = c->npdcch + k, len = c->len[sfi][k], nb_rx = c->nb_rx, NS = c->nsymb * c->N;
  rg32_t *map = (rg32_t *)(c->map + c->map_off[sfi][k]);
  const size_t oo = (size_t)sf * c->llr_stride + c->llr_off[sfi][k];
  const uint32_t sh = shift[sf], base = c->llr_off[sfi][k];
  rg32_t *gold = (rg32_t *)(c->gold + (size_t)sfi * c->gold_words);
  for (uint32_t j = threadIdx.x; j < len; j += blockDim.x) {
    const uint32_t mw = map[j];
    const bool neg = (j & 1u) != 0;
    int16_t c0r[2], c0i[2], r0r[2], r0i[2], c1r = 0, c1i = 0, q2r = 0, q2i = 0, m1 = 0;
#pragma unroll
    for (uint32_t a = 0; a < 2; a++) {
      const uint32_t aa = a < nb_rx ? a : 0u;
      const uint32_t yv = (uint32_t)rxF[((size_t)sf * nb_rx + aa) * NS + (size_t)l * c->N + (mw & 0xFFFFu)];
      const uint32_t h0 = rx_est<PIL>(c, est, plane, aa, sf, l, mw >> 16), h1 = rx_est<PIL>(c, est, plane, 2 + aa, sf, l, mw >> 16);
      const uint32_t p0 = rx_prec_tm3(h0, h1, neg), p1 = rx_prec_tm3_s1(h0, h1, neg);
      rx_conj_mul(p0, yv, sh, c0r[a], c0i[a]);
      rx_conj_mul(p0, p1, sh, r0r[a], r0i[a]);
      if (a == 0) {
        rx_conj_mul(p1, yv, sh, c1r, c1i);
        if (QM1 == 2) rx_conj_mul(p1, p0, sh, q2r, q2i);
        if (QM1 > 2) {                                              /* dl_ch_mag1 of antenna 0 */
          const int16_t hr = (int16_t)p1, hi = (int16_t)(p1 >> 16);
          const int16_t m = rx_sat16(rx_madd(hr, hr, hi, hi) >> sh);
          m1 = (int16_t)((((int32_t)m * (QM1 == 4 ? 20724 : 20225)) >> 16) << 1);   /* QAM16_n1 / QAM64_n1 */
        }
      }
    }
    if (nb_rx > 1) {                                            /* dlsch_detection_mrc: stream 0, rho */
      c0r[0] = rx_sat16((c0r[0] >> 1) + (c0r[1] >> 1));
      c0i[0] = rx_sat16((c0i[0] >> 1) + (c0i[1] >> 1));
      r0r[0] = rx_sat16((r0r[0] >> 1) + (r0r[1] >> 1));
      r0i[0] = rx_sat16((r0i[0] >> 1) + (r0i[1] >> 1));
    }
    int16_t v[6];
    if (QM1 == 2) rx_qq_llr(c0r[0], c0i[0], c1r, c1i, r0r[0], r0i[0], v);
    else rx_qx_llr<QM1>(c0r[0], c0i[0], c1r, c1i, m1, r0r[0], r0i[0], v);
    rx_llr_store<2>(v, unscramble ? gold : nullptr, base + 2 * j, llr0 + oo + 2 * j);
    if (QM1 == 2 && llr1) {
      rx_qq_llr(c1r, c1i, c0r[0], c0i[0], q2r, q2i, v);
      rx_llr_store<2>(v, unscramble ? gold : nullptr, base + 2 * j, llr1 + oo + 2 * j);
    }
  }
}

template <bool PIL>
static hipError_t launch_rx_tm3qq(const rx_dev_t *d_cfg, const rx_dev_t *h_cfg, int n_sf, const int32_t *d_rxF,
                                  const int32_t *d_est, size_t plane, int16_t *d_llr0, int16_t *d_llr1, uint8_t *d_shift,
                                  int unscramble, hipStream_t s)
{
  hipLaunchKernelGGL(k_rx_level_tm3<PIL>, dim3(n_sf), dim3(256), 0, s, d_cfg, d_est, plane, d_shift);
  const dim3 g(h_cfg->n_sym, n_sf), b(256);
  if (h_cfg->qm1 == 4)
    hipLaunchKernelGGL((k_rx_llr_tm3qq<4, PIL>), g, b, 0, s, d_cfg, d_rxF, d_est, plane, d_llr0, nullptr, d_shift, unscramble);
  else if (h_cfg->qm1 == 6)
    hipLaunchKernelGGL((k_rx_llr_tm3qq<6, PIL>), g, b, 0, s, d_cfg, d_rxF, d_est, plane, d_llr0, nullptr, d_shift, unscramble);
  else
    hipLaunchKernelGGL((k_rx_llr_tm3qq<2, PIL>), g, b, 0, s, d_cfg, d_rxF, d_est, plane, d_llr0, d_llr1, d_shift, unscramble);
  return hipGetLastError();
}

hipError_t oai4g_launch_rx_tm3qq(const rx_dev_t *d_cfg, const rx_dev_t *h_cfg, int n_sf, const int32_t *d_rxF,
                                 const int32_t *d_est, size_t plane, int16_t *d_llr0, int16_t *d_llr1,
                                 uint8_t *d_shift, int unscramble, hipStream_t s, int pil)
{
  if (n_sf <= 0) return hipSuccess;
  return pil ? launch_rx_tm3qq<true>(d_cfg, h_cfg, n_sf, d_rxF, d_est, plane, d_llr0, d_llr1, d_shift, unscramble, s)
             : launch_rx_tm3qq<false>(d_cfg, h_cfg, n_sf, d_rxF, d_est, plane, d_llr0, d_llr1, d_shift, unscramble, s);
}

template <bool PIL>
static hipError_t launch_rx_tm3(const rx_dev_t *d_cfg, const rx_dev_t *h_cfg, int n_sf, const int32_t *d_rxF,
                                const int32_t *d_est, size_t plane, int16_t *d_llr, uint8_t *d_shift, int unscramble,
                                hipStream_t s)
{
  hipLaunchKernelGGL(k_rx_level_tm3<PIL>, dim3(n_sf), dim3(256), 0, s, d_cfg, d_est, plane, d_shift);
  const dim3 g(h_cfg->n_sym, n_sf), b(256);
  if (h_cfg->Qm == 4)
    hipLaunchKernelGGL((k_rx_llr_tm3<4, PIL>), g, b, 0, s, d_cfg, d_rxF, d_est, plane, d_llr, d_shift, unscramble);
  else
    hipLaunchKernelGGL((k_rx_llr_tm3<6, PIL>), g, b, 0, s, d_cfg, d_rxF, d_est, plane, d_llr, d_shift, unscramble);
  return hipGetLastError();
}

hipError_t oai4g_launch_rx_tm3(const rx_dev_t *d_cfg, const rx_dev_t *h_cfg, int n_sf, const int32_t *d_rxF,
                               const int32_t *d_est, size_t plane, int16_t *d_llr, uint8_t *d_shift, int unscramble,
                               hipStream_t s, int pil)
{
  if (n_sf <= 0) return hipSuccess;
  return pil ? launch_rx_tm3<true>(d_cfg, h_cfg, n_sf, d_rxF, d_est, plane, d_llr, d_shift, unscramble, s)
             : launch_rx_tm3<false>(d_cfg, h_cfg, n_sf, d_rxF, d_est, plane, d_llr, d_shift, unscramble, s);
}

/* ======================================================================================
 * TM2 (ALAMOUTI, two TX ports) with dlsim's UE (rx_pdsch, dual_stream_flag = 0):
 *   dlsch_extract_rbs_dual      (the TM3 map)
 *   dlsch_channel_level         :2777-2838 per (port, RX antenna): int32 |h|^2 sum / (nb_rb nre),
 *                               log2_maxh = log2_approx(max(0, max avg)) / 2 (:276-285)
 *   dlsch_channel_compensation  :801-980 per (port, RX antenna)
 *   dlsch_detection_mrc         :2583-2621 per port
 *   dlsch_alamouti              :3067-3160 pairs (2k, 2k + 1) of extracted REs, int16 wrap sums,
 *                               magnitudes (m0 +sat m1) >> 1, mulhi(., 23170) << 1
 *   dlsch_qpsk / 16qam / 64qam_llr, unscrambled
 * One thread per RE pair; planes and layouts as for TM3.
 * ==================================================================================== */
__global__ void __launch_bounds__(256) k_rx_level_tm2(const rx_dev_t *__restrict__ c, const int32_t *__restrict__ est,
                                                      size_t plane, uint8_t *__restrict__ shift)
{
  __shared__ uint32_t tot[4];
  const uint32_t sf = blockIdx.x, sfi = (c->first_sf + sf * c->sf_step) % 10, l = c->npdcch;
  if (threadIdx.x < 4) tot[threadIdx.x] = 0;
  __syncthreads();
  rg32_t *map = (rg32_t *)(c->map + c->map_off[sfi][0]);
  const size_t so = ((size_t)sf * c->nsymb + l) * c->N;
  uint32_t part[4] = {0, 0, 0, 0};
  for (uint32_t j = threadIdx.x; j < c->lvl_n[sfi]; j += blockDim.x) {
    const uint32_t col = map[j] >> 16;
#pragma unroll
    for (uint32_t pa = 0; pa < 4; pa++)
      if ((pa & 1u) < c->nb_rx) part[pa] += rx_h2((uint32_t)est[pa * plane + so + col]);
  }
#pragma unroll
  for (int pa = 0; pa < 4; pa++)
    if (part[pa]) atomicAdd(&tot[pa], part[pa]);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint8_t m = 0;
    for (uint32_t pa = 0; pa < 4; pa++)
      if ((pa & 1u) < c->nb_rx) {
        const uint8_t v = rx_shift_of((int32_t)tot[pa], c->lvl_div[sfi]);   /* log2 monotone: max of shifts */
        m = v > m ? v : m;
      }
    shift[sf] = m;
  }
}

template <int QM>
__global__ void __launch_bounds__(256) k_rx_llr_tm2(const rx_dev_t *__restrict__ c, const int32_t *__restrict__ rxF,
                                                    const int32_t *__restrict__ est, size_t plane,
                                                    int16_t *__restrict__ llr, const uint8_t *__restrict__ shift,
                                                    int unscramble)
{
  const uint32_t sf = blockIdx.y, k = blockIdx.x, sfi = (c->first_sf + sf * c->sf_step) % 10;
  const uint32_t l = c->npdcch + k, len = c->len[sfi][k], nb_rx = c->nb_rx, NS = c->nsymb * c->N;
  rg32_t *map = (rg32_t *)(c->map + c->map_off[sfi][k]);
  const size_t eo = ((size_t)sf * c->nsymb + l) * c->N;
  int16_t *out = llr + (size_t)sf * c->llr_stride + c->llr_off[sfi][k];
  const uint32_t sh = shift[sf], base = c->llr_off[sfi][k];
  rg32_t *gold = (rg32_t *)(c->gold + (size_t)sfi * c->gold_words);
  const int16_t a1 = c->a1, a2 = c->a2;
  for (uint32_t q = threadIdx.x; 2 * q < len; q += blockDim.x) {
    /* the pair's two REs (the config guarantees map entries up to len rounded up to even) */
    const uint32_t m0 = map[2 * q], m1 = map[2 * q + 1];
    int16_t cr[2][2], ci[2][2], mg[2][2], mgb[2][2];            /* [port][RE of the pair] */
#pragma unroll
    for (int e = 0; e < 2; e++) {
      const uint32_t mw = e ? m1 : m0;
      int16_t r_[2][2], i_[2][2], g_[2][2], gb_[2][2];        /* [port][antenna] */
#pragma unroll
      for (uint32_t a = 0; a < 2; a++) {
        const uint32_t aa = a < nb_rx ? a : 0u;
        const uint32_t yv = (uint32_t)rxF[((size_t)sf * nb_rx + aa) * NS + (size_t)l * c->N + (mw & 0xFFFFu)];
        const int16_t yr = (int16_t)yv, yi = (int16_t)(yv >> 16);
#pragma unroll
        for (uint32_t p = 0; p < 2; p++) {
          const uint32_t hv = (uint32_t)est[(2 * p + aa) * plane + eo + (mw >> 16)];
          const int16_t hr = (int16_t)hv, hi = (int16_t)(hv >> 16), nhi = (int16_t)(-(int32_t)hi);
          r_[p][a] = rx_sat16(rx_madd(hr, yr, hi, yi) >> sh);
          i_[p][a] = rx_sat16(rx_madd(nhi, yr, hr, yi) >> sh);
          if (QM > 2) {
            const int16_t m = rx_sat16(rx_madd(hr, hr, hi, hi) >> sh);
            g_[p][a] = (int16_t)((((int32_t)m * a1) >> 16) << 1);
            gb_[p][a] = (int16_t)((((int32_t)m * a2) >> 16) << 1);
          } else {
            g_[p][a] = gb_[p][a] = 0;
          }
        }
      }
#pragma unroll
      for (int p = 0; p < 2; p++) {
        if (nb_rx > 1) {                                        /* dlsch_detection_mrc */
          cr[p][e] = rx_sat16((r_[p][0] >> 1) + (r_[p][1] >> 1));
          ci[p][e] = rx_sat16((i_[p][0] >> 1) + (i_[p][1] >> 1));
          mg[p][e] = rx_sat16((g_[p][0] >> 1) + (g_[p][1] >> 1));
          mgb[p][e] = rx_sat16((gb_[p][0] >> 1) + (gb_[p][1] >> 1));
        } else {
          cr[p][e] = r_[p][0]; ci[p][e] = i_[p][0]; mg[p][e] = g_[p][0]; mgb[p][e] = gb_[p][0];
        }
      }
    }
    /* dlsch_alamouti (C short arithmetic: wraps) */
    const int16_t y0r = (int16_t)(cr[0][0] + cr[1][1]), y0i = (int16_t)(ci[0][0] - ci[1][1]);
    const int16_t y1r = (int16_t)(cr[0][1] - cr[1][0]), y1i = (int16_t)(ci[0][1] + ci[1][0]);
    const int16_t yr2[2] = {y0r, y1r}, yi2[2] = {y0i, y1i};
#pragma unroll
    for (int e = 0; e < 2; e++) {
      const uint32_t j = 2 * q + e;
      if (j >= len) break;
      const int16_t m = (int16_t)(rx_sat16((int32_t)mg[0][e] + mg[1][e]) >> 1);
      const int16_t mb = (int16_t)(rx_sat16((int32_t)mgb[0][e] + mgb[1][e]) >> 1);
      const int16_t xr = (int16_t)((((int32_t)yr2[e] * 23170) >> 16) << 1), xi = (int16_t)((((int32_t)yi2[e] * 23170) >> 16) << 1);
      int16_t v[6];
      rx_llr_values<QM>(xr, xi, m, mb, v);
      rx_llr_store<QM>(v, unscramble ? gold : nullptr, base + j * QM, out + QM * j);
    }
  }
}

hipError_t oai4g_launch_rx_tm2(const rx_dev_t *d_cfg, const rx_dev_t *h_cfg, int n_sf, const int32_t *d_rxF,
                               const int32_t *d_est, size_t plane, int16_t *d_llr, uint8_t *d_shift, int unscramble,
                               hipStream_t s)
{
  if (n_sf <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_rx_level_tm2, dim3(n_sf), dim3(256), 0, s, d_cfg, d_est, plane, d_shift);
  const dim3 g(h_cfg->n_sym, n_sf), b(256);
  if (h_cfg->Qm == 2)
    hipLaunchKernelGGL(k_rx_llr_tm2<2>, g, b, 0, s, d_cfg, d_rxF, d_est, plane, d_llr, d_shift, unscramble);
  else if (h_cfg->Qm == 4)
    hipLaunchKernelGGL(k_rx_llr_tm2<4>, g, b, 0, s, d_cfg, d_rxF, d_est, plane, d_llr, d_shift, unscramble);
  else
    hipLaunchKernelGGL(k_rx_llr_tm2<6>, g, b, 0, s, d_cfg, d_rxF, d_est, plane, d_llr, d_shift, unscramble);
  return hipGetLastError();
}

/* dlsch_unscrambling drop-in: llr[k] *= 2 c(k) - 1 (int16), c = the words of the Gold sequence */
__global__ void __launch_bounds__(256) k_rx_unscramble(int16_t *__restrict__ llr, const uint32_t *__restrict__ c,
                                                       uint32_t n)
{
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x)
    if (!((c[k >> 5] >> (k & 31)) & 1u)) llr[k] = (int16_t)(-(int32_t)llr[k]);
}

hipError_t oai4g_launch_unscramble(int16_t *d_llr, const uint32_t *d_c, int n, hipStream_t s)
{
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_rx_unscramble, dim3(min((n + 255) / 256, 1024)), dim3(256), 0, s, d_llr, d_c, (uint32_t)n);
  return hipGetLastError();
}

hipError_t oai4g_launch_rx(const rx_dev_t *d_cfg, const rx_dev_t *h_cfg, int n_sf, const int32_t *d_rxF,
                           const int32_t *d_ch, int16_t *d_llr, uint8_t *d_shift, int unscramble, hipStream_t s)
{
  if (n_sf <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_rx_level, dim3(n_sf), dim3(256), 0, s, d_cfg, d_ch, d_shift);
  const dim3 g(h_cfg->n_sym, n_sf), b(256);                  /* 256 x RX_R >= 1200 REs per symbol */
  if (h_cfg->Qm == 2)
    hipLaunchKernelGGL(k_rx_llr<2>, g, b, 0, s, d_cfg, d_rxF, d_ch, d_llr, d_shift, unscramble);
  else if (h_cfg->Qm == 4)
    hipLaunchKernelGGL(k_rx_llr<4>, g, b, 0, s, d_cfg, d_rxF, d_ch, d_llr, d_shift, unscramble);
  else
    hipLaunchKernelGGL(k_rx_llr<6>, g, b, 0, s, d_cfg, d_rxF, d_ch, d_llr, d_shift, unscramble);
  return hipGetLastError();
}
