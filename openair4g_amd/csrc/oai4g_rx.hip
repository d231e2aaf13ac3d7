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
