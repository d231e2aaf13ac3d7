/*
 * gfx950 kernels for the UE's downlink channel estimation from the cell-specific reference
 * signals:
 *   lte_dl_channel_estimation   PHY/LTE_ESTIMATION/lte_dl_channel_estimation.c:37-336 (6 / 50 / 100
 *                               PRB interpolator), 338-533 (25 PRB: the DC-pair filters),
 *                               535-623 (15 PRB: f / f2 only, its second-half start), 629-701 (temporal interpolation with
 *                               high_speed_flag = 1, dlsim.c:2057)
 *   lte_dl_cell_spec_rx         PHY/LTE_REFSIG/lte_dl_cell_spec.c:205-260
 *   multadd_real_vector_complex_scalar / multadd_complex_vector_real_scalar  PHY/TOOLS/cmult_sv.c:55-122
 *
 * The reference walks the pilots of a symbol left to right and saturating-adds each pilot's
 * 24-tap filter response into the estimate row (adds_epi16), so an estimate entry is the ordered
 * saturating sum of the <= 4 pilots whose windows cover it.  Here one thread owns one subcarrier
 * column of a subframe: a workgroup first computes the conjugate-pilot products of every pilot
 * its 256 columns see (5 pilot symbols: 0, 4, 7, 11 and the next subframe's symbol 0) into LDS,
 * then each thread sums its column's covering pilots in ascending pilot order (the reference's
 * order, so the saturation points agree), applies the temporal interpolation of every row and
 * writes the subframe's 14 estimate rows once — coalesced, no read-modify-write of the estimate
 * buffer.  HBM traffic per subframe = 14 N words written + the pilot REs read.
 */
#include "oai4g_rx_prims.h"

namespace {

constexpr uint32_t CE_WG = 256;
constexpr uint32_t CE_MAXP = 64;   /* pilots a 256-column window can see: 2 (ceil(283 / 12) + 1) = 50 */

__device__ __forceinline__ int16_t ce_sat16(int32_t v) { return (int16_t)max(-32768, min(32767, v)); }

/* mulhi_epi16 then slli_epi16 by s (the shift wraps in 16 bits) */
__device__ __forceinline__ int16_t ce_mulhi_shl(int16_t a, int16_t b, uint32_t s)
{
  return (int16_t)(uint16_t)((uint32_t)(((int32_t)a * b) >> 16) << s);
}

/* conj(pilot m) * rx >> 15 of one pilot symbol (lte_dl_channel_estimation.c:214-215) */
__device__ uint32_t ce_pilot_ch(const chest_dev_t *__restrict__ c, const int32_t *__restrict__ row, uint32_t Ns,
                                uint32_t l01, uint32_t m)
{
  const uint32_t k = c->k[l01], N_RB = c->N_RB, mp = 110 - N_RB + m;
  const uint32_t idx = (c->gold[Ns][l01][mp >> 4] >> (2 * (mp & 15))) & 3u;
  /* lte_dl_cell_spec_rx's conjugated QPSK: (a,-a), (-a,-a), (a,a), (-a,a), a = ONE_OVER_SQRT2_Q15 */
  const int32_t pr = (idx & 1u) ? -23170 : 23170, pi = idx < 2 ? -23170 : 23170;
  const uint32_t bin = m < N_RB ? c->fco + k + 6 * m : c->off2[l01] + 6 * (m - N_RB);
  const uint32_t w = (uint32_t)row[bin];
  const int32_t rr = (int16_t)w, ri = (int16_t)(w >> 16);
  const int16_t chr = (int16_t)((pr * rr - pi * ri) >> 15), chi = (int16_t)((pr * ri + pi * rr) >> 15);
  return (uint32_t)(uint16_t)chr | ((uint32_t)(uint16_t)chi << 16);
}

/* filter of pilot m (of 2 N_RB): the edge filters except at 15 PRB, the DC pair (24, 25) at 25 PRB
 * (lte_dl_channel_estimation.c:212-623) */
__device__ __forceinline__ uint32_t ce_kind(uint32_t N_RB, uint32_t m)
{
  if (N_RB != 15) {
    if (m < 2) return m;
    if (m + 2 >= 2 * N_RB) return 4 + (m + 2 - 2 * N_RB);
    if (N_RB == 25 && (m >> 1) == 12) return 6 + (m & 1u);
  }
  return 2 + (m & 1u);
}

/* first pair index whose windows [12 q, 12 q + 28) can cover column j */
__device__ __forceinline__ uint32_t ce_qlo(uint32_t j) { return j >= 27 ? (j - 16) / 12 : 0; }

/* estimate entry j of one pilot symbol: ordered saturating sum over the covering pilots */
__device__ uint32_t ce_column(uint32_t N_RB, const int16_t (*__restrict__ f)[24], const uint32_t *__restrict__ chl,
                              uint32_t m_base, uint32_t j)
{
  int32_t ar = 0, ai = 0;
  const uint32_t q_hi = min(N_RB - 1, j / 12);
  for (uint32_t q = ce_qlo(j); q <= q_hi; q++)
    for (uint32_t h = 0; h < 2; h++) {
      const uint32_t m = 2 * q + h, s = 12 * q + 4 * h;
      if (j < s || j - s >= 24) continue;
      const int16_t tap = f[ce_kind(N_RB, m)][j - s];
      if (!tap) continue;                                   /* adds of 0: exact to skip */
      const uint32_t v = chl[m - m_base];
      ar = ce_sat16(ar + ce_mulhi_shl((int16_t)v, tap, 2));
      ai = ce_sat16(ai + ce_mulhi_shl((int16_t)(v >> 16), tap, 2));
    }
  return (uint32_t)(uint16_t)ar | ((uint32_t)(uint16_t)ai << 16);
}

/* one interpolated entry: mulhi(a, wa) << 1, then adds mulhi(b, wb) << 1 (cmult_sv.c:55-80) */
__device__ __forceinline__ int32_t ce_ip(uint32_t a, int16_t wa, uint32_t b, int16_t wb)
{
  const int16_t r = ce_sat16((int32_t)ce_mulhi_shl((int16_t)a, wa, 1) + ce_mulhi_shl((int16_t)b, wb, 1));
  const int16_t i = ce_sat16((int32_t)ce_mulhi_shl((int16_t)(a >> 16), wa, 1) + ce_mulhi_shl((int16_t)(b >> 16), wb, 1));
  return (int32_t)((uint32_t)(uint16_t)r | ((uint32_t)(uint16_t)i << 16));
}

/* the temporal interpolation that follows the estimate `cur` of pilot symbol `symbol`, with `prev`
 * the estimate of the preceding pilot symbol (lte_dl_channel_estimation.c:639-698) */
__device__ __forceinline__ void ce_interp(int32_t *__restrict__ E, uint32_t N, uint32_t Ncp, uint32_t symbol,
                                          uint32_t prev, uint32_t cur)
{
  const uint32_t p1 = Ncp ? 3 : 4, p2 = Ncp ? 6 : 7, p3 = Ncp ? 9 : 11;
  if (symbol == 0) {
    E[(p3 + 1) * N] = ce_ip(prev, 21845, cur, 10923);
    E[(p3 + 2) * N] = ce_ip(prev, 10923, cur, 21845);
  } else if (symbol == p2) {
    E[(p1 + 1) * N] = ce_ip(prev, 21845, cur, 10923);
    E[(p1 + 2) * N] = ce_ip(prev, 10923, cur, 21845);
  } else {                                                   /* pilot1 (from row 0) or pilot3 (from pilot2) */
    const uint32_t r0 = symbol == p1 ? 1 : p2 + 1;
    if (Ncp == 0) {
      E[r0 * N] = ce_ip(prev, 24576, cur, 8192);
      E[(r0 + 1) * N] = ce_ip(prev, 16384, cur, 16384);
      E[(r0 + 2) * N] = ce_ip(prev, 8192, cur, 24576);
    } else {                                                 /* the reference's 1/3, 2/3 weights, as written */
      E[r0 * N] = ce_ip(prev, 10923, cur, 21845);
      E[(r0 + 1) * N] = ce_ip(prev, 21845, cur, 10923);
    }
  }
}

/* pilot index range a workgroup's columns [j0, j0 + 256) need */
__device__ __forceinline__ void ce_window(uint32_t N_RB, uint32_t j0, uint32_t j1, uint32_t &m_base, uint32_t &n_p)
{
  const uint32_t q_lo = ce_qlo(j0), q_hi = min(N_RB - 1, (j1 - 1) / 12);
  m_base = 2 * q_lo;
  n_p = q_hi >= q_lo ? 2 * (q_hi - q_lo + 1) : 0;
}

}  // namespace

/* batch: grid (ceil(N / 256), n_sf); rxF = n_sf subframes of nsymb x N words followed by the
 * symbol 0 of the subframe after the batch; est = n_sf x nsymb x N.  PIL: only the 5 frequency-
 * interpolated pilot rows (symbols 0, p1, p2, p3 and the next subframe's 0), stored as the 4 pairs
 * of consecutive pilot rows, est = n_sf x 4 x N x 2 words (pair k at column j = (P_k, P_k+1)): every
 * estimate row is one 8-byte load of a pair, coalesced across the columns.  Only the columns a
 * pilot reaches are written (the grid stops at 12 N_RB + 16); the demodulator forms the rows itself
 * (rx_est, the same temporal interpolation) */
template <bool PIL>
__global__ void __launch_bounds__(CE_WG) k_chest(const chest_dev_t *__restrict__ c, const int32_t *__restrict__ rxF,
                                                 int32_t *__restrict__ est)
{
  __shared__ uint32_t chl[5][CE_MAXP];
  __shared__ int16_t flt[2][8][24];
  const uint32_t sf = blockIdx.y, N = c->N, nsymb = c->nsymb, Ncp = c->Ncp, N_RB = c->N_RB;
  const uint32_t sfi = (c->first_sf + sf * c->sf_step) % 10;
  const uint32_t p1 = Ncp ? 3 : 4, p2 = Ncp ? 6 : 7, p3 = Ncp ? 9 : 11;
  const uint32_t j0 = blockIdx.x * CE_WG, j1 = min(N, j0 + CE_WG);
  uint32_t m_base, n_p;
  ce_window(N_RB, j0, j1, m_base, n_p);
  for (uint32_t i = threadIdx.x; i < 2 * 8 * 24; i += CE_WG) (&flt[0][0][0])[i] = (&c->filt[0][0][0])[i];
  const int32_t *base = rxF + (size_t)sf * c->elem_syms * N;
  if (c->branch)
    for (uint32_t i = threadIdx.x; i < 5 * n_p; i += CE_WG) {
      const uint32_t in = i / n_p, m = m_base + i % n_p;
      const uint32_t sym = in == 0 ? 0 : in == 1 ? p1 : in == 2 ? p2 : in == 3 ? p3 : c->next_syms;  /* next sf */
      const uint32_t Ns = in < 2 ? 2 * sfi : in < 4 ? 2 * sfi + 1 : (2 * sfi + 2) % 20;
      chl[in][i % n_p] = ce_pilot_ch(c, base + (size_t)sym * N, Ns, in & 1u, m);
    }
  __syncthreads();
  const uint32_t j = j0 + threadIdx.x;
  if (j >= N) return;
  uint32_t P[5] = {0, 0, 0, 0, 0};
  if (c->branch)
    for (uint32_t in = 0; in < 5; in++) P[in] = ce_column(N_RB, flt[in & 1u], chl[in], m_base, j);
  if constexpr (PIL) {
    typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
    u32x2_t *E2 = (u32x2_t *)est + (size_t)sf * 4 * N + j;
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) E2[k * N] = (u32x2_t){P[k], P[k + 1]};
    return;
  }
  int32_t *E = est + (size_t)sf * nsymb * N + j;
  E[0] = (int32_t)P[0];
  E[p1 * N] = (int32_t)P[1];
  E[p2 * N] = (int32_t)P[2];
  E[p3 * N] = (int32_t)P[3];
  ce_interp(E, N, Ncp, p1, P[0], P[1]);
  ce_interp(E, N, Ncp, p2, P[1], P[2]);
  ce_interp(E, N, Ncp, p3, P[2], P[3]);
  ce_interp(E, N, Ncp, 0, P[3], P[4]);
}

/* one call of lte_dl_channel_estimation (drop-in): row `symbol` from the pilot symbol rxF_sym,
 * then the interpolation of the rows it closes, reading the previous pilot row from est */
__global__ void __launch_bounds__(CE_WG) k_chest_symbol(const chest_dev_t *__restrict__ c,
                                                        const int32_t *__restrict__ rxF_sym, int32_t *__restrict__ est,
                                                        uint32_t Ns, uint32_t l01, uint32_t symbol)
{
  __shared__ uint32_t chl[CE_MAXP];
  __shared__ int16_t flt[8][24];
  const uint32_t N = c->N, Ncp = c->Ncp, N_RB = c->N_RB;
  const uint32_t p1 = Ncp ? 3 : 4, p2 = Ncp ? 6 : 7, p3 = Ncp ? 9 : 11;
  const uint32_t j0 = blockIdx.x * CE_WG, j1 = min(N, j0 + CE_WG);
  uint32_t m_base, n_p;
  ce_window(N_RB, j0, j1, m_base, n_p);
  for (uint32_t i = threadIdx.x; i < 8 * 24; i += CE_WG) (&flt[0][0])[i] = (&c->filt[l01][0][0])[i];
  if (c->branch)
    for (uint32_t i = threadIdx.x; i < n_p; i += CE_WG) chl[i] = ce_pilot_ch(c, rxF_sym, Ns, l01, m_base + i);
  __syncthreads();
  const uint32_t j = j0 + threadIdx.x;
  if (j >= N) return;
  const uint32_t cur = c->branch ? ce_column(N_RB, flt, chl, m_base, j) : 0u;
  int32_t *E = est + j;
  const uint32_t prev_row = symbol == 0 ? p3 : symbol == p1 ? 0 : symbol == p2 ? p1 : p2;
  const uint32_t prev = (uint32_t)E[prev_row * N];
  E[symbol * N] = (int32_t)cur;
  ce_interp(E, N, Ncp, symbol, prev, cur);
}

/* ======================================================================================
 * Fused estimation + demodulation (batch path): the estimate rows rx_pdsch would read are never
 * written to HBM.  One 256-thread workgroup per subframe: the conjugate-pilot products of the 5
 * pilot symbols (LDS), their frequency-interpolated rows over the 12 N_RB estimate columns
 * (LDS, the k_chest sums), then the channel level of the first PDSCH symbol and the LLRs of
 * every PDSCH RE, each RE's estimate formed from the two pilot rows of its symbol with the
 * temporal interpolation's weights.  Bit-identical to k_chest followed by k_rx_level / k_rx_llr.
 * ==================================================================================== */
/* estimate row l as (instance a, weight wa, instance b, weight wb); wb = 0: pilot row a itself.
 * Instances: 0 = symbol 0, 1 = pilot1, 2 = pilot2, 3 = pilot3, 4 = next subframe's symbol 0
 * (lte_dl_channel_estimation.c:639-698 with high_speed_flag = 1) */
__device__ __forceinline__ void ce_row_src(uint32_t Ncp, uint32_t l, uint32_t &a, int16_t &wa, uint32_t &b, int16_t &wb)
{
  if (Ncp == 0) {
    switch (l) {
      case 0: a = 0; b = 0; wa = 0; wb = 0; return;
      case 1: a = 0; b = 1; wa = 24576; wb = 8192; return;
      case 2: a = 0; b = 1; wa = 16384; wb = 16384; return;
      case 3: a = 0; b = 1; wa = 8192; wb = 24576; return;
      case 4: a = 1; b = 1; wa = 0; wb = 0; return;
      case 5: a = 1; b = 2; wa = 21845; wb = 10923; return;
      case 6: a = 1; b = 2; wa = 10923; wb = 21845; return;
      case 7: a = 2; b = 2; wa = 0; wb = 0; return;
      case 8: a = 2; b = 3; wa = 24576; wb = 8192; return;
      case 9: a = 2; b = 3; wa = 16384; wb = 16384; return;
      case 10: a = 2; b = 3; wa = 8192; wb = 24576; return;
      case 11: a = 3; b = 3; wa = 0; wb = 0; return;
      case 12: a = 3; b = 4; wa = 21845; wb = 10923; return;
      default: a = 3; b = 4; wa = 10923; wb = 21845; return;
    }
  }
  switch (l) {
    case 0: a = 0; b = 0; wa = 0; wb = 0; return;
    case 1: a = 0; b = 1; wa = 10923; wb = 21845; return;
    case 2: a = 0; b = 1; wa = 21845; wb = 10923; return;
    case 3: a = 1; b = 1; wa = 0; wb = 0; return;
    case 4: a = 1; b = 2; wa = 21845; wb = 10923; return;
    case 5: a = 1; b = 2; wa = 10923; wb = 21845; return;
    case 6: a = 2; b = 2; wa = 0; wb = 0; return;
    case 7: a = 2; b = 3; wa = 10923; wb = 21845; return;
    case 8: a = 2; b = 3; wa = 21845; wb = 10923; return;
    case 9: a = 3; b = 3; wa = 0; wb = 0; return;
    case 10: a = 3; b = 4; wa = 21845; wb = 10923; return;
    default: a = 3; b = 4; wa = 10923; wb = 21845; return;
  }
}

constexpr uint32_t RXC_COLS = 1200;          /* 12 N_RB estimate columns, N_RB <= 100 */
constexpr uint32_t RXC_WG = 512;
constexpr uint32_t RXC_R = 3;                /* REs per thread and symbol: 512 x 3 >= 1200 */
constexpr uint32_t RXC_S = 2;                /* symbols whose loads are in flight together */

template <int QM>
__global__ void __launch_bounds__(RXC_WG) k_rx_chest(const chest_dev_t *__restrict__ ce, const rx_dev_t *__restrict__ c,
                                                     const int32_t *__restrict__ rxF, int16_t *__restrict__ llr,
                                                     uint8_t *__restrict__ shift, int unscramble)
{
  __shared__ uint32_t chl[5][2 * 100];
  __shared__ int16_t flt[2][8][24];
  __shared__ uint32_t P[5][RXC_COLS];
  __shared__ uint32_t acc;
  const uint32_t sf = blockIdx.x, N = ce->N, nsymb = ce->nsymb, Ncp = ce->Ncp, N_RB = ce->N_RB;
  const uint32_t sfi = (ce->first_sf + sf * ce->sf_step) % 10;
  const uint32_t p1 = Ncp ? 3 : 4, p2 = Ncp ? 6 : 7, p3 = Ncp ? 9 : 11, np = 2 * N_RB, ncol = 12 * N_RB;
  const int32_t *base = rxF + (size_t)sf * ce->elem_syms * N;
  for (uint32_t i = threadIdx.x; i < 2 * 8 * 24; i += RXC_WG) (&flt[0][0][0])[i] = (&ce->filt[0][0][0])[i];
  if (threadIdx.x == 0) acc = 0;
  if (ce->branch)
    for (uint32_t i = threadIdx.x; i < 5 * np; i += RXC_WG) {
      const uint32_t in = i / np, m = i - in * np;
      const uint32_t sym = in == 0 ? 0 : in == 1 ? p1 : in == 2 ? p2 : in == 3 ? p3 : ce->next_syms;
      const uint32_t Ns = in < 2 ? 2 * sfi : in < 4 ? 2 * sfi + 1 : (2 * sfi + 2) % 20;
      chl[in][m] = ce_pilot_ch(ce, base + (size_t)sym * N, Ns, in & 1u, m);
    }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < 5 * ncol; i += RXC_WG) {
    const uint32_t in = i / ncol, col = i - in * ncol;
    P[in][col] = ce->branch ? ce_column(N_RB, flt[in & 1u], chl[in], 0, 5 + col) : 0u;
  }
  __syncthreads();
  auto est = [&](uint32_t l, uint32_t col) -> uint32_t {
    uint32_t a, b;
    int16_t wa, wb;
    ce_row_src(Ncp, l, a, wa, b, wb);
    return wb == 0 ? P[a][col] : (uint32_t)ce_ip(P[a][col], wa, P[b][col], wb);
  };
  /* dlsch_channel_level over the first PDSCH symbol */
  {
    const uint32_t l = c->npdcch;
    rg32_t *map = (rg32_t *)(c->map + c->map_off[sfi][0]);
    uint32_t part = 0;
    for (uint32_t j = threadIdx.x; j < c->lvl_n[sfi]; j += RXC_WG) part += rx_h2(est(l, (map[j] >> 16) - 5));
    atomicAdd(&acc, part);
  }
  __syncthreads();
  const uint32_t sh = rx_shift_of((int32_t)acc, c->lvl_div[sfi]);
  if (threadIdx.x == 0) shift[sf] = (uint8_t)sh;
  rg32_t *gold = unscramble ? (rg32_t *)(c->gold + (size_t)sfi * c->gold_words) : nullptr;
  const int16_t a1 = c->a1, a2 = c->a2;
  for (uint32_t k0 = 0; k0 < c->n_sym; k0 += RXC_S) {
    /* all map words, then all received words of RXC_S symbols, then the arithmetic */
    uint32_t mw[RXC_S][RXC_R], yv[RXC_S][RXC_R];
#pragma unroll
    for (uint32_t u = 0; u < RXC_S; u++) {
      const uint32_t k = k0 + u, len = k < c->n_sym ? c->len[sfi][k] : 0u;
      rg32_t *map = (rg32_t *)(c->map + c->map_off[sfi][k < c->n_sym ? k : 0]);
#pragma unroll
      for (uint32_t r = 0; r < RXC_R; r++) {
        const uint32_t j = threadIdx.x + RXC_WG * r;
        mw[u][r] = j < len ? map[j] : 5u << 16;
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < RXC_S; u++) {
      const int32_t *y = base + (size_t)(c->npdcch + k0 + u < nsymb ? c->npdcch + k0 + u : 0) * N;
#pragma unroll
      for (uint32_t r = 0; r < RXC_R; r++) yv[u][r] = (uint32_t)y[mw[u][r] & 0xFFFFu];
    }
#pragma unroll
    for (uint32_t u = 0; u < RXC_S; u++) {
      const uint32_t k = k0 + u;
      if (k >= c->n_sym) break;
      const uint32_t l = c->npdcch + k, len = c->len[sfi][k], lb = c->llr_off[sfi][k];
      int16_t *out = llr + (size_t)sf * c->llr_stride + lb;
#pragma unroll
      for (uint32_t r = 0; r < RXC_R; r++) {
        const uint32_t j = threadIdx.x + RXC_WG * r;
        if (j >= len) break;
        rx_re_llr<QM>(est(l, (mw[u][r] >> 16) - 5), yv[u][r], sh, a1, a2, gold, lb + j * QM, out + QM * j);
      }
    }
  }
}

hipError_t oai4g_launch_rx_chest(const chest_dev_t *d_ce, const rx_dev_t *d_rx, const rx_dev_t *h_rx, int n_sf,
                                 const int32_t *d_rxF, int16_t *d_llr, uint8_t *d_shift, int unscramble, hipStream_t s)
{
  if (n_sf <= 0) return hipSuccess;
  if (h_rx->Qm == 2)
    hipLaunchKernelGGL(k_rx_chest<2>, dim3(n_sf), dim3(RXC_WG), 0, s, d_ce, d_rx, d_rxF, d_llr, d_shift, unscramble);
  else if (h_rx->Qm == 4)
    hipLaunchKernelGGL(k_rx_chest<4>, dim3(n_sf), dim3(RXC_WG), 0, s, d_ce, d_rx, d_rxF, d_llr, d_shift, unscramble);
  else
    hipLaunchKernelGGL(k_rx_chest<6>, dim3(n_sf), dim3(RXC_WG), 0, s, d_ce, d_rx, d_rxF, d_llr, d_shift, unscramble);
  return hipGetLastError();
}

hipError_t oai4g_launch_chest(const chest_dev_t *d_cfg, const chest_dev_t *h_cfg, int n_sf, const int32_t *d_rxF,
                              int32_t *d_est, hipStream_t s)
{
  if (n_sf <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_chest<false>, dim3((h_cfg->N + CE_WG - 1) / CE_WG, n_sf), dim3(CE_WG), 0, s, d_cfg, d_rxF, d_est);
  return hipGetLastError();
}

hipError_t oai4g_launch_chest_pilots(const chest_dev_t *d_cfg, const chest_dev_t *h_cfg, int n_sf, const int32_t *d_rxF,
                                     int32_t *d_pil, hipStream_t s)
{
  if (n_sf <= 0) return hipSuccess;
  const uint32_t span = min(h_cfg->N, 12 * h_cfg->N_RB + 16);   /* columns a pilot window reaches */
  hipLaunchKernelGGL(k_chest<true>, dim3((span + CE_WG - 1) / CE_WG, n_sf), dim3(CE_WG), 0, s, d_cfg, d_rxF, d_pil);
  return hipGetLastError();
}

hipError_t oai4g_launch_chest_symbol(const chest_dev_t *d_cfg, const chest_dev_t *h_cfg, const int32_t *d_rxF_sym,
                                     int32_t *d_est, int Ns, int l, int symbol, hipStream_t s)
{
  hipLaunchKernelGGL(k_chest_symbol, dim3((h_cfg->N + CE_WG - 1) / CE_WG), dim3(CE_WG), 0, s, d_cfg, d_rxF_sym, d_est,
                     (uint32_t)Ns, (uint32_t)(l == 0 ? 0 : 1), (uint32_t)symbol);
  return hipGetLastError();
}

/* ======================================================================================
 * lte_est_freq_offset's integer part (PHY/LTE_ESTIMATION/lte_est_freq_offset.c:45-166, antenna 0):
 * one wave per estimate plane.  dl_channel_level of row l from RE 12 (re^2 + im^2 over N_RB * 12
 * REs, wrapping 32-bit sums, C int division), dl_ch_shift = 6 + log2_approx(level) / 2, then
 * dot_product (PHY/TOOLS/cdot_prod.c:40-118: per RE (xr yr + xi yi) >> shift and
 * (xr yi - xi yr) >> shift, wrapping sums, packs to int16) of row l against the previous pilot
 * row over the upper half (from RE (N_RB / 2 + 1) * 12, (N_RB / 2 - 1) * 12 REs); omega = twice it,
 * int16 wrap per component, as re | im << 16: the reference's omega_cpx points at omega itself
 * (:152), so its upper-half dot product (:164) overwrites the lower half's (:150) before
 * omega_cpx->r += omega.r (:165-166) — the lower half never counts (tests/test_ref_pin_fo_cpu.py).
 * Sums are mod 2^32, so the wave's reduction order gives the reference's lane sums exactly.
 * ==================================================================================== */
static __device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v)
{
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += (uint32_t)__shfl_xor((int)v, m, 64);
  return v;
}

static __device__ __forceinline__ int16_t fo_sat16(int32_t v) { return (int16_t)max(-32768, min(32767, v)); }

__global__ void __launch_bounds__(64) k_freq_offset(const int32_t *__restrict__ est, size_t est_stride, int n_jobs,
                                                    int N_RB, uint32_t row_off, uint32_t prev_off,
                                                    int32_t *__restrict__ omega)
{
  const int j = blockIdx.x;
  if (j >= n_jobs) return;
  const int lane = threadIdx.x;
  const uint32_t *p = (const uint32_t *)est + (size_t)j * est_stride;
  const int nre = N_RB * 12;
  uint32_t acc = 0;
  for (int i = lane; i < nre; i += 64) {
    const uint32_t w = p[row_off + 12 + i];
    const int32_t re = (int16_t)(w & 0xFFFF), im = (int16_t)(w >> 16);
    acc += (uint32_t)(re * re) + (uint32_t)(im * im);
  }
  acc = wave_sum_u32(acc);
  const int32_t avg = (int32_t)acc / nre;
  const uint32_t x = (uint32_t)avg & 0x7FFFFFFFu;      /* log2_approx: bits 0..30 */
  const uint32_t shift = 6 + (x ? 32u - __clz(x) : 0u) / 2;
  const int n = (N_RB / 2 - 1) * 12, hi = (N_RB / 2 + 1) * 12;
  int16_t out_re = 0, out_im = 0;
  {
    const int base = hi;
    uint32_t sre = 0, sim = 0;
    for (int i = lane; i < n; i += 64) {
      const uint32_t a = p[row_off + base + i], b = p[prev_off + base + i];
      const int32_t xr = (int16_t)(a & 0xFFFF), xi = (int16_t)(a >> 16);
      const int32_t yr = (int16_t)(b & 0xFFFF), yi = (int16_t)(b >> 16);
      const int32_t nyr = (int16_t)(-yr);                 /* _mm_sign_epi16: -(-32768) = -32768 */
      sre += (uint32_t)((int32_t)((uint32_t)(xr * yr) + (uint32_t)(xi * yi)) >> shift);
      sim += (uint32_t)((int32_t)((uint32_t)(xr * yi) + (uint32_t)(xi * nyr)) >> shift);
    }
    sre = wave_sum_u32(sre);
    sim = wave_sum_u32(sim);
    out_re = fo_sat16((int32_t)sre);
    out_im = fo_sat16((int32_t)sim);
    out_re = (int16_t)(out_re + out_re);
    out_im = (int16_t)(out_im + out_im);
  }
  if (lane == 0) omega[j] = (int32_t)((uint32_t)(uint16_t)out_re | ((uint32_t)(uint16_t)out_im << 16));
}

hipError_t oai4g_launch_freq_offset(const int32_t *d_est, size_t est_stride, int n_jobs, int N_RB, uint32_t row_off,
                                    uint32_t prev_off, int32_t *d_omega, hipStream_t s)
{
  if (n_jobs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_freq_offset, dim3(n_jobs), dim3(64), 0, s, d_est, est_stride, n_jobs, N_RB, row_off, prev_off,
                     d_omega);
  return hipGetLastError();
}
