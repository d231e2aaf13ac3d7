/*
 * gfx950 kernels for the downlink control region of the transmit grid:
 *   generate_pcfich (PHY/LTE_TRANSPORT/pcfich.c:144-228): CFI codeword (pcfich_b, :138-142),
 *   Gold scrambling with c_init = ((2 Nid + 1)(subframe + 1)) << 9 + Nid (pcfich_scrambling
 *   :86-109, lte_gold_generic lte_gold.c:151-177), QPSK with the SISO or ALAMOUTI gain and
 *   precoding (:168-197), and the four-REG mapping of symbol 0 that skips the two CRS positions of
 *   each 6-RE group (:200-227).
 * One 64-lane wave does everything: lane 0 runs the Gold warm-up, every lane derives the bits it
 * needs from the broadcast scrambling word, lanes 0..15 each own one RE of every antenna.
 */
#include "oai4g_internal.h"

static __device__ __forceinline__ void pcfich_gold_step(uint32_t &x1, uint32_t &x2)
{
  x1 = (x1 >> 1) ^ (x1 >> 4);
  x1 = x1 ^ (x1 << 31) ^ (x1 << 28);
  x2 = (x2 >> 1) ^ (x2 >> 2) ^ (x2 >> 3) ^ (x2 >> 4);
  x2 = x2 ^ (x2 << 31) ^ (x2 << 30) ^ (x2 << 29) ^ (x2 << 28);
}

/* pcfich_b[cfi - 1][i] (pcfich.c:138-142): CFI 1..3 repeat (0,1,1) / (1,0,1) / (1,1,0) */
static __device__ __forceinline__ uint32_t cfi_bit(uint32_t cfi, uint32_t i) { return (0xEEu >> (3 * (cfi - 1) + i % 3)) & 1u; }

__global__ void __launch_bounds__(64) k_pcfich(int32_t *__restrict__ g0, int32_t *__restrict__ g1, pcfich_args_t a)
{
  __shared__ uint32_t s_word;
  const uint32_t lane = threadIdx.x;
  if (lane == 0) {   /* lte_gold_generic(reset = 1): 50 word steps, the 50th word is the output */
    uint32_t x1 = 1u + (1u << 31), x2 = a.c_init;
    x2 = x2 ^ ((x2 ^ (x2 >> 1) ^ (x2 >> 2) ^ (x2 >> 3)) << 31);
    for (int n = 1; n < 50; n++) pcfich_gold_step(x1, x2);
    pcfich_gold_step(x1, x2);
    s_word = x1 ^ x2;
  }
  __syncthreads();
  if (lane >= 16) return;
  const uint32_t s = s_word, m = lane;
  auto bt = [&](uint32_t i) { return cfi_bit(a.cfi, i) ^ ((s >> i) & 1u); };
  const int16_t g = a.gain;
  int16_t d0r, d0i, d1r, d1i;
  if (a.mode1) {
    d0r = d1r = bt(2 * m) ? (int16_t)-g : g;
    d0i = d1i = bt(2 * m + 1) ? (int16_t)-g : g;
  } else {
    const uint32_t i = m & ~1u;               /* the pair (i, i + 1) of :182-196 */
    const int16_t x0r = bt(2 * i) ? (int16_t)-g : g, x0i = bt(2 * i + 1) ? (int16_t)-g : g;
    const int16_t y1r = bt(2 * i + 2) ? g : (int16_t)-g, y1i = bt(2 * i + 3) ? (int16_t)-g : g;   /* -x1* */
    if ((m & 1u) == 0) { d0r = x0r; d0i = x0i; d1r = y1r; d1i = y1i; }
    else { d0r = (int16_t)-y1r; d0i = y1i; d1r = x0r; d1i = (int16_t)-x0i; }
  }
  /* RE m = the (m mod 4)-th non-CRS position of REG m / 4 */
  const uint32_t q = m >> 2, k = m & 3, ns3 = a.nushift3;
  uint32_t pos = 0, seen = 0;
  for (uint32_t i = 0; i < 6; i++)
    if (i != ns3 && i != ns3 + 3) {
      if (seen == k) pos = i;
      seen++;
    }
  const uint32_t idx = a.reg_off[q] + pos;
  g0[idx] = (int32_t)((uint16_t)d0r | ((uint32_t)(uint16_t)d0i << 16));
  if (a.n_ant > 1) g1[idx] = (int32_t)((uint16_t)d1r | ((uint32_t)(uint16_t)d1i << 16));
}

hipError_t oai4g_launch_pcfich(int32_t *d_g0, int32_t *d_g1, const pcfich_args_t &a, hipStream_t s)
{
  hipLaunchKernelGGL(k_pcfich, dim3(1), dim3(64), 0, s, d_g0, d_g1, a);
  return hipGetLastError();
}
