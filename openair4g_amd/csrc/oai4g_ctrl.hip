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

/* ======================================================================================
 * PDCCH: generate_dci_top (PHY/LTE_TRANSPORT/dci.c:2024-2346) after the PCFICH.
 * One 256-thread workgroup:
 *   1. every DCI, one wave each: CRC16 over the A payload bits with the reference's partial-byte
 *      step (crc_byte.c:155-171), XOR with the RNTI (ccoding_byte_lte.c:84-92); then each lane
 *      produces rate-matched bits e_k directly: k -> (stream s, compacted index j) of the
 *      circular buffer without <NULL> (lte_rate_matching.c:637-680) -> (column, row) of the
 *      32-column sub-block interleaver (:133-190) -> input bit i -> the tail-biting TBCC output
 *      d^(s)_i = parity(g_s & c_i..c_{i-6} mod D) (the LUT encoder of ccodelte_encode restated as
 *      a circular convolution), written at 72 nCCE + k of the <NIL>-initialised bit array;
 *   2. the Gold words of c_init = (subframe << 9) + Nid (one lane) and the scrambling of the
 *      non-<NIL> bits (pdcch_scrambling, dci.c:1905-1930);
 *   3. every mapped RE: its QPSK symbol (SISO with <NIL> -> 0, or the ALAMOUTI pair with
 *      <NIL> -> +gain, :2170-2224) from the host's interleaving + REG map (pdcch_interleaving
 *      :277-341, REG allocation :2234-2340).
 * ==================================================================================== */
#define DCI_EBITS ((2 * 33 + 22) * 72 + 8 * 72)

__constant__ uint8_t c_bitrev_cc[32] = {1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31,   /* 36.212 T 5.1.4-2 */
                                        0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30};

static __device__ uint32_t crc16_byte(uint32_t v)   /* crc16Table[v] (crc_byte.c:95) */
{
  uint32_t reg = 0;
  for (int i = 7; i >= 0; i--) {
    const uint32_t fb = ((reg >> 15) ^ (v >> i)) & 1u;
    reg = (reg << 1) & 0xFFFFu;
    if (fb) reg ^= 0x1021u;
  }
  return reg;
}

__global__ void __launch_bounds__(256) k_dci(dci_args_t a, const uint32_t *__restrict__ map,
                                             const uint16_t *__restrict__ src, int32_t *__restrict__ g0,
                                             int32_t *__restrict__ g1)
{
  __shared__ uint8_t e[DCI_EBITS];
  __shared__ uint32_t gold[DCI_EBITS / 32 + 2];
  __shared__ uint8_t cb[OAI4G_MAX_DCI][64 + 16];     /* c = a || (crc ^ rnti) of every DCI */
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  for (uint32_t i = tid; i < DCI_EBITS; i += blockDim.x) e[i] = 2;
  if (tid == 64) {           /* lte_gold_generic: word w is the output after 50 + w steps */
    uint32_t x1 = 1u + (1u << 31), x2 = a.c_init;
    x2 = x2 ^ ((x2 ^ (x2 >> 1) ^ (x2 >> 2) ^ (x2 >> 3)) << 31);
    for (int n = 1; n < 50; n++) pcfich_gold_step(x1, x2);
    const uint32_t nw = (a.nbits + 31) >> 5;
    for (uint32_t w = 0; w < nw; w++) {
      pcfich_gold_step(x1, x2);
      gold[w] = x1 ^ x2;
    }
  }
  /* c bits of every DCI: payload bits, then the RNTI-masked CRC16 (one lane per DCI) */
  for (uint32_t di = wave; di < a.n_dci; di += 4) {
    const dci_dev_t &d = a.dci[di];
    for (uint32_t i = lane; i < d.A; i += 64) cb[di][i] = (uint8_t)((d.flip[i >> 3] >> (7 - (i & 7))) & 1u);
    if (lane == 0) {
      uint32_t crc = 0;
      const uint32_t full = d.A >> 3, r = d.A & 7u;
      for (uint32_t b = 0; b < full; b++) crc = (crc << 8) ^ (crc16_byte(d.flip[b] ^ (crc >> 24)) << 16);
      if (r) crc = (crc << r) ^ (crc16_byte((((uint32_t)d.flip[full] >> (8 - r)) ^ (crc >> (32 - r))) & 0xFFu) << 16);
      crc ^= d.rnti << 16;
      for (uint32_t i = 0; i < 16; i++) cb[di][d.A + i] = (uint8_t)((crc >> (31 - i)) & 1u);
    }
  }
  __syncthreads();
  /* rate-matched bits of every DCI, all 256 threads over the concatenated (DCI, k) space */
  for (uint32_t di = 0; di < a.n_dci; di++) {
    const dci_dev_t &d = a.dci[di];
    if (d.nCCE < 0) continue;                        /* not transmitted (dci.c:2119, 2138) */
    const uint32_t D = d.A + 16u, R = (D + 31) >> 5, ND = 32 * R - D, E = 72u << d.L;
    const uint8_t *c = cb[di];
    for (uint32_t k = tid; k < E; k += blockDim.x) {
      const uint32_t jj = k % (3 * D), s = jj / D;
      uint32_t j = jj - s * D, col = 0;
      for (; col < 32; col++) {                      /* column holding the j-th non-<NULL> entry */
        const uint32_t n = R - (c_bitrev_cc[col] < ND ? 1u : 0u);
        if (j < n) break;
        j -= n;
      }
      const uint32_t row = j + (c_bitrev_cc[col] < ND ? 1u : 0u);
      const uint32_t i = 32 * row + c_bitrev_cc[col] - ND;   /* TBCC input position */
      const uint32_t g = s == 0 ? 0133u : (s == 1 ? 0171u : 0165u);
      uint32_t par = 0;
#pragma unroll
      for (uint32_t t = 0; t < 7; t++)               /* tap t: c_{i-t}, generator bit 6 - t */
        par ^= ((g >> (6 - t)) & 1u) & c[(i + D - t) % D];
      e[72 * (uint32_t)d.nCCE + k] = (uint8_t)par;
    }
    __syncthreads();                                 /* DCIs land in generate_dci_top's order */
  }
  __syncthreads();
  for (uint32_t i = tid; i < a.nbits; i += blockDim.x)   /* pdcch_scrambling: <NIL> stays */
    if (e[i] != 2) e[i] = (uint8_t)(e[i] ^ ((gold[i >> 5] >> (i & 31)) & 1u));
  __syncthreads();
  const int16_t gq = a.gain;
  for (uint32_t r = tid; r < a.n_re; r += blockDim.x) {
    const uint32_t sym = src[r];
    int16_t y0r, y0i, y1r, y1i;
    if (a.mode1) {
      const uint8_t b0 = e[2 * sym], b1 = e[2 * sym + 1];
      y0r = y1r = b0 == 2 ? (int16_t)0 : (b0 == 1 ? (int16_t)-gq : gq);
      y0i = y1i = b1 == 2 ? (int16_t)0 : (b1 == 1 ? (int16_t)-gq : gq);
    } else {
      const uint32_t p = sym & ~1u;                  /* ALAMOUTI pair (p, p + 1), bits 2p .. 2p + 3 */
      const int16_t s0 = e[2 * p] == 1 ? (int16_t)-gq : gq, s1 = e[2 * p + 1] == 1 ? (int16_t)-gq : gq;
      const int16_t s2 = e[2 * p + 2] == 1 ? (int16_t)-gq : gq, s3 = e[2 * p + 3] == 1 ? (int16_t)-gq : gq;
      if ((sym & 1u) == 0) { y0r = s0; y0i = s1; y1r = (int16_t)-s2; y1i = s3; }   /* x0, -x1* */
      else { y0r = s2; y0i = s3; y1r = s0; y1i = (int16_t)-s1; }                   /* x1, x0* */
    }
    const uint32_t off = map[r];
    g0[off] = (int32_t)((uint16_t)y0r | ((uint32_t)(uint16_t)y0i << 16));
    if (a.n_ant > 1) g1[off] = (int32_t)((uint16_t)y1r | ((uint32_t)(uint16_t)y1i << 16));
  }
}

hipError_t oai4g_launch_dci(const dci_args_t &a, const uint32_t *d_map, const uint16_t *d_src, int32_t *d_g0,
                            int32_t *d_g1, uint32_t g1_stride, hipStream_t s)
{
  (void)g1_stride;
  hipLaunchKernelGGL(k_dci, dim3(1), dim3(256), 0, s, a, d_map, d_src, d_g0, d_g1);
  return hipGetLastError();
}
