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

/* ======================================================================================
 * PSS / SSS (pss.c:50-103, sss.c:47-92): one thread per sequence element m = 0..61 of the
 * inner 62 subcarriers, k = N - 31 + m with the DC skip; every antenna gets the same value,
 * written with '=' as the reference does.
 * ==================================================================================== */
struct sync_ptrs_t {
  int32_t *g[4];
};

__global__ void __launch_bounds__(64) k_sync(sync_ptrs_t p, sync_args_t a)
{
  const uint32_t m = threadIdx.x;
  if (m >= 62) return;
  uint32_t k = a.N - 31 + m;
  if (k >= a.N) k = k + 1 - a.N;                       /* k++ (skip DC), k -= N */
  int16_t re, im;
  if (a.pss) {
    re = (int16_t)(((int32_t)a.a * a.val[m][0]) >> 15);
    im = (int16_t)(((int32_t)a.a * a.val[m][1]) >> 15);
  } else {
    re = (int16_t)((int32_t)a.a * a.val[m][0]);
    im = 0;
  }
  const int32_t v = (int32_t)((uint16_t)re | ((uint32_t)(uint16_t)im << 16));
  for (uint32_t aa = 0; aa < a.n_ant; aa++) p.g[aa][k] = v;
}

hipError_t oai4g_launch_sync(int32_t *const *d_sym, const sync_args_t &a, hipStream_t s)
{
  sync_ptrs_t p = {};
  for (uint32_t aa = 0; aa < a.n_ant && aa < 4; aa++) p.g[aa] = d_sym[aa];
  hipLaunchKernelGGL(k_sync, dim3(1), dim3(64), 0, s, p, a);
  return hipGetLastError();
}

/* ======================================================================================
 * PBCH (pbch.c:161-420).  One 256-thread workgroup:
 *   1. (frame_mod4 == 0) lane 0: CRC16 of the 24 MIB bits XOR the antenna mask
 *      (ccodelte_encode add_crc = 2, ccoding_byte_lte.c:84-92); every thread then produces
 *      rate-matched bits e_k directly: k -> (stream, compacted index) of the circular buffer
 *      (lte_rate_matching.c:637-680) -> (column, row) of the 32-column interleaver
 *      (:133-190) -> TBCC output d^(s)_i as a circular convolution of c; scrambled with the
 *      Gold words of c_init = Nid_cell (pbch_scrambling :760-783) and stored as bytes (the
 *      reference's eNB_pbch->pbch_e, kept for frame_mod4 = 1..3);
 *   2. the quarter frame_mod4 of e mapped to the 240 (216) REs of slot 1 symbols 0..3: RE slot
 *      j = the j-th non-pilot subcarrier of the 72 around DC, k first then l; QPSK with
 *      gain (amp 23170) >> 15, SISO on every antenna or the ALAMOUTI pair (j, j + 1) with the
 *      reference's 1/sqrt2 floor scaling and the partner written from the accumulated values
 *      of RE j (allocate_pbch_REs_in_RB :62-158); '+=' into the grid.
 * ==================================================================================== */
struct pbch_ptrs_t {
  int32_t *g[4];
};

static __device__ __forceinline__ int32_t pk16(int16_t re, int16_t im)
{
  return (int32_t)((uint16_t)re | ((uint32_t)(uint16_t)im << 16));
}
static __device__ __forceinline__ int16_t lo16(int32_t v) { return (int16_t)(v & 0xFFFF); }
static __device__ __forceinline__ int16_t hi16(int32_t v) { return (int16_t)((uint32_t)v >> 16); }

__global__ void __launch_bounds__(256) k_pbch(pbch_ptrs_t p, uint8_t *__restrict__ ebytes, pbch_args_t a)
{
  __shared__ uint8_t c[40];
  __shared__ uint32_t gold[64];
  __shared__ uint8_t e[1920];
  const uint32_t tid = threadIdx.x;
  if (a.encode) {
    if (tid == 0) {
      uint32_t crc = 0;                                  /* crc16 over 3 whole bytes (crc_byte.c:155-171) */
      for (int b = 0; b < 3; b++) crc = (crc << 8) ^ (crc16_byte(a.a[b] ^ ((crc >> 24) & 0xFFu)) << 16);
      crc ^= (uint32_t)a.amask << 16;
      for (int i = 0; i < 24; i++) c[i] = (uint8_t)((a.a[i >> 3] >> (7 - (i & 7))) & 1u);
      for (int i = 0; i < 16; i++) c[24 + i] = (uint8_t)((crc >> (31 - i)) & 1u);
    }
    if (tid == 64) {                                     /* lte_gold_generic, c_init = Nid */
      uint32_t x1 = 1u + (1u << 31), x2 = a.Nid;
      x2 = x2 ^ ((x2 ^ (x2 >> 1) ^ (x2 >> 2) ^ (x2 >> 3)) << 31);
      for (int n = 1; n < 50; n++) pcfich_gold_step(x1, x2);
      for (uint32_t w = 0; w < (a.E + 31u) / 32u; w++) {
        pcfich_gold_step(x1, x2);
        gold[w] = x1 ^ x2;
      }
    }
    __syncthreads();
    const uint32_t D = 40, R = 2, ND = 32 * R - D;
    for (uint32_t k = tid; k < a.E; k += blockDim.x) {
      const uint32_t jj = k % (3 * D), s = jj / D;
      uint32_t j = jj - s * D, col = 0;
      for (; col < 32; col++) {
        const uint32_t n = R - (c_bitrev_cc[col] < ND ? 1u : 0u);
        if (j < n) break;
        j -= n;
      }
      const uint32_t row = j + (c_bitrev_cc[col] < ND ? 1u : 0u);
      const uint32_t i = 32 * row + c_bitrev_cc[col] - ND;
      const uint32_t g = s == 0 ? 0133u : (s == 1 ? 0171u : 0165u);
      uint32_t par = 0;
#pragma unroll
      for (uint32_t t = 0; t < 7; t++) par ^= ((g >> (6 - t)) & 1u) & c[(i + D - t) % D];
      e[k] = (uint8_t)(par ^ ((gold[k >> 5] >> (k & 31)) & 1u));
    }
    __syncthreads();
    for (uint32_t k = tid; k < a.E; k += blockDim.x) ebytes[k] = e[k];
  } else {
    for (uint32_t k = tid; k < a.E; k += blockDim.x) e[k] = ebytes[k];
  }
  __syncthreads();
  /* RE slots of the quarter: 4 symbols, 72 subcarriers each minus the pilot positions */
  const uint8_t *x = e + a.quarter * (a.E >> 2);
  const uint32_t nre = (a.E >> 2) >> 1;
  const int16_t g = a.gain;
  auto bin = [&](uint32_t sc) {                            /* subcarrier 0..71 around DC -> grid bin */
    const uint32_t b = a.N - 36 + sc;
    return b >= a.N ? b - a.N + 1 : b;
  };
  auto pos = [&](uint32_t j) {                             /* RE slot -> offset in the 4-symbol window */
    uint32_t l = 0;
    for (; l < 4; l++) {
      const uint32_t n = ((a.pil_mask >> l) & 1u) ? 48u : 72u;
      if (j < n) break;
      j -= n;
    }
    uint32_t sc = j;
    if ((a.pil_mask >> l) & 1u) {                         /* the j-th of the 8 non-pilot REs per RB */
      const uint32_t rb = j >> 3, q = j & 7u;
      uint32_t cnt = 0, re = 0;
      for (uint32_t r = 0; r < 12; r++)
        if (r % 3 != a.nushift3) {
          if (cnt == q) re = r;
          cnt++;
        }
      sc = 12 * rb + re;
    }
    return l * a.N + bin(sc);
  };
  if (a.mode1) {
    for (uint32_t j = tid; j < nre; j += blockDim.x) {
      const uint32_t o = pos(j);
      const int16_t re = x[2 * j] == 1 ? (int16_t)-g : g, im = x[2 * j + 1] == 1 ? (int16_t)-g : g;
      for (uint32_t aa = 0; aa < a.n_ant; aa++) {
        const int32_t v = p.g[aa][o];
        p.g[aa][o] = pk16((int16_t)(lo16(v) + re), (int16_t)(hi16(v) + im));
      }
    }
  } else {
    for (uint32_t j = 2 * tid; j < nre; j += 2 * blockDim.x) {
      const uint32_t o = pos(j), o2 = pos(j + 1);
      const int16_t t1r = x[2 * j] == 1 ? (int16_t)-g : g, t1i = x[2 * j + 1] == 1 ? (int16_t)-g : g;
      const int16_t t2r = x[2 * j + 2] == 1 ? g : (int16_t)-g, t2i = x[2 * j + 3] == 1 ? (int16_t)-g : g;
      const int32_t v0 = p.g[0][o], v1 = p.g[1][o];
      const int16_t y0r = (int16_t)(lo16(v0) + (int16_t)((t1r * 23170) >> 15));
      const int16_t y0i = (int16_t)(hi16(v0) + (int16_t)((t1i * 23170) >> 15));
      const int16_t y1r = (int16_t)(lo16(v1) + (int16_t)((t2r * 23170) >> 15));
      const int16_t y1i = (int16_t)(hi16(v1) + (int16_t)((t2i * 23170) >> 15));
      p.g[0][o] = pk16(y0r, y0i);
      p.g[1][o] = pk16(y1r, y1i);
      const int32_t w0 = p.g[0][o2], w1 = p.g[1][o2];
      p.g[0][o2] = pk16((int16_t)(lo16(w0) - y1r), (int16_t)(hi16(w0) + y1i));
      p.g[1][o2] = pk16((int16_t)(lo16(w1) + y0r), (int16_t)(hi16(w1) - y0i));
    }
  }
}

hipError_t oai4g_launch_pbch(int32_t *const *d_g, uint8_t *d_e, const pbch_args_t &a, hipStream_t s)
{
  pbch_ptrs_t p = {};
  for (uint32_t aa = 0; aa < a.n_ant && aa < 4; aa++) p.g[aa] = d_g[aa];
  hipLaunchKernelGGL(k_pbch, dim3(1), dim3(256), 0, s, p, d_e, a);
  return hipGetLastError();
}

/* ======================================================================================
 * PHICH (generate_phich, phich.c:401-780, normal CP).  One thread per (PHICH, symbol i of 12):
 * the scrambling word of the PHICH's c_init (one Gold word), the orthogonal-sequence sign,
 * BPSK with the gain, SISO or the ALAMOUTI pair (i even: (x0, -x1*), i odd: (x1, x0*)), RE =
 * the (i mod 4)-th non-RS position of REG i / 4.  Several PHICHs may share REs, and the
 * reference accumulates int16 with wrap-around, so contributions go through int32 atomics and
 * are folded into the grid afterwards (wrap-add commutes).
 * ==================================================================================== */
struct phich_ptrs_t {
  int32_t *g[2];
};

__global__ void __launch_bounds__(256) k_phich(phich_ptrs_t p, int32_t *__restrict__ acc, phich_args_t a)
{
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < 4 * a.win; i += blockDim.x) acc[i] = 0;
  __syncthreads();
  for (uint32_t t = tid; t < 12 * a.n; t += blockDim.x) {
    const phich_item_t &it = a.it[t / 12];
    const uint32_t i = t % 12;
    uint32_t x1 = 1u + (1u << 31), x2 = it.c_init;
    x2 = x2 ^ ((x2 ^ (x2 >> 1) ^ (x2 >> 2) ^ (x2 >> 3)) << 31);
    for (int n = 1; n < 50; n++) pcfich_gold_step(x1, x2);
    pcfich_gold_step(x1, x2);
    const uint32_t sw = x1 ^ x2;
    const int hi = it.hi ? 1 : 0;
    auto dsym = [&](uint32_t q, int &re, int &im) {   /* d[2q], d[2q + 1] of phich.c:455-536 */
      const int cs = ((sw >> q) & 1u) == 0 ? 1 - 2 * hi : 2 * hi - 1;
      const uint32_t w = it.nseq & 3u;                /* +-1 pattern of Table 6.9.1-2 */
      const int sg = ((w == 1 && (q & 1)) || (w == 2 && (q & 2)) || (w == 3 && ((q ^ (q >> 1)) & 1))) ? -1 : 1;
      const int v = sg * cs;
      if (it.nseq < 4) { re = v; im = v; }
      else { re = -v; im = v; }
    };
    int re0, im0;
    dsym(i, re0, im0);
    int y0r, y0i, y1r = 0, y1i = 0;
    const int g = a.gain;
    if (a.mode1) {
      y0r = (int16_t)(re0 * g);
      y0i = (int16_t)(im0 * g);
    } else {
      const uint32_t i0 = i & ~1u;
      int ar, ai, br, bi;
      dsym(i0, ar, ai);
      dsym(i0 + 1, br, bi);
      const int16_t a0r = (int16_t)(ar * g), a0i = (int16_t)(ai * g);
      const int16_t b1r = (int16_t)(-br * g), b1i = (int16_t)(bi * g);   /* -x1* */
      if ((i & 1u) == 0) { y0r = a0r; y0i = a0i; y1r = b1r; y1i = b1i; }
      else { y0r = (int16_t)-b1r; y0i = b1i; y1r = a0r; y1i = (int16_t)-a0i; }
    }
    const uint32_t q = i >> 2, m = i & 3u;
    uint32_t pos = 0, cnt = 0;
    for (uint32_t r = 0; r < 6; r++)
      if (r != a.nushift && r != a.nushift + 3) {
        if (cnt == m) pos = r;
        cnt++;
      }
    const uint32_t o = it.reg_off[q] + pos;
    atomicAdd(&acc[o], y0r);
    atomicAdd(&acc[a.win + o], y0i);
    if (a.n_ant > 1) {
      atomicAdd(&acc[2 * a.win + o], y1r);
      atomicAdd(&acc[3 * a.win + o], y1i);
    }
  }
  __syncthreads();
  for (uint32_t o = tid; o < a.win; o += blockDim.x)
    for (uint32_t aa = 0; aa < a.n_ant; aa++) {
      const int32_t ar = acc[2 * aa * a.win + o], ai = acc[(2 * aa + 1) * a.win + o];
      if (ar == 0 && ai == 0) continue;
      const int32_t v = p.g[aa][o];
      p.g[aa][o] = pk16((int16_t)(lo16(v) + (int16_t)ar), (int16_t)(hi16(v) + (int16_t)ai));
    }
}

hipError_t oai4g_launch_phich(int32_t *const *d_g, int32_t *d_acc, const phich_args_t &a, hipStream_t s)
{
  if (a.n == 0) return hipSuccess;
  phich_ptrs_t p = {};
  for (uint32_t aa = 0; aa < a.n_ant && aa < 2; aa++) p.g[aa] = d_g[aa];
  hipLaunchKernelGGL(k_phich, dim3(1), dim3(256), 0, s, p, d_acc, a);
  return hipGetLastError();
}
