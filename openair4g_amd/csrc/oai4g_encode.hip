/*
 * gfx950 kernels for the bit-domain half of the PDSCH transmit path:
 *   CRC-24A/B (crc_byte.c:98-153), code-block segmentation (lte_segmentation.c:39-170),
 *   turbo encoding (3gpplte_sse.c:380-476), sub-block interleaving (lte_rate_matching.c:51-130),
 *   circular-buffer rate matching (lte_rate_matching.c:464-566) and Gold scrambling
 *   (dlsch_scrambling.c:51-97, lte_gold.c:151-177).
 *
 * Fused encoder: one 256-thread workgroup per (subframe, codeword).  Bits live in LDS as
 * LSB-first 32-bit words.  The recursive systematic convolutional encoders are linear over
 * GF(2), so each 32-bit chunk is encoded from a zero state, the chunk exit states are combined
 * with a Hillis-Steele scan over 3-bit states (x -> A^32 x), and every chunk is re-encoded
 * from its true entry state: O(K/32) parallel work instead of a K-step serial recursion.
 * The sub-block interleaver and the circular-buffer read are never materialised: every
 * output bit e[k] is traced back (k -> compacted index -> w position -> (stream, index)) and
 * read from the encoder's streams; scrambling XORs whole 32-bit Gold words produced by a
 * 64-lane jump-ahead generator (x2 state advanced by precomputed powers of its step matrix).
 * Output: packed, scrambled e bits per codeword ([n_sf][n_cw][ebits_words] words).
 */
#include "oai4g_internal.h"

/* ---------------------------------------------------------------------------------------
 * RSC trellis (3gpplte_sse.c:96-102) at nibble granularity, built at compile time.
 * state bits (s2 s1 s0), s2 newest: out = u^s2^s1, s' = ((u^s1^s0)<<2) | (s2<<1) | s1.
 * ------------------------------------------------------------------------------------- */
struct rsc_tables_t {
  uint8_t next[8][16];   /* state after 4 input bits (LSB-first nibble) */
  uint8_t par[8][16];    /* 4 parity bits, LSB-first */
  uint8_t apow[8][8];    /* zero-input propagation by 32*2^d steps: apow[d][s] */
};

static constexpr uint8_t rsc_step_c(uint8_t u, uint8_t s, uint8_t *out)
{
  *out = (uint8_t)((u ^ (s >> 2) ^ (s >> 1)) & 1);
  return (uint8_t)((((u << 2) ^ (s >> 1)) ^ ((s >> 1) << 2) ^ (s << 2)) & 7);
}

static constexpr rsc_tables_t make_rsc_tables()
{
  rsc_tables_t t{};
  for (int s = 0; s < 8; s++)
    for (int nib = 0; nib < 16; nib++) {
      uint8_t st = (uint8_t)s, p = 0;
      for (int b = 0; b < 4; b++) {
        uint8_t o = 0;
        st = rsc_step_c((uint8_t)((nib >> b) & 1), st, &o);
        p |= (uint8_t)(o << b);
      }
      t.next[s][nib] = st;
      t.par[s][nib] = p;
    }
  for (int d = 0; d < 8; d++)
    for (int s = 0; s < 8; s++) {
      uint8_t st = (uint8_t)s;
      for (int n = 0; n < (32 << d); n++) {
        uint8_t o = 0;
        st = rsc_step_c(0, st, &o);
      }
      t.apow[d][s] = st;
    }
  return t;
}

__constant__ rsc_tables_t c_rsc = make_rsc_tables();

static __constant__ uint8_t c_colperm[32] = {0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30,
                                             1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31};

static __device__ __forceinline__ uint32_t lsw(uint32_t w) { return w + (w >> 5); } /* stream word swizzle */

/* 4 MSB-first bytes (little-endian word) -> 32 bits LSB-first in sequence order */
static __device__ __forceinline__ uint32_t bytes_to_seq(uint32_t le) { return __builtin_bswap32(__builtin_bitreverse32(le)); }

/* ---------------------------------------------------------------------------------------
 * CRC-24 helpers: 24-bit register, MSB-first, zero init (reference returns reg << 8).
 * ------------------------------------------------------------------------------------- */
static __device__ __forceinline__ uint32_t crc_mulmod(uint32_t a, uint32_t b, uint32_t poly)
{
  uint32_t r = 0;
  for (int i = 23; i >= 0; i--) {
    r <<= 1;
    if (r & 0x1000000u) r ^= 0x1000000u | poly;
    if ((b >> i) & 1u) r ^= a;
  }
  return r;
}

/* x^(8n) mod P by square-and-multiply on x^8 */
static __device__ __forceinline__ uint32_t crc_xpow8(uint32_t n, uint32_t poly)
{
  uint32_t result = 1, base = 0x100;   /* x^8 (degree < 24) */
  while (n) {
    if (n & 1u) result = crc_mulmod(result, base, poly);
    base = crc_mulmod(base, base, poly);
    n >>= 1;
  }
  return result;
}

/* Workgroup-cooperative CRC of buf[0..nbytes) (LDS bytes).  tab: 256-entry LDS table of the
 * 24-bit byte remainders.  Returns the 24-bit CRC in every thread.  red: >= 8 LDS words. */
static __device__ uint32_t crc24_block(const uint8_t *buf, uint32_t nbytes, uint32_t poly, const uint32_t *tab,
                                       uint32_t *red)
{
  const uint32_t tid = threadIdx.x, nth = blockDim.x;
  uint32_t per = (nbytes + nth - 1) / nth;
  uint32_t start = tid * per, end = min(start + per, nbytes);
  uint32_t reg = 0;
  for (uint32_t i = start; i < end; i++) reg = ((reg << 8) ^ tab[((reg >> 16) ^ buf[i]) & 0xffu]) & 0xffffffu;
  if (start < nbytes && end < nbytes && reg) reg = crc_mulmod(reg, crc_xpow8(nbytes - end, poly), poly);
  if (start >= nbytes) reg = 0;
  /* xor-reduce: wave, then across waves */
  for (int off = 32; off > 0; off >>= 1) reg ^= __shfl_xor(reg, off, 64);
  __syncthreads();
  if ((tid & 63) == 0) red[tid >> 6] = reg;
  __syncthreads();
  uint32_t tot = 0;
  for (uint32_t wv = 0; wv < (nth + 63) / 64; wv++) tot ^= red[wv];
  __syncthreads();
  return tot;
}

static __device__ void crc_table_init(uint32_t *tab, uint32_t poly)
{
  for (uint32_t v = threadIdx.x; v < 256; v += blockDim.x) {
    uint32_t r = v << 16;
    for (int i = 0; i < 8; i++) r = (r & 0x800000u) ? ((r << 1) ^ poly) & 0xffffffu : (r << 1) & 0xffffffu;
    tab[v] = r;
  }
}

/* ---------------------------------------------------------------------------------------
 * Gold sequence jump-ahead (lte_gold.c:151-177): word w = X1(50+w) ^ X2(50+w).
 * Lane l < 64 generates words [64l, 64l+64).
 * ------------------------------------------------------------------------------------- */
static __device__ __forceinline__ void gold_step(uint32_t &x1, uint32_t &x2)
{
  x1 = (x1 >> 1) ^ (x1 >> 4);
  x1 = x1 ^ (x1 << 31) ^ (x1 << 28);
  x2 = (x2 >> 1) ^ (x2 >> 2) ^ (x2 >> 3) ^ (x2 >> 4);
  x2 = x2 ^ (x2 << 31) ^ (x2 << 30) ^ (x2 << 29) ^ (x2 << 28);
}

static __device__ void gold_generate(uint32_t *gold, uint32_t nwords, uint32_t c_init, const uint32_t *gx1,
                                     const uint32_t *gx2j)
{
  uint32_t l = threadIdx.x;
  if (l >= 64 || 64 * l >= nwords) return;
  uint32_t x2i = c_init ^ ((c_init ^ (c_init >> 1) ^ (c_init >> 2) ^ (c_init >> 3)) << 31);
  uint32_t x2 = 0;
  const uint32_t *col = gx2j + 32 * l;
  for (int b = 0; b < 32; b++)
    if ((x2i >> b) & 1u) x2 ^= col[b];
  uint32_t x1 = gx1[l];
  uint32_t w0 = 64 * l, wend = min(w0 + 64, nwords);
  gold[w0] = x1 ^ x2;
  for (uint32_t w = w0 + 1; w < wend; w++) {
    gold_step(x1, x2);
    gold[w] = x1 ^ x2;
  }
}

/* ---------------------------------------------------------------------------------------
 * Turbo encoding of all code blocks of a codeword held in LDS.
 * streams: per block r, 3 streams (sys, p1, p2) of sw words each (swizzled), at
 * strm + r*3*sw.  tails: 2 words per block (6 tail bits per constituent encoder).
 * scan: 1 byte per (block, encoder, chunk).
 * ------------------------------------------------------------------------------------- */
struct cb_geom_t {
  uint32_t C;
  uint32_t sw;              /* stream words per block (swizzled, padded) */
  uint32_t K[OAI4G_MAX_CB];
  uint32_t f1[OAI4G_MAX_CB], f2[OAI4G_MAX_CB];
};

/* input word of chunk j for encoder e (0: systematic, 1: QPP-interleaved systematic) */
static __device__ __forceinline__ uint32_t enc_input(const uint32_t *sys, uint32_t K, uint32_t f1, uint32_t f2,
                                                     uint32_t j, int e)
{
  if (e == 0) return sys[lsw(j)];
  uint32_t k = 32 * j;
  uint32_t n = min(32u, K - k);
  uint64_t kk = k;
  uint32_t pi = (uint32_t)((f1 * kk + (uint64_t)f2 * kk * kk) % K);
  uint32_t dl = (uint32_t)((f1 + (uint64_t)f2 * (2 * kk + 1)) % K);
  uint32_t d2 = (2u * f2) % K;
  uint32_t word = 0;
  for (uint32_t b = 0; b < n; b++) {
    word |= ((sys[lsw(pi >> 5)] >> (pi & 31)) & 1u) << b;
    pi += dl;
    if (pi >= K) pi -= K;
    dl += d2;
    if (dl >= K) dl -= K;
  }
  return word;
}

static __device__ void turbo_encode_blocks(uint32_t *strm, uint32_t *tails, uint8_t *scan, const cb_geom_t &g)
{
  const uint32_t tid = threadIdx.x, nth = blockDim.x;
  /* flattened item list: for r, e, j ; per-(r,e) offsets */
  uint32_t nitems = 0;
  uint32_t base[OAI4G_MAX_CB];
  for (uint32_t r = 0; r < g.C; r++) {
    base[r] = nitems;
    nitems += 2 * ((g.K[r] + 31) >> 5);
  }
  /* pass 1: zero-start exit state of every chunk */
  for (uint32_t it = tid; it < nitems; it += nth) {
    uint32_t r = 0;
    while (r + 1 < g.C && it >= base[r + 1]) r++;
    uint32_t nch = (g.K[r] + 31) >> 5, loc = it - base[r];
    int e = loc >= nch;
    uint32_t j = e ? loc - nch : loc;
    const uint32_t *sys = strm + r * 3 * g.sw;
    uint32_t u = enc_input(sys, g.K[r], g.f1[r], g.f2[r], j, e);
    uint32_t nnib = min(32u, g.K[r] - 32 * j) >> 2;
    uint8_t s = 0;
    for (uint32_t q = 0; q < nnib; q++) s = c_rsc.next[s][(u >> (4 * q)) & 15u];
    scan[it] = s;
  }
  __syncthreads();
  /* pass 2: segmented inclusive scan v[j] ^= A^(32*2^d) v[j-2^d] */
  for (int d = 0; d < 8; d++) {
    uint32_t span = 1u << d;
    uint8_t tmp[24];
    int cnt = 0;
    for (uint32_t it = tid; it < nitems; it += nth, cnt++) {
      uint32_t r = 0;
      while (r + 1 < g.C && it >= base[r + 1]) r++;
      uint32_t nch = (g.K[r] + 31) >> 5, loc = it - base[r];
      uint32_t j = loc >= nch ? loc - nch : loc;
      uint8_t v = scan[it];
      if (j >= span) v ^= c_rsc.apow[d][scan[it - span]];
      if (cnt < 24) tmp[cnt] = v;
    }
    __syncthreads();
    cnt = 0;
    for (uint32_t it = tid; it < nitems; it += nth, cnt++)
      if (cnt < 24) scan[it] = tmp[cnt];
    __syncthreads();
  }
  /* pass 3: re-encode each chunk from its entry state -> parity words, tails */
  for (uint32_t it = tid; it < nitems; it += nth) {
    uint32_t r = 0;
    while (r + 1 < g.C && it >= base[r + 1]) r++;
    uint32_t nch = (g.K[r] + 31) >> 5, loc = it - base[r];
    int e = loc >= nch;
    uint32_t j = e ? loc - nch : loc;
    uint32_t *sys = strm + r * 3 * g.sw;
    uint32_t u = enc_input(sys, g.K[r], g.f1[r], g.f2[r], j, e);
    uint8_t s = j ? scan[it - 1] : 0;
    uint32_t nnib = min(32u, g.K[r] - 32 * j) >> 2, par = 0;
    for (uint32_t q = 0; q < nnib; q++) {
      uint32_t nib = (u >> (4 * q)) & 15u;
      par |= (uint32_t)c_rsc.par[s][nib] << (4 * q);
      s = c_rsc.next[s][nib];
    }
    sys[(1 + e) * g.sw + lsw(j)] = par;
    if (j == nch - 1) {
      /* trellis termination (3gpplte_sse.c:104-109, 440-471): bits x,z per step */
      uint32_t tb = 0;
      for (int stp = 0; stp < 3; stp++) {
        uint32_t z = ((s >> 2) ^ s) & 1u, x = (s ^ (s >> 1)) & 1u;
        s >>= 1;
        tb |= (x << (2 * stp)) | (z << (2 * stp + 1));
      }
      tails[2 * r + e] = tb;
    }
  }
  __syncthreads();
}

/* tail bit m (0..11) of block r: t[0..5] from encoder 1, t[6..11] from encoder 2 */
static __device__ __forceinline__ uint32_t tail_bit(const uint32_t *tails, uint32_t r, uint32_t m)
{
  return m < 6 ? (tails[2 * r] >> m) & 1u : (tails[2 * r + 1] >> (m - 6)) & 1u;
}

/* value of d^(s)_idx for block r: stream bit if idx < K, else tail (lte_rate_matching.c:75-110) */
static __device__ __forceinline__ uint32_t dstream_bit(const uint32_t *blk, uint32_t sw, const uint32_t *tails,
                                                       uint32_t r, uint32_t K, uint32_t s, uint32_t idx)
{
  if (idx < K) return (blk[s * sw + lsw(idx >> 5)] >> (idx & 31)) & 1u;
  return tail_bit(tails, r, 3 * (idx - K) + s);
}

/* walker over the sub-block interleaver output w (lte_rate_matching.c:51-130) */
struct wwalk_t {
  uint32_t p, region, col, row, which;
};

static __device__ __forceinline__ void wwalk_init(wwalk_t &w, uint32_t p, uint32_t R, uint32_t Kpi)
{
  w.p = p;
  if (p < Kpi) {
    w.region = 0; w.col = p / R; w.row = p - w.col * R; w.which = 0;
  } else {
    uint32_t q = p - Kpi;
    w.region = 1; w.col = q / (2 * R);
    uint32_t rr = q - w.col * 2 * R;
    w.row = rr >> 1; w.which = rr & 1u;
  }
}

static __device__ __forceinline__ void wwalk_next(wwalk_t &w, uint32_t R)
{
  w.p++;
  if (w.region == 0) {
    if (++w.row == R) { w.row = 0; if (++w.col == 32) { w.region = 1; w.col = 0; } }
  } else {
    w.which ^= 1u;
    if (w.which == 0 && ++w.row == R) { w.row = 0; if (++w.col == 32) { w.region = 0; w.col = 0; w.p = 0; } }
  }
}

static __device__ __forceinline__ uint32_t wwalk_bit(const wwalk_t &w, const uint32_t *blk, uint32_t sw,
                                                     const uint32_t *tails, uint32_t r, uint32_t K, uint32_t ND,
                                                     uint32_t Kpi)
{
  uint32_t j = c_colperm[w.col] + 32 * w.row;
  if (w.region == 0) return dstream_bit(blk, sw, tails, r, K, 0, j - ND);
  if (w.which == 0) return dstream_bit(blk, sw, tails, r, K, 1, j - ND);
  uint32_t j2 = (j + 1 == Kpi) ? 0 : j + 1;
  return dstream_bit(blk, sw, tails, r, K, 2, j2 - ND);
}

/* is w[p] a NULL (dummy) entry? (lte_rate_matching.c:51-130) */
static __device__ __forceinline__ bool wwalk_null(const wwalk_t &w, uint32_t R, uint32_t ND)
{
  if (w.row != 0) return (w.region == 1 && w.which == 1 && w.col == 31 && w.row == R - 1 && ND > 0);
  uint32_t cp = c_colperm[w.col];
  if (w.region == 0 || w.which == 0) return cp < ND;
  return (cp + 1 < ND) || (w.col == 31 && R == 1 && ND > 0);
}

/* position of the ci-th non-NULL entry of w (sorted NULL positions np[0..nn)) */
static __device__ __forceinline__ uint32_t compact_to_pos(uint32_t ci, const uint16_t *np, uint32_t nn, uint32_t &m)
{
  uint32_t lo = 0, hi = nn; /* m = #{i : np[i] - i <= ci} */
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if ((uint32_t)np[mid] - mid <= ci) lo = mid + 1;
    else hi = mid;
  }
  m = lo;
  return ci + lo;
}

/* ---------------------------------------------------------------------------------------
 * The fused encoder.
 * ------------------------------------------------------------------------------------- */
struct enc_lds_t {
  uint32_t *tb;     /* TB || CRC bytes */
  uint32_t *strm;
  uint32_t *gold;
  uint32_t *tails;  /* 2 per block */
  uint8_t *scan;    /* 2 * sum(K/32) bytes */
  uint32_t *crctab; /* 256 */
  uint32_t *red;    /* 8 */
  uint16_t *np;     /* 2 * OAI4G_MAX_NULLS */
};

template <bool DEBUG>
static __device__ void encode_codeword(const cfg_dev_t *__restrict__ c, uint32_t sf, uint32_t cwi,
                                       const uint8_t *__restrict__ payload, uint32_t *__restrict__ ebits,
                                       enc_debug_t dbg, uint32_t *lds_base)
{
  const cw_dev_t &cw = c->cw[cwi];
  const uint32_t tid = threadIdx.x, nth = blockDim.x;
  const uint32_t sfi = DEBUG ? sf : (c->first_sf + sf * c->sf_step) % 10;
  const uint32_t C = cw.C;
  const uint32_t sw = cw.stream_words;
  enc_lds_t L;
  L.tb = lds_base;
  L.strm = L.tb + c->lds_tb_words;
  L.gold = L.strm + c->lds_stream_words;
  L.tails = L.gold + c->lds_gold_words;
  L.crctab = L.tails + 2 * OAI4G_MAX_CB;
  L.red = L.crctab + 256;
  L.np = (uint16_t *)(L.red + 8);
  L.scan = (uint8_t *)(L.np + 2 * OAI4G_MAX_NULLS);
  uint8_t *tbb = (uint8_t *)L.tb;
  const uint32_t G = cw.G[sfi], Gw = (G + 31) >> 5;

  /* ---- phase 0: TB bytes -> LDS, Gold words, NULL lists, CRC table ---- */
  const uint8_t *src = payload + (size_t)(DEBUG ? 0 : (sf * c->n_cw + cwi)) * c->payload_stride;
  const uint32_t Ab = cw.A_bytes;
  for (uint32_t i = tid; i < c->lds_tb_words; i += nth) {
    uint32_t v = 0;
    if (4 * i < Ab) {
      v = *(const uint32_t *)(src + 4 * i);
      uint32_t valid = Ab - 4 * i;
      if (valid < 4) v &= (1u << (8 * valid)) - 1u;
    }
    L.tb[i] = v;
  }
  const uint32_t c_init = (c->rnti << 14) + (cw.q << 13) + (sfi << 9) + c->Nid_cell; /* Ns>>1 = subframe */
  gold_generate(L.gold, Gw, c_init, c->gold_x1, c->gold_x2j);
  for (uint32_t i = tid; i < 2 * OAI4G_MAX_NULLS; i += nth) L.np[i] = cw.nullpos[i / OAI4G_MAX_NULLS][i % OAI4G_MAX_NULLS];
  crc_table_init(L.crctab, 0x864cfbu);
  __syncthreads();

  /* ---- phase 1: CRC-24A (dlsch_coding.c:296-300) ---- */
  uint32_t crc = crc24_block(tbb, Ab, 0x864cfbu, L.crctab, L.red);
  if (tid == 0) {
    tbb[Ab] = (uint8_t)(crc >> 16);
    tbb[Ab + 1] = (uint8_t)(crc >> 8);
    tbb[Ab + 2] = (uint8_t)crc;
  }
  __syncthreads();
  if (DEBUG && dbg.b)
    for (uint32_t i = tid; i < Ab + 3; i += nth) dbg.b[i] = tbb[i];

  /* ---- phase 2: segmentation -> per-block systematic streams (+ CRC-24B when C > 1) ---- */
  crc_table_init(L.crctab, 0x800063u);
  __syncthreads();
  uint32_t crcb[OAI4G_MAX_CB];
  for (uint32_t r = 0; r < C; r++) {
    crcb[r] = 0;
    if (C > 1) crcb[r] = crc24_block(tbb + cw.src[r], cw.ncopy[r], 0x800063u, L.crctab, L.red);
  }
  for (uint32_t r = 0; r < C; r++) {
    uint32_t K = cw.K[r], nw = (K + 31) >> 5, fill = cw.fill[r], ncopy = cw.ncopy[r], s0 = cw.src[r];
    uint32_t *sys = L.strm + r * 3 * sw;
    for (uint32_t j = tid; j < nw; j += nth) {
      uint32_t le = 0;
      for (uint32_t q = 0; q < 4; q++) {
        uint32_t i = 4 * j + q, byte = 0;
        if (i < fill) byte = 0;
        else if (i < fill + ncopy) byte = tbb[s0 + i - fill];
        else if (C > 1 && i < fill + ncopy + 3) byte = (crcb[r] >> (8 * (2 - (i - fill - ncopy)))) & 0xffu;
        le |= byte << (8 * q);
      }
      uint32_t wv = bytes_to_seq(le);
      if (32 * (j + 1) > K) wv &= (1u << (K - 32 * j)) - 1u;
      sys[lsw(j)] = wv;
    }
  }
  __syncthreads();

  /* ---- phase 3: turbo encoding of every block ---- */
  cb_geom_t g;
  g.C = C;
  g.sw = sw;
  for (uint32_t r = 0; r < C; r++) { g.K[r] = cw.K[r]; g.f1[r] = cw.f1[r]; g.f2[r] = cw.f2[r]; }
  turbo_encode_blocks(L.strm, L.tails, L.scan, g);

  if (DEBUG) {
    /* reference-layout intermediates: c[r] bytes, d[r] (NULL prefix + 3K+12 (+side effect)), w[r] */
    for (uint32_t r = 0; r < C; r++) {
      uint32_t K = cw.K[r], R = cw.R[r], Kpi = cw.Kpi[r], ND = cw.ND[r];
      const uint32_t *blk = L.strm + r * 3 * sw;
      if (dbg.c)
        for (uint32_t i = tid; i < K / 8; i += nth) {
          uint32_t wv = blk[lsw(i >> 2)];
          uint32_t byte = (wv >> (8 * (i & 3))) & 0xffu;
          dbg.c[r * (8 + 3 + 768) + i] = (uint8_t)(__builtin_bitreverse32(byte) >> 24);
        }
      if (dbg.d) {
        uint8_t *d = dbg.d + (size_t)r * OAI4G_D_BYTES;
        for (uint32_t i = tid; i < 96; i += nth) d[i] = OAI4G_LTE_NULL;
        for (uint32_t i = tid; i < 3 * K + 12; i += nth) {
          uint32_t kk = i / 3, s = i - 3 * kk;
          d[96 + i] = (uint8_t)(kk < K ? dstream_bit(blk, sw, L.tails, r, K, s, kk) : tail_bit(L.tails, r, i - 3 * K));
        }
        /* d[3D+2] = d[2] (lte_rate_matching.c:75) */
        if (tid == 0) d[96 + 3 * (K + 4) + 2] = (uint8_t)dstream_bit(blk, sw, L.tails, r, K, 2, 0);
      }
      if (dbg.w) {
        uint8_t *w = dbg.w + (size_t)r * OAI4G_W_BYTES;
        for (uint32_t p = tid; p < 3 * Kpi; p += nth) {
          wwalk_t wk;
          wwalk_init(wk, p, R, Kpi);
          w[p] = wwalk_null(wk, R, ND) ? OAI4G_LTE_NULL : (uint8_t)wwalk_bit(wk, blk, sw, L.tails, r, K, ND, Kpi);
        }
      }
    }
  }

  if (DEBUG && !dbg.e) return;
  /* ---- phase 4: rate matching + scrambling -> packed e words ---- */
  const uint32_t *roff = cw.roff[sfi];
  uint32_t *eout = DEBUG ? nullptr : ebits + (size_t)(sf * c->n_cw + cwi) * c->ebits_words;
  for (uint32_t wi = tid; wi < Gw; wi += nth) {
    uint32_t k0 = 32 * wi;
    uint32_t r = 0;
    while (r + 1 < C && k0 >= roff[r + 1]) r++;
    uint32_t out = 0;
    uint32_t nb = min(32u, G - k0);
    uint32_t b = 0;
    while (b < nb && r < C) {
      /* walk the run of bits belonging to block r */
      uint32_t kl = k0 + b - roff[r];
      uint32_t Er = roff[r + 1] - roff[r];
      uint32_t run = min(nb - b, Er - kl);
      uint32_t K = cw.K[r], R = cw.R[r], Kpi = cw.Kpi[r], ND = cw.ND[r], Nnn = cw.Nnn[r], Ncb = cw.Ncb[r];
      const uint16_t *np = L.np + cw.kidx[r] * OAI4G_MAX_NULLS;
      uint32_t nn = cw.nnull[cw.kidx[r]];
      const uint32_t *blk = L.strm + r * 3 * sw;
      uint32_t ci = (cw.k0c[r] + kl) % Nnn, m;
      uint32_t p = compact_to_pos(ci, np, nn, m);
      wwalk_t wk;
      wwalk_init(wk, p, R, Kpi);
      for (uint32_t x = 0; x < run; x++) {
        if (x) {
          /* advance to the next non-NULL position, wrapping at Ncb */
          do {
            wwalk_next(wk, R);
            if (wk.p >= Ncb) wwalk_init(wk, 0, R, Kpi);
          } while (wwalk_null(wk, R, ND));
        }
        uint32_t bit = wwalk_bit(wk, blk, sw, L.tails, r, K, ND, Kpi);
        if (DEBUG && dbg.e) dbg.e[k0 + b + x] = (uint8_t)bit;
        out |= bit << (b + x);
      }
      (void)m;
      b += run;
      r++;
    }
    if (!DEBUG) eout[wi] = out ^ (L.gold[wi] & (nb == 32 ? 0xffffffffu : ((1u << nb) - 1u)));
  }
}

__global__ void __launch_bounds__(256) k_encode(const cfg_dev_t *__restrict__ c, const uint8_t *__restrict__ payload,
                                                uint32_t *__restrict__ ebits)
{
  extern __shared__ uint32_t lds_dyn[];
  uint32_t sf = blockIdx.x / c->n_cw, cwi = blockIdx.x % c->n_cw;
  enc_debug_t none = {nullptr, nullptr, nullptr, nullptr, nullptr};
  encode_codeword<false>(c, sf, cwi, payload, ebits, none, lds_dyn);
}

__global__ void __launch_bounds__(256) k_encode_debug(const cfg_dev_t *__restrict__ c, uint32_t sf, uint32_t cwi,
                                                      const uint8_t *__restrict__ payload, enc_debug_t dbg)
{
  extern __shared__ uint32_t lds_dyn[];
  encode_codeword<true>(c, sf, cwi, payload, nullptr, dbg, lds_dyn);
}

static size_t enc_lds_bytes(const cfg_dev_t *h)
{
  uint32_t scan_bytes = 0;
  for (int cw = 0; cw < (int)h->n_cw; cw++) {
    uint32_t s = 0;
    for (uint32_t r = 0; r < h->cw[cw].C; r++) s += 2 * ((h->cw[cw].K[r] + 31) >> 5);
    scan_bytes = s > scan_bytes ? s : scan_bytes;
  }
  size_t words = (size_t)h->lds_tb_words + h->lds_stream_words + h->lds_gold_words + 2 * OAI4G_MAX_CB + 256 + 8 +
                 OAI4G_MAX_NULLS + (scan_bytes + 3) / 4 + 4;
  return words * 4;
}

hipError_t oai4g_launch_encode(const cfg_dev_t *d_cfg, const cfg_dev_t *h_cfg, int n_sf, const uint8_t *d_payload,
                               uint32_t *d_ebits, hipStream_t s)
{
  size_t lds = enc_lds_bytes(h_cfg);
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void *)k_encode, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void *)k_encode_debug, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  hipLaunchKernelGGL(k_encode, dim3(n_sf * h_cfg->n_cw), dim3(256), lds, s, d_cfg, d_payload, d_ebits);
  return hipGetLastError();
}

hipError_t oai4g_launch_encode_debug(const cfg_dev_t *d_cfg, const cfg_dev_t *h_cfg, int cw, int sf,
                                     const uint8_t *d_payload, enc_debug_t dbg, hipStream_t s)
{
  size_t lds = enc_lds_bytes(h_cfg);
  hipFuncSetAttribute((const void *)k_encode_debug, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipLaunchKernelGGL(k_encode_debug, dim3(1), dim3(256), lds, s, d_cfg, (uint32_t)sf, (uint32_t)cw, d_payload, dbg);
  return hipGetLastError();
}

/* =======================================================================================
 * Drop-in byte-layout kernels
 * ===================================================================================== */

/* crc24a/crc24b over an arbitrary bit length (crc_byte.c:117-153), one workgroup */
__global__ void __launch_bounds__(256) k_crc24(const uint8_t *__restrict__ in, int bitlen, uint32_t poly,
                                               uint32_t *__restrict__ out)
{
  __shared__ uint32_t tab[256];
  __shared__ uint32_t red[8];
  extern __shared__ uint8_t buf[];
  uint32_t nbytes = (uint32_t)bitlen / 8, rem = (uint32_t)bitlen % 8;
  for (uint32_t i = threadIdx.x; i < nbytes + (rem ? 1 : 0); i += blockDim.x) buf[i] = in[i];
  crc_table_init(tab, poly);
  __syncthreads();
  uint32_t reg = crc24_block(buf, nbytes, poly, tab, red);
  if (threadIdx.x == 0) {
    if (rem) {
      /* crc = (crc << rem) ^ T[(byte >> (8-rem)) ^ (crc >> (32-rem))] on the <<8 register */
      uint32_t r32 = reg << 8;
      uint32_t idx = ((uint32_t)buf[nbytes] >> (8 - rem)) ^ (r32 >> (32 - rem));
      r32 = (r32 << rem) ^ (tab[idx & 0xffu] << 8);
      out[0] = r32;
    } else {
      out[0] = reg << 8;
    }
  }
}

hipError_t oai4g_launch_crc24(const uint8_t *d_in, int bitlen, uint32_t poly_top, uint32_t *d_out, hipStream_t s)
{
  uint32_t nbytes = (uint32_t)(bitlen + 7) / 8;
  hipLaunchKernelGGL(k_crc24, dim3(1), dim3(256), nbytes + 4, s, d_in, bitlen, poly_top >> 8, d_out);
  return hipGetLastError();
}

/* threegpplte_turbo_encoder: c bytes -> d bytes (3K+12), one workgroup */
__global__ void __launch_bounds__(256) k_turbo_bytes(const uint8_t *__restrict__ cin, uint32_t K, uint32_t f1,
                                                     uint32_t f2, uint8_t *__restrict__ dout)
{
  __shared__ uint32_t strm[3 * 200];
  __shared__ uint32_t tails[2];
  __shared__ uint8_t scan[2 * 192];
  const uint32_t sw = 200;
  uint32_t nw = (K + 31) >> 5;
  for (uint32_t j = threadIdx.x; j < nw; j += blockDim.x) {
    uint32_t le = 0;
    for (uint32_t q = 0; q < 4; q++) {
      uint32_t i = 4 * j + q;
      le |= (uint32_t)(i < K / 8 ? cin[i] : 0) << (8 * q);
    }
    uint32_t wv = bytes_to_seq(le);
    if (32 * (j + 1) > K) wv &= (1u << (K - 32 * j)) - 1u;
    strm[lsw(j)] = wv;
  }
  __syncthreads();
  cb_geom_t g;
  g.C = 1;
  g.sw = sw;
  g.K[0] = K;
  g.f1[0] = f1;
  g.f2[0] = f2;
  turbo_encode_blocks(strm, tails, scan, g);
  for (uint32_t i = threadIdx.x; i < 3 * K + 12; i += blockDim.x) {
    uint32_t kk = i / 3, s = i - 3 * kk;
    dout[i] = (uint8_t)(kk < K ? dstream_bit(strm, sw, tails, 0, K, s, kk) : tail_bit(tails, 0, i - 3 * K));
  }
}

hipError_t oai4g_launch_turbo_bytes(const uint8_t *d_c, int nbytes, uint8_t *d_out, uint32_t f1, uint32_t f2,
                                    hipStream_t s)
{
  hipLaunchKernelGGL(k_turbo_bytes, dim3(1), dim3(256), 0, s, d_c, (uint32_t)nbytes * 8, f1, f2, d_out);
  return hipGetLastError();
}

/* sub_block_interleaving_turbo on caller bytes.  dfull points at the buffer start: d = dfull+96. */
__global__ void __launch_bounds__(256) k_subblock_bytes(uint32_t D, const uint8_t *__restrict__ dfull,
                                                        uint8_t *__restrict__ w)
{
  uint32_t R = (D + 31) >> 5, Kpi = R << 5, ND = Kpi - D;
  const uint8_t *base = dfull + 96 - 3 * ND;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < Kpi; k += gridDim.x * blockDim.x) {
    uint32_t col = k / R, row = k - col * R;
    uint32_t j = c_colperm[col] + 32 * row;
    w[k] = base[3 * j];
    w[Kpi + 2 * k] = base[3 * j + 1];
    /* base[3j+5] with the d[3D+2] = d[2] alias (lte_rate_matching.c:75) */
    uint32_t i5 = 3 * j + 5;
    w[Kpi + 2 * k + 1] = (i5 == 3 * Kpi + 2) ? dfull[96 + 2] : base[i5];
    if (ND > 0 && k == Kpi - 1) w[3 * Kpi - 1] = OAI4G_LTE_NULL;
  }
}

hipError_t oai4g_launch_subblock_bytes(uint32_t D, const uint8_t *d_dfull, uint8_t *d_w, hipStream_t s)
{
  hipLaunchKernelGGL(k_subblock_bytes, dim3(32), dim3(256), 0, s, D, d_dfull, d_w);
  return hipGetLastError();
}

/* lte_rate_matching_turbo on caller bytes: compaction of the non-NULL entries of w[0..Ncb)
 * (block-wide prefix count), then e[k] = compact[(start + k) mod nnz].  One workgroup. */
__global__ void __launch_bounds__(256) k_rm_bytes(const uint8_t *__restrict__ w, uint32_t Ncb, uint32_t k0,
                                                   uint32_t E, uint8_t *__restrict__ e, uint32_t *status)
{
  extern __shared__ uint8_t comp[];
  __shared__ uint32_t wsum[4];
  __shared__ uint32_t s_start, s_total;
  const uint32_t tid = threadIdx.x, nth = blockDim.x;
  uint32_t per = (Ncb + nth - 1) / nth, a = tid * per, b = min(a + per, Ncb);
  uint32_t cnt = 0, before_k0 = 0;
  for (uint32_t i = a; i < b; i++)
    if (w[i] != OAI4G_LTE_NULL) { cnt++; if (i < k0) before_k0++; }
  /* exclusive scan of cnt over threads (wave shuffles + LDS) */
  uint32_t lane = tid & 63, wv = tid >> 6, incl = cnt;
  for (int off = 1; off < 64; off <<= 1) {
    uint32_t v = __shfl_up(incl, off, 64);
    if (lane >= (uint32_t)off) incl += v;
  }
  if (lane == 63) wsum[wv] = incl;
  if (tid == 0) { s_start = 0; s_total = 0; }
  __syncthreads();
  uint32_t wbase = 0;
  for (uint32_t i = 0; i < wv; i++) wbase += wsum[i];
  uint32_t excl = wbase + incl - cnt;
  uint32_t o = excl;
  for (uint32_t i = a; i < b; i++)
    if (w[i] != OAI4G_LTE_NULL) comp[o++] = w[i];
  atomicAdd(&s_start, before_k0);
  atomicAdd(&s_total, cnt);
  __syncthreads();
  uint32_t nnz = s_total, st = s_start;
  if (nnz == 0) { if (tid == 0) status[0] = 1; return; }
  for (uint32_t k = tid; k < E; k += nth) e[k] = comp[(st + k) % nnz];
  if (tid == 0) status[0] = 0;
}

hipError_t oai4g_launch_rm_bytes(const uint8_t *d_w, uint32_t Ncb, uint32_t k0, uint32_t E, uint8_t *d_e,
                                 uint32_t *d_status, hipStream_t s)
{
  hipLaunchKernelGGL(k_rm_bytes, dim3(1), dim3(256), (Ncb + 15) & ~15u, s, d_w, Ncb, k0, E, d_e, d_status);
  return hipGetLastError();
}

/* dlsch_scrambling on bytes, in place, (1 + G/32)*32 entries (dlsch_scrambling.c:83-92) */
__global__ void __launch_bounds__(256) k_scramble_bytes(uint8_t *__restrict__ e, uint32_t n_entries, uint32_t c_init,
                                                        const uint32_t *__restrict__ gx1,
                                                        const uint32_t *__restrict__ gx2j)
{
  extern __shared__ uint32_t gold[];
  uint32_t nwords = (n_entries + 31) >> 5;
  gold_generate(gold, nwords, c_init, gx1, gx2j);
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < n_entries; k += blockDim.x)
    e[k] = (uint8_t)((e[k] & 1u) ^ ((gold[k >> 5] >> (k & 31)) & 1u));
}

hipError_t oai4g_launch_scramble_bytes(uint8_t *d_e, int n_entries, uint32_t c_init, const uint32_t *d_gold_x1,
                                       const uint32_t *d_gold_x2j, hipStream_t s)
{
  uint32_t nwords = ((uint32_t)n_entries + 31) >> 5;
  if (nwords > OAI4G_MAX_GOLD_WORDS) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_scramble_bytes, dim3(1), dim3(256), nwords * 4, s, d_e, (uint32_t)n_entries, c_init,
                     d_gold_x1, d_gold_x2j);
  return hipGetLastError();
}

/* deterministic payload: byte i = low byte of splitmix64(seed + i/8) >> (8*(i%8)) */
__global__ void k_fill(uint8_t *__restrict__ d, size_t bytes, uint64_t seed)
{
  size_t nw = bytes / 8;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < (bytes + 7) / 8; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + 0x9e3779b97f4a7c15ull * (i + 1);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    z ^= z >> 31;
    if (i < nw) ((uint64_t *)d)[i] = z;
    else
      for (size_t b = 0; b < bytes - 8 * i; b++) d[8 * i + b] = (uint8_t)(z >> (8 * b));
  }
}

hipError_t oai4g_launch_fill(uint8_t *d, size_t bytes, uint64_t seed, hipStream_t s)
{
  hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, s, d, bytes, seed);
  return hipGetLastError();
}
