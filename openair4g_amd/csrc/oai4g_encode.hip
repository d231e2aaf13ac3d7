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
  /* The RSC is linear and time-invariant over GF(2).  For a 32-bit input chunk u and
   * entry state s:  parity = clmul_lo(u, hz) ^ zs[s],  exit = apow[0][s] ^ F(u) with
   * F(u)_i = parity(u & fm[i]). */
  uint32_t hz;           /* impulse response of the parity output (32 steps) */
  uint32_t zs[8];        /* zero-input parity response from state s */
  uint32_t fm[3];        /* input -> exit-state masks */
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
  for (int s = 0; s < 8; s++) {
    uint8_t st = (uint8_t)s;
    uint32_t z = 0;
    for (int k = 0; k < 32; k++) {
      uint8_t o = 0;
      st = rsc_step_c(k == 0 && s == 0 ? 1 : 0, st, &o);
      z |= (uint32_t)o << k;
    }
    if (s == 0) t.hz = z; /* input = impulse at k = 0 from the zero state */
    uint8_t st2 = (uint8_t)s;
    uint32_t z2 = 0;
    for (int k = 0; k < 32; k++) {
      uint8_t o = 0;
      st2 = rsc_step_c(0, st2, &o);
      z2 |= (uint32_t)o << k;
    }
    t.zs[s] = z2;
  }
  for (int k = 0; k < 32; k++) {
    uint8_t st = 0;
    for (int n = 0; n < 32; n++) {
      uint8_t o = 0;
      st = rsc_step_c(n == k ? 1 : 0, st, &o);
    }
    for (int i = 0; i < 3; i++)
      if ((st >> i) & 1) t.fm[i] |= 1u << k;
  }
  return t;
}

static constexpr rsc_tables_t k_rsc = make_rsc_tables();

/* truncated carry-less product u * hz.  hz = g / f over GF(2)[D] mod D^32 with the feedback
 * f = 1 + D^2 + D^3 and the parity taps g = 1 + D + D^3; f divides 1 + D^7, so
 * 1 / f = (1 + D^2 + D^3 + D^4)(1 + D^7 + D^14 + D^21 + D^28) mod D^32 and the product takes
 * 13 shift / xor steps instead of one per tap of hz (20) */
/* v = u / f mod D^32: the feedback register's input sequence from the zero state, so bit k of v is
 * the newest state bit after step k and the zero-start exit state (s2 s1 s0) = (v31 v30 v29) = v >> 29 */
static __device__ __forceinline__ uint32_t rsc_feedback_word(uint32_t u)
{
  const uint32_t x = u ^ (u << 2) ^ (u << 3) ^ (u << 4);
  uint32_t y = x ^ (x << 7);
  y ^= y << 14;
  return y ^ (x << 28);
}
/* zero-start parity word = v g */
static __device__ __forceinline__ uint32_t rsc_parity_of_feedback(uint32_t v) { return v ^ (v << 1) ^ (v << 3); }
[[maybe_unused]] static __device__ __forceinline__ uint32_t rsc_parity_word(uint32_t u)
{
  static_assert(k_rsc.hz == 0xe9d3a74fu, "RSC impulse response");
  return rsc_parity_of_feedback(rsc_feedback_word(u));
}

[[maybe_unused]] static __device__ __forceinline__ uint32_t rsc_exit_input(uint32_t u)
{
  return (__builtin_popcount(u & k_rsc.fm[0]) & 1u) | ((__builtin_popcount(u & k_rsc.fm[1]) & 1u) << 1) |
         ((__builtin_popcount(u & k_rsc.fm[2]) & 1u) << 2);
}

__constant__ rsc_tables_t c_rsc = k_rsc;



/* 4 MSB-first bytes (little-endian word) -> 32 bits LSB-first in sequence order */
static __device__ __forceinline__ uint32_t bytes_to_seq(uint32_t le) { return __builtin_bswap32(__builtin_bitreverse32(le)); }

/* CRC byte table: tab[v] = v * x^24 mod P (24-bit register form of crc_byte.c:98-105) */
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

typedef const __attribute__((address_space(1))) uint32_t gu32_t;

/* Gold words 0..nwords-1 (word w = state after 50+w steps): lane l jumps to word S l with the
 * host's M^(50+S l) tables and steps S = OAI4G_GOLD_STRIDE words.  Needs blockDim.x ==
 * OAI4G_GOLD_LANES. */
[[maybe_unused]] static __device__ __forceinline__ void gold_generate(uint32_t *gold, uint32_t nwords, uint32_t c_init,
                                                     const uint32_t *gx1, const uint32_t *gx2j)
{
  const uint32_t l = threadIdx.x, w0 = OAI4G_GOLD_STRIDE * l;
  if (l >= OAI4G_GOLD_LANES || w0 >= nwords) return;
  const uint32_t x2i = c_init ^ ((c_init ^ (c_init >> 1) ^ (c_init >> 2) ^ (c_init >> 3)) << 31);
  gu32_t *col = (gu32_t *)(gx2j + l);            /* column b of lane l at [b][lane] */
  uint32_t cv[32];
#pragma unroll
  for (int b = 0; b < 32; b++) cv[b] = col[OAI4G_GOLD_LANES * b];
  uint32_t x2 = 0;
#pragma unroll
  for (int b = 0; b < 32; b++) x2 ^= cv[b] & (0u - ((x2i >> b) & 1u));
  uint32_t x1 = *(gu32_t *)(gx1 + l);
  const uint32_t wend = min(w0 + OAI4G_GOLD_STRIDE, nwords);
  gold[w0] = x1 ^ x2;
  for (uint32_t w = w0 + 1; w < wend; w++) {
    gold_step(x1, x2);
    gold[w] = x1 ^ x2;
  }
}

/* ---------------------------------------------------------------------------------------
 * CRC-24 (crc_byte.c:98-153 restated for wavefronts).  The message is virtually
 * front-padded with zero bytes (which leave a zero-initialised register unchanged) so that
 * every lane hashes exactly `per` bytes; lanes are then combined pairwise up a tree:
 * crc(L||R) = crc(L) * x^(8|R|) ^ crc(R) mod P.  The constant multipliers of every tree
 * level come from the host as nibble tables, so a combine is 6 independent LDS lookups.
 * ------------------------------------------------------------------------------------- */
static __device__ __forceinline__ uint32_t crc_step(uint32_t reg, uint32_t byte, const uint32_t *tab)
{
  return ((reg << 8) & 0xffffffu) ^ tab[((reg >> 16) ^ byte) & 0xffu];
}

static __device__ __forceinline__ uint32_t crc_mul_tab(uint32_t a, const uint32_t *t /* [6][16] */)
{
  return t[a & 15u] ^ t[16 + ((a >> 4) & 15u)] ^ t[32 + ((a >> 8) & 15u)] ^ t[48 + ((a >> 12) & 15u)] ^
         t[64 + ((a >> 16) & 15u)] ^ t[80 + ((a >> 20) & 15u)];
}

/* lane chunk CRC of virtual bytes [lane*per, (lane+1)*per) of a message padded to nl*per
 * (per % 4 == 0): four byte reads are issued ahead of their four dependent table steps; the
 * virtual zero bytes in front leave the zero register unchanged */
static __device__ __forceinline__ uint32_t crc_chunk(const uint8_t *buf, uint32_t nbytes, uint32_t per, uint32_t lane,
                                                     uint32_t nl, const uint32_t *tab)
{
  const int vstart = (int)(lane * per) - (int)(per * nl - nbytes);
  uint32_t reg = 0;
  for (uint32_t i = 0; i < per; i += 4) {
    uint32_t b[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int idx = vstart + (int)i + q;
      b[q] = idx >= 0 ? (uint32_t)buf[idx] : 0u;
    }
#pragma unroll
    for (int q = 0; q < 4; q++) reg = crc_step(reg, b[q], tab);
  }
  return reg;
}

/* lane chunk CRC over 4-byte words: bytes [lane per, (lane + 1) per) of the message base8 + start
 * of nbytes bytes, virtually front-padded to nl per bytes (per % 4 == 0; the zero bytes in front
 * leave the zero register unchanged), one unaligned word read per 4 bytes.  The register is kept
 * in the top 24 bits (tab8[v] = crc_byte.c's table entry << 8), so a byte step is
 * reg = (reg << 8) ^ tab8[(reg >> 24) ^ byte]. */
static __device__ __forceinline__ uint32_t crc_chunk_w(const uint32_t *base32, uint32_t start, uint32_t nbytes,
                                                       uint32_t per, uint32_t lane, uint32_t nl, const uint32_t *tab8)
{
  const int vstart = (int)(lane * per) - (int)(per * nl - nbytes);
  uint32_t reg = 0;
  for (uint32_t i = 0; i < per; i += 4) {
    const int o = vstart + (int)i;
    const uint32_t a = start + (uint32_t)(o > 0 ? o : 0), wi = a >> 2;
    uint32_t w = __builtin_amdgcn_alignbit(base32[wi + 1], base32[wi], (a & 3u) * 8u);
    if (o < 0) w = o <= -4 ? 0u : w << (8 * (uint32_t)(-o));   /* bytes before the message are zero */
    reg = (reg << 8) ^ tab8[(reg >> 24) ^ (w & 0xffu)];
    reg = (reg << 8) ^ tab8[(reg >> 24) ^ ((w >> 8) & 0xffu)];
    reg = (reg << 8) ^ tab8[(reg >> 24) ^ ((w >> 16) & 0xffu)];
    reg = (reg << 8) ^ tab8[(reg >> 24) ^ (w >> 24)];
  }
  return reg >> 8;
}

/* crc_chunk_w for both generator polynomials at once (two independent table chains over the same
 * word reads: ra over P_A, rb over P_B), in reflected form: with r = bitrev32(reg) the MSB-first step
 * reg' = (reg << 8) ^ T8[(reg >> 24) ^ b] becomes r' = (r >> 8) ^ R[(r ^ bitrev8(b)) & 0xff],
 * R[x] = bitrev32(T8[bitrev8(x)]).  Registers and tables are kept shifted left by 2 (r2 = r << 2,
 * R2 = R << 2), so (r2 ^ x2) & 0x3fc is the entry's byte offset (one bitop3; bits 0-1 of r2 pick up
 * bits that the next mask and shift drop): a byte step is bitop3, base add, ds_read, shift, xor --
 * four fast VALU ops against five (two of them slow: lshl, lshl_add) in crc_chunk_w's form.  Bytes of a
 * word enter in order: bitrev32 puts byte q reversed at bits 31-8q..24-8q. */
static __device__ __forceinline__ void crc_chunk_w2r(const uint32_t *base32, uint32_t start, uint32_t nbytes,
                                                     uint32_t per, uint32_t pos, uint32_t nl, const uint8_t *r2a,
                                                     const uint8_t *r2b, uint32_t &ra, uint32_t &rb)
{
  const int vstart = (int)(pos * per) - (int)(per * nl - nbytes);
  uint32_t a = 0, b = 0;
  for (uint32_t i = 0; i < per; i += 4) {
    const int o = vstart + (int)i;
    const uint32_t ad = start + (uint32_t)(o > 0 ? o : 0), wi = ad >> 2;
    uint32_t w = __builtin_amdgcn_alignbit(base32[wi + 1], base32[wi], (ad & 3u) * 8u);
    if (o < 0) w = o <= -4 ? 0u : w << (8 * (uint32_t)(-o));   /* bytes before the block are zero */
    const uint32_t wr = __builtin_bitreverse32(w);
    const uint32_t x[4] = {wr >> 22, wr >> 14, wr >> 6, wr << 2};
#pragma unroll
    for (int q = 0; q < 4; q++) {
      a = (a >> 8) ^ *(const uint32_t *)(r2a + ((a ^ x[q]) & 0x3fcu));
      b = (b >> 8) ^ *(const uint32_t *)(r2b + ((b ^ x[q]) & 0x3fcu));
    }
  }
  ra = __builtin_bitreverse32(a >> 2) >> 8;
  rb = __builtin_bitreverse32(b >> 2) >> 8;
}

/* crc_wave_tree2 over aligned groups of lpb lanes (16, 32 or 64; pos = lane within the group), both
 * polynomials; the results are in every lane of the group */
static __device__ __forceinline__ void crc_group_tree2(uint32_t &ra, uint32_t &rb, uint32_t pos, uint32_t lpb,
                                                       const uint32_t (*ma)[8][96], const uint32_t (*mb)[8][96])
{
  const uint32_t j0 = 7 - (pos & 7), j1 = (lpb >> 3) - 1 - (pos >> 3);
  ra = crc_mul_tab(ra, ma[0][j0]);
  rb = crc_mul_tab(rb, mb[0][j0]);
#pragma unroll
  for (int m = 1; m < 8; m <<= 1) {
    ra ^= __shfl_xor(ra, m, 64);
    rb ^= __shfl_xor(rb, m, 64);
  }
  ra = crc_mul_tab(ra, ma[1][j1]);
  rb = crc_mul_tab(rb, mb[1][j1]);
  for (uint32_t m = 8; m < lpb; m <<= 1) {
    ra ^= __shfl_xor(ra, (int)m, 64);
    rb ^= __shfl_xor(rb, (int)m, 64);
  }
}

/* 6-level in-wave tree; mul = [6][6][16] tables; result valid in lane 0 */
[[maybe_unused]] static __device__ __forceinline__ uint32_t crc_wave_tree(uint32_t reg, const uint32_t *mul)
{
  const uint32_t lane = threadIdx.x & 63;
  for (int d = 0; d < 6; d++) {
    uint32_t other = __shfl_down(reg, 1u << d, 64);
    if ((lane & ((2u << d) - 1u)) == 0) reg = crc_mul_tab(reg, mul + d * 96) ^ other;
  }
  return reg;
}

/* two-level in-wave combine (cw_dev_t crc2_*): every lane multiplies once by its position in its
 * group of 8, the groups XOR-reduce, the group sums multiply by the group's position, the wave
 * XOR-reduces; the result is in every lane.  Multiplier tables read from global memory (L1 / L2). */
static __device__ __forceinline__ uint32_t crc_wave_tree2(uint32_t reg, const uint32_t (*mul)[8][96])
{
  const uint32_t lane = threadIdx.x & 63;
  reg = crc_mul_tab(reg, mul[0][7 - (lane & 7)]);
  reg ^= __shfl_xor(reg, 1, 64);
  reg ^= __shfl_xor(reg, 2, 64);
  reg ^= __shfl_xor(reg, 4, 64);
  reg = crc_mul_tab(reg, mul[1][7 - (lane >> 3)]);
  reg ^= __shfl_xor(reg, 8, 64);
  reg ^= __shfl_xor(reg, 16, 64);
  reg ^= __shfl_xor(reg, 32, 64);
  return reg;
}

/* generic one-wave CRC (drop-in path): multipliers computed on the fly */
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

static __device__ uint32_t crc24_wave(const uint8_t *buf, uint32_t nbytes, uint32_t poly, const uint32_t *tab)
{
  const uint32_t lane = threadIdx.x & 63;
  uint32_t per = (((nbytes + 63) >> 6) + 3) & ~3u;   /* crc_chunk wants a multiple of 4 */
  if (nbytes == 0) return 0;
  uint32_t reg = crc_chunk(buf, nbytes, per, lane, 64, tab);
  uint32_t m = 1;
  for (uint32_t i = 0; i < per; i++) m = crc_step(m, 0, tab);   /* x^(8 per) mod P */
  for (int d = 0; d < 6; d++) {
    uint32_t other = __shfl_down(reg, 1u << d, 64);
    if ((lane & ((2u << d) - 1u)) == 0) reg = crc_mulmod(reg, m, poly) ^ other;
    m = crc_mulmod(m, m, poly);
  }
  return __shfl(reg, 0, 64);
}

/* ---------------------------------------------------------------------------------------
 * Turbo encoding.  One wavefront per (block, constituent encoder) segment; lane l owns
 * qp consecutive 32-bit chunks (qp = 1, 2 or 4).  Zero-start chunk exit states are composed
 * lane-locally, scanned across lanes with shuffles (x -> A^(32 qp 2^d) x), and each chunk
 * is then re-encoded from its true entry state.  No barriers, no LDS scan buffers.
 * ------------------------------------------------------------------------------------- */
struct enc_tabs_t {            /* LDS copy of the RSC tables (lane-varying indices) */
  uint8_t next[8][16];
  uint8_t par[8][16];
  uint8_t apow[8][8];
  uint32_t zs[8];
};

/* QPP walk start of chunk j: Pi(32j) | (Pi(32j+1) - Pi(32j) mod K) << 16 */
static __device__ __forceinline__ uint32_t qpp_start(uint32_t K, uint32_t f1, uint32_t f2, uint32_t j)
{
  uint32_t k = 32 * j;
  uint32_t pi = (((f2 * k) % K) * k + f1 * k) % K;            /* fits 32 bits for K <= 6144 */
  uint32_t dl = (f1 + ((f2 * ((2 * k + 1) % K)) % K)) % K;     /* Pi(k+1) - Pi(k) */
  return pi | (dl << 16);
}

/* interleaved input word of chunk j: bits c'_k = c_Pi(k), Pi(k) = (f1 k + f2 k^2) mod K walked by
 * first and second differences (3gpplte.c:50-74) */
static __device__ __forceinline__ uint32_t qpp_gather_word(const uint32_t *sys, uint32_t K, uint32_t start,
                                                           uint32_t d2, uint32_t j)
{
  uint32_t pi = start & 0xffffu, dl = start >> 16, word = 0;
#pragma unroll
  for (int b = 0; b < 32; b++) {
    word |= __builtin_amdgcn_ubfe(sys[pi >> 5], pi & 31u, 1u) << b;
    pi += dl;
    pi = min(pi, pi - K);
    dl += d2;
    dl = min(dl, dl - K);
  }
  const uint32_t n = K - 32 * j;
  return n >= 32 ? word : word & ((1u << n) - 1u);
}

/* encode one segment (block r, encoder e) with the calling wavefront */
static __device__ __forceinline__ void turbo_segment(const uint32_t *in, uint32_t *par_out, uint32_t K,
                                                     uint32_t *tail_out, const enc_tabs_t *tb)
{
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nch = (K + 31) >> 5;
  const uint32_t lq = nch <= 64 ? 0 : (nch <= 128 ? 1 : 2), qp = 1u << lq;
  uint32_t u[4], v[4];
  uint32_t S = 0;
#pragma unroll
  for (int t = 0; t < 4; t++) {
    u[t] = 0;
    uint32_t j = lane * qp + t;
    if (t < (int)qp && j < nch) u[t] = in[j];
    /* zero-start exit state of a full chunk: the feedback word's last three bits (partial chunks
     * only feed later lanes, whose values are not used) */
    v[t] = rsc_feedback_word(u[t]);
    if (t < (int)qp) S = tb->apow[0][S] ^ (v[t] >> 29);
  }
  /* inclusive scan over lanes: S_l ^= A^(32 qp 2^d) S_(l - 2^d) */
#pragma unroll
  for (int d = 0; d < 6; d++) {
    uint32_t other = __shfl_up(S, 1u << d, 64);
    if (lane >= (1u << d)) S ^= tb->apow[lq + d][other];
  }
  uint32_t s = __shfl_up(S, 1, 64);
  if (lane == 0) s = 0;
#pragma unroll
  for (int t = 0; t < 4; t++) {
    uint32_t j = lane * qp + t;
    if (t < (int)qp && j < nch) {
      uint32_t n = min(32u, K - 32 * j);
      uint32_t par = rsc_parity_of_feedback(v[t]) ^ tb->zs[s];
      if (n < 32) {
        par &= (1u << n) - 1u;
        for (uint32_t q = 0; q < (n >> 2); q++) s = tb->next[s][(u[t] >> (4 * q)) & 15u];
      } else {
        s = tb->apow[0][s] ^ (v[t] >> 29);
      }
      par_out[j] = par;
      if (j == nch - 1) {
        /* trellis termination (3gpplte_sse.c:104-109, 440-471): (x, z) per step */
        uint32_t tbits = 0;
        for (int stp = 0; stp < 3; stp++) {
          uint32_t z = ((s >> 2) ^ s) & 1u, x = (s ^ (s >> 1)) & 1u;
          s >>= 1;
          tbits |= (x << (2 * stp)) | (z << (2 * stp + 1));
        }
        *tail_out = tbits;
      }
    }
  }
}

/* tail bit m (0..11) of block r: t[0..5] from encoder 1, t[6..11] from encoder 2 */
static __device__ __forceinline__ uint32_t tail_bit(const uint32_t *tails, uint32_t r, uint32_t m)
{
  return m < 6 ? (tails[2 * r] >> m) & 1u : (tails[2 * r + 1] >> (m - 6)) & 1u;
}

/* value of d^(s)_idx for block r: stream bit if idx < K, else tail */
static __device__ __forceinline__ uint32_t dstream_bit(const uint32_t *blk, uint32_t sw, const uint32_t *tails,
                                                       uint32_t r, uint32_t K, uint32_t s, uint32_t idx)
{
  if (idx < K) return (blk[s * sw + (idx >> 5)] >> (idx & 31)) & 1u;
  return tail_bit(tails, r, 3 * (idx - K) + s);
}

static __device__ __forceinline__ uint32_t colperm(uint32_t col) { return __builtin_bitreverse32(col) >> 27; }

/* ---- debug-only walker over w (reference layout dumps) ---- */
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

static __device__ __forceinline__ uint32_t wwalk_bit(const wwalk_t &w, const uint32_t *blk, uint32_t sw,
                                                     const uint32_t *tails, uint32_t r, uint32_t K, uint32_t ND,
                                                     uint32_t Kpi)
{
  uint32_t j = colperm(w.col) + 32 * w.row;
  if (w.region == 0) return dstream_bit(blk, sw, tails, r, K, 0, j - ND);
  if (w.which == 0) return dstream_bit(blk, sw, tails, r, K, 1, j - ND);
  uint32_t j2 = (j + 1 == Kpi) ? 0 : j + 1;
  return dstream_bit(blk, sw, tails, r, K, 2, j2 - ND);
}

static __device__ __forceinline__ bool wwalk_null(const wwalk_t &w, uint32_t R, uint32_t ND)
{
  if (w.row != 0) return (w.region == 1 && w.which == 1 && w.col == 31 && w.row == R - 1 && ND > 0);
  uint32_t cp = colperm(w.col);
  if (w.region == 0 || w.which == 0) return cp < ND;
  return (cp + 1 < ND) || (w.col == 31 && R == 1 && ND > 0);
}

/* 32 bits of a packed LSB-first LDS bit array starting at bit `pos` (pos >= -32: zeros before 0) */
[[maybe_unused]] static __device__ __forceinline__ uint32_t sx32(const uint32_t *a, int pos)
{
  const int wi = pos >> 5;
  const uint32_t lo = a[(uint32_t)max(wi, 0)] & (wi >= 0 ? 0xffffffffu : 0u);
  const uint32_t hi = a[(uint32_t)(wi + 1)];
  return __builtin_amdgcn_alignbit(hi, lo, (uint32_t)pos & 31u);
}

/* lane l ^ J of the 32-lane half without the LDS pipe: DPP quad permutes for 1 and 2, the half-row
 * mirror (l ^ 7) then quad_perm [3,2,1,0] (l ^ 3) for 4, a row rotate by 8 for 8, and
 * v_permlane16_swap for 16 (it swaps odd rows of its first operand with even rows of its second:
 * with both = x, the second result holds row 1 in row 0 and the first holds row 0 in row 1) */
#ifndef OAI4G_ENC_XOR_DPP
/* lane l ^ J of the 32-lane half: DPP quad permutes for 1 and 2, ds_swizzle (bit mode) above.
 * (OAI4G_ENC_XOR_DPP: the same without the LDS pipe, below; measured slower: the kernel is bound
 * by VALU issue and the DPP forms of 4 / 16 take two VALU ops where ds_swizzle takes none) */
template <uint32_t J>
static __device__ __forceinline__ uint32_t xor_lane(uint32_t x)
{
  if constexpr (J == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xf, 0xf, false);   /* [1,0,3,2] */
  else if constexpr (J == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xf, 0xf, false); /* [2,3,0,1] */
  else return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, (int)((J << 10) | 0x1f));
}
#else
template <uint32_t J>
static __device__ __forceinline__ uint32_t xor_lane(uint32_t x)
{
  if constexpr (J == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xf, 0xf, false);   /* [1,0,3,2] */
  else if constexpr (J == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xf, 0xf, false); /* [2,3,0,1] */
  else if constexpr (J == 4) {
    const int m = __builtin_amdgcn_mov_dpp((int)x, 0x141, 0xf, 0xf, false);                          /* half mirror */
    return (uint32_t)__builtin_amdgcn_mov_dpp(m, 0x1B, 0xf, 0xf, false);                               /* [3,2,1,0] */
  } else if constexpr (J == 8) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x128, 0xf, 0xf, false);                         /* row_ror:8 */
  } else {
    static_assert(J == 16, "xor_lane");
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return (threadIdx.x & 16u) ? (uint32_t)r[0] : (uint32_t)r[1];
  }
}
#endif

/* 32x32 bit transpose across the 32 lanes of a half-wave: lane c ends with bit i = bit c of
 * lane i's input.  Branch-free butterfly: stage j exchanges the j-bit blocks that differ between
 * partners l and l^j.  The byte-granular stages (16, 8) are one v_perm each: the lane's selector
 * (sel[0] / sel[1], per lane) takes its kept blocks from x and the partner's from p.  The finer
 * stages rotate the partner's word into place (right by j in the upper lane, left by j in the
 * lower) and merge with a bit-field mux whose mask flips with the lane. */
struct tp_lane_t {
  uint32_t sel16, sel8;        /* v_perm selectors of stages 16 and 8 */
  uint32_t rot[3], mm[3];      /* stages 4, 2, 1: rotate amount and kept-bit mask */
};

static __device__ __forceinline__ tp_lane_t tp_lane(uint32_t lane32)
{
  tp_lane_t t;
  /* v_perm bytes 0-3 = second operand (x), 4-7 = first (partner p) */
  t.sel16 = (lane32 & 16u) ? 0x03020706u : 0x05040100u;   /* hi: [p2 p3 x2 x3], lo: [x0 x1 p0 p1] */
  t.sel8 = (lane32 & 8u) ? 0x03070105u : 0x06020400u;     /* hi: [p1 x1 p3 x3], lo: [x0 p0 x2 p2] */
  const uint32_t M[3] = {0x0f0f0f0fu, 0x33333333u, 0x55555555u};
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const uint32_t J = 4u >> k;
    const bool hi = (lane32 & J) != 0;
    t.rot[k] = hi ? J : 32u - J;
    t.mm[k] = hi ? ~M[k] : M[k];
  }
  return t;
}

template <int K = 0>
static __device__ __forceinline__ uint32_t transpose32_t(uint32_t x, const tp_lane_t &t)
{
  if constexpr (K == 5) {
    return x;
  } else if constexpr (K < 2) {
    const uint32_t p = xor_lane<(16u >> K)>(x);
    return transpose32_t<K + 1>(__builtin_amdgcn_perm(p, x, K == 0 ? t.sel16 : t.sel8), t);
  } else {
    const uint32_t p = xor_lane<(16u >> K)>(x);
    const uint32_t sh = __builtin_amdgcn_alignbit(p, p, t.rot[K - 2]);
    /* (x & mm) | (sh & ~mm) as one fast-rate v_bitop3 mux (0xe4: c ? a : b); the compiler's
     * v_and + v_and_or pair has a slow-rate op */
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe4" : "=v"(r) : "v"(x), "v"(sh), "v"(t.mm[K - 2]));
    return transpose32_t<K + 1>(r, t);
  }
}

/* OR 32 bits into an LDS bit array at bit offset `bit` (LDS atomics: tiles of neighbouring
 * columns share boundary words) */
static __device__ __forceinline__ void or_bits(uint32_t *w, uint32_t bit, uint32_t v)
{
  if (!v) return;
  const uint32_t wi = bit >> 5, sh = bit & 31u;
  atomicOr(&w[wi], v << sh);
  if (sh && (v >> (32 - sh))) atomicOr(&w[wi + 1], v >> (32 - sh));
}

/* the same without the tests: both words always (an OR of zero into the second is harmless; the
 * caller guarantees word bit / 32 + 1 is inside the array), the pair from one 64-bit shift */
static __device__ __forceinline__ void or_bits2(uint32_t *w, uint32_t bit, uint32_t v)
{
  const uint64_t s = (uint64_t)v << (bit & 31u);
  uint32_t *p = w + (bit >> 5);
  atomicOr(p, (uint32_t)s);
  atomicOr(p + 1, (uint32_t)(s >> 32));
}

/* ---------------------------------------------------------------------------------------
 * The fused encoder.
 * ------------------------------------------------------------------------------------- */
template <bool DEBUG>
static __device__ void encode_codeword(const cfg_dev_t *__restrict__ c, uint32_t sf, uint32_t cwi,
                                       const uint8_t *__restrict__ payload, uint32_t *__restrict__ ebits,
                                       enc_debug_t dbg, uint32_t *lds_base, int stop_phase = 99, uint32_t sf0 = 0)
{
  const cw_dev_t &cw = c->cw[cwi];
  const uint32_t tid = threadIdx.x, nth = blockDim.x, lane = tid & 63, nwaves = nth >> 6;
  /* the wave index as an SGPR: every loop over waves (phases 3b, 4) is then a scalar loop */
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t sfi = DEBUG ? sf : (c->first_sf + (sf0 + sf) * c->sf_step) % 10;
  /* wave-uniform: SGPRs, so the per-block stream offsets (r 3 sw) are scalar arithmetic */
  const uint32_t C = __builtin_amdgcn_readfirstlane(cw.C), sw = __builtin_amdgcn_readfirstlane(cw.stream_words);
  /* LDS carve-up.  Region A: TB || CRC (phases 0-2), the QPP-interleaved words (phase 3), one half
   * of the e words (phase 4).  Region B: the CRC byte tables (phases 0-1), then the constituent
   * streams (the QPP planes in the parity slots during phase 3a). */
  uint32_t *tbw = lds_base;
  uint32_t *strm = lds_base + c->lds_a_words;
  /* the CRC byte tables live in region B until segmentation writes the streams (phases 0-1) */
  uint32_t *crctab_a = strm;
  uint32_t *crctab_b = crctab_a + 256;
  uint32_t *tails = strm + c->lds_b_words;
  uint32_t *crcs = tails + 2 * OAI4G_MAX_CB;             /* [0] = CRC24A, [1+r] = CRC24B of block r */
  uint32_t *red = crcs + OAI4G_MAX_CB + 2;               /* 4 per-wave partials */
  enc_tabs_t *tabs = (enc_tabs_t *)(red + 4);
  uint32_t *dbg_ebuf = (uint32_t *)(tabs + 1);          /* k_encode_debug only: the whole codeword's e words */
  uint8_t *tbb = (uint8_t *)tbw;
  const uint32_t G = cw.G[sfi];

  /* block geometry as wave-uniform scalars: n0 blocks of size kk0 (kw0 words) then blocks of size
   * kk1; word i of the interleaved space -> block r, word j, block size K without per-lane table
   * walks */
  const uint32_t nw = cw.ilv_off[C], u0 = cw.u0, n0 = cw.n0;
  const uint32_t kw0 = __builtin_amdgcn_readfirstlane(cw.kw[0]), kw1 = __builtin_amdgcn_readfirstlane(cw.kw[1]);
  const uint32_t km0 = __builtin_amdgcn_readfirstlane(cw.kmag[0]), km1 = __builtin_amdgcn_readfirstlane(cw.kmag[1]);
  const uint32_t kk0 = __builtin_amdgcn_readfirstlane(cw.kk[0]), kk1 = __builtin_amdgcn_readfirstlane(cw.kk[1]);
  /* the block's filler bytes, copied bytes and TB offset in closed form (lte_segmentation.c:52-166:
   * fill F / 8 in block 0 only; every block copies K / 8 - L / 8 bytes less its fill; offsets are
   * the running sum): no per-lane loads of cw.fill / ncopy / src ahead of a barrier */
  const uint32_t L8 = __builtin_amdgcn_readfirstlane(cw.L) >> 3, F8 = __builtin_amdgcn_readfirstlane(cw.F) >> 3;
  const uint32_t cb0 = (kk0 >> 3) - L8, cb1 = (kk1 >> 3) - L8;
  auto seg_of = [&](uint32_t r, uint32_t &fill, uint32_t &ncopy, uint32_t &s0) {
    const uint32_t ki = r >= n0 ? 1u : 0u;
    fill = r == 0 ? F8 : 0u;
    ncopy = (ki ? cb1 : cb0) - fill;
    s0 = r == 0 ? 0u : (ki ? n0 * cb0 + (r - n0) * cb1 : r * cb0) - F8;
  };

  /* ---- phase 0: TB bytes, stream words past each block's data, tables ---- */
  const uint8_t *src = payload + (size_t)(DEBUG ? 0 : (sf * c->n_cw + cwi)) * c->payload_stride;
  const uint32_t Ab = cw.A_bytes;
  {
    const uint32_t ct = tid, cn = nth;
    for (uint32_t i = ct; i < c->lds_tb_words; i += cn) {
      uint32_t v = 0;
      if (4 * i < Ab) {
        v = *(const uint32_t *)(src + 4 * i);
        uint32_t valid = Ab - 4 * i;
        if (valid < 4) v &= (1u << (8 * valid)) - 1u;
      }
      tbw[i] = v;
    }
    if (ct == 0) crcs[0] = 0u;                    /* phase 1's XOR accumulator (C > 1) */
    if (C > 1) {
      for (uint32_t v = ct; v < 256; v += cn) {   /* reflected, << 2 (crc_chunk_w2r) */
        const uint32_t iv = __builtin_bitreverse32(v) >> 24;
        crctab_a[v] = __builtin_bitreverse32(c->crctab[0][iv] << 8) << 2;
        crctab_b[v] = __builtin_bitreverse32(c->crctab[1][iv] << 8) << 2;
      }
    } else {
      for (uint32_t v = ct; v < 256; v += cn)     /* the register-in-the-top-24-bits form */
        crctab_a[v] = c->crctab[0][v] << 8;
    }
    for (uint32_t i = ct; i < 128; i += cn) {
      (&tabs->next[0][0])[i] = (&c_rsc.next[0][0])[i];
      (&tabs->par[0][0])[i] = (&c_rsc.par[0][0])[i];
      if (i < 64) (&tabs->apow[0][0])[i] = (&c_rsc.apow[0][0])[i];
      if (i < 8) tabs->zs[i] = c_rsc.zs[i];
    }
  }
  __syncthreads();
  if (stop_phase <= 0) return;

  /* ---- phase 1: CRC-24A over the TB (dlsch_coding.c:296-300) and CRC-24B of every block's data
   * bytes (lte_segmentation.c:156-166) ---- */
  if (C > 1) {
    /* one pass for both: crc_lpb lanes per block, each lane a chunk of one block through both byte
     * tables; the groups combine their chunks per block (-> CRC-24B) and multiply the block's
     * CRC-24A part into place (crcmul_blk), LDS XOR atomics sum the TB's */
    const uint32_t lpb = __builtin_amdgcn_readfirstlane(cw.crc_lpb), per = __builtin_amdgcn_readfirstlane(cw.crc_per_cb);
    const uint32_t pos = tid & (lpb - 1);
    for (uint32_t r = tid / lpb; r < C; r += nth / lpb) {
      uint32_t fill, n, s0;
      seg_of(r, fill, n, s0);
      if (s0 + n > Ab) n = Ab > s0 ? Ab - s0 : 0;
      uint32_t ra, rb;
      crc_chunk_w2r(tbw, s0, n, per, pos, lpb, (const uint8_t *)crctab_a, (const uint8_t *)crctab_b, ra, rb);
      crc_group_tree2(ra, rb, pos, lpb, cw.crc2_cb[0], cw.crc2_cb[1]);
      if (pos == 0) {
        crcs[1 + r] = rb;
        atomicXor(&crcs[0], crc_mul_tab(ra, cw.crcmul_blk[r]));
      }
    }
    __syncthreads();
    if (tid == 0) {
      const uint32_t crc = crcs[0];
      tbb[Ab] = (uint8_t)(crc >> 16);
      tbb[Ab + 1] = (uint8_t)(crc >> 8);
      tbb[Ab + 2] = (uint8_t)crc;
      /* the TB-CRC bytes end the last block's data (lte_segmentation.c: the last block copies the
       * TB through its CRC-24A), folded into its CRC-24B through the reflected LDS table
       * (crc_chunk_w2r's register form) */
      uint32_t a = __builtin_bitreverse32(crcs[C] << 8) << 2;
      const uint8_t *r2b = (const uint8_t *)crctab_b;
      a = (a >> 8) ^ *(const uint32_t *)(r2b + ((a ^ (__builtin_bitreverse32(crc >> 16) >> 22)) & 0x3fcu));
      a = (a >> 8) ^ *(const uint32_t *)(r2b + ((a ^ (__builtin_bitreverse32((crc >> 8) & 0xffu) >> 22)) & 0x3fcu));
      a = (a >> 8) ^ *(const uint32_t *)(r2b + ((a ^ (__builtin_bitreverse32(crc & 0xffu) >> 22)) & 0x3fcu));
      crcs[C] = __builtin_bitreverse32(a >> 2) >> 8;
    }
  } else {
    uint32_t reg = crc_chunk_w(tbw, 0, Ab, cw.crc_per_tb, tid, nth, crctab_a);
    reg = crc_wave_tree2(reg, cw.crc2_tb);
    if (lane == 0) red[wave] = reg;
    __syncthreads();
    if (tid == 0) {
      uint32_t v01 = crc_mul_tab(red[0], cw.crcmul_tb[6][0]) ^ red[1];
      uint32_t v23 = crc_mul_tab(red[2], cw.crcmul_tb[6][0]) ^ red[3];
      uint32_t crc = crc_mul_tab(v01, cw.crcmul_tb[7][0]) ^ v23;
      tbb[Ab] = (uint8_t)(crc >> 16);
      tbb[Ab + 1] = (uint8_t)(crc >> 8);
      tbb[Ab + 2] = (uint8_t)crc;
    }
  }
  __syncthreads();
  if (DEBUG && dbg.b)
    for (uint32_t i = tid; i < Ab + 3; i += nth) dbg.b[i] = tbb[i];
  if (stop_phase <= 1) return;

  /* stream words past the data of each block (tail bits, read-ahead; region B held the CRC tables
   * until here); the data words are fully written by segmentation (systematic) and the phase-3
   * planes / turbo (parity) */
  /* ---- phase 2: segmentation -> systematic streams (LSB-first words), one word per thread over
   * the words of all blocks; a word inside the copied bytes is one unaligned 4-byte read ---- */
  for (uint32_t i = tid; i < C * 3 * 4; i += nth) {
    const uint32_t slot = i >> 2, r = slot / 3;
    const uint32_t w = (r < n0 ? kw0 : kw1) + (i & 3u);
    if (w < sw) strm[slot * sw + w] = 0u;
  }
  auto unit_of = [&](uint32_t i, uint32_t &r, uint32_t &j, uint32_t &K, uint32_t &ki) {
    ki = i >= u0 ? 1u : 0u;
    const uint32_t ii = ki ? i - u0 : i, kw = ki ? kw1 : kw0;
    const uint32_t rr = __umul24(ii, ki ? km1 : km0) >> 20;
    j = ii - __umul24(rr, kw);
    r = ki ? n0 + rr : rr;
    K = ki ? kk1 : kk0;
  };
  for (uint32_t i = tid; i < nw; i += nth) {
    uint32_t r, j, K, ki;
    unit_of(i, r, j, K, ki);
    uint32_t fill, ncopy, s0;
    seg_of(r, fill, ncopy, s0);
    const uint32_t i0 = 4 * j;
    uint32_t le;
    if (i0 >= fill) {
      /* the data bytes as one unaligned read; a block's last word (or two) also takes the CRC-24B
       * bytes from byte sh = fill + ncopy - i0 on, spliced in without a byte loop (bytes past the
       * block are masked off below) */
      const uint32_t a = s0 + i0 - fill, wi = a >> 2;
      le = __builtin_amdgcn_alignbit(tbw[wi + 1], tbw[wi], (a & 3u) * 8u);
      const int sh = (int)(fill + ncopy) - (int)i0;
      if (C > 1 && sh < 4) {                                   /* sh in [-2, 3] */
        const uint32_t crcle = __builtin_bswap32(crcs[1 + r] << 8);   /* CRC bytes MSB first */
        const uint32_t cw32 = (uint32_t)(((uint64_t)crcle << (8 * (sh + 4))) >> 32);
        le = (sh > 0 ? le & (0xffffffffu >> (32 - 8 * sh)) : 0u) | cw32;
      }
    } else {
      const uint32_t crcb = C > 1 ? crcs[1 + r] : 0;
      le = 0;
      for (uint32_t q = 0; q < 4; q++) {
        const uint32_t ib = i0 + q;
        uint32_t byte = 0;
        if (ib < fill) byte = 0;
        else if (ib < fill + ncopy) byte = tbb[s0 + ib - fill];
        else if (C > 1 && ib < fill + ncopy + 3) byte = (crcb >> (8 * (2 - (ib - fill - ncopy)))) & 0xffu;
        le |= byte << (8 * q);
      }
    }
    uint32_t wv = bytes_to_seq(le);
    if (32 * (j + 1) > K) wv &= (1u << (K - 32 * j)) - 1u;
    strm[r * 3 * sw + j] = wv;
  }
  __syncthreads();
  if (stop_phase <= 2) return;

  /* ---- phase 3a: QPP-interleaved input words of every block, folded by quarters.  With
   * Q = K/4, Pi(k + qQ) = Pi(k) + q c4 (mod K), so one walk over k < Q reads output bits k, k+Q,
   * k+2Q, k+3Q from four rotations of c at the same position Pi(k): plane_r[x] = c[(x + rQ) mod K].
   * Plane 0 is the systematic stream, planes 1 / 2 are staged in the (not yet written) parity
   * stream slots of the block, plane 3 in region A behind the interleaved words. ---- */
  uint32_t *ilv = lds_base;
  /* byte-interleaved planes of every block, over x' < Q only: word w holds positions x' = 8w..8w+7,
   * byte q = plane q (c[x' + qQ]); plane p at x = x' + uQ is byte (p + u) mod 4 there, so one
   * rotate by 8u + (x' & 7) aligns all four bits of position x.  Built from four 32-bit plane words
   * per 32 positions with byte permutes.  A block's planes (K / 32 words) live in its first parity
   * stream's slot, which the turbo encoder writes only in phase 3b: region A holds just the
   * interleaved words. */
  for (uint32_t r = 0; r < C; r++) {
    const uint32_t K = r < n0 ? kk0 : kk1, Kw = (K + 31) >> 5, Q = K >> 2, io = r < n0 ? r * kw0 : u0 + (r - n0) * kw1;
    const uint32_t *sys = strm + r * 3 * sw;
    for (uint32_t w = tid; w < Kw; w += nth) ilv[io + w] = 0u;
    const uint32_t ng = (Q + 31) >> 5, nbw = (Q + 7) >> 3;
    for (uint32_t g = tid; g < ng; g += nth) {
      uint32_t P[4];
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {
        const uint32_t src = 32 * g + q * Q, wi = src >> 5;                  /* src < K */
        const uint32_t lo = sys[wi], hi = wi + 1 < Kw ? sys[wi + 1] : 0u;    /* bits >= K are zero */
        uint32_t v = __builtin_amdgcn_alignbit(hi, lo, src);
        if (src + 32 > K) v |= sys[0] << (K - src);                          /* wrap to c_0.. */
        P[q] = v;
      }
#pragma unroll
      for (uint32_t jb = 0; jb < 4; jb++) {
        const uint32_t t01 = __builtin_amdgcn_perm(P[1], P[0], 0x0c0c0000u | jb | ((4 + jb) << 8));
        const uint32_t t23 = __builtin_amdgcn_perm(P[3], P[2], 0x00000c0cu | (jb << 16) | ((4 + jb) << 24));
        if (4 * g + jb < nbw) strm[(r * 3 + 1) * sw + 4 * g + jb] = t01 | t23;
      }
    }
  }
  __syncthreads();
  {
    /* 8-step units: unit j of block r walks k = 8j .. 8j+7 (< Q) through the host table and
     * yields one byte of each quarter; ceil(K/32) units per block, indexed like the interleaved words */
    const bool s3a = __builtin_amdgcn_readfirstlane(cw.qpp_s3[0]) != 0, s3b = __builtin_amdgcn_readfirstlane(cw.qpp_s3[1]) != 0;
    for (uint32_t i = tid; i < nw; i += nth) {
      uint32_t r, j, K, ki;
      unit_of(i, r, j, K, ki);
      const uint32_t Q = K >> 2;
      const uint4 e4 = *(const uint4 *)&cw.qpp_tab[ki][4 * j];
      const uint32_t ew[4] = {e4.x, e4.y, e4.z, e4.w};
      const uint32_t *b8 = strm + (r * 3 + 1) * sw;     /* block r's planes */
      uint32_t acc = 0;
#pragma unroll
      for (int b = 0; b < 8; b++) {
        /* entry: rotate in bits 0-4 (alignbit reads only those), plane word in bits 7-14, so the
         * word's byte offset is one field extract of bits 5-14 (bits 5-6 are zero) */
        const uint32_t e = (b & 1) ? ew[b >> 1] >> 16 : ew[b >> 1];
        const uint32_t D = *(const uint32_t *)((const uint8_t *)b8 + __builtin_amdgcn_ubfe(e, 5, 10));
        acc |= __builtin_amdgcn_alignbit(D, D, e) & (0x01010101u << b);
      }
      uint32_t a0 = acc & 0xffu, a1 = (acc >> 8) & 0xffu, a2 = (acc >> 16) & 0xffu, a3 = acc >> 24;
      const uint32_t n = Q - 8 * j;
      if (n < 8) {
        const uint32_t m = (1u << n) - 1u;
        a0 &= m; a1 &= m; a2 &= m; a3 &= m;
      }
      /* output quarter q reads plane (q c4 / Q) mod 4 */
      const bool s3 = ki ? s3b : s3a;
      const uint32_t q1 = s3 ? a3 : a1, q3 = s3 ? a1 : a3;
      uint32_t *o = ilv + (i - j);
      if ((Q & 7u) == 0) {                                  /* byte-aligned quarters (32 | K) */
        uint8_t *ob = (uint8_t *)o + j;
        const uint32_t qb = Q >> 3;
        ob[0] = (uint8_t)a0; ob[qb] = (uint8_t)q1; ob[2 * qb] = (uint8_t)a2; ob[3 * qb] = (uint8_t)q3;
      } else {
        or_bits(o, 8 * j, a0);
        or_bits(o, Q + 8 * j, q1);
        or_bits(o, 2 * Q + 8 * j, a2);
        or_bits(o, 3 * Q + 8 * j, q3);
      }
    }
  }
  __syncthreads();
  if (stop_phase == 23) return;   /* diagnostics: QPP interleaving only */

  /* ---- phase 3b: turbo encoding, one wave per (block, encoder) ---- */
  for (uint32_t seg = wave; seg < 2 * C; seg += nwaves) {
    const uint32_t r = seg >> 1, e = seg & 1u;
    uint32_t *blk = strm + r * 3 * sw;
    const uint32_t io = r < n0 ? r * kw0 : u0 + (r - n0) * kw1;
    turbo_segment(e ? ilv + io : blk, blk + (1 + e) * sw, r < n0 ? kk0 : kk1, &tails[2 * r + e], tabs);
  }
  __syncthreads();
  if (stop_phase <= 3) return;

  if (DEBUG) {
    /* reference-layout intermediates: c[r] bytes, d[r] (NULL prefix + 3K+12 + side effect), w[r] */
    for (uint32_t r = 0; r < C; r++) {
      uint32_t K = cw.K[r], R = cw.R[r], Kpi = cw.Kpi[r], ND = cw.ND[r];
      const uint32_t *blk = strm + r * 3 * sw;
      if (dbg.c)
        for (uint32_t i = tid; i < K / 8; i += nth) {
          uint32_t wv = blk[(i >> 2)];
          uint32_t byte = (wv >> (8 * (i & 3))) & 0xffu;
          dbg.c[r * (8 + 3 + 768) + i] = (uint8_t)(__builtin_bitreverse32(byte) >> 24);
        }
      if (dbg.d) {
        uint8_t *d = dbg.d + (size_t)r * OAI4G_D_BYTES;
        for (uint32_t i = tid; i < 96; i += nth) d[i] = OAI4G_LTE_NULL;
        for (uint32_t i = tid; i < 3 * K + 12; i += nth) {
          uint32_t kk = i / 3, s = i - 3 * kk;
          d[96 + i] = (uint8_t)(kk < K ? dstream_bit(blk, sw, tails, r, K, s, kk) : tail_bit(tails, r, i - 3 * K));
        }
        if (tid == 0) d[96 + 3 * (K + 4) + 2] = (uint8_t)dstream_bit(blk, sw, tails, r, K, 2, 0);
      }
      if (dbg.w) {
        uint8_t *w = dbg.w + (size_t)r * OAI4G_W_BYTES;
        for (uint32_t p = tid; p < 3 * Kpi; p += nth) {
          wwalk_t wk;
          wwalk_init(wk, p, R, Kpi);
          w[p] = wwalk_null(wk, R, ND) ? OAI4G_LTE_NULL : (uint8_t)wwalk_bit(wk, blk, sw, tails, r, K, ND, Kpi);
        }
      }
    }
    if (!dbg.e) return;
  }

  /* append the 4 tail bits of each constituent stream at bit K (d^(s)_K..K+3) */
  const uint32_t nd0 = __builtin_amdgcn_readfirstlane(cw.NDk[0]), nd1 = __builtin_amdgcn_readfirstlane(cw.NDk[1]);
  for (uint32_t r = tid; r < C; r += nth) {
    const uint32_t K = r < n0 ? kk0 : kk1, ND = r < n0 ? nd0 : nd1;
    uint32_t *blk = strm + r * 3 * sw;
    for (uint32_t s = 0; s < 3; s++) {
      uint32_t t4 = tail_bit(tails, r, s) | (tail_bit(tails, r, 3 + s) << 1) | (tail_bit(tails, r, 6 + s) << 2) |
                    (tail_bit(tails, r, 9 + s) << 3);
      uint32_t w0 = K >> 5, off = K & 31;
      blk[s * sw + w0] |= t4 << off;
      if (off > 28) blk[s * sw + (w0 + 1)] |= t4 >> (32 - off);
    }
    /* phase 4's RM_SRC_LAST lane reads y^(2)_0 = d^(2)_0 at stream-2 position Kpi - ND = K + 4
     * when ND = 0: the reference's own d[3D + 2] = d[2] copy (lte_rate_matching.c:74-75) in stream form */
    if (ND == 0) blk[2 * sw + ((K + 4) >> 5)] |= (blk[2 * sw] & 1u) << ((K + 4) & 31u);
  }
  __syncthreads();

  /* ---- phase 4: sub-block interleaving (lte_rate_matching.c:51-130) and rate matching
   * (:464-566) fused.  Each half-wave takes a 32x32 bit tile of one block's streams and transposes
   * it (5 shuffle stages) so that lane c holds a run of 32 consecutive w bits of column
   * bitrev5(c): v^(0) tiles are 32 rows of y^(0); interlaced tiles are 16 rows of y^(1) and y^(2)
   * alternating (lane 2i: y^(1) row, lane 2i+1: y^(2) row, pre-shifted by one for the
   * (pi(k)+1) mod Kpi rule), so the transposed run is already w's v^(1)/v^(2) interlacing.  w is
   * never materialised: NULLs sit only at row 0 of a column (and at w[3Kpi-1]), so the run's
   * position among the non-NULL entries of w is closed-form, and the run goes straight to its
   * place(s) in the circular-buffer output: e index (ci - k0c) mod Nnn (+ j Nnn while < E),
   * positions >= Ncb excluded.  Region A (the interleaved words are dead) holds the output. ---- */
  /* The e words are staged per half of the blocks: blocks [0, hb) then [hb, C), each half's words
   * (its first word may be shared with the previous half: carried over) zeroed, ORed into, then
   * scrambled and stored.  Region A holds one half (the host sizes it, lds_a_words), so the
   * three streams and the output are never resident in full together.  The debug kernel stages
   * the whole codeword in one pass behind the tables (dbg.ebuf). */
  {
    const tp_lane_t tpl = tp_lane(tid & 31);
    const uint32_t sw3 = __builtin_amdgcn_readfirstlane(3 * sw);
    const uint32_t nt0 = __builtin_amdgcn_readfirstlane(cw.ntk[0]), nt1 = __builtin_amdgcn_readfirstlane(cw.ntk[1]);
    const uint32_t Nnn0 = __builtin_amdgcn_readfirstlane(cw.Nnnk[0]), Nnn1 = __builtin_amdgcn_readfirstlane(cw.Nnnk[1]);
    const uint32_t es = __builtin_amdgcn_readfirstlane(cw.esplit[sfi]);
    const uint32_t Elo = __builtin_amdgcn_readfirstlane(cw.E[sfi][0]), Ehi = __builtin_amdgcn_readfirstlane(cw.E[sfi][C - 1]);
    const uint32_t wrapt0 = __builtin_amdgcn_readfirstlane(cw.rm_wrapt[0]), wrapt1 = __builtin_amdgcn_readfirstlane(cw.rm_wrapt[1]);
    /* no repetition (E <= Nnn for every block): a run lands once at most */
    const bool once = Ehi <= min(Nnn0, Nnn1) && Elo <= min(Nnn0, Nnn1) && wrapt0 != ~1u && wrapt1 != ~1u;
    const uint32_t pp0 = (nt0 + 1) >> 1, pp1 = (nt1 + 1) >> 1;            /* tile pairs per block */
    const uint32_t psplit = n0 * pp0;
    const uint32_t pm0 = ((1u << 20) + pp0 - 1) / pp0, pm1 = ((1u << 20) + pp1 - 1) / pp1;
    auto ro_of = [&](uint32_t r) { return r >= es ? es * Elo + (r - es) * Ehi : r * Elo; };   /* e bit offset of block r */
    auto pair0 = [&](uint32_t r) { return r < n0 ? r * pp0 : psplit + (r - n0) * pp1; };      /* first tile pair of block r */
    /* tile pair P -> (block size, block, first tile); the pair's plan rows are contiguous, so a
     * lane's plan words sit at a wave-uniform base + 4 lane.  Loaded one pair ahead. */
    auto decode = [&](uint32_t P, uint32_t &ki, uint32_t &r, uint32_t &t0) {
      ki = P >= psplit ? 1u : 0u;
      const uint32_t PP = ki ? P - psplit : P, pp = ki ? pp1 : pp0;
      const uint32_t rr = (PP * (ki ? pm1 : pm0)) >> 20, rem = PP - rr * pp;
      r = ki ? n0 + rr : rr;
      t0 = 2 * rem;
    };
    gu32_t *gold = (gu32_t *)(c->gold_tab + (size_t)(sfi * c->n_cw + cwi) * c->ebits_words);
    uint32_t *eout = DEBUG ? nullptr : ebits + (size_t)(sf * c->n_cw + cwi) * c->ebits_words;
    uint32_t *ebuf = DEBUG ? dbg_ebuf : lds_base;
    const uint32_t hb = DEBUG ? C : (C + 1) >> 1, nhalf = DEBUG ? 1u : 2u;
    uint32_t carry = 0;                          /* the boundary word of the first half */
    for (uint32_t h = 0; h < nhalf; h++) {
      const uint32_t rb0 = h ? hb : 0, rb1 = h ? C : hb;
      const uint32_t eb0 = ro_of(rb0), eb1 = rb1 < C ? ro_of(rb1) : G;   /* e bits [eb0, eb1) */
      const uint32_t w0 = eb0 >> 5, nwh = ((eb1 + 31) >> 5) - w0;       /* staged words */
      /* nwh + 1 words: or_bits2 always writes word bit / 32 + 1 as well, so the word past the half's last
       * is zeroed too; the host reserves it (derive_cfg: lds_a_words >= w1, w2 = staged words + 1; the
       * debug kernel's dbg_ebuf holds the whole codeword + 1) */
      for (uint32_t i = tid; i < nwh + 1; i += nth) ebuf[i] = (i == 0 && h) ? carry : 0u;
      __syncthreads();
      const uint32_t pb = pair0(rb0), pe = pair0(rb1), bit0 = 32 * w0;
      /* plan rows of pair (ki, t0): a wave-uniform word offset (scalar) from the plan base, so the
       * loads take an SGPR base and the lane offset, with no vector address arithmetic */
      const uint32_t *rsrc0 = &cw.rm_src[0][0][0], *rdst0 = &cw.rm_dst[0][0][0];
      auto row_of = [&](uint32_t ki, uint32_t t0) {
        return __builtin_amdgcn_readfirstlane(ki * ((OAI4G_RM_TILES + 1) * 32) + t0 * 32);
      };
      /* round-robin pairs P = pb + wave + k nwaves, stepped rather than decoded: the next pair is
       * nwaves pairs on (2 nwaves tiles), carried over block ends; a block's scalars change only
       * there.  Plan words loaded one pair ahead. */
      /* The pair loop, versioned on `once` (wave-uniform, loop-invariant) so that neither version
       * tests it per pair; a block's scalars (stream offset, E, e offset, Nnn, wrap tile) are
       * refreshed only when the walk enters the next block. */
      auto pair_loop = [&](auto ONCE) {
        uint32_t P = pb + wave;
        uint32_t ki = 0, r = 0, t0 = 0;
        uint32_t nsrc = 1u << 5, ndst = 0;
        if (P < pe) {
          decode(P, ki, r, t0);
          const uint32_t ro = row_of(ki, t0);
          nsrc = (rsrc0 + ro)[lane];
          ndst = (rdst0 + ro)[lane];
        }
        uint32_t bbo = 0, E = 0, rob = 0, Nnn = 0, wtc = 0, tpb = 0, rowb = 0;
        auto enter = [&](uint32_t rr, uint32_t kk) {
          bbo = __builtin_amdgcn_readfirstlane(rr * sw3);
          E = rr >= es ? Ehi : Elo;
          rob = ro_of(rr) - bit0;
          Nnn = kk ? Nnn1 : Nnn0;
          wtc = kk ? wrapt1 : wrapt0;
          tpb = 2 * (kk ? pp1 : pp0);                                        /* tiles per block (pairs x 2) */
          rowb = kk * ((OAI4G_RM_TILES + 1) * 32);                           /* the block size's plan rows */
        };
        enter(r, ki);
        for (; P < pe; P += nwaves) {    /* scalar loop: wave is an SGPR */
          const uint32_t src = nsrc, dst = ndst;
          /* the next pair of this wave (crossing into later blocks only at a block end) */
          uint32_t k2 = ki, r2 = r, t2 = t0 + 2 * nwaves, rowb2 = rowb;
          if (t2 >= tpb) {
            uint32_t tpb2 = tpb;
            do {
              t2 -= tpb2;
              r2++;
              k2 = r2 >= n0 ? 1u : 0u;
              tpb2 = 2 * (k2 ? pp1 : pp0);
            } while (t2 >= tpb2);
            rowb2 = k2 * ((OAI4G_RM_TILES + 1) * 32);
          }
          if (P + nwaves < pe) {
            const uint32_t ro = __builtin_amdgcn_readfirstlane(rowb2 + t2 * 32);
            nsrc = (rsrc0 + ro)[lane];
            ndst = (rdst0 + ro)[lane];
          }
          const uint32_t *bb = strm + bbo - 1;                               /* block streams - 1 word (scalar offset) */
          const uint32_t *wp = bb + ((src >> 5) & 0x7fffu);
          uint32_t y = __builtin_amdgcn_alignbit(wp[1], wp[0], src);          /* bits before 0 are NULLs */
          /* the RM_SRC_LAST lane (row R - 1 of y2, j = Kpi - 1 reads y^(2)_0 at bit 31) needs no
           * test: its bit 31 is stream-2 position Kpi - ND, which holds d^(2)_0 when ND = 0 (copied
           * there with the tail bits) and is past the run (a NULL, m excludes it) when ND > 0 */
          y = transpose32_t<0>(y, tpl);
          y >>= (dst >> 16) & 31u;                                           /* leading NULLs z */
          const uint32_t o = dst & 0xffffu, m = __builtin_amdgcn_ubfe(dst, 21, 6);
          const uint32_t ro = rob;                                           /* relative to the staged words */
          if constexpr (decltype(ONCE)::value) {
            /* no repetition (E <= Nnn): the run's part below E, then (the one run that straddles
             * the circular buffer's end: a block's wrap tile, scalar test first) its wrapped part at 0 */
            const int l = min((int)m, (int)E - (int)o);
            if (l > 0) or_bits2(ebuf, ro + o, y & (0xffffffffu >> (32 - l)));
            if (wtc - t0 < 2u) {                                             /* t0 or t0 + 1 is the wrap tile */
              asm volatile("" ::: "memory");   /* keeps the lane test below behind the scalar one */
              if (dst & OAI4G_RM_DST_WRAP) {
                const uint32_t ma = Nnn - o;                                 /* 1 .. m - 1 */
                const uint32_t l2 = min(m - ma, E);
                or_bits2(ebuf, ro, (y >> ma) & (0xffffffffu >> (32 - l2)));
              }
            }
          } else if (m) {
            y &= 0xffffffffu >> (32 - m);
            /* the run may straddle the wrap back to k0c; E > Nnn repeats the buffer */
            const uint32_t ma = min(m, Nnn - o);
            for (uint32_t part = 0; part < 2; part++) {
              const uint32_t len = part ? m - ma : ma, os = part ? 0u : o;
              const uint32_t v = part ? (ma < 32 ? y >> ma : 0u) : (ma < 32 ? y & ((1u << ma) - 1u) : y);
              for (uint32_t x = os; len && x < E; x += Nnn) {                   /* repetition rounds */
                const uint32_t l = min(len, E - x);
                or_bits(ebuf, ro + x, v & (0xffffffffu >> (32 - l)));
              }
            }
          }
          if (r2 != r) enter(r2, k2);
          ki = k2;
          r = r2;
          t0 = t2;
        }
      };
      if (once) pair_loop(std::true_type{});
      else pair_loop(std::false_type{});
      __syncthreads();
      if (DEBUG) {
        for (uint32_t k = tid; k < G; k += nth) dbg.e[k] = (uint8_t)((ebuf[k >> 5] >> (k & 31)) & 1u);
        return;
      }
      /* scrambling (dlsch_scrambling.c:51-97): c_init = rnti 2^14 + q 2^13 + subframe 2^9 + Nid_cell
       * depends only on (subframe index, codeword), so the Gold words come from the configuration's
       * table (L2-resident) and are XORed into the RM output on the way out.  A first half that ends
       * inside a word leaves that word to the second. */
      const uint32_t nst = stop_phase <= 4 ? 0u : ((h + 1 < nhalf && (eb1 & 31u)) ? nwh - 1 : nwh);
      for (uint32_t i = tid; i < nst; i += nth) {
        const uint32_t wi = w0 + i;
        uint32_t v = ebuf[i] ^ gold[wi];
        const uint32_t nb = min(32u, G - 32 * wi);
        if (nb < 32) v &= (1u << nb) - 1u;
        eout[wi] = v;
      }
      if (h + 1 < nhalf) {
        carry = (eb1 & 31u) ? ebuf[nwh - 1] : 0u;
        __syncthreads();
      }
    }
  }
}

__global__ void __launch_bounds__(256) k_encode(const cfg_dev_t *__restrict__ c, const uint8_t *__restrict__ payload,
                                                uint32_t *__restrict__ ebits, int stop_phase, uint32_t sf0)
{
  extern __shared__ uint32_t lds_dyn[];
  uint32_t sf = blockIdx.x / c->n_cw, cwi = blockIdx.x % c->n_cw;
  enc_debug_t none = {nullptr, nullptr, nullptr, nullptr, nullptr};
  encode_codeword<false>(c, sf, cwi, payload, ebits, none, lds_dyn, stop_phase, sf0);
}

__global__ void __launch_bounds__(256) k_encode_debug(const cfg_dev_t *__restrict__ c, uint32_t sf, uint32_t cwi,
                                                      const uint8_t *__restrict__ payload, enc_debug_t dbg)
{
  extern __shared__ uint32_t lds_dyn[];
  encode_codeword<true>(c, sf, cwi, payload, nullptr, dbg, lds_dyn);
}

static size_t enc_lds_bytes(const cfg_dev_t *h)
{
  size_t words = (size_t)h->lds_a_words + h->lds_b_words + 2 * OAI4G_MAX_CB + OAI4G_MAX_CB + 2 + 4;
  size_t bytes = words * 4 + sizeof(enc_tabs_t);
#ifdef OAI4G_ENC_LDS_PAD
  bytes += OAI4G_ENC_LDS_PAD;   /* DIAGNOSTIC: unused LDS, fewer resident workgroups per CU */
#endif
  return (bytes + 15) & ~(size_t)15;
}

static hipError_t launch_encode_impl(const cfg_dev_t *d_cfg, const cfg_dev_t *h_cfg, int sf0, int n_sf,
                                     const uint8_t *d_payload, uint32_t *d_ebits, int stop_phase, hipStream_t s);

/* subframes [sf0, sf0 + n_sf) of a batch whose payloads / e-bit words start at d_payload / d_ebits */
hipError_t oai4g_launch_encode(const cfg_dev_t *d_cfg, const cfg_dev_t *h_cfg, int sf0, int n_sf,
                               const uint8_t *d_payload, uint32_t *d_ebits, hipStream_t s)
{
  return launch_encode_impl(d_cfg, h_cfg, sf0, n_sf, d_payload, d_ebits, 99, s);
}

hipError_t oai4g_launch_encode_phase(const cfg_dev_t *d_cfg, const cfg_dev_t *h_cfg, int n_sf,
                                     const uint8_t *d_payload, uint32_t *d_ebits, int stop_phase, hipStream_t s)
{
  return launch_encode_impl(d_cfg, h_cfg, 0, n_sf, d_payload, d_ebits, stop_phase, s);
}

static hipError_t launch_encode_impl(const cfg_dev_t *d_cfg, const cfg_dev_t *h_cfg, int sf0, int n_sf,
                                     const uint8_t *d_payload, uint32_t *d_ebits, int stop_phase, hipStream_t s)
{
  if (n_sf <= 0) return hipSuccess;
  d_payload += (size_t)sf0 * h_cfg->n_cw * h_cfg->payload_stride;
  d_ebits += (size_t)sf0 * h_cfg->n_cw * h_cfg->ebits_words;
  size_t lds = enc_lds_bytes(h_cfg);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void *)k_encode, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void *)k_encode_debug, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  hipLaunchKernelGGL(k_encode, dim3(n_sf * h_cfg->n_cw), dim3(256), lds, s, d_cfg, d_payload, d_ebits, stop_phase,
                     (uint32_t)sf0);
  return hipGetLastError();
}

/* resident k_encode workgroups per CU at this configuration's dynamic LDS (diagnostic) */
hipError_t oai4g_encode_occupancy(const cfg_dev_t *h_cfg, int *blocks_per_cu, size_t *lds_bytes)
{
  *lds_bytes = enc_lds_bytes(h_cfg);
  (void)hipFuncSetAttribute((const void *)k_encode, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_encode, 256, *lds_bytes);
}

hipError_t oai4g_launch_encode_debug(const cfg_dev_t *d_cfg, const cfg_dev_t *h_cfg, int cw, int sf,
                                     const uint8_t *d_payload, enc_debug_t dbg, hipStream_t s)
{
  size_t lds = enc_lds_bytes(h_cfg) + 4 * ((size_t)h_cfg->lds_gold_words + 1);   /* + dbg_ebuf */
  (void)hipFuncSetAttribute((const void *)k_encode_debug, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipLaunchKernelGGL(k_encode_debug, dim3(1), dim3(256), lds, s, d_cfg, (uint32_t)sf, (uint32_t)cw, d_payload, dbg);
  return hipGetLastError();
}

/* =======================================================================================
 * Drop-in byte-layout kernels
 * ===================================================================================== */

/* crc24a/crc24b over an arbitrary bit length (crc_byte.c:117-153); wave 0 of one workgroup */
__global__ void __launch_bounds__(64) k_crc24(const uint8_t *__restrict__ in, int bitlen, uint32_t poly,
                                              uint32_t *__restrict__ out)
{
  __shared__ uint32_t tab[256];
  extern __shared__ uint8_t buf[];
  uint32_t nbytes = (uint32_t)bitlen / 8, rem = (uint32_t)bitlen % 8;
  for (uint32_t i = threadIdx.x; i < nbytes + (rem ? 1 : 0); i += blockDim.x) buf[i] = in[i];
  crc_table_init(tab, poly);
  __syncthreads();
  uint32_t reg = crc24_wave(buf, nbytes, poly, tab);
  if (threadIdx.x == 0) {
    if (rem) {
      /* crc = (crc << rem) ^ T[(byte >> (8-rem)) ^ (crc >> (32-rem))] on the <<8 register */
      uint32_t r32 = reg << 8;
      uint32_t idx = ((uint32_t)buf[nbytes] >> (8 - rem)) ^ (r32 >> (32 - rem));
      out[0] = (r32 << rem) ^ (tab[idx & 0xffu] << 8);
    } else {
      out[0] = reg << 8;
    }
  }
}

hipError_t oai4g_launch_crc24(const uint8_t *d_in, int bitlen, uint32_t poly_top, uint32_t *d_out, hipStream_t s)
{
  uint32_t nbytes = (uint32_t)(bitlen + 7) / 8;
  hipLaunchKernelGGL(k_crc24, dim3(1), dim3(64), nbytes + 4, s, d_in, bitlen, poly_top >> 8, d_out);
  return hipGetLastError();
}

/* threegpplte_turbo_encoder: c bytes -> d bytes (3K+12), one workgroup (waves 0/1 encode) */
__global__ void __launch_bounds__(256) k_turbo_bytes(const uint8_t *__restrict__ cin, uint32_t K, uint32_t f1,
                                                     uint32_t f2, uint8_t *__restrict__ dout)
{
  const uint32_t sw = 208;
  __shared__ uint32_t strm[3 * sw];
  __shared__ uint32_t tails[2];
  __shared__ enc_tabs_t tabs;
  uint32_t nw = (K + 31) >> 5;
  for (uint32_t i = threadIdx.x; i < 3 * sw; i += blockDim.x) strm[i] = 0;
  if (threadIdx.x < 128) {
    (&tabs.next[0][0])[threadIdx.x] = (&c_rsc.next[0][0])[threadIdx.x];
    (&tabs.par[0][0])[threadIdx.x] = (&c_rsc.par[0][0])[threadIdx.x];
    if (threadIdx.x < 64) (&tabs.apow[0][0])[threadIdx.x] = (&c_rsc.apow[0][0])[threadIdx.x];
    if (threadIdx.x < 8) tabs.zs[threadIdx.x] = c_rsc.zs[threadIdx.x];
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < nw; j += blockDim.x) {
    uint32_t le = 0;
    for (uint32_t q = 0; q < 4; q++) {
      uint32_t i = 4 * j + q;
      le |= (uint32_t)(i < K / 8 ? cin[i] : 0) << (8 * q);
    }
    uint32_t wv = bytes_to_seq(le);
    if (32 * (j + 1) > K) wv &= (1u << (K - 32 * j)) - 1u;
    strm[j] = wv;
  }
  __syncthreads();
  __shared__ uint32_t ilv[OAI4G_MAX_CHUNKS];
  const uint32_t d2 = (2 * f2) % K;
  for (uint32_t j = threadIdx.x; j < nw; j += blockDim.x) ilv[j] = qpp_gather_word(strm, K, qpp_start(K, f1, f2, j), d2, j);
  __syncthreads();
  uint32_t wave = threadIdx.x >> 6;
  if (wave < 2) turbo_segment(wave ? ilv : strm, strm + (1 + wave) * sw, K, &tails[wave], &tabs);
  __syncthreads();
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
    uint32_t j = colperm(col) + 32 * row;
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

/* deterministic payload: 8-byte word w = splitmix64 output for the counter seed + gamma (w + 1) */
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

/* =======================================================================================
 * PMC calibration (diagnostic): stream a known byte count with the access width the
 * pipeline kernels use (4 B per lane, coalesced), mode 0 = read, 1 = write.  rocprofv3's
 * FETCH_SIZE / WRITE_SIZE of this dispatch calibrate the counters (MI355X_MICROARCH.md:
 * "other access widths are uncalibrated").
 * ===================================================================================== */
__global__ void __launch_bounds__(256) k_diag_stream(const uint32_t *__restrict__ src, uint32_t *__restrict__ dst,
                                                     size_t n_words, int mode)
{
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (mode == 1) {
    for (; i < n_words; i += stride) dst[i] = (uint32_t)i;
    return;
  }
  uint32_t acc = 0;
  for (; i < n_words; i += stride) acc ^= src[i];
  if (acc == 0x9e3779b9u) dst[0] = acc;    /* keeps the loads live; practically never stores */
}

hipError_t oai4g_launch_diag_stream(const void *src, void *dst, size_t bytes, int mode, hipStream_t s)
{
  hipLaunchKernelGGL(k_diag_stream, dim3(4096), dim3(256), 0, s, (const uint32_t *)src, (uint32_t *)dst, bytes / 4,
                     mode);
  return hipGetLastError();
}

