/*
 * Host side of openair4g_amd: C ABI (include/oai4g.h), configuration derivation, drop-in
 * entry points and the batched transmit path.  All arithmetic on samples / bits runs in the
 * gfx950 kernels; this file only derives parameters (what the reference recomputes on every
 * call: segmentation, rate-matching geometry, RE maps), moves buffers and launches.
 */
#include <hip/hip_runtime.h>
#include <math.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>
#include <map>
#include <mutex>
#include <vector>

#include "../../include/oai4g.h"
#include "../../include/oai4g_qpp.h"
#include "../../include/oai4g_tbs.h"
#include "oai4g_internal.h"

/* ------------------------------------------------------------------------------------------
 * errors
 * ---------------------------------------------------------------------------------------- */
static thread_local char g_err[512] = "";

static void set_err(const char *fmt, ...)
{
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" const char *oai4g_last_error(void) { return g_err; }

/* the error slot for the library's other translation units (oai4g_dist.cpp) */
void oai4g_set_error(const char *fmt, ...)
{
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

#define HCK(call, ret)                                                                          \
  do {                                                                                          \
    hipError_t e_ = (call);                                                                     \
    if (e_ != hipSuccess) {                                                                     \
      set_err("%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), __FILE__, __LINE__);       \
      fprintf(stderr, "[openair4g_amd] %s\n", g_err);                                           \
      return ret;                                                                               \
    }                                                                                           \
  } while (0)

/* ------------------------------------------------------------------------------------------
 * global device tables: twiddles, Gold jump-ahead
 * ---------------------------------------------------------------------------------------- */
static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static int g_init_status = -1;
static char g_init_err[512] = "";
static uint32_t *g_tw = nullptr, *g_twf = nullptr, *g_gx1 = nullptr, *g_gx2j = nullptr;
static int g_n_cu = 256;
static uint32_t h_gx1[OAI4G_GOLD_LANES], h_gx2j[OAI4G_GOLD_LANES * 32];

static void twiddle_host(int N, int m, int16_t *re, int16_t *im)
{
  /* W_N^m in Q15: (floor(32767 cos), floor(-32767 sin)) — reproduces lte_dfts.c tw* tables */
  double a = 2.0 * M_PI * (double)m / (double)N;
  *re = (int16_t)floor(32767.0 * cos(a));
  *im = (int16_t)floor(-32767.0 * sin(a));
}

/* forward DFT operand pair (a, b) with x * W = (dot2(x, a), dot2(x, b)): a = (Wr, -Wi), b = (Wi, Wr)
 * for cmult (tw1024, tw2048) and the packed_cmult2 tables tw16a/b … tw512a/b; tw256a alone holds
 * floor(32767 sin) as its second entry (lte_dfts.c:2162 vs :2167) */
static void dft_twiddle_ab_host(int N, int m, int16_t a[2], int16_t b[2])
{
  int16_t wr, wi;
  twiddle_host(N, m, &wr, &wi);
  a[0] = wr;
  a[1] = (N == 256) ? (int16_t)floor(32767.0 * sin(2.0 * M_PI * (double)m / (double)N)) : (int16_t)-wi;
  b[0] = wi;
  b[1] = wr;
}

static void gold_step_h(uint32_t *x1, uint32_t *x2)
{
  *x1 = (*x1 >> 1) ^ (*x1 >> 4);
  *x1 = *x1 ^ (*x1 << 31) ^ (*x1 << 28);
  *x2 = (*x2 >> 1) ^ (*x2 >> 2) ^ (*x2 >> 3) ^ (*x2 >> 4);
  *x2 = *x2 ^ (*x2 << 31) ^ (*x2 << 30) ^ (*x2 << 29) ^ (*x2 << 28);
}

/* lte_gold (LTE_REFSIG/lte_gold.c:52-93): CRS Gold words [ns][pilot l][14] */
/* 14 CRS Gold words of slot ns, symbol lsym of the slot: c_init = 2^10 (7(ns+1) + lsym + 1)
 * (2 Nid + 1) + 2 Nid + N_CP (lte_gold.c:52-93; lsym = 1 for the port-2/3 extension) */
static void gold_words_h(const oai4g_frame_parms_t *fp, uint32_t ns, uint32_t lsym, uint32_t w[14])
{
  const uint32_t Ncp = 1 - fp->Ncp, Nid = fp->Nid_cell;
  uint32_t x1 = 1u + (1u << 31);
  uint32_t x2 = Ncp + (Nid << 1) + (((1 + (Nid << 1)) * (1 + lsym + 7 * (1 + ns))) << 10);
  x2 ^= (x2 ^ (x2 >> 1) ^ (x2 >> 2) ^ (x2 >> 3)) << 31;
  for (int n = 1; n < 50; n++) gold_step_h(&x1, &x2);
  for (int n = 0; n < 14; n++) {
    gold_step_h(&x1, &x2);
    w[n] = x1 ^ x2;
  }
}

static void lte_gold_table_h(const oai4g_frame_parms_t *fp, uint32_t t[20][2][14])
{
  for (uint32_t ns = 0; ns < 20; ns++)
    for (uint32_t l = 0; l < 2; l++) gold_words_h(fp, ns, (fp->Ncp == 0 ? 4 : 3) * l, t[ns][l]);
}

/* CRS pilot RE of port p, pilot l (0: symbol 0 of the slot, 1: symbol 4 / 3), index m
 * (lte_dl_cell_spec.c:147-200): subcarrier bin and QPSK index into qpsk[] */
static uint32_t crs_bin(const oai4g_frame_parms_t *fp, uint32_t p, uint32_t l, uint32_t m)
{
  const uint32_t nu = (p == 0) ? (l == 0 ? 0 : 3) : (l == 0 ? 3 : 0);
  uint32_t k = nu + fp->nushift;
  if (k > 5) k -= 6;
  k += fp->first_carrier_offset + 6 * m;
  if (k >= fp->ofdm_symbol_size) k = k + 1 - fp->ofdm_symbol_size;     /* DC skip */
  return k;
}
/* CRS RE of port 2/3 (4-TX extension, 36.211 6.10.1.2): symbol 1 of slot ns, nu = 3 (ns mod 2)
 * for p = 2, 3 + 3 (ns mod 2) for p = 3 */
static uint32_t crs_bin_p23(const oai4g_frame_parms_t *fp, uint32_t p, uint32_t ns, uint32_t m)
{
  uint32_t k = ((p == 2 ? 0u : 3u) + 3u * (ns & 1u) + fp->nushift) % 6u + fp->first_carrier_offset + 6 * m;
  if (k >= fp->ofdm_symbol_size) k = k + 1 - fp->ofdm_symbol_size;
  return k;
}
static uint32_t crs_qpsk(int16_t amp, uint32_t idx)
{
  const int16_t a = (int16_t)((amp * 23170) >> 15);                  /* ONE_OVER_SQRT2_Q15 */
  const int16_t re = (idx & 1) ? (int16_t)-a : a, im = (idx & 2) ? (int16_t)-a : a;
  return (uint16_t)re | ((uint32_t)(uint16_t)im << 16);
}

static bool g_init_done = false;
static int g_device = 0;                           /* the device the tables live on (do_init) */
static void do_init(void)
{
  g_init_done = true;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0) {
    snprintf(g_init_err, sizeof(g_init_err), "no HIP device available (%s)",
             e == hipSuccess ? "0 devices" : hipGetErrorString(e));
    g_init_status = -1;
    return;
  }
  int dev = 0;
  hipGetDevice(&dev);
  g_device = dev;                                  /* every later thread binds to this device */
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess || strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    snprintf(g_init_err, sizeof(g_init_err), "device %d is not gfx950 (%s)", dev, prop.gcnArchName);
    g_init_status = -2;
    return;
  }
  g_n_cu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  /* twiddles */
  std::vector<uint32_t> tw(2 * OAI4G_TW_TOTAL);   /* t, then the rotated companions (-t.im, t.re) */
  const int sizes[] = {4, 6, 7, 8, 9, 10, 11};
  for (int log2s : sizes) {
    int N = 1 << log2s;
    uint32_t off = oai4g_tw_offset(log2s);
    for (int m = 0; m < N; m++) {
      int16_t re, im;
      twiddle_host(N, m, &re, &im);
      tw[off + m] = (uint16_t)re | ((uint32_t)(uint16_t)im << 16);
      tw[OAI4G_TW_TOTAL + off + m] = (uint16_t)(int16_t)(-im) | ((uint32_t)(uint16_t)re << 16);
    }
  }
  std::vector<uint32_t> twf(2 * OAI4G_TW_TOTAL);  /* forward: a, then b */
  for (int log2s : sizes) {
    int N = 1 << log2s;
    uint32_t off = oai4g_tw_offset(log2s);
    for (int m = 0; m < N; m++) {
      int16_t a[2], b[2];
      dft_twiddle_ab_host(N, m, a, b);
      twf[off + m] = (uint16_t)a[0] | ((uint32_t)(uint16_t)a[1] << 16);
      twf[OAI4G_TW_TOTAL + off + m] = (uint16_t)b[0] | ((uint32_t)(uint16_t)b[1] << 16);
    }
  }
  /* Gold: x1 after 50+S l word steps; x2 step-matrix powers M2^(50+S l) (columns), S = OAI4G_GOLD_STRIDE */
  uint32_t x1 = 1u + (1u << 31), cols[32];
  for (int b = 0; b < 32; b++) cols[b] = 1u << b;
  int steps_done = 0;
  for (int l = 0; l < OAI4G_GOLD_LANES; l++) {
    int target = 50 + OAI4G_GOLD_STRIDE * l;
    while (steps_done < target) {
      uint32_t dummy = 0;
      gold_step_h(&x1, &dummy);
      for (int b = 0; b < 32; b++) {
        uint32_t z = 0;
        gold_step_h(&z, &cols[b]);
      }
      steps_done++;
    }
    h_gx1[l] = x1;
    for (int b = 0; b < 32; b++) h_gx2j[OAI4G_GOLD_LANES * b + l] = cols[b];   /* [b][lane]: coalesced */
  }
  if (hipMalloc(&g_tw, tw.size() * 4) != hipSuccess || hipMalloc(&g_twf, twf.size() * 4) != hipSuccess ||
      hipMemcpy(g_twf, twf.data(), twf.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMalloc(&g_gx1, sizeof(h_gx1)) != hipSuccess ||
      hipMalloc(&g_gx2j, sizeof(h_gx2j)) != hipSuccess ||
      hipMemcpy(g_tw, tw.data(), tw.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(g_gx1, h_gx1, sizeof(h_gx1), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(g_gx2j, h_gx2j, sizeof(h_gx2j), hipMemcpyHostToDevice) != hipSuccess) {
    snprintf(g_init_err, sizeof(g_init_err), "device table upload failed");
    g_init_status = -3;
    return;
  }
  g_init_status = 0;
}

extern "C" int oai4g_set_device(int device)
{
  /* before the first oai4g_init: the process's rank drives `device` (one process per GPU) */
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
    set_err("set_device: device %d of %d", device, n);
    return -1;
  }
  if (g_init_done && g_device != device) {
    set_err("set_device: the library is already initialised on device %d", g_device);
    return -1;
  }
  HCK(hipSetDevice(device), -1);
  return 0;
}

/* hipSetDevice is per thread: every library call binds the calling thread to the library's device
 * before it creates streams, buffers or launches (the device tables live there).  Checked on every
 * call, not cached: the application may switch the thread's device in between (hipSetDevice,
 * torch.cuda.set_device).  The binding stays in effect after the call (include/oai4g.h).  Called by
 * NEED_INIT. */
static int bind_thread_device(void)
{
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess) return -1;
  if (cur != g_device && hipSetDevice(g_device) != hipSuccess) {
    set_err("thread bind: hipSetDevice(%d) failed", g_device);
    return -1;
  }
  return 0;
}
int oai4g_bind_thread(void) { return bind_thread_device(); }

extern "C" int oai4g_init(void)
{
  pthread_once(&g_once, do_init);
  if (g_init_status != 0) {
    set_err("openair4g_amd: %s", g_init_err);
    fprintf(stderr, "[openair4g_amd] %s\n", g_err);
  }
  return g_init_status;
}

extern "C" int oai4g_device_name(char *buf, int len)
{
  if (oai4g_init() != 0) return -1;
  int dev = 0;
  hipGetDevice(&dev);
  hipDeviceProp_t prop;
  HCK(hipGetDeviceProperties(&prop, dev), -1);
  snprintf(buf, len, "%s (%s, %d CUs)", prop.name, prop.gcnArchName, prop.multiProcessorCount);
  return 0;
}

/* ------------------------------------------------------------------------------------------
 * per-thread scratch (drop-in path): one stream + one growable device buffer
 * ---------------------------------------------------------------------------------------- */
struct scratch_t {
  hipStream_t s = nullptr;
  uint8_t *buf = nullptr;
  size_t cap = 0;
};
static thread_local scratch_t g_scr;

static uint8_t *scratch(size_t bytes)
{
  if (!g_scr.s && hipStreamCreateWithFlags(&g_scr.s, hipStreamNonBlocking) != hipSuccess) return nullptr;
  if (bytes > g_scr.cap) {
    if (g_scr.buf) hipFree(g_scr.buf);
    size_t cap = bytes < (64u << 20) ? (64u << 20) : bytes;
    if (hipMalloc(&g_scr.buf, cap) != hipSuccess) {
      g_scr.buf = nullptr;
      g_scr.cap = 0;
      return nullptr;
    }
    g_scr.cap = cap;
  }
  return g_scr.buf;
}

#define NEED_INIT(ret)                                          \
  do {                                                          \
    if (oai4g_init() != 0 || bind_thread_device() != 0) return ret; \
  } while (0)

/* ------------------------------------------------------------------------------------------
 * parameter helpers (lte_parms.c, lte_mcs.c)
 * ---------------------------------------------------------------------------------------- */
extern "C" int oai4g_init_frame_parms(oai4g_frame_parms_t *fp, uint16_t N_RB_DL, uint16_t Nid_cell, uint8_t Ncp,
                                      uint8_t nb_antennas_tx, uint8_t mode1_flag, uint8_t frame_type)
{
  memset(fp, 0, sizeof(*fp));
  fp->N_RB_DL = N_RB_DL;
  fp->Nid_cell = Nid_cell;
  fp->Ncp = Ncp;
  fp->nushift = (uint8_t)(Nid_cell % 6);
  fp->nb_antennas_tx = nb_antennas_tx;
  fp->mode1_flag = mode1_flag;
  fp->frame_type = frame_type;
  uint16_t cp0 = Ncp ? 512 : 160, cp = Ncp ? 512 : 144;
  fp->symbols_per_tti = Ncp ? 12 : 14;
  int sh;
  switch (N_RB_DL) {
  case 100: fp->ofdm_symbol_size = 2048; fp->log2_symbol_size = 11; sh = 0; break;
  case 50: fp->ofdm_symbol_size = 1024; fp->log2_symbol_size = 10; sh = 1; break;
  case 25: fp->ofdm_symbol_size = 512; fp->log2_symbol_size = 9; sh = 2; break;
  case 15: fp->ofdm_symbol_size = 256; fp->log2_symbol_size = 8; sh = 3; break;
  case 6: fp->ofdm_symbol_size = 128; fp->log2_symbol_size = 7; sh = 4; break;
  default: set_err("init_frame_parms: unsupported N_RB_DL %u", N_RB_DL); return -1;
  }
  fp->samples_per_tti = 30720u >> sh;
  fp->first_carrier_offset = (uint16_t)(fp->ofdm_symbol_size - 6 * N_RB_DL);
  fp->nb_prefix_samples = (uint16_t)(cp >> sh);
  fp->nb_prefix_samples0 = (uint16_t)(cp0 >> sh);
  fp->phich_resource = 6;                 /* Ng = one (dlsim.c:138) */
  fp->phich_duration = 0;
  fp->tdd_config = 3;
  fp->nb_antennas_tx_eNB = nb_antennas_tx; /* dlsim.c:137 */
  return 0;
}

extern "C" uint8_t oai4g_get_Qm(uint8_t mcs) { return mcs < 10 ? 2 : (mcs < 17 ? 4 : 6); }

/* get_Qm_ul (lte_mcs.c:57) */
extern "C" uint8_t oai4g_get_Qm_ul(uint8_t mcs) { return mcs < 11 ? 2 : (mcs < 21 ? 4 : 6); }

/* get_I_TBS (lte_mcs.c:69-82): 36.213 Table 7.1.7.1-1 */
extern "C" uint8_t oai4g_get_I_TBS(uint8_t mcs)
{
  if (mcs < 10) return mcs;
  if (mcs == 10) return 9;
  if (mcs < 17) return (uint8_t)(mcs - 1);
  if (mcs == 17) return 15;
  return (uint8_t)(mcs - 2);
}

/* get_I_TBS_UL (lte_mcs.c:84-95): its `I_MCS == 10` branch is unreachable after `<= 10`, kept as is */
extern "C" uint8_t oai4g_get_I_TBS_UL(uint8_t mcs)
{
  if (mcs <= 10) return mcs;
  if (mcs < 21) return (uint8_t)(mcs - 1);
  return (uint8_t)(mcs - 2);
}

/* TBStable[I_TBS][N_PRB-1] (dlsch_tbs_full.h:34) in bits; 0 outside the table */
extern "C" uint32_t oai4g_tbs_bits(uint8_t I_TBS, uint16_t nb_rb)
{
  if (I_TBS > 26 || nb_rb < 1 || nb_rb > 110) return 0;
  return oai4g_tbs_by_prb[nb_rb - 1][I_TBS];
}

/* get_TBS_DL (lte_mcs.c:118-137): transport block size in BYTES (TBStable >> 3), 0 for nb_rb = 0
 * or mcs >= 29 — the reference's unit, which its callers multiply back by 8 */
extern "C" uint32_t oai4g_get_TBS_DL(uint8_t mcs, uint16_t nb_rb)
{
  if (nb_rb == 0 || mcs >= 29) return 0;
  return oai4g_tbs_bits(oai4g_get_I_TBS(mcs), nb_rb) >> 3;
}

/* get_TBS_UL (lte_mcs.c:137-155), same unit */
extern "C" uint32_t oai4g_get_TBS_UL(uint8_t mcs, uint16_t nb_rb)
{
  if (nb_rb == 0 || mcs >= 29) return 0;
  return oai4g_tbs_bits(oai4g_get_I_TBS_UL(mcs), nb_rb) >> 3;
}

static int rb_bit(const uint32_t *rb_alloc, int rb)
{
  if (rb < 32) return (rb_alloc[0] >> rb) & 1;
  if (rb < 64) return (rb_alloc[1] >> (rb - 32)) & 1;
  if (rb < 96) return (rb_alloc[2] >> (rb - 64)) & 1;
  if (rb < 100) return (rb_alloc[3] >> (rb - 96)) & 1;
  return 0;
}

/* adjust_G (lte_mcs.c:249-334) */
static int adjust_G(const oai4g_frame_parms_t *fp, const uint32_t *rb_alloc, int Qm, int subframe)
{
  if (subframe != 0 && subframe != 5 && subframe != 6) return 0;
  int re = 0, half = fp->N_RB_DL >> 1;
  if (fp->N_RB_DL & 1) {
    for (int rb = half - 3; rb <= half + 3; rb++)
      if (rb_bit(rb_alloc, rb)) re += (rb == half - 3 || rb == half + 3) ? 6 : 12;
  } else {
    for (int rb = half - 3; rb < half + 3; rb++)
      if (rb_bit(rb_alloc, rb)) re += 12;
  }
  int Ncp = fp->Ncp;
  if (subframe == 0) {
    if (fp->frame_type == 1)
      return fp->mode1_flag == 0 ? (-Ncp + 14) * re * Qm / 3 : (-Ncp + 29) * re * Qm / 6;
    return fp->mode1_flag == 0 ? (-Ncp + 17) * re * Qm / 3 : (-Ncp + 35) * re * Qm / 6;
  }
  if (subframe == 5) return (fp->frame_type == 0 ? 2 : 1) * re * Qm;
  if (subframe == 6 && fp->frame_type == 1) return re * Qm;
  return 0;
}

/* get_G (lte_mcs.c:336-368); PMCH subframes are not part of this path */
extern "C" int oai4g_get_G(const oai4g_frame_parms_t *fp, uint16_t nb_rb, const uint32_t *rb_alloc,
                           uint8_t mod_order, uint8_t Nl, uint8_t num_pdcch_symbols, int frame, uint8_t subframe)
{
  (void)frame;
  int adj = adjust_G(fp, rb_alloc, mod_order, subframe);
  int nd = fp->Ncp == 0 ? 11 : 9;
  if (fp->mode1_flag == 0) return (((int)nb_rb * mod_order * ((nd - num_pdcch_symbols) * 12 + 3 * 8)) - adj) * Nl;
  return ((int)nb_rb * mod_order * ((nd - num_pdcch_symbols) * 12 + 3 * 10)) - adj;
}

/* lte_segmentation parameter math (lte_segmentation.c:39-126) */
static int seg_params(uint32_t B, uint32_t *C, uint32_t *Cplus, uint32_t *Cminus, uint32_t *Kplus, uint32_t *Kminus,
                      uint32_t *F, uint32_t *L)
{
  uint32_t Bp;
  if (B <= 6144) { *L = 0; *C = 1; Bp = B; }
  else { *L = 24; *C = (B + (6144 - 24) - 1) / (6144 - 24); Bp = B + *C * 24; }
  if (*C > OAI4G_MAX_SEGMENTS) {
    printf("lte_segmentation.c: too many segments %u\n", *C);
    return -1;
  }
  uint32_t per = Bp / *C;
  if (per <= 40) { *Kplus = 40; *Kminus = 0; }
  else if (per <= 512) { *Kplus = (per >> 3) << 3; *Kminus = per - 8; }
  else if (per <= 1024) { *Kplus = ((per + 15) >> 4) << 4; *Kminus = *Kplus - 16; }
  else if (per <= 2048) { *Kplus = ((per + 31) >> 5) << 5; *Kminus = *Kplus - 32; }
  else if (per <= 6144) { *Kplus = ((per + 63) >> 6) << 6; *Kminus = *Kplus - 64; }
  else {
    printf("lte_segmentation.c: Illegal codeword size !!!\n");
    return -1;
  }
  if (*C == 1) { *Cplus = 1; *Kminus = 0; *Cminus = 0; }
  else { *Cminus = (*C * *Kplus - Bp) / (*Kplus - *Kminus); *Cplus = *C - *Cminus; }
  *F = *Cplus * *Kplus + *Cminus * *Kminus - Bp;
  return 0;
}

/* NULL positions of the sub-block interleaver output for block size K (by simulating
 * sub_block_interleaving_turbo on a marker input: lte_rate_matching.c:51-130) */
static const uint8_t k_colperm[32] = {0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30,
                                      1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31};
static int null_positions(uint32_t K, uint16_t *out, uint32_t maxn)
{
  uint32_t D = K + 4, R = (D + 31) >> 5, Kpi = R << 5, ND = Kpi - D;
  std::vector<uint8_t> d(96 + 3 * D + 16, 0);
  memset(d.data(), OAI4G_LTE_NULL, 96);
  uint8_t *dd = d.data() + 96;
  dd[3 * D + 2] = dd[2];
  const uint8_t *base = dd - 3 * ND;
  std::vector<uint8_t> w(3 * Kpi);
  uint32_t k = 0;
  for (uint32_t col = 0; col < 32; col++)
    for (uint32_t row = 0; row < R; row++, k++) {
      uint32_t j = k_colperm[col] + 32 * row;
      w[k] = base[3 * j];
      w[Kpi + 2 * k] = base[3 * j + 1];
      w[Kpi + 2 * k + 1] = base[3 * j + 5];
    }
  if (ND > 0) w[3 * Kpi - 1] = OAI4G_LTE_NULL;
  uint32_t n = 0;
  for (uint32_t p = 0; p < 3 * Kpi; p++)
    if (w[p] == OAI4G_LTE_NULL) {
      if (n >= maxn) return -1;
      out[n++] = (uint16_t)p;
    }
  return (int)n;
}

/* GF(2)[x] products modulo a CRC-24 polynomial (24-bit register, x^24 implicit) */
static uint32_t crc_mulmod_h(uint32_t a, uint32_t b, uint32_t poly)
{
  uint32_t r = 0;
  for (int i = 23; i >= 0; i--) {
    r <<= 1;
    if (r & 0x1000000u) r ^= 0x1000000u | poly;
    if ((b >> i) & 1u) r ^= a;
  }
  return r;
}

static uint32_t crc_xpow8_h(uint64_t n, uint32_t poly)   /* x^(8n) mod P */
{
  uint32_t result = 1, base = 0x100;
  while (n) {
    if (n & 1u) result = crc_mulmod_h(result, base, poly);
    base = crc_mulmod_h(base, base, poly);
    n >>= 1;
  }
  return result;
}

/* tab[d][k][v] = (v * x^(4k)) * x^(8*per*2^d) mod P, so a*m_d = xor_k tab[d][k][nibble_k(a)] */
/* nibble tables of the two-level combine: [0][j] = x^(8 per j), [1][j] = x^(64 per j) mod P */
static void crc_mul_tables2(uint32_t per, uint32_t poly, uint32_t (*tab)[8][96])
{
  for (int lv = 0; lv < 2; lv++)
    for (uint32_t j = 0; j < 8; j++) {
      const uint32_t m = crc_xpow8_h((uint64_t)per * j * (lv ? 8u : 1u), poly);
      for (int k = 0; k < 6; k++)
        for (uint32_t v = 0; v < 16; v++) tab[lv][j][16 * k + v] = crc_mulmod_h((v << (4 * k)) & 0xffffffu, m, poly);
    }
}

static void crc_mul_tables(uint32_t per, int levels, uint32_t poly, uint32_t (*tab)[6][16])
{
  for (int d = 0; d < levels; d++) {
    uint32_t m = crc_xpow8_h((uint64_t)per << d, poly);
    for (int k = 0; k < 6; k++)
      for (uint32_t v = 0; v < 16; v++) tab[d][k][v] = crc_mulmod_h((v << (4 * k)) & 0xffffffu, m, poly);
  }
}

/* QAM tables (dlsch_modulation.c:79-103, 1223-1246).  The raw tables are int (LTE_TRANSPORT/
 * vars.h:72): the outer 64-QAM level 35393 exceeds int16 and is only narrowed after the scaling. */
static void qam_tables_scaled(int Qm, int16_t amp, int16_t srho_a, int16_t srho_b, bool alamouti, cw_dev_t &c)
{
  int32_t q16[4], q64[8];
  for (int a = -1; a <= 1; a += 2)
    for (int b = -1; b <= 1; b += 2) {
      q16[(1 + a) + (1 + b) / 2] = -a * (20724 + b * 10362);
      for (int cc = -1; cc <= 1; cc += 2)
        q64[(1 + a) * 2 + (1 + b) + (1 + cc) / 2] = -a * (20225 + b * (10112 + cc * 5056));
    }
  int16_t amp_a = (int16_t)(((int32_t)amp * srho_a) >> 13), amp_b = (int16_t)(((int32_t)amp * srho_b) >> 13);
  c.qpsk_a = (int16_t)((amp_a * 23170) >> 15);
  c.qpsk_b = (int16_t)((amp_b * 23170) >> 15);
  /* ALAMOUTI normalises for two antennas: amp/sqrt2 times the raw table (:364, :398-399) */
  const int16_t sa = alamouti ? (int16_t)(((int32_t)amp_a * 23170) >> 15) : amp_a;
  const int16_t sb = alamouti ? (int16_t)(((int32_t)amp_b * 23170) >> 15) : amp_b;
  for (int i = 0; i < 8; i++) {
    const int32_t v = Qm == 4 ? q16[i & 3] : q64[i];
    c.qam_a[i] = (int16_t)((v * sa) >> 15);
    c.qam_b[i] = (int16_t)((v * sb) >> 15);
  }
  /* ALAMOUTI QPSK (:371-386): +-gain, then * ONE_OVER_SQRT2_Q15 >> 15 */
  const int16_t g[2] = {c.qpsk_a, c.qpsk_b};
  for (int pil = 0; pil < 2; pil++) {
    c.alm_qpsk[pil][0] = (int16_t)(((int32_t)g[pil] * 23170) >> 15);
    c.alm_qpsk[pil][1] = (int16_t)(((int32_t)(int16_t)-g[pil] * 23170) >> 15);
  }
}

/* ------------------------------------------------------------------------------------------
 * Range check for k_modofdm's no-saturation IDFT forms (ibfly4_shr1_ns and r4inv<NS>,
 * oai4g_dft_prims.h).  The 2048-point transform is DIT: a 64-level value (before its >> 3) is part
 * of a 64-point DFT over the subcarriers of one residue class mod 32, a 256-level value one of a
 * 256-point DFT over a class mod 8 scaled by 1/8 (the 64-level's shift), a 1024-level value one over
 * a class mod 2 scaled by 1/16, a 2048-level sum (before mulhi) one over every subcarrier scaled by
 * 1/32; the leaf's are parts of 16-point DFTs, inside the 64-level's classes.
 * Every twiddle has modulus < 1 (Q15, |t| <= 32767.7), so a value's modulus is at most (occupied
 * subcarriers of its class) x (largest input modulus) x scale, plus the truncations of the levels
 * below (< 64 in modulus).  Every transform input is a QAM word (TM1), a sign-flipped / swapped one
 * (ALAMOUTI), a CDD pair (floor((x0 + x1) / 2), +-floor((x0 - x1) / 2)) of two (LARGE_CDD) or a halved
 * one (4-port CDD): components <= the largest level V of the configuration's QAM / QPSK tables,
 * modulus <= sqrt(2) V, and only 12 N_RB_DL subcarriers carry anything.  When the four bounds stay inside
 * int16 with a margin of 128, no add of those levels saturates or wraps, packs_epi32 never clamps
 * and no operand is -32768, whatever the bits: the no-saturation forms are then the reference's
 * arithmetic.  (C3: V = 553, R = 782.1; 39 R + 128 = 30629, 151 R / 8 + 128 = 14890, 601 R / 16 +
 * 128 = 29505, 1201 R / 32 + 128 = 29480.)  With CRS or static REs (PCFICH, PDCCH, PHICH, PSS, SSS,
 * PBCH) in the grid, V also covers their components (v_static: the largest over the CRS table and the
 * static-RE table, re-checked whenever oai4g_tx_config_set_control / _set_common rebuild it).
 * OAI4G_MOD_SAT (test hook) keeps the saturating forms.
 * ---------------------------------------------------------------------------------------- */
static uint32_t mod_nosat_ok(const cfg_dev_t &h, int v_static)
{
  if (h.log2N != 11 || h.nsymb != 14 || getenv("OAI4G_MOD_SAT")) return 0;
  int v = v_static;
  for (uint32_t cw = 0; cw < h.n_cw; cw++) {
    const cw_dev_t &c = h.cw[cw];
    for (int i = 0; i < 8; i++) v = std::max(v, std::max(std::abs((int)c.qam_a[i]), std::abs((int)c.qam_b[i])));
    v = std::max(v, std::max(std::abs((int)c.qpsk_a), std::abs((int)c.qpsk_b)));
    for (int i = 0; i < 2; i++)
      v = std::max(v, std::max(std::abs((int)c.alm_qpsk[i][0]), std::abs((int)c.alm_qpsk[i][1])));
  }
  const double R = std::sqrt(2.0) * v, band = 12.0 * h.N_RB_DL;
  const double c32 = std::ceil(band / 32) + 1, c8 = std::ceil(band / 8) + 1, c2 = std::ceil(band / 2) + 1;
  return (c32 * R + 128 <= 32767 && c8 * R / 8 + 128 <= 32767 && c2 * R / 16 + 128 <= 32767 &&
          (band + 1) * R / 32 + 128 <= 32767) ? 1u : 0u;
}

static int packed_iq_max(const std::vector<uint32_t> &t)
{
  int v = 0;
  for (uint32_t w : t) v = std::max(v, std::max(std::abs((int)(int16_t)(w & 0xFFFFu)), std::abs((int)(int16_t)(w >> 16))));
  return v;
}

/* ------------------------------------------------------------------------------------------
 * RE map: restatement of dlsch_modulation's control flow (dlsch_modulation.c:1258-1493 and
 * allocate_REs_in_RB :139-249, 745-748) producing, per symbol, the data-RE order.
 * Returns REs allocated, or -1 for an unsupported mode.
 * ---------------------------------------------------------------------------------------- */
static int not_pilot(int pilots, int re, int nushift, int use2nd)
{
  int off = (pilots == 2) ? 3 : 0, v = nushift % 3;
  if (pilots == 0) return 1;
  if (use2nd) return (re != nushift + off) && (re != ((nushift + 6 + off) % 12));
  return (re != v) && (re != v + 6) && (re != v + 3) && (re != v + 9);
}

static int build_remap(const oai4g_frame_parms_t *fp, const uint32_t *rb_alloc, int num_pdcch, int subframe,
                       int mimo_mode, uint16_t *remap /* [14][N] */, uint32_t *symbase /* [14] */,
                       int *re_alloc /* the reference's re_allocated */)
{
  const bool alm = mimo_mode == OAI4G_ALAMOUTI;
  int ralloc = 0;
  int N = fp->ofdm_symbol_size, nsymb = fp->Ncp == 0 ? 14 : 12, half = fp->N_RB_DL >> 1;
  int use2nd = fp->mode1_flag == 1;
  for (int i = 0; i < 14 * N; i++) remap[i] = 0xFFFF;
  uint32_t total = 0;
  for (int l = 0; l < 14; l++) symbase[l] = 0;
  for (int l = num_pdcch; l < nsymb; l++) {
    symbase[l] = total;
    uint32_t idx = 0;
    int pilots;
    if (fp->Ncp == 0) pilots = (l == 4 || l == 11) ? 2 : (l == 7 ? 1 : 0);
    else pilots = (l == 3 || l == 9) ? 2 : (l == 6 ? 1 : 0);
    if (fp->nb_antennas_tx == 4 && l % (nsymb >> 1) == 1) pilots = 3;   /* port-2/3 CRS (4-TX extension) */
    int re_offset = fp->first_carrier_offset;
    for (int rb = 0; rb < fp->N_RB_DL; rb++) {
      int alloc = rb_bit(rb_alloc, rb), skip_half = 0, skip_dc = 0;
      if (fp->N_RB_DL & 1) {
        skip_dc = (rb == half);
        if (subframe == 0 && rb > half - 3 && rb < half + 3 && l >= (nsymb >> 1) && l < (nsymb >> 1) + 4) alloc = 0;
        if (subframe == 0 && rb == half - 3 && l >= (nsymb >> 1) && l < (nsymb >> 1) + 4) skip_half = 1;
        else if (subframe == 0 && rb == half + 3 && l >= (nsymb >> 1) && l < (nsymb >> 1) + 4) skip_half = 2;
        if (fp->frame_type == 1) {
          if ((subframe == 0 || subframe == 5) && rb > half - 3 && rb < half + 3 && l == nsymb - 1) alloc = 0;
          if ((subframe == 0 || subframe == 5) && rb == half - 3 && l == nsymb - 1) skip_half = 1;
          else if ((subframe == 0 || subframe == 5) && rb == half + 3 && l == nsymb - 1) skip_half = 2;
          if ((subframe == 1 || subframe == 6) && rb > half - 3 && rb < half + 3 && l == 2) alloc = 0;
          if ((subframe == 1 || subframe == 6) && rb == half - 3 && l == 2) skip_half = 1;
          else if ((subframe == 1 || subframe == 6) && rb == half + 3 && l == 2) skip_half = 2;
        } else {
          int ls = (nsymb >> 1) - 1, lp = (nsymb >> 1) - 2;
          if ((subframe == 0 || subframe == 5) && rb > half - 3 && rb < half + 3 && l == ls) alloc = 0;
          if ((subframe == 0 || subframe == 5) && rb == half - 3 && l == ls) skip_half = 1;
          else if ((subframe == 0 || subframe == 5) && rb == half + 3 && l == ls) skip_half = 2;
          if ((subframe == 0 || subframe == 5) && rb > half - 3 && rb < half + 3 && l == lp) alloc = 0;
          if ((subframe == 0 || subframe == 5) && rb == half - 3 && l == lp) skip_half = 1;
          else if ((subframe == 0 || subframe == 5) && rb == half + 3 && l == lp) skip_half = 2;
        }
      } else {
        if (subframe == 0 && rb >= half - 3 && rb < half + 3 && l >= (nsymb >> 1) && l < (nsymb >> 1) + 4) alloc = 0;
        if (fp->frame_type == 1) {
          if ((subframe == 0 || subframe == 5) && rb >= half - 3 && rb < half + 3 && l == nsymb - 1) alloc = 0;
          if ((subframe == 1 || subframe == 6) && rb >= half - 3 && rb < half + 3 && l == 2) alloc = 0;
        } else {
          if ((subframe == 0 || subframe == 5) && rb >= half - 3 && rb < half + 3 && l == (nsymb >> 1) - 2) alloc = 0;
          if ((subframe == 0 || subframe == 5) && rb >= half - 3 && rb < half + 3 && l == (nsymb >> 1) - 1) alloc = 0;
        }
      }
      if (alloc) {
        int first = 0, last = 12, re_off = re_offset, par = 0;
        if (skip_half == 1) last = 6;
        else if (skip_half == 2) first = 6;
        for (int re = first; re < last; re++) {
          if (skip_dc && re == 6) re_off = re_off - N + 1;
          if (!not_pilot(pilots, re, fp->nushift, use2nd)) continue;
          int k = re_off + re;
          if (k < 0 || k >= N) return -1;
          if (alm) {
            /* ALAMOUTI pair (:362-546, :868-876): symbols 2i, 2i+1 at RE n and its partner, the
             * next carrier or the one after when that is a pilot (linear grid index); code =
             * 2i | role.  A partner outside this symbol's row or on an RE that is written twice
             * would need accumulation: not produced by any supported grid, rejected here. */
            int k2 = k + (not_pilot(pilots, re + 1, fp->nushift, use2nd) ? 1 : 2);
            if (k2 >= N || remap[l * N + k] != 0xFFFF || remap[l * N + k2] != 0xFFFF) return -1;
            remap[l * N + k] = (uint16_t)idx;
            remap[l * N + k2] = (uint16_t)(idx | 1u);
            idx += 2;
            ralloc += 2;
            re++;
            if (!not_pilot(pilots, re, fp->nushift, use2nd)) {
              re++;
              ralloc++;          /* the reference also counts the pilot it steps over */
            }
            continue;
          }
          remap[l * N + k] = (uint16_t)(idx | (par << 15));
          idx++;
          ralloc++;
          par ^= 1;
        }
      }
      re_offset += 12;
      if (re_offset >= N) re_offset = skip_dc == 0 ? 1 : 7;
    }
    total += idx;
  }
  if (re_alloc) *re_alloc = ralloc;
  return (int)total;
}

/* ------------------------------------------------------------------------------------------
 * configuration
 * ---------------------------------------------------------------------------------------- */
struct oai4g_tx_config {
  oai4g_tx_params_t p;
  oai4g_frame_parms_t fp;
  cfg_dev_t h;                      /* host mirror */
  cfg_dev_t *d = nullptr;           /* device copy */
  uint16_t *d_remap = nullptr;
  std::vector<uint16_t> h_remap;
  uint32_t *d_crs = nullptr;
  uint32_t *d_gold = nullptr;           /* [10][n_cw][ebits_words] scrambling words */
  std::vector<uint32_t> h_crs;          /* [10][4][200] packed CRS IQ */
  uint32_t *d_ctl = nullptr;            /* static RE values [10][14][2][N] (set_control / set_common) */
  std::vector<uint32_t> h_ctl;          /* host copy of d_ctl's table (empty when no control REs) */
  uint32_t *d_stat = nullptr;           /* cfg_dev_t::stat_tm */
  int ctl_vmax = 0;                     /* largest I / Q magnitude in the static-RE table (mod_nosat_ok) */
  std::vector<oai4g_dci_alloc_t> dci;   /* oai4g_tx_config_set_control's DCI set */
  uint8_t n_ue_dci = 0, n_common_dci = 0;
  bool common_on = false;
  oai4g_common_sig_t common;            /* oai4g_tx_config_set_common's signals */
  int re_count[10];
  int re_alloc[10];                 /* dlsch_modulation's return value (ALAMOUTI counts skipped pilots) */
  /* optional pipelined batches (OAI4G_PIPE_CHUNK=n): the encoder runs on the caller's stream, the
   * modulator/IDFT on s_mod, chunk by chunk.  Off by default: measured slower on MI355X than the
   * serial pair (the persistent modulator grid already fills every CU). */
  hipStream_t s_mod = nullptr;
  hipEvent_t ev_enc[OAI4G_PIPE_MAX_CHUNKS] = {};
  hipEvent_t ev_done = nullptr;
  int pipe_chunk = 0;
};

/* The sub-block interleaver + rate matcher plan of block size ki (k_encode phase 4;
 * lte_rate_matching.c:51-130, 464-566).  Tile t: v0 tiles cover 32 rows of y0, interlaced tiles 16
 * rows of y1 / y2 alternating per lane (lane 2i: y1 row, 2i + 1: y2 row, shifted by one for the
 * (pi(k) + 1) mod Kpi rule).  After the half-wave's 32x32 transpose lane c holds matrix column c =
 * w column bitrev5(c), rows of the tile: its NULLs (row 0 of the column) lead the run, and the
 * run's place in the NULL-free circular buffer is closed-form. */
static void rm_plan(cw_dev_t &c, int ki)
{
  const uint32_t R = c.Rk[ki], ND = c.NDk[ki], Ncb = c.Ncbk[ki], Nnn = c.Nnnk[ki], k0c = c.k0ck[ki];
  const uint32_t tz = c.t0k[ki], nt = c.ntk[ki], sw = c.stream_words;
  memset(c.rm_dst[ki], 0, sizeof(c.rm_dst[ki]));
  c.rm_wrapt[ki] = ~0u;
  for (uint32_t t = 0; t <= OAI4G_RM_TILES; t++)
    for (uint32_t L = 0; L < 32; L++) c.rm_src[ki][t][L] = 1u << 5;   /* idle: word 0 of stream 0 */
  for (uint32_t t = 0; t < nt; t++) {
    const bool il = t >= tz;
    const uint32_t rb = il ? t - tz : t;
    for (uint32_t L = 0; L < 32; L++) {
      /* source: row of the tile this lane loads */
      const uint32_t row = il ? 16 * rb + (L >> 1) : 32 * rb + L, s = il ? 1 + (L & 1) : 0;
      if (row < R) {
        const int pos = (int)(32 * row) - (int)ND + (s == 2 ? 1 : 0);     /* >= -32 */
        const uint32_t wrel = (uint32_t)((int)(s * sw) + (pos >> 5) + 1);
        c.rm_src[ki][t][L] = ((uint32_t)pos & 31u) | (wrel << 5) | (s == 2 && row == R - 1 ? OAI4G_RM_SRC_LAST : 0u);
      }   /* past the last row: the idle word (any bits, beyond the run) */
      /* destination: the run of matrix column L = w column wc */
      uint32_t wc = 0;
      for (int b = 0; b < 5; b++) wc |= ((L >> b) & 1u) << (4 - b);
      uint32_t b0 = 0, b1 = 0;           /* NULL-headed w columns before wc in v0 / v1, v2 */
      for (uint32_t w2 = 0; w2 < wc; w2++) {
        uint32_t p2 = 0;
        for (int b = 0; b < 5; b++) p2 |= ((w2 >> b) & 1u) << (4 - b);
        b0 += p2 < ND ? 1u : 0u;
        b1 += p2 + 1 < ND ? 1u : 0u;
      }
      const uint32_t z0 = L < ND ? 1u : 0u, z1 = z0 + (L + 1 < ND ? 1u : 0u);
      const uint32_t zc = il ? z1 : z0;
      const uint32_t cs = il ? 32 * R - ND + 2 * wc * R - b0 - b1 : wc * R - b0;   /* compact index of the column's first entry */
      const uint32_t pc = il ? 32 * R + 2 * wc * R : wc * R;                       /* w position of the column start */
      const int left = il ? 2 * ((int)R - 16 * (int)rb) : (int)R - 32 * (int)rb;
      int n = left < 32 ? left : 32;
      if (il && L == 31 && ND > 0 && left <= 32 && n) n--;                         /* w[3Kpi-1] is NULL */
      const uint32_t z = rb ? 0u : zc, ci0 = rb ? cs + 32 * rb - zc : cs, p0 = pc + 32 * rb;
      const int m = p0 + (uint32_t)n > Ncb ? (int)Ncb - (int)(p0 + z) : n - (int)z;   /* limited buffer */
      if (m <= 0) continue;
      uint32_t o = ci0 + Nnn - k0c;
      o = o >= Nnn ? o - Nnn : o;
      c.rm_dst[ki][t][L] = o | (z << 16) | ((uint32_t)m << 21) | (o + (uint32_t)m > Nnn ? OAI4G_RM_DST_WRAP : 0u);
      /* runs are disjoint intervals of the circular buffer, so at most one straddles its end; ~1
       * (never expected) sends the encoder down its general placement path */
      if (o + (uint32_t)m > Nnn) c.rm_wrapt[ki] = c.rm_wrapt[ki] == ~0u || c.rm_wrapt[ki] == t ? t : ~1u;
    }
  }
  /* test hook: OAI4G_ENC_GENERAL_RM set sends every block size down the encoder's general placement
   * path (the ~1 plan), which no LTE geometry reaches by itself (tests/test_gpu_rm_paths.py) */
  if (getenv("OAI4G_ENC_GENERAL_RM")) c.rm_wrapt[ki] = ~1u;
}

static int derive_cfg(oai4g_tx_config *cfg, const oai4g_tx_params_t *p, const uint8_t Nl[2], bool need_remap,
                      int only_sf)
{
  memset(&cfg->h, 0, sizeof(cfg->h));
  cfg->p = *p;
  oai4g_frame_parms_t &fp = cfg->fp;
  if (oai4g_init_frame_parms(&fp, p->N_RB_DL, p->Nid_cell, p->Ncp, p->nb_antennas_tx, p->mode1_flag,
                             p->frame_type) != 0)
    return -1;
  cfg_dev_t &h = cfg->h;
  if (p->n_cw < 1 || p->n_cw > 2) { set_err("n_cw must be 1 or 2"); return -1; }
  if (p->mimo_mode != OAI4G_SISO && p->mimo_mode != OAI4G_LARGE_CDD && p->mimo_mode != OAI4G_ALAMOUTI) {
    set_err("mimo_mode %u not supported (SISO, ALAMOUTI and LARGE_CDD)", p->mimo_mode);
    return -1;
  }
  if (p->mimo_mode == OAI4G_ALAMOUTI && (p->nb_antennas_tx != 2 || p->n_cw != 1)) {
    set_err("ALAMOUTI requires 2 TX antennas and one codeword (dlsch_modulation.c:362)");
    return -1;
  }
  if (p->mimo_mode == OAI4G_LARGE_CDD && ((p->nb_antennas_tx != 2 && p->nb_antennas_tx != 4) || p->n_cw != 2)) {
    set_err("LARGE_CDD requires 2 (dlsch_modulation.c:551) or 4 (C4 extension) TX antennas and 2 codewords");
    return -1;
  }
  if (p->nb_antennas_tx == 4 && p->mimo_mode != OAI4G_LARGE_CDD) {
    set_err("4 TX antennas: LARGE_CDD only (C4 extension)");
    return -1;
  }
  if (p->payload_stride % 4) { set_err("payload_stride must be a multiple of 4"); return -1; }
  h.N_RB_DL = fp.N_RB_DL;
  h.N = fp.ofdm_symbol_size;
  h.log2N = fp.log2_symbol_size;
  h.cp0 = fp.nb_prefix_samples0;
  h.cp = fp.nb_prefix_samples;
  h.spt = fp.samples_per_tti;
  h.nsymb = fp.symbols_per_tti;
  h.n_ant = fp.nb_antennas_tx;
  h.first_carrier = fp.first_carrier_offset;
  h.n_cw = p->n_cw;
  h.mimo_mode = p->mimo_mode;
  h.num_pdcch = p->num_pdcch_symbols;
  h.rnti = p->rnti;
  h.Nid_cell = p->Nid_cell;
  h.first_sf = p->first_subframe % 10;
  h.sf_step = p->subframe_step;
  h.payload_stride = p->payload_stride;
  for (uint32_t v = 0; v < 256; v++) {            /* crc_byte.c:98-105 */
    uint32_t ra = v << 16, rb = v << 16;
    for (int i = 0; i < 8; i++) {
      ra = (ra & 0x800000u) ? ((ra << 1) ^ 0x864cfbu) & 0xffffffu : (ra << 1) & 0xffffffu;
      rb = (rb & 0x800000u) ? ((rb << 1) ^ 0x800063u) & 0xffffffu : (rb << 1) & 0xffffffu;
    }
    h.crctab[0][v] = ra;
    h.crctab[1][v] = rb;
  }
  uint32_t max_tb_words = 0, max_stream_words = 0, max_gw = 0, max_bits = 0, max_w = 0, max_inw = 0;
  bool rm_fail = false;
  for (int cw = 0; cw < p->n_cw; cw++) {
    cw_dev_t &c = h.cw[cw];
    c.TBS = p->TBS[cw];
    if (c.TBS == 0 || (c.TBS & 7)) { set_err("TBS[%d]=%u must be a positive multiple of 8", cw, c.TBS); return -1; }
    c.A_bytes = c.TBS >> 3;
    if (p->payload_stride < ((c.A_bytes + 3) & ~3u)) {
      set_err("payload_stride %u < TBS/8 rounded to 4 (%u)", p->payload_stride, (c.A_bytes + 3) & ~3u);
      return -1;
    }
    c.Qm = oai4g_get_Qm(p->mcs[cw]);
    c.q = p->q[cw];
    uint32_t C, Cp, Cm, Kp, Km, F, L;
    if (seg_params(c.TBS + 24, &C, &Cp, &Cm, &Kp, &Km, &F, &L) < 0) { set_err("segmentation failed"); return -1; }
    c.C = C; c.Cminus = Cm; c.Kplus = Kp; c.Kminus = Km; c.F = F; c.L = L;
    uint32_t src = 0, maxK = 0;
    for (uint32_t r = 0; r < C; r++) {
      uint32_t K = r < Cm ? Km : Kp;
      int qi = oai4g_qpp_index(K);
      if (qi < 0) { set_err("illegal code block size %u", K); return -1; }
      c.K[r] = K;
      c.f1[r] = oai4g_qpp_table[qi].f1;
      c.f2[r] = oai4g_qpp_table[qi].f2;
      c.fill[r] = r == 0 ? F / 8 : 0;
      c.ncopy[r] = (K - L) / 8 - c.fill[r];
      c.src[r] = src;
      src += c.ncopy[r];
      maxK = K > maxK ? K : maxK;
      /* rate matching geometry */
      uint32_t D = K + 4, R = (D + 31) >> 5, Kpi = R << 5;
      c.R[r] = R; c.Kpi[r] = Kpi; c.ND[r] = Kpi - D;
      uint32_t Kw = 3 * Kpi;
      uint32_t Nir = OAI4G_NSOFT / p->Kmimo / (p->Mdlharq < 8 ? p->Mdlharq : 8);
      uint32_t Ncb = (Nir / C < Kw) ? Nir / C : Kw;
      if (Ncb < Kw && !p->rm_limited_buffer) {
        printf("Exiting, RM condition (Nir %u, Nsoft %u, Kw %u\n", Nir, OAI4G_NSOFT, Kw);
        set_err("RM condition: Ncb %u < Kw %u (the reference emits E=0, lte_rate_matching.c:518-521)", Ncb, Kw);
        rm_fail = true;
        Ncb = Kw;
      }   /* else (opt-in): the circular buffer is w[0..Ncb), 36.212 5.1.4.1.2 */
      c.Ncb[r] = Ncb;
      c.kidx[r] = (C > 1 && r < Cm) ? 0 : 1;
    }
    if (src != (c.TBS + 24) / 8) { set_err("segmentation byte accounting mismatch"); return -1; }
    /* QPP walk tables per block size (Kminus list 0, Kplus list 1) and interleaved-word offsets */
    for (int ki = 0; ki < 2; ki++) {
      uint32_t K = ki == 0 ? Km : Kp;
      if (K == 0 || (ki == 0 && !(C > 1 && Cm > 0))) continue;
      int qi = oai4g_qpp_index(K);
      uint64_t f1 = oai4g_qpp_table[qi].f1, f2 = oai4g_qpp_table[qi].f2;
      for (uint32_t j = 0; j < (K + 31) / 32; j++) {   /* k = 8j < K/4: walk starts of the quarter fold */
        uint64_t k = 8 * j;
        uint32_t pi = (uint32_t)((f1 * k + f2 * k * k) % K), pi1 = (uint32_t)((f1 * (k + 1) + f2 * (k + 1) * (k + 1)) % K);
        c.qpp0[ki][j] = pi | (((pi1 + K - pi) % K) << 16);
      }
      c.qpp_d2[ki] = (uint32_t)((2 * f2) % K);
      memset(c.qpp_tab[ki], 0, sizeof(c.qpp_tab[ki]));
      /* entry k: plane word xp/8 (bits 7-14) and the rotate (bits 0-4) that lands bit (8u + xp%8) of
       * it at bit k%8 of each byte (the walk's step index is folded into the rotate, so the kernel
       * needs no shift) */
      for (uint64_t k = 0; k < K / 4; k++) {
        const uint32_t x = (uint32_t)((f1 * k + f2 * k * k) % K), Q = K / 4, xp = x % Q, u = x / Q;
        const uint32_t rot = (8 * u + (xp & 7) + 32 - (uint32_t)(k & 7)) & 31u;
        c.qpp_tab[ki][k >> 1] |= (((xp >> 3) << 7) | rot) << (16 * (k & 1));
      }
      c.qpp_s3[ki] = (uint32_t)((f1 * (K / 4)) % K) == K / 4 ? 0u : 1u;
    }
    {
      uint32_t o = 0;
      for (uint32_t r = 0; r < C; r++) {
        c.ilv_off[r] = o;
        o += (c.K[r] + 31) / 32;
      }
      c.ilv_off[C] = o;
      c.n0 = (C > 1) ? Cm : 0;
      c.kk[0] = c.n0 ? Km : Kp;
      c.kk[1] = Kp;
      for (int ki = 0; ki < 2; ki++) {
        c.kw[ki] = (c.kk[ki] + 31) / 32;
        c.kmag[ki] = ((1u << 20) + c.kw[ki] - 1) / c.kw[ki];
      }
      c.u0 = c.n0 * c.kw[0];
    }
    c.crc_per_tb = (((c.A_bytes + 255) / 256) + 3) & ~3u;   /* bytes per lane, a multiple of 4 */
    crc_mul_tables(c.crc_per_tb, 8, 0x864cfbu, c.crcmul_tb);
    crc_mul_tables2(c.crc_per_tb, 0x864cfbu, c.crc2_tb);
    uint32_t ncb_max = 0;
    for (uint32_t r = 0; r < C; r++) {
      uint32_t n = c.ncopy[r];
      if (c.src[r] + n > c.A_bytes) n = c.A_bytes > c.src[r] ? c.A_bytes - c.src[r] : 0;
      ncb_max = n > ncb_max ? n : ncb_max;
    }
    /* C > 1: the CRC-24A and every CRC-24B in one pass, crc_lpb lanes per block (k_encode phase 1) */
    c.crc_lpb = C <= 4 ? 64u : (C <= 8 ? 32u : 16u);
    c.crc_per_cb = (((ncb_max + c.crc_lpb - 1) / c.crc_lpb) + 3) & ~3u;
    crc_mul_tables2(c.crc_per_cb ? c.crc_per_cb : 1, 0x864cfbu, c.crc2_cb[0]);
    crc_mul_tables2(c.crc_per_cb ? c.crc_per_cb : 1, 0x800063u, c.crc2_cb[1]);
    for (uint32_t r = 0; r < C; r++) {
      uint32_t end = c.src[r] + c.ncopy[r];
      if (end > c.A_bytes) end = c.A_bytes;
      const uint32_t m = crc_xpow8_h(c.A_bytes - (end > c.src[r] ? end : c.src[r]), 0x864cfbu);
      for (int k = 0; k < 6; k++)
        for (uint32_t v = 0; v < 16; v++) c.crcmul_blk[r][16 * k + v] = crc_mulmod_h((v << (4 * k)) & 0xffffffu, m, 0x864cfbu);
    }
    for (int ki = 0; ki < 2; ki++) {
      uint32_t K = ki == 0 ? (Km ? Km : Kp) : Kp;
      int n = null_positions(K, c.nullpos[ki], OAI4G_MAX_NULLS);
      if (n < 0) { set_err("too many NULL positions"); return -1; }
      c.nnull[ki] = (uint32_t)n;
    }
    for (uint32_t r = 0; r < C; r++) {
      uint32_t R = c.R[r], Ncb = c.Ncb[r], nn = c.nnull[c.kidx[r]];
      const uint16_t *np = c.nullpos[c.kidx[r]];
      uint32_t ncol8 = R << 3;
      uint32_t k0 = R * (2 + p->rvidx[cw] * ((Ncb % ncol8 ? 1 : 0) + Ncb / ncol8) * 2);
      uint32_t before = 0, inbuf = 0;
      for (uint32_t i = 0; i < nn; i++) {
        if (np[i] < k0) before++;
        if (np[i] < Ncb) inbuf++;             /* NULLs inside the (possibly limited) circular buffer */
      }
      c.k0c[r] = k0 - before;
      c.Nnn[r] = Ncb - inbuf;
    }
    uint32_t nw = (maxK + 31) >> 5;
    c.stream_words = nw + 3;   /* + tail word + read-ahead words */
    uint32_t inw = 0;
    for (uint32_t r = 0; r < C; r++) inw += (c.K[r] + 31) >> 5;
    max_inw = inw > max_inw ? inw : max_inw;
    /* packed w of every block (3 Kpi bits = 3R words, + 2 read-ahead words each) and the
     * 32x32 transpose tiles of the sub-block interleaver (3 streams x ceil(R/32) per block) */
    uint32_t wwords = 0, ntask = 0;
    for (uint32_t r = 0; r < C; r++) {
      c.wpk_off[r] = wwords;
      wwords += 3 * c.R[r] + 2;
      for (uint32_t rb = 0; rb < (c.R[r] + 31) / 32; rb++) c.tasks[ntask++] = (uint16_t)(r | (rb << 5));
      for (uint32_t rb = 0; rb < (c.R[r] + 15) / 16; rb++) c.tasks[ntask++] = (uint16_t)(r | (1u << 4) | (rb << 5));
    }
    c.wpk_off[C] = wwords;
    c.ntask = ntask;
    for (uint32_t r = 0; r < C; r++) {   /* every block of one size shares its geometry */
      const uint32_t ki = r < c.n0 ? 0 : 1;
      if (c.K[r] != c.kk[ki]) { set_err("block size order"); return -1; }
      c.Rk[ki] = c.R[r]; c.NDk[ki] = c.ND[r]; c.Ncbk[ki] = c.Ncb[r]; c.Nnnk[ki] = c.Nnn[r]; c.k0ck[ki] = c.k0c[r];
    }
    for (uint32_t r = 0; r < C; r++) {
      const uint32_t ki = r < c.n0 ? 0 : 1;
      if (c.R[r] != c.Rk[ki] || c.ND[r] != c.NDk[ki] || c.Ncb[r] != c.Ncbk[ki] || c.Nnn[r] != c.Nnnk[ki] ||
          c.k0c[r] != c.k0ck[ki] || c.kidx[r] != ki) {
        set_err("per-size block geometry differs");
        return -1;
      }
    }
    if (c.n0 == 0) { c.Rk[0] = c.Rk[1]; c.NDk[0] = c.NDk[1]; c.Ncbk[0] = c.Ncbk[1]; c.Nnnk[0] = c.Nnnk[1]; c.k0ck[0] = c.k0ck[1]; }
    for (int ki = 0; ki < 2; ki++) {
      c.nullcol[ki][0] = c.nullcol[ki][1] = 0;
      for (uint32_t wc = 0; wc < 32; wc++) {
        uint32_t pc = 0;
        for (int b = 0; b < 5; b++) pc |= ((wc >> b) & 1u) << (4 - b);   /* bitrev5 column permutation */
        if (pc < c.NDk[ki]) c.nullcol[ki][0] |= 1u << wc;
        if (pc + 1 < c.NDk[ki]) c.nullcol[ki][1] |= 1u << wc;
      }
      c.t0k[ki] = (c.Rk[ki] + 31) / 32;
      c.ntk[ki] = c.t0k[ki] + (c.Rk[ki] + 15) / 16;
      c.ntmag[ki] = ((1u << 20) + c.ntk[ki] - 1) / c.ntk[ki];
      if (c.ntk[ki] > OAI4G_RM_TILES) { set_err("rate-matching plan: %u tiles", c.ntk[ki]); return -1; }
      rm_plan(c, ki);
    }
    max_w = wwords > max_w ? wwords : max_w;
    uint32_t tbw = (c.A_bytes + 3 + 3) / 4 + 1;
    max_tb_words = tbw > max_tb_words ? tbw : max_tb_words;
    uint32_t strw = C * 3 * c.stream_words;
    max_stream_words = strw > max_stream_words ? strw : max_stream_words;
    for (int sf = 0; sf < 10; sf++) {
      int G;
      if (fp.nb_antennas_tx == 4) {
        /* 4-TX extension: the reference's get_G formula knows no port-2/3 CRS; G = the RE map's
         * PDSCH RE count x Qm (one layer per codeword) */
        std::vector<uint16_t> tmp((size_t)14 * fp.ofdm_symbol_size);
        uint32_t sb[14];
        int n = build_remap(&fp, p->rb_alloc, p->num_pdcch_symbols, sf, p->mimo_mode, tmp.data(), sb, nullptr);
        G = n < 0 ? -1 : n * (int)c.Qm;
      } else {
        G = oai4g_get_G(&fp, p->nb_rb, p->rb_alloc, (uint8_t)c.Qm, Nl[cw], p->num_pdcch_symbols, 0, (uint8_t)sf);
      }
      if (G <= 0 || G > OAI4G_MAX_CHANNEL_BITS) { set_err("G=%d out of range", G); return -1; }
      c.G[sf] = (uint32_t)G;
      uint32_t Gp = (uint32_t)G / Nl[cw] / c.Qm, GpmodC = Gp % C, off = 0;
      for (uint32_t r = 0; r < C; r++) {
        uint32_t E = (r < C - GpmodC) ? Nl[cw] * c.Qm * (Gp / C) : Nl[cw] * c.Qm * ((GpmodC ? 1 : 0) + Gp / C);
        c.E[sf][r] = E;
        c.roff[sf][r] = off;
        off += E;
      }
      c.roff[sf][C] = off;
      c.esplit[sf] = C - GpmodC;
      for (int h = 0; h < 2; h++) {
        const uint32_t E = c.E[sf][h ? C - 1 : 0], w = (E + 31) / 32;
        c.ew[sf][h] = w;
        c.emag[sf][h] = w ? (uint32_t)(((1ull << 32) + w - 1) / w) : 0u;
      }
      uint32_t gw = (off + 31) / 32;
      max_gw = gw > max_gw ? gw : max_gw;
      max_bits = (uint32_t)G > max_bits ? (uint32_t)G : max_bits;
    }
    qam_tables_scaled((int)c.Qm, p->amp, p->sqrt_rho_a, p->sqrt_rho_b, p->mimo_mode == OAI4G_ALAMOUTI, c);
  }
  if (max_gw > OAI4G_MAX_GOLD_WORDS) { set_err("G too large"); return -1; }
  h.lds_tb_words = max_tb_words;
  h.lds_stream_words = max_stream_words;
  h.lds_gold_words = max_gw + 1;
  h.lds_w_words = max_w;
  (void)max_inw;
  /* encoder LDS regions with phase-disjoint lifetimes (see oai4g_encode.hip) */
  h.lds_a_words = max_tb_words;
  for (int cw = 0; cw < p->n_cw; cw++) {
    const cw_dev_t &c = h.cw[cw];
    /* region A also holds the interleaved words in phase 3 (the planes sit in the parity slots) */
    if (c.ilv_off[c.C] > h.lds_a_words) h.lds_a_words = c.ilv_off[c.C];
    /* and, in phase 4, the e words of one half of the blocks at a time (k_encode): blocks [0, hb)
     * then [hb, C), each half from the word holding its first bit, + 1 word for or_bits */
    const uint32_t hb = (c.C + 1) / 2;
    for (int sf = 0; sf < 10; sf++) {
      const uint32_t G = c.G[sf], eb = hb < c.C ? c.roff[sf][hb] : G;
      const uint32_t w1 = (eb + 31) / 32 + 1, w2 = (G + 31) / 32 - eb / 32 + 1;
      if (w1 > h.lds_a_words) h.lds_a_words = w1;
      if (w2 > h.lds_a_words) h.lds_a_words = w2;
    }
  }
  h.lds_b_words = max_stream_words;
  if (h.lds_b_words < OAI4G_ENC_CRC_TABLE_WORDS) h.lds_b_words = OAI4G_ENC_CRC_TABLE_WORDS;   /* the CRC tables, phases 0-1 */

  /* RE maps */
  if (need_remap) {
    uint32_t N = h.N;
    cfg->h_remap.assign((size_t)10 * 14 * N, 0xFFFF);
    for (int sf = 0; sf < 10; sf++) {
      if (only_sf >= 0 && sf != only_sf) continue;
      int n = build_remap(&fp, p->rb_alloc, p->num_pdcch_symbols, sf, p->mimo_mode,
                          cfg->h_remap.data() + (size_t)sf * 14 * N, h.symbase[sf], &cfg->re_alloc[sf]);
      if (n < 0) { set_err("RE map construction failed"); return -1; }
      cfg->re_count[sf] = n;
      if (p->with_crs) {
        /* pilots.c:43-168: port 0 on antenna 0; antenna 1 port 0 (mode1) or port 1 */
        uint32_t gt[20][2][14];
        lte_gold_table_h(&fp, gt);
        const uint32_t sps = fp.Ncp == 0 ? 7 : 6, psym[4] = {0, sps - 3, sps, 2 * sps - 3};   /* l' = 0, 4 (3) per slot */
        const int nports = (fp.nb_antennas_tx > 1 && !fp.mode1_flag) ? 2 : 1;
        cfg->h_crs.resize((size_t)10 * 6 * 200);
        for (uint32_t i = 0; i < 4; i++) {
          const uint32_t Ns = 2 * sf + (i >> 1), l = i & 1;
          for (uint32_t m = 0; m < 2u * fp.N_RB_DL; m++) {
            const uint32_t mp = 110 - fp.N_RB_DL + m;
            cfg->h_crs[((size_t)sf * 6 + i) * 200 + m] = crs_qpsk(p->amp, (gt[Ns][l][mp >> 4] >> (2 * (mp & 15))) & 3);
            for (int port = 0; port < nports; port++) {
              uint16_t &code = cfg->h_remap[((size_t)sf * 14 + psym[i]) * N + crs_bin(&fp, port, l, m)];
              if (code != 0xFFFF) { set_err("CRS RE collides with a PDSCH RE"); return -1; }
              code = (uint16_t)(OAI4G_CRS_CODE | (i << 9) | ((uint32_t)port << 8) | m);
            }
          }
        }
        if (fp.nb_antennas_tx == 4)   /* ports 2/3: pilot entries 4, 5 = symbol 1 of each slot */
          for (uint32_t s = 0; s < 2; s++) {
            const uint32_t Ns = 2 * sf + s;
            uint32_t gw[14];
            gold_words_h(&fp, Ns, 1, gw);
            for (uint32_t m = 0; m < 2u * fp.N_RB_DL; m++) {
              const uint32_t mp = 110 - fp.N_RB_DL + m;
              cfg->h_crs[((size_t)sf * 6 + 4 + s) * 200 + m] = crs_qpsk(p->amp, (gw[mp >> 4] >> (2 * (mp & 15))) & 3);
              for (uint32_t port = 2; port < 4; port++) {
                uint16_t &code = cfg->h_remap[((size_t)sf * 14 + s * sps + 1) * N + crs_bin_p23(&fp, port, Ns, m)];
                if (code != 0xFFFF) { set_err("CRS RE collides with a PDSCH RE"); return -1; }
                code = (uint16_t)(OAI4G_CRS_CODE | ((4 + s) << 9) | ((port & 1u) << 8) | m);
              }
            }
          }
      }
      /* symbols whose QAM levels use rho_B (CRS-bearing: dlsch_modulation.c:1223-1246) */
      h.pilmask = 0;
      for (uint32_t l = 0, hs = h.nsymb >> 1; l < h.nsymb; l++) {
        const uint32_t ls = l % hs;
        if (ls == 0 || ls == hs - 3 || (fp.nb_antennas_tx == 4 && ls == 1)) h.pilmask |= 1u << l;
      }
      for (int l = 0; l < 14; l++) {
        uint32_t next = l + 1 < (int)h.nsymb ? h.symbase[sf][l + 1] : (uint32_t)n;
        h.symnre[sf][l] = (uint32_t)(l < p->num_pdcch_symbols || l >= (int)h.nsymb ? 0 : next - h.symbase[sf][l]);
      }
      for (int cw = 0; cw < p->n_cw; cw++) {
        uint32_t bits = (uint32_t)n * h.cw[cw].Qm;
        max_bits = bits > max_bits ? bits : max_bits;
      }
    }
  }
  h.ebits_words = (max_bits + 31) / 32 + 2;
  return rm_fail ? -2 : 0;
}

/* cfg_dev_t::stat_tm from the RE map, the CRS values and the control table: for kernel antenna `ant`
 * (TM1: the one transform) the value the modulator's static-RE step used to produce per RE
 * (pilots.c:43-168: port p's pilot on antenna p, every port's in the single TM1 transform; the
 * control REs of generate_dci_top on antennas 0 / 1 only), in remap_tm's thread-major order */
static int build_stat_tm(oai4g_tx_config *cfg)
{
  if (cfg->d_stat) hipFree(cfg->d_stat);
  cfg->d_stat = nullptr;
  cfg->h.stat_tm = nullptr;
  cfg->h.stat_planes = 0;
  if (cfg->h_remap.empty() || (cfg->h_crs.empty() && cfg->h_ctl.empty())) return 0;
  const size_t N = cfg->h.N, T = N >> 4, nsl = cfg->h_remap.size() / N;
  const uint32_t planes = cfg->h.mimo_mode == OAI4G_SISO ? 1u : cfg->h.n_ant;
  std::vector<uint32_t> st(nsl * planes * N, 0u);
  for (size_t sl = 0; sl < nsl; sl++) {
    const size_t sf = sl / 14;
    for (size_t pos = 0; pos < N; pos++) {
      const uint32_t cd = cfg->h_remap[sl * N + pos];
      const size_t t = pos % T, k = pos / T;
      for (uint32_t ant = 0; ant < planes; ant++) {
        uint32_t v = 0;
        if (cd != 0xFFFFu && (cd & 0xE000u) == OAI4G_CRS_CODE) {
          const uint32_t ci = (cd >> 9) & 7u, m = cd & 0xFFu, port = ((cd >> 8) & 1u) | (ci >= 4 ? 2u : 0u);
          if (!cfg->h_crs.empty() && (planes == 1 || ant == port)) v = cfg->h_crs[(sf * 6 + ci) * 200 + m];
        } else if ((cd & 0xE000u) == OAI4G_CTL_CODE) {
          if (!cfg->h_ctl.empty() && ant < 2) v = cfg->h_ctl[(sl * 2 + ant) * N + pos];
        }
        st[(sl * planes + ant) * N + t * 16 + k] = v;
      }
    }
  }
  HCK(hipMalloc(&cfg->d_stat, st.size() * 4), -1);
  HCK(hipMemcpy(cfg->d_stat, st.data(), st.size() * 4, hipMemcpyHostToDevice), -1);
  cfg->h.stat_tm = cfg->d_stat;
  cfg->h.stat_planes = planes;
  return 0;
}

static int upload_remap(oai4g_tx_config *cfg)
{
  if (cfg->d_remap) hipFree(cfg->d_remap);
  cfg->d_remap = nullptr;
  if (!cfg->h_remap.empty()) {
    /* natural layout followed by the thread-major copy the fused kernel reads */
    const size_t n = cfg->h_remap.size(), N = cfg->h.N, T = N >> 4;
#if OAI4G_MOD_STAGE
    /* k_modofdm stages 4 entries per quad of data REs below a sentinel at 3N/4 */
    for (int sf = 0; sf < 10; sf++)
      for (int l = 0; l < 14; l++)
        if (cfg->h.symnre[sf][l] + 3u > (3u * N) / 4u) { set_err("too many data REs per symbol for the modulator"); return -1; }
#endif
    /* natural, thread-major, thread-major with the non-data codes on the zero sentinel */
    std::vector<uint16_t> both(3 * n);
    std::copy(cfg->h_remap.begin(), cfg->h_remap.end(), both.begin());
    /* staged entries: 2-byte QAM-table addresses, or (OAI4G_MOD_PRE, the 2048-point kernels) 8-byte
     * (y0, d) pairs of two-antenna LARGE_CDD / 4-byte QAM words of TM1 */
    const bool pre = OAI4G_MOD_STAGE && OAI4G_MOD_PRE && cfg->h.mimo_mode == OAI4G_LARGE_CDD && cfg->h.n_ant == 2 &&
                     cfg->h.log2N == 11;
    const bool pre1 = OAI4G_MOD_STAGE && OAI4G_MOD_PRE && cfg->h.mimo_mode == OAI4G_SISO && cfg->h.log2N == 11;
    const uint32_t esh = pre ? 3u : pre1 ? 2u : 1u;
    const uint16_t sentinel = (uint16_t)(((3u * (uint32_t)N) / 4u) << esh);   /* modofdm_geom::SENT, bytes */
    for (size_t sl = 0; sl < n / N; sl++)
      for (size_t t = 0; t < T; t++)
        for (size_t k = 0; k < 16; k++) {
          uint16_t code = cfg->h_remap[sl * N + t + T * k];
#if OAI4G_MOD_STAGE
          /* data RE (idx | parity << 15, idx < 3N/4): the byte offset of its staged entry (2 idx, or 8 idx
           * for the precoded pairs: < 8 * 1536 < 2^15) */
          if (code < OAI4G_CTL_CODE) {
            /* the precoded pairs carry the CDD sign already: the staging step stores -d for an odd
             * data index.  The reference alternates the sign per RE within each RB
             * (dlsch_modulation.c:733-749) and every RB of a two-port grid holds an even number of
             * data REs (12, 8 beside the 4 CRS REs, 6 / 4 in a half RB), so the parity is the index's;
             * checked here for every RE */
            const uint32_t idx = code & 0x3FFFu, par = code >> 15;
            if (pre && par != (idx & 1u)) { set_err("LARGE_CDD: CDD parity differs from the RE index parity"); return -1; }
            code = (uint16_t)(((pre || pre1 ? 0u : par) << 15) | (idx << esh));
          }
#endif
          both[n + sl * N + t * 16 + k] = code;
#if OAI4G_MOD_STAGE
          both[2 * n + sl * N + t * 16 + k] = code < OAI4G_CTL_CODE ? code : sentinel;
#else
          /* the unstaged modulator tests code < OAI4G_CTL_CODE itself: keep the non-data codes */
          (void)sentinel;
          both[2 * n + sl * N + t * 16 + k] = code;
#endif
        }
    HCK(hipMalloc(&cfg->d_remap, both.size() * 2), -1);
    HCK(hipMemcpy(cfg->d_remap, both.data(), both.size() * 2, hipMemcpyHostToDevice), -1);
    cfg->h.remap_tm = cfg->d_remap + n;
    cfg->h.remap_tm0 = cfg->d_remap + 2 * n;
  } else {
    cfg->h.remap_tm = nullptr;
    cfg->h.remap_tm0 = nullptr;
  }
  if (build_stat_tm(cfg) != 0) return -1;
  cfg->h.remap = cfg->d_remap;
  return 0;
}

/* the scrambling words of every (subframe index, codeword): lte_gold_generic (lte_gold.c:151-177)
 * with c_init = rnti 2^14 + q 2^13 + subframe 2^9 + Nid_cell (dlsch_scrambling.c:74-76) */
static int upload_gold(oai4g_tx_config *cfg)
{
  const cfg_dev_t &h = cfg->h;
  const size_t stride = h.ebits_words;
  std::vector<uint32_t> g((size_t)10 * h.n_cw * stride, 0u);
  for (uint32_t sf = 0; sf < 10; sf++)
    for (uint32_t cw = 0; cw < h.n_cw; cw++) {
      const uint32_t c_init = (h.rnti << 14) + (h.cw[cw].q << 13) + (sf << 9) + h.Nid_cell;
      uint32_t x1 = 1u + (1u << 31), x2 = c_init ^ ((c_init ^ (c_init >> 1) ^ (c_init >> 2) ^ (c_init >> 3)) << 31);
      auto step = [&]() {
        x1 = (x1 >> 1) ^ (x1 >> 4);
        x1 = x1 ^ (x1 << 31) ^ (x1 << 28);
        x2 = (x2 >> 1) ^ (x2 >> 2) ^ (x2 >> 3) ^ (x2 >> 4);
        x2 = x2 ^ (x2 << 31) ^ (x2 << 30) ^ (x2 << 29) ^ (x2 << 28);
      };
      for (int n = 1; n < 50; n++) step();
      const size_t nw = std::min(stride, (size_t)(h.cw[cw].G[sf] + 31) / 32);
      uint32_t *o = g.data() + ((size_t)sf * h.n_cw + cw) * stride;
      for (size_t w = 0; w < nw; w++) {
        step();
        o[w] = x1 ^ x2;
      }
    }
  if (cfg->d_gold) hipFree(cfg->d_gold);
  cfg->d_gold = nullptr;
  HCK(hipMalloc(&cfg->d_gold, g.size() * 4), -1);
  HCK(hipMemcpy(cfg->d_gold, g.data(), g.size() * 4, hipMemcpyHostToDevice), -1);
  cfg->h.gold_tab = cfg->d_gold;
  return 0;
}

static int upload_cfg(oai4g_tx_config *cfg)
{
  if (upload_remap(cfg) != 0) return -1;
  if (upload_gold(cfg) != 0) return -1;
  if (!cfg->h_crs.empty()) {
    HCK(hipMalloc(&cfg->d_crs, cfg->h_crs.size() * 4), -1);
    HCK(hipMemcpy(cfg->d_crs, cfg->h_crs.data(), cfg->h_crs.size() * 4, hipMemcpyHostToDevice), -1);
  }
  cfg->h.crs_tab = cfg->d_crs;
  cfg->h.with_crs = cfg->d_crs ? 1u : 0u;
  cfg->h.mod_nosat = mod_nosat_ok(cfg->h, std::max(packed_iq_max(cfg->h_crs), cfg->ctl_vmax));
  cfg->h.n_cu = (uint32_t)g_n_cu;
  cfg->h.gold_x1 = g_gx1;
  cfg->h.gold_x2j = g_gx2j;
  cfg->h.tw = g_tw;
  HCK(hipMalloc(&cfg->d, sizeof(cfg_dev_t)), -1);
  HCK(hipMemcpy(cfg->d, &cfg->h, sizeof(cfg_dev_t), hipMemcpyHostToDevice), -1);
  return 0;
}

static void release_cfg(oai4g_tx_config *cfg)
{
  for (auto &e : cfg->ev_enc)
    if (e) hipEventDestroy(e);
  if (cfg->ev_done) hipEventDestroy(cfg->ev_done);
  if (cfg->s_mod) hipStreamDestroy(cfg->s_mod);
  cfg->s_mod = nullptr;
  cfg->ev_done = nullptr;
  if (cfg->d) hipFree(cfg->d);
  if (cfg->d_remap) hipFree(cfg->d_remap);
  if (cfg->d_crs) hipFree(cfg->d_crs);
  if (cfg->d_ctl) hipFree(cfg->d_ctl);
  if (cfg->d_stat) hipFree(cfg->d_stat);
  if (cfg->d_gold) hipFree(cfg->d_gold);
  cfg->d_stat = nullptr;
  cfg->d_gold = nullptr;
  cfg->d_crs = nullptr;
  cfg->d_ctl = nullptr;
  cfg->d = nullptr;
  cfg->d_remap = nullptr;
}

extern "C" oai4g_tx_config_t *oai4g_tx_config_create(const oai4g_tx_params_t *p)
{
  NEED_INIT(nullptr);
  if (p->N_RB_DL != 6 && p->N_RB_DL != 15 && p->N_RB_DL != 25 && p->N_RB_DL != 50 && p->N_RB_DL != 100) {
    set_err("batched path supports N_RB_DL 6, 15, 25, 50, 100 (IDFT 128/256/512/1024/2048)");
    return nullptr;
  }
  oai4g_tx_config *cfg = new oai4g_tx_config();
  uint8_t Nl[2] = {1, 1};
  if (derive_cfg(cfg, p, Nl, true, -1) != 0 || upload_cfg(cfg) != 0) {   /* RM condition (-2) is an error here */
    release_cfg(cfg);
    delete cfg;
    return nullptr;
  }
  bool ok = hipStreamCreateWithFlags(&cfg->s_mod, hipStreamNonBlocking) == hipSuccess &&
            hipEventCreateWithFlags(&cfg->ev_done, hipEventDisableTiming) == hipSuccess;
  for (auto &e : cfg->ev_enc) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    set_err("stream/event creation failed");
    release_cfg(cfg);
    delete cfg;
    return nullptr;
  }
  if (const char *pc = getenv("OAI4G_PIPE_CHUNK")) cfg->pipe_chunk = atoi(pc);
  return cfg;
}

extern "C" void oai4g_tx_config_destroy(oai4g_tx_config_t *cfg)
{
  if (!cfg) return;
  release_cfg(cfg);
  delete cfg;
}

extern "C" uint32_t oai4g_tx_G(const oai4g_tx_config_t *cfg, int cw, int subframe)
{
  return cfg->h.cw[cw].G[subframe % 10];
}
extern "C" uint32_t oai4g_tx_ebits_words(const oai4g_tx_config_t *cfg) { return cfg->h.ebits_words; }
extern "C" uint32_t oai4g_tx_iq_samples(const oai4g_tx_config_t *cfg) { return cfg->h.spt; }
extern "C" size_t oai4g_tx_workspace_bytes(const oai4g_tx_config_t *cfg, int n_sf)
{
  return (size_t)n_sf * cfg->h.n_cw * cfg->h.ebits_words * 4;
}

extern "C" int oai4g_tx_encode(const oai4g_tx_config_t *cfg, int n_sf, const uint8_t *d_payload, void *d_work,
                               void *stream)
{
  NEED_INIT(-1);
  HCK(oai4g_launch_encode(cfg->d, &cfg->h, 0, n_sf, d_payload, (uint32_t *)d_work, (hipStream_t)stream), -1);
  return 0;
}

/* the 2048-point modulator stores sample pairs as 8-byte words */
static int iq_aligned(const int32_t *d_iq)
{
  if ((uintptr_t)d_iq & 7u) {
    set_err("iq buffer must be 8-byte aligned");
    return 0;
  }
  return 1;
}

extern "C" int oai4g_tx_batch(const oai4g_tx_config_t *cfg, int n_sf, const uint8_t *d_payload, void *d_work,
                              int32_t *d_iq, void *stream)
{
  NEED_INIT(-1);
  if (n_sf <= 0) return 0;
  if (!iq_aligned(d_iq)) return -1;
  hipStream_t s = (hipStream_t)stream;
  uint32_t *ew = (uint32_t *)d_work;
  int chunk = cfg->pipe_chunk;
  if (chunk <= 0 || n_sf < 2 * chunk) {
    HCK(oai4g_launch_encode(cfg->d, &cfg->h, 0, n_sf, d_payload, ew, s), -1);
    HCK(oai4g_launch_modofdm(cfg->d, &cfg->h, 0, n_sf, ew, d_iq, s), -1);
    return 0;
  }
  int nch = (n_sf + chunk - 1) / chunk;
  if (nch > OAI4G_PIPE_MAX_CHUNKS) {
    nch = OAI4G_PIPE_MAX_CHUNKS;
    chunk = (n_sf + nch - 1) / nch;
  }
  /* the modulator stream must not start before work already queued on the caller's stream */
  HCK(hipEventRecord(cfg->ev_done, s), -1);
  HCK(hipStreamWaitEvent(cfg->s_mod, cfg->ev_done, 0), -1);
  for (int i = 0; i < nch; i++) {
    const int sf0 = i * chunk, n = n_sf - sf0 < chunk ? n_sf - sf0 : chunk;
    HCK(oai4g_launch_encode(cfg->d, &cfg->h, sf0, n, d_payload, ew, s), -1);
    HCK(hipEventRecord(cfg->ev_enc[i], s), -1);
    HCK(hipStreamWaitEvent(cfg->s_mod, cfg->ev_enc[i], 0), -1);
    HCK(oai4g_launch_modofdm(cfg->d, &cfg->h, sf0, n, ew, d_iq, cfg->s_mod), -1);
  }
  HCK(hipEventRecord(cfg->ev_done, cfg->s_mod), -1);
  HCK(hipStreamWaitEvent(s, cfg->ev_done, 0), -1);
  return 0;
}

extern "C" int oai4g_tx_batch_timed(const oai4g_tx_config_t *cfg, int n_sf, const uint8_t *d_payload, void *d_work,
                                    int32_t *d_iq, void *stream, float *kernel_ms)
{
  NEED_INIT(-1);
  if (!iq_aligned(d_iq)) return -1;
  hipStream_t s = (hipStream_t)stream;
  hipEvent_t ev[3];
  for (int i = 0; i < 3; i++) HCK(hipEventCreate(&ev[i]), -1);
  HCK(hipEventRecord(ev[0], s), -1);
  HCK(oai4g_launch_encode(cfg->d, &cfg->h, 0, n_sf, d_payload, (uint32_t *)d_work, s), -1);
  HCK(hipEventRecord(ev[1], s), -1);
  HCK(oai4g_launch_modofdm(cfg->d, &cfg->h, 0, n_sf, (const uint32_t *)d_work, d_iq, s), -1);
  HCK(hipEventRecord(ev[2], s), -1);
  HCK(hipEventSynchronize(ev[2]), -1);
  HCK(hipEventElapsedTime(&kernel_ms[0], ev[0], ev[1]), -1);
  HCK(hipEventElapsedTime(&kernel_ms[1], ev[1], ev[2]), -1);
  for (int i = 0; i < 3; i++) hipEventDestroy(ev[i]);
  return 0;
}

extern "C" int oai4g_tx_modulate(const oai4g_tx_config_t *cfg, int n_sf, const void *d_work, int32_t *d_iq,
                                 void *stream)
{
  NEED_INIT(-1);
  if (!cfg || !iq_aligned(d_iq)) return -1;
  HCK(oai4g_launch_modofdm(cfg->d, &cfg->h, 0, n_sf, (const uint32_t *)d_work, d_iq, (hipStream_t)stream), -1);
  return 0;
}

extern "C" int oai4g_tx_mod_nosat(const oai4g_tx_config_t *cfg) { return cfg ? (int)cfg->h.mod_nosat : 0; }

/* Diagnostics: time the encoder with an early exit after phase `stop_phase`
 * (0 load/Gold, 1 CRC, 2 segmentation, 3 turbo, 4 w build, 99 full). Outputs are invalid. */
extern "C" int oai4g_diag_encode_phase_ms(const oai4g_tx_config_t *cfg, int n_sf, const uint8_t *d_payload,
                                          void *d_work, int stop_phase, int reps, float *ms)
{
  NEED_INIT(-1);
  hipEvent_t a, b;
  HCK(hipEventCreate(&a), -1);
  HCK(hipEventCreate(&b), -1);
  HCK(oai4g_launch_encode_phase(cfg->d, &cfg->h, n_sf, d_payload, (uint32_t *)d_work, stop_phase, nullptr), -1);
  HCK(hipEventRecord(a, nullptr), -1);
  for (int i = 0; i < reps; i++)
    HCK(oai4g_launch_encode_phase(cfg->d, &cfg->h, n_sf, d_payload, (uint32_t *)d_work, stop_phase, nullptr), -1);
  HCK(hipEventRecord(b, nullptr), -1);
  HCK(hipEventSynchronize(b), -1);
  HCK(hipEventElapsedTime(ms, a, b), -1);
  *ms /= reps;
  hipEventDestroy(a);
  hipEventDestroy(b);
  return 0;
}

/* Diagnostics: resident encoder workgroups per CU and the dynamic LDS bytes of one workgroup */
extern "C" int oai4g_diag_encode_occupancy(const oai4g_tx_config_t *cfg, int *blocks_per_cu, size_t *lds_bytes)
{
  NEED_INIT(-1);
  if (!cfg || !blocks_per_cu || !lds_bytes) { set_err("diag_encode_occupancy: bad arguments"); return -1; }
  HCK(oai4g_encode_occupancy(&cfg->h, blocks_per_cu, lds_bytes), -1);
  return 0;
}

/* PMC calibration: stream `bytes` at 4 B per lane (mode 0 read from src, 1 write to dst) */
extern "C" int oai4g_diag_stream(const void *d_src, void *d_dst, size_t bytes, int mode, void *stream)
{
  NEED_INIT(-1);
  HCK(oai4g_launch_diag_stream(d_src, d_dst, bytes, mode, (hipStream_t)stream), -1);
  return 0;
}

/* ------------------------------------------------------------------------------------------
 * device memory helpers
 * ---------------------------------------------------------------------------------------- */
extern "C" void *oai4g_dev_alloc(size_t bytes)
{
  NEED_INIT(nullptr);
  void *p = nullptr;
  HCK(hipMalloc(&p, bytes), nullptr);
  return p;
}
extern "C" void oai4g_dev_free(void *p)
{
  if (p) hipFree(p);
}
extern "C" int oai4g_memcpy_h2d(void *dst, const void *src, size_t bytes)
{
  NEED_INIT(-1);
  HCK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice), -1);
  return 0;
}
extern "C" int oai4g_memcpy_d2h(void *dst, const void *src, size_t bytes)
{
  NEED_INIT(-1);
  HCK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost), -1);
  return 0;
}
extern "C" int oai4g_memset_d(void *dst, int value, size_t bytes)
{
  NEED_INIT(-1);
  HCK(hipMemset(dst, value, bytes), -1);
  return 0;
}
extern "C" int oai4g_sync(void)
{
  NEED_INIT(-1);
  HCK(hipDeviceSynchronize(), -1);
  return 0;
}
/* ------------------------------------------------------------------------------------------
 * dlsim's channel stage (dlsim.c:2714-2866): tx_lev and AWGN, device batches and the host drop-in
 * ---------------------------------------------------------------------------------------- */
extern "C" int oai4g_signal_energy_batch(const int32_t *d_x, int n, size_t stride, uint32_t length, int32_t *d_energy,
                                         void *stream)
{
  NEED_INIT(-1);
  if (n < 0 || length < 2 || (n > 0 && (!d_x || !d_energy))) { set_err("signal_energy_batch: bad arguments"); return -1; }
  HCK(oai4g_launch_signal_energy(d_x, n, stride, length, d_energy, (hipStream_t)stream), -1);
  return 0;
}

extern "C" int32_t oai4g_signal_energy(const int32_t *input, uint32_t length)
{
  NEED_INIT(-1);
  if (!input || length < 2) { set_err("signal_energy: bad arguments"); return -1; }
  int32_t e = -1;
  uint8_t *buf = scratch((size_t)length * 4 + 256);
  if (!buf) { set_err("signal_energy: scratch allocation failed"); return -1; }
  int32_t *d_x = (int32_t *)buf, *d_e = (int32_t *)(buf + (((size_t)length * 4 + 127) & ~(size_t)127));
  if (hipMemcpyAsync(d_x, input, (size_t)length * 4, hipMemcpyHostToDevice, g_scr.s) != hipSuccess ||
      oai4g_launch_signal_energy(d_x, 1, 0, length, d_e, g_scr.s) != hipSuccess ||
      hipMemcpyAsync(&e, d_e, 4, hipMemcpyDeviceToHost, g_scr.s) != hipSuccess || hipStreamSynchronize(g_scr.s) != hipSuccess) {
    set_err("signal_energy: device call failed");
    return -1;
  }
  return e;
}

extern "C" int oai4g_awgn_batch(const int32_t *d_tx, size_t tx_stride, uint32_t tx_len, const int32_t *d_tail,
                                uint32_t tail_len, int32_t *d_rx, size_t rx_stride, int n, const int32_t *d_tx_lev,
                                double offset_db, uint64_t seed, uint32_t first_vector, void *stream)
{
  NEED_INIT(-1);
  if (n < 0 || (n > 0 && (!d_tx || !d_rx || !d_tx_lev || (tail_len && !d_tail))) || n > 65535 ||
      tx_len + tail_len == 0) {
    set_err("awgn_batch: bad arguments");
    return -1;
  }
  HCK(oai4g_launch_awgn(d_tx, tx_stride, tx_len, d_tail, tail_len, d_rx, rx_stride, n, d_tx_lev, offset_db, seed,
                        first_vector, (hipStream_t)stream), -1);
  return 0;
}

extern "C" int oai4g_fill_payload(uint8_t *d_payload, size_t bytes, uint64_t seed, void *stream)
{
  NEED_INIT(-1);
  HCK(oai4g_launch_fill(d_payload, bytes, seed, (hipStream_t)stream), -1);
  return 0;
}

/* ------------------------------------------------------------------------------------------
 * dlsch containers (new_eNB_dlsch / free_eNB_dlsch, dlsch_coding.c:85-220)
 * ---------------------------------------------------------------------------------------- */
extern "C" oai4g_dlsch_t *oai4g_new_dlsch(uint8_t Kmimo, uint8_t Mdlharq, uint8_t N_RB_DL)
{
  int bw_scaling = N_RB_DL == 6 ? 16 : (N_RB_DL == 25 ? 4 : (N_RB_DL == 50 ? 2 : 1));
  oai4g_dlsch_t *d = (oai4g_dlsch_t *)calloc(1, sizeof(oai4g_dlsch_t));
  if (!d) return nullptr;
  d->Kmimo = Kmimo;
  d->Mdlharq = Mdlharq;
  d->sqrt_rho_a = 8192;
  d->sqrt_rho_b = 8192;
  for (int i = 0; i < Mdlharq && i < 8; i++) {
    oai4g_dl_harq_t *h = (oai4g_dl_harq_t *)calloc(1, sizeof(oai4g_dl_harq_t));
    d->harq_processes[i] = h;
    h->b = (uint8_t *)calloc(OAI4G_MAX_SEGMENTS * 768 / bw_scaling + 8, 1);
    h->e = (uint8_t *)calloc(OAI4G_MAX_CHANNEL_BITS + 64, 1);
    h->Nl = 1;
    for (int r = 0; r < OAI4G_MAX_SEGMENTS; r++) {
      h->c[r] = (uint8_t *)calloc(8 + 3 + 768, 1);
      h->d[r] = (uint8_t *)calloc(OAI4G_D_BYTES + 16, 1);
      h->w[r] = (uint8_t *)calloc(OAI4G_W_BYTES, 1);
      memset(h->d[r], OAI4G_LTE_NULL, 96);
    }
  }
  return d;
}

extern "C" void oai4g_free_dlsch(oai4g_dlsch_t *d)
{
  if (!d) return;
  for (int i = 0; i < 8; i++) {
    oai4g_dl_harq_t *h = d->harq_processes[i];
    if (!h) continue;
    for (int r = 0; r < OAI4G_MAX_SEGMENTS; r++) { free(h->c[r]); free(h->d[r]); free(h->w[r]); }
    free(h->b);
    free(h->e);
    free(h);
  }
  free(d);
}

/* lte_gold_generic (lte_gold.c:151-177): host-side scalar helper */
extern "C" uint32_t oai4g_lte_gold_generic(uint32_t *x1, uint32_t *x2, uint8_t reset)
{
  if (reset) {
    *x1 = 1u + (1u << 31);
    *x2 = *x2 ^ ((*x2 ^ (*x2 >> 1) ^ (*x2 >> 2) ^ (*x2 >> 3)) << 31);
    for (int n = 1; n < 50; n++) gold_step_h(x1, x2);
  }
  gold_step_h(x1, x2);
  return *x1 ^ *x2;
}

/* ------------------------------------------------------------------------------------------
 * drop-in coding entry points
 * ---------------------------------------------------------------------------------------- */
static uint32_t crc_dropin(const uint8_t *in, int bitlen, uint32_t poly_top)
{
  NEED_INIT(0);
  uint32_t nbytes = (uint32_t)(bitlen + 7) / 8;
  uint8_t *buf = scratch(nbytes + 64);
  if (!buf) { set_err("scratch allocation failed"); return 0; }
  uint32_t *d_out = (uint32_t *)(buf + ((nbytes + 15) & ~15u));
  uint32_t out = 0;
  HCK(hipMemcpyAsync(buf, in, nbytes, hipMemcpyHostToDevice, g_scr.s), 0);
  HCK(oai4g_launch_crc24(buf, bitlen, poly_top, d_out, g_scr.s), 0);
  HCK(hipMemcpyAsync(&out, d_out, 4, hipMemcpyDeviceToHost, g_scr.s), 0);
  HCK(hipStreamSynchronize(g_scr.s), 0);
  return out;
}

extern "C" uint32_t oai4g_crc24a(const uint8_t *in, int bitlen) { return crc_dropin(in, bitlen, 0x864cfb00u); }
extern "C" uint32_t oai4g_crc24b(const uint8_t *in, int bitlen) { return crc_dropin(in, bitlen, 0x80006300u); }

extern "C" int oai4g_lte_segmentation(const uint8_t *input_buffer, uint8_t **output_buffers, uint32_t B, uint32_t *C,
                                      uint32_t *Cplus, uint32_t *Cminus, uint32_t *Kplus, uint32_t *Kminus,
                                      uint32_t *F)
{
  uint32_t L;
  if (seg_params(B, C, Cplus, Cminus, Kplus, Kminus, F, &L) < 0) return -1;
  if (input_buffer && output_buffers) {
    uint32_t k = 0, s = 0;
    for (; k < (*F >> 3); k++) output_buffers[0][k] = 0;
    for (uint32_t r = 0; r < *C; r++) {
      uint32_t Kr = r < *Cminus ? *Kminus : *Kplus;
      for (; k < ((Kr - L) >> 3); k++) output_buffers[r][k] = input_buffer[s++];
      if (*C > 1) {
        uint32_t crc = oai4g_crc24b(output_buffers[r], (int)(Kr - 24)) >> 8;
        output_buffers[r][(Kr - 24) >> 3] = (uint8_t)(crc >> 16);
        output_buffers[r][1 + ((Kr - 24) >> 3)] = (uint8_t)(crc >> 8);
        output_buffers[r][2 + ((Kr - 24) >> 3)] = (uint8_t)crc;
      }
      k = 0;
    }
  }
  return 0;
}

extern "C" void oai4g_threegpplte_turbo_encoder(const uint8_t *input, uint16_t input_length_bytes, uint8_t *output,
                                                uint8_t F, uint16_t f1, uint16_t f2)
{
  (void)F; /* the reference's SSE encoder ignores F (3gpplte_sse.c:380-476) */
  NEED_INIT();
  uint32_t K = (uint32_t)input_length_bytes * 8;
  if (oai4g_qpp_index(K) < 0) {
    printf("Illegal frame length!\n");
    return;
  }
  uint8_t *buf = scratch(1024 + 3 * 6144 + 64);
  if (!buf) return;
  HCK(hipMemcpyAsync(buf, input, input_length_bytes, hipMemcpyHostToDevice, g_scr.s), );
  HCK(oai4g_launch_turbo_bytes(buf, input_length_bytes, buf + 1024, f1, f2, g_scr.s), );
  HCK(hipMemcpyAsync(output, buf + 1024, 3 * K + 12, hipMemcpyDeviceToHost, g_scr.s), );
  HCK(hipStreamSynchronize(g_scr.s), );
}

extern "C" uint32_t oai4g_sub_block_interleaving_turbo(uint32_t D, uint8_t *d, uint8_t *w)
{
  NEED_INIT(0);
  uint32_t R = (D + 31) >> 5, Kpi = R << 5;
  size_t dbytes = 96 + 3 * (size_t)D + 3;
  uint8_t *buf = scratch(dbytes + 3 * Kpi + 64);
  if (!buf) return 0;
  HCK(hipMemcpyAsync(buf, d - 96, dbytes, hipMemcpyHostToDevice, g_scr.s), 0);
  HCK(oai4g_launch_subblock_bytes(D, buf, buf + ((dbytes + 15) & ~(size_t)15), g_scr.s), 0);
  HCK(hipMemcpyAsync(w, buf + ((dbytes + 15) & ~(size_t)15), 3 * Kpi, hipMemcpyDeviceToHost, g_scr.s), 0);
  HCK(hipStreamSynchronize(g_scr.s), 0);
  d[3 * D + 2] = d[2]; /* side effect kept (lte_rate_matching.c:75) */
  return R;
}

extern "C" uint32_t oai4g_lte_rate_matching_turbo(uint32_t RTC, uint32_t G, const uint8_t *w, uint8_t *e, uint8_t C,
                                                  uint32_t Nsoft, uint8_t Mdlharq, uint8_t Kmimo, uint8_t rvidx,
                                                  uint8_t Qm, uint8_t Nl, uint8_t r, uint8_t nb_rb, uint8_t m)
{
  (void)nb_rb;
  (void)m;
  NEED_INIT(0);
  uint32_t Kw = 3 * (RTC << 5);
  uint32_t Nir = Nsoft / Kmimo / (Mdlharq < 8 ? Mdlharq : 8);
  uint32_t Ncb = (Nir / C < Kw) ? Nir / C : Kw;
  if (Ncb < Kw) {
    printf("Exiting, RM condition (Nir %u, Nsoft %u, Kw %u\n", Nir, Nsoft, Kw);
    return 0;
  }
  uint32_t Gp = G / Nl / Qm, GpmodC = Gp % C, E;
  if (r < (C - GpmodC)) E = Nl * Qm * (Gp / C);
  else E = Nl * Qm * ((GpmodC == 0 ? 0 : 1) + (Gp / C));
  uint32_t ncol8 = RTC << 3;
  uint32_t k0 = RTC * (2 + rvidx * ((Ncb % ncol8 ? 1 : 0) + Ncb / ncol8) * 2);
  size_t woff = 0, eoff = (Ncb + 63) & ~(size_t)63, soff = eoff + ((E + 63) & ~(size_t)63);
  uint8_t *buf = scratch(soff + 64);
  if (!buf) return 0;
  HCK(hipMemcpyAsync(buf + woff, w, Ncb, hipMemcpyHostToDevice, g_scr.s), 0);
  HCK(oai4g_launch_rm_bytes(buf + woff, Ncb, k0, E, buf + eoff, (uint32_t *)(buf + soff), g_scr.s), 0);
  HCK(hipMemcpyAsync(e, buf + eoff, E, hipMemcpyDeviceToHost, g_scr.s), 0);
  HCK(hipStreamSynchronize(g_scr.s), 0);
  return E;
}

/* parameter block for a single-DLSCH drop-in call */
static void params_from_dlsch(const oai4g_frame_parms_t *fp, uint8_t num_pdcch, const oai4g_dlsch_t *d0,
                              const oai4g_dlsch_t *d1, uint8_t subframe, oai4g_tx_params_t *p, uint8_t Nl[2])
{
  memset(p, 0, sizeof(*p));
  const oai4g_dl_harq_t *h0 = d0->harq_processes[d0->current_harq_pid];
  p->N_RB_DL = fp->N_RB_DL;
  p->Nid_cell = fp->Nid_cell;
  p->Ncp = fp->Ncp;
  p->nb_antennas_tx = fp->nb_antennas_tx;
  p->mode1_flag = fp->mode1_flag;
  p->frame_type = fp->frame_type;
  p->n_cw = d1 ? 2 : 1;
  p->mimo_mode = h0->mimo_mode;
  p->num_pdcch_symbols = num_pdcch;
  p->Kmimo = d0->Kmimo;
  p->Mdlharq = d0->Mdlharq;
  p->first_subframe = subframe;
  p->subframe_step = 0;
  p->rnti = d0->rnti;
  p->amp = 512;
  p->sqrt_rho_a = d0->sqrt_rho_a;
  p->sqrt_rho_b = d0->sqrt_rho_b;
  memcpy(p->rb_alloc, h0->rb_alloc, sizeof(p->rb_alloc));
  p->nb_rb = h0->nb_rb;
  p->mcs[0] = h0->mcs;
  p->rvidx[0] = h0->rvidx;
  p->TBS[0] = h0->TBS;
  Nl[0] = h0->Nl ? h0->Nl : 1;
  Nl[1] = 1;
  if (d1) {
    const oai4g_dl_harq_t *h1 = d1->harq_processes[d0->current_harq_pid];
    p->mcs[1] = h1->mcs;
    p->rvidx[1] = h1->rvidx;
    p->TBS[1] = h1->TBS;
    Nl[1] = h1->Nl ? h1->Nl : 1;
  }
  uint32_t maxA = p->TBS[0] / 8;
  if (d1 && p->TBS[1] / 8 > maxA) maxA = p->TBS[1] / 8;
  p->payload_stride = (maxA + 3 + 15) & ~15u;
}

extern "C" int oai4g_dlsch_encoding(uint8_t *a, const oai4g_frame_parms_t *frame_parms, uint8_t num_pdcch_symbols,
                                    oai4g_dlsch_t *dlsch, int frame, uint8_t subframe)
{
  (void)frame;
  NEED_INIT(-1);
  oai4g_dl_harq_t *h = dlsch->harq_processes[dlsch->current_harq_pid];
  if (h->round != 0) {
    set_err("dlsch_encoding: retransmission rounds re-use the stored w (not supported by the drop-in yet)");
    return -1;
  }
  oai4g_tx_params_t p;
  uint8_t Nl[2];
  params_from_dlsch(frame_parms, num_pdcch_symbols, dlsch, nullptr, subframe, &p, Nl);
  if (p.mimo_mode == OAI4G_ALAMOUTI || p.mimo_mode == OAI4G_LARGE_CDD) p.mimo_mode = OAI4G_SISO; /* coding only */
  if (p.N_RB_DL != 6 && p.N_RB_DL != 15 && p.N_RB_DL != 25 && p.N_RB_DL != 50 && p.N_RB_DL != 100) return -1;
  oai4g_tx_config cfg;
  int rc = derive_cfg(&cfg, &p, Nl, false, -1);
  bool rm_fail = rc == -2; /* reference: every block's rate matcher returns E = 0, e untouched */
  if (rc != 0 && !rm_fail) return -1;
  if (upload_cfg(&cfg) != 0) { release_cfg(&cfg); return -1; }
  cw_dev_t &c = cfg.h.cw[0];
  uint32_t G = c.G[subframe % 10];
  size_t off_pay = 0, off_b = 16 * 1024, off_c = off_b + 16 * 1024, off_d = off_c + 16 * (8 + 3 + 768),
         off_w = off_d + 16 * (size_t)OAI4G_D_BYTES, off_e = off_w + 16 * (size_t)OAI4G_W_BYTES;
  uint8_t *buf = scratch(off_e + OAI4G_MAX_CHANNEL_BITS + 64);
  if (!buf) { release_cfg(&cfg); return -1; }
  HCK(hipMemcpyAsync(buf + off_pay, a, c.A_bytes, hipMemcpyHostToDevice, g_scr.s), -1);
  enc_debug_t dbg = {buf + off_c, buf + off_d, buf + off_w, rm_fail ? nullptr : buf + off_e, buf + off_b};
  HCK(oai4g_launch_encode_debug(cfg.d, &cfg.h, 0, subframe % 10, buf + off_pay, dbg, g_scr.s), -1);
  std::vector<uint8_t> hb(off_e + G);
  HCK(hipMemcpyAsync(hb.data(), buf, off_e + G, hipMemcpyDeviceToHost, g_scr.s), -1);
  HCK(hipStreamSynchronize(g_scr.s), -1);
  release_cfg(&cfg);
  /* CRC appended into the caller's buffer and copied to b (dlsch_coding.c:296-305) */
  memcpy(a + c.A_bytes, hb.data() + off_b + c.A_bytes, 3);
  h->B = c.TBS + 24;
  memcpy(h->b, a, c.A_bytes + 4); /* memcpy(b, a, A/8 + 4) (dlsch_coding.c:305) */
  h->C = c.C; h->Cplus = c.C - c.Cminus; h->Cminus = c.Cminus; h->Kplus = c.Kplus; h->Kminus = c.Kminus; h->F = c.F;
  for (uint32_t r = 0; r < c.C; r++) {
    uint32_t K = c.K[r];
    memcpy(h->c[r], hb.data() + off_c + r * (8 + 3 + 768), K / 8);
    memcpy(h->d[r], hb.data() + off_d + r * (size_t)OAI4G_D_BYTES, 96 + 3 * (K + 4) + 3);
    memcpy(h->w[r], hb.data() + off_w + r * (size_t)OAI4G_W_BYTES, 3 * c.Kpi[r]);
    h->RTC[r] = c.R[r];
  }
  if (!rm_fail) memcpy(h->e, hb.data() + off_e, G);
  return 0;
}

extern "C" void oai4g_dlsch_scrambling(const oai4g_frame_parms_t *frame_parms, int mbsfn_flag, oai4g_dlsch_t *dlsch,
                                       int G, uint8_t q, uint8_t Ns)
{
  NEED_INIT();
  uint8_t *e = dlsch->harq_processes[dlsch->current_harq_pid]->e;
  uint32_t x2 = mbsfn_flag == 0 ? ((uint32_t)dlsch->rnti << 14) + ((uint32_t)q << 13) + ((uint32_t)(Ns >> 1) << 9) +
                                      frame_parms->Nid_cell
                                : ((uint32_t)(Ns >> 1) << 9) + frame_parms->Nid_cell_mbsfn;   /* :70-72 */
  int n = (1 + (G >> 5)) * 32; /* the reference writes past G (dlsch_scrambling.c:83-92) */
  uint8_t *buf = scratch((size_t)n + 64);
  if (!buf) return;
  HCK(hipMemcpyAsync(buf, e, n, hipMemcpyHostToDevice, g_scr.s), );
  HCK(oai4g_launch_scramble_bytes(buf, n, x2, g_gx1, g_gx2j, g_scr.s), );
  HCK(hipMemcpyAsync(e, buf, n, hipMemcpyDeviceToHost, g_scr.s), );
  HCK(hipStreamSynchronize(g_scr.s), );
}

extern "C" int oai4g_dlsch_modulation(int32_t **txdataF, int16_t amp, uint32_t subframe_offset,
                                      const oai4g_frame_parms_t *frame_parms, uint8_t num_pdcch_symbols,
                                      oai4g_dlsch_t *dlsch0, oai4g_dlsch_t *dlsch1)
{
  NEED_INIT(-1);
  oai4g_tx_params_t p;
  uint8_t Nl[2];
  params_from_dlsch(frame_parms, num_pdcch_symbols, dlsch0, dlsch1, (uint8_t)(subframe_offset % 10), &p, Nl);
  const oai4g_dl_harq_t *h0 = dlsch0->harq_processes[dlsch0->current_harq_pid];
  if (h0->Nlayers > 1) return -1;
  p.amp = amp;
  if (p.mimo_mode == OAI4G_LARGE_CDD && !dlsch1) p.n_cw = 1;
  if (p.mimo_mode == OAI4G_ALAMOUTI) p.n_cw = 1;       /* both symbols of a pair come from dlsch0 */
  if (p.mimo_mode != OAI4G_SISO && p.mimo_mode != OAI4G_LARGE_CDD && p.mimo_mode != OAI4G_ALAMOUTI) {
    set_err("dlsch_modulation: mimo_mode %u not supported", p.mimo_mode);
    return -1;
  }
  /* coding geometry is irrelevant here; use the grid-only derivation */
  oai4g_tx_config cfg;
  if (p.mimo_mode == OAI4G_LARGE_CDD && p.n_cw == 1) {
    set_err("LARGE_CDD with one codeword is not supported");
    return -1;
  }
  int rc = derive_cfg(&cfg, &p, Nl, true, (int)(subframe_offset % 10));
  if (rc != 0 && rc != -2) return -1;
  if (upload_cfg(&cfg) != 0) { release_cfg(&cfg); return -1; }
  int sf = (int)(subframe_offset % 10);
  uint32_t N = cfg.h.N, nsymb = cfg.h.nsymb, nant = cfg.h.n_ant;
  size_t grid_bytes = (size_t)nant * nsymb * N * 4;
  uint32_t n_re = (uint32_t)cfg.re_count[sf];
  size_t e0_bytes = (size_t)n_re * cfg.h.cw[0].Qm + 64, e1_bytes = p.n_cw > 1 ? (size_t)n_re * cfg.h.cw[1].Qm + 64 : 0;
  size_t off_e0 = (grid_bytes + 255) & ~(size_t)255, off_e1 = off_e0 + ((e0_bytes + 255) & ~(size_t)255);
  uint8_t *buf = scratch(off_e1 + e1_bytes + 64);
  if (!buf) { release_cfg(&cfg); return -1; }
  size_t sym_off = (size_t)N * subframe_offset * nsymb;
  for (uint32_t aa = 0; aa < nant; aa++)
    HCK(hipMemcpyAsync(buf + (size_t)aa * nsymb * N * 4, txdataF[aa] + sym_off, (size_t)nsymb * N * 4,
                       hipMemcpyHostToDevice, g_scr.s), -1);
  HCK(hipMemcpyAsync(buf + off_e0, h0->e, (size_t)n_re * cfg.h.cw[0].Qm, hipMemcpyHostToDevice, g_scr.s), -1);
  if (p.n_cw > 1)
    HCK(hipMemcpyAsync(buf + off_e1, dlsch1->harq_processes[dlsch0->current_harq_pid]->e,
                       (size_t)n_re * cfg.h.cw[1].Qm, hipMemcpyHostToDevice, g_scr.s), -1);
  HCK(oai4g_launch_modulate_bytes(cfg.d, &cfg.h, sf, buf + off_e0, p.n_cw > 1 ? buf + off_e1 : nullptr,
                                  (int32_t *)buf, g_scr.s), -1);
  for (uint32_t aa = 0; aa < nant; aa++)
    HCK(hipMemcpyAsync(txdataF[aa] + sym_off, buf + (size_t)aa * nsymb * N * 4, (size_t)nsymb * N * 4,
                       hipMemcpyDeviceToHost, g_scr.s), -1);
  HCK(hipStreamSynchronize(g_scr.s), -1);
  const int ret = cfg.re_alloc[sf];
  release_cfg(&cfg);
  return ret;
}

/* ------------------------------------------------------------------------------------------
 * drop-in OFDM entry points
 * ---------------------------------------------------------------------------------------- */
static int run_ofdm(const int32_t *input, size_t in_n, int32_t *output, size_t out_lo, size_t out_n, int log2n,
                    int nsym, const ofdm_sym_t *syms, int scale)
{
  NEED_INIT(-1);
  size_t in_bytes = in_n * 4, out_off = (in_bytes + 255) & ~(size_t)255;
  uint8_t *buf = scratch(out_off + out_n * 4 + 64);
  if (!buf) return -1;
  int32_t *d_in = (int32_t *)buf, *d_out = (int32_t *)(buf + out_off);
  HCK(hipMemcpyAsync(d_in, input, in_bytes, hipMemcpyHostToDevice, g_scr.s), -1);
  /* the output window is read-modify-write: samples outside the written symbols stay intact */
  HCK(hipMemcpyAsync(d_out, output + out_lo, out_n * 4, hipMemcpyHostToDevice, g_scr.s), -1);
  HCK(oai4g_launch_ofdm(d_in, d_out, log2n, nsym, syms, scale, g_tw, g_scr.s), -1);
  HCK(hipMemcpyAsync(output + out_lo, d_out, out_n * 4, hipMemcpyDeviceToHost, g_scr.s), -1);
  HCK(hipStreamSynchronize(g_scr.s), -1);
  return 0;
}

static bool log2n_ok(int l) { return l >= 6 && l <= 11; }
/* PHY_ofdm_mod's switch (ofdm_mod.c:103-127) names idft128..idft2048; any other size falls to its
 * default (idft512 over a 2^log2 stride, overlapping symbols), which the drop-in refuses instead */
static bool ofdm_log2_ok(int l) { return l >= 7 && l <= 11; }

extern "C" void oai4g_PHY_ofdm_mod(const int32_t *input, int32_t *output, uint8_t log2fftsize, uint8_t nb_symbols,
                                   uint16_t nb_prefix_samples, int etype)
{
  if (etype != OAI4G_CYCLIC_PREFIX) {
    set_err("PHY_ofdm_mod: only CYCLIC_PREFIX is supported");
    return;
  }
  if (!ofdm_log2_ok(log2fftsize) || nb_symbols == 0 || nb_symbols > 28) {
    set_err("PHY_ofdm_mod: unsupported size 2^%u or symbol count %u", log2fftsize, nb_symbols);
    return;
  }
  ofdm_sym_t syms[28];
  uint32_t N = 1u << log2fftsize;
  if (nb_prefix_samples > N) { /* the CP loop (ofdm_mod.c:167-171) would read in front of the symbol */
    set_err("PHY_ofdm_mod: prefix %u longer than the symbol", nb_prefix_samples);
    return;
  }
  for (int i = 0; i < nb_symbols; i++) {
    syms[i].in_off = (uint32_t)i * N;
    syms[i].out_off = (uint32_t)i * N + (uint32_t)(1 + i) * nb_prefix_samples;
    syms[i].cp = nb_prefix_samples;
  }
  size_t out_n = (size_t)nb_symbols * (N + nb_prefix_samples);
  run_ofdm(input, (size_t)nb_symbols * N, output, 0, out_n, log2fftsize, nb_symbols, syms, 1);
}

/* one slot = symbol 0 with CP0, then symbols 1..nsymb-1 with CP, in a single launch */
static void slot_syms(const oai4g_frame_parms_t *fp, uint32_t in_base, uint32_t out_base, int nsym_slot,
                      ofdm_sym_t *syms)
{
  uint32_t N = fp->ofdm_symbol_size;
  syms[0].in_off = in_base;
  syms[0].out_off = out_base + fp->nb_prefix_samples0;
  syms[0].cp = fp->nb_prefix_samples0;
  for (int i = 1; i < nsym_slot; i++) {
    syms[i].in_off = in_base + (uint32_t)i * N;
    syms[i].out_off = out_base + N + fp->nb_prefix_samples0 + (uint32_t)(i - 1) * N + (uint32_t)i * fp->nb_prefix_samples;
    syms[i].cp = fp->nb_prefix_samples;
  }
}

extern "C" void oai4g_normal_prefix_mod(const int32_t *txdataF, int32_t *txdata, uint8_t nsymb,
                                        const oai4g_frame_parms_t *fp)
{
  if (!ofdm_log2_ok(fp->log2_symbol_size)) { set_err("normal_prefix_mod: unsupported FFT size"); return; }
  uint32_t N = fp->ofdm_symbol_size;
  int short_offset = (2 * nsymb) < fp->symbols_per_tti;
  int nslots = short_offset + 2 * nsymb / fp->symbols_per_tti;
  ofdm_sym_t syms[28];
  int ns = 0;
  for (int i = 0; i < nslots; i++) {
    int per = short_offset ? 2 : (fp->symbols_per_tti >> 1);
    slot_syms(fp, (uint32_t)((i * N * fp->symbols_per_tti) >> 1), (uint32_t)((i * fp->samples_per_tti) >> 1), per,
              syms + ns);
    ns += per;
  }
  uint32_t in_n = 0, out_hi = 0;
  for (int i = 0; i < ns; i++) {
    in_n = syms[i].in_off + N > in_n ? syms[i].in_off + N : in_n;
    out_hi = syms[i].out_off + N > out_hi ? syms[i].out_off + N : out_hi;
  }
  run_ofdm(txdataF, in_n, txdata, 0, out_hi, fp->log2_symbol_size, ns, syms, 1);
}

extern "C" void oai4g_do_OFDM_mod(int32_t **txdataF, int32_t **txdata, uint32_t frame, uint16_t next_slot,
                                  const oai4g_frame_parms_t *fp)
{
  (void)frame;
  uint32_t slot_offset_F = (uint32_t)next_slot * fp->ofdm_symbol_size * (fp->Ncp == 1 ? 6 : 7);
  uint32_t slot_offset = (uint32_t)next_slot * (fp->samples_per_tti >> 1);
  for (int aa = 0; aa < fp->nb_antennas_tx; aa++) {
    if (fp->Ncp == 1)
      oai4g_PHY_ofdm_mod(txdataF[aa] + slot_offset_F, txdata[aa] + slot_offset, fp->log2_symbol_size, 6,
                         fp->nb_prefix_samples, OAI4G_CYCLIC_PREFIX);
    else
      oai4g_normal_prefix_mod(txdataF[aa] + slot_offset_F, txdata[aa] + slot_offset, 7, fp);
  }
}

/* ------------------------------------------------------------------------------------------
 * Cell-specific reference signals (pilots.c:43-168, lte_dl_cell_spec.c:123-203)
 * ---------------------------------------------------------------------------------------- */
static int run_crs(int32_t *const *grids, int n_grids, size_t grid_res, const crs_job_t *jobs, int n_jobs, int16_t amp,
                   const oai4g_frame_parms_t *fp)
{
  uint32_t gt[20][2][14];
  lte_gold_table_h(fp, gt);
  const size_t gbytes = sizeof(gt), jbytes = (size_t)n_jobs * sizeof(crs_job_t), dbytes = (size_t)n_grids * grid_res * 4;
  uint8_t *buf = scratch(gbytes + jbytes + dbytes + 256);
  if (!buf) return -1;
  uint32_t *d_gold = (uint32_t *)buf;
  crs_job_t *d_jobs = (crs_job_t *)(buf + ((gbytes + 15) & ~(size_t)15));
  int32_t *d_grid = (int32_t *)(buf + ((gbytes + 15) & ~(size_t)15) + ((jbytes + 255) & ~(size_t)255));
  HCK(hipMemcpyAsync(d_gold, gt, gbytes, hipMemcpyHostToDevice, g_scr.s), -1);
  HCK(hipMemcpyAsync(d_jobs, jobs, jbytes, hipMemcpyHostToDevice, g_scr.s), -1);
  for (int g = 0; g < n_grids; g++)
    HCK(hipMemcpyAsync(d_grid + g * grid_res, grids[g], grid_res * 4, hipMemcpyHostToDevice, g_scr.s), -1);
  HCK(oai4g_launch_crs(d_grid, d_jobs, n_jobs, d_gold, amp, fp->ofdm_symbol_size, fp->N_RB_DL, fp->nushift,
                       fp->first_carrier_offset, g_scr.s), -1);
  for (int g = 0; g < n_grids; g++)
    HCK(hipMemcpyAsync(grids[g], d_grid + g * grid_res, grid_res * 4, hipMemcpyDeviceToHost, g_scr.s), -1);
  HCK(hipStreamSynchronize(g_scr.s), -1);
  return 0;
}

extern "C" void oai4g_generate_pilots(int32_t **txdataF, int16_t amp, const oai4g_frame_parms_t *fp, uint16_t Ntti)
{
  NEED_INIT();
  const uint32_t N = fp->ofdm_symbol_size, Nsymb = fp->Ncp == 0 ? 14 : 12, second = fp->Ncp == 0 ? 4 : 3;
  const int n_ant = fp->nb_antennas_tx > 1 ? 2 : 1;
  std::vector<crs_job_t> jobs;
  for (uint32_t tti = 0; tti < Ntti; tti++) {
    const uint32_t base = tti * N * Nsymb, slot = (tti * 2) % 20;
    const uint32_t sym[4] = {0, second, Nsymb >> 1, (Nsymb >> 1) + second};
    for (int i = 0; i < 4; i++)
      for (int a = 0; a < n_ant; a++) {
        const size_t grid_res = (size_t)Ntti * N * Nsymb;
        crs_job_t j;
        j.off = (uint32_t)(a * grid_res + base + sym[i] * N);
        j.Ns = (uint8_t)(slot + (i >> 1));
        j.l = (uint8_t)(i & 1);
        j.p = (uint8_t)(a == 0 || fp->mode1_flag ? 0 : 1);
        j.pad = 0;
        jobs.push_back(j);
      }
  }
  run_crs(txdataF, n_ant, (size_t)Ntti * N * Nsymb, jobs.data(), (int)jobs.size(), amp, fp);
}

extern "C" int oai4g_lte_dl_cell_spec(int32_t *output, int16_t amp, const oai4g_frame_parms_t *fp, uint8_t Ns,
                                      uint8_t l, uint8_t p)
{
  NEED_INIT(-1);
  if (p > 1 || l > 1 || Ns >= 20) {
    set_err("lte_dl_cell_spec: p %d, l %d -> ERROR", p, l);
    return -1;
  }
  crs_job_t j = {0, Ns, l, p, 0};
  return run_crs(&output, 1, fp->ofdm_symbol_size, &j, 1, amp, fp);
}

/* ------------------------------------------------------------------------------------------
 * Uplink turbo decoding (3gpplte_turbo_decoder_sse_16bit.c, lte_rate_matching.c)
 * ---------------------------------------------------------------------------------------- */
/* init_td16 (:898-943) for block size K: pi4 | pi5 | pi6 as uint16, uploaded once per K */
static const uint16_t *td_tables(uint32_t K)
{
  static std::mutex mu;
  static std::map<uint32_t, uint16_t *> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(K);
  if (it != cache.end()) return it->second;
  const int qi = oai4g_qpp_index(K);
  if (qi < 0) return nullptr;
  const uint64_t f1 = oai4g_qpp_table[qi].f1, f2 = oai4g_qpp_table[qi].f2;
  std::vector<uint32_t> pi2(K);
  for (uint32_t i = 0, i2 = 0; i2 < 8; i2++)
    for (uint32_t i3 = 0, j = i2; i3 < K / 8; i3++, i++, j += 8) pi2[i] = j;
  std::vector<uint16_t> t(3 * (size_t)K);
  for (uint32_t i = 0; i < K; i++) {
    const uint32_t pi = (uint32_t)((f1 * i + f2 * (uint64_t)i * i) % K), pi3 = pi2[pi];
    t[pi2[i]] = (uint16_t)pi3;          /* pi4 */
    t[K + pi3] = (uint16_t)pi2[i];      /* pi5 */
    t[2 * K + pi] = (uint16_t)pi2[i];   /* pi6 */
  }
  uint16_t *d = nullptr;
  if (hipMalloc(&d, t.size() * 2) != hipSuccess || hipMemcpy(d, t.data(), t.size() * 2, hipMemcpyHostToDevice) != hipSuccess) {
    set_err("decoder table upload failed");
    return nullptr;
  }
  cache[K] = d;
  return d;
}

/* init_td8 (3gpplte_turbo_decoder_sse_8bit.c:846-892) for K % 16 == 0: 16 windows */
static const uint16_t *td8_tables(uint32_t K)
{
  static std::mutex mu;
  static std::map<uint32_t, uint16_t *> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(K);
  if (it != cache.end()) return it->second;
  const int qi = oai4g_qpp_index(K);
  if (qi < 0 || (K & 15)) return nullptr;
  const uint64_t f1 = oai4g_qpp_table[qi].f1, f2 = oai4g_qpp_table[qi].f2;
  std::vector<uint32_t> pi2(K);
  for (uint32_t i = 0, j = 0; i < K; i++, j += 16) {
    if (j >= K) j -= (K - 1);
    pi2[i] = j;
  }
  std::vector<uint16_t> t(3 * (size_t)K);
  for (uint32_t i = 0; i < K; i++) {
    const uint32_t pi = (uint32_t)((f1 * i + f2 * (uint64_t)i * i) % K), pi3 = pi2[pi];
    t[pi2[i]] = (uint16_t)pi3;          /* pi4 */
    t[K + pi3] = (uint16_t)pi2[i];      /* pi5 */
    t[2 * K + pi] = (uint16_t)pi2[i];   /* pi6 */
  }
  uint16_t *d = nullptr;
  if (hipMalloc(&d, t.size() * 2) != hipSuccess || hipMemcpy(d, t.data(), t.size() * 2, hipMemcpyHostToDevice) != hipSuccess) {
    set_err("decoder8 table upload failed");
    return nullptr;
  }
  cache[K] = d;
  return d;
}

extern "C" size_t oai4g_td8_scratch_bytes(uint16_t K, int n_cb) { return (size_t)((n_cb + 3) / 4) * oai4g_td8_wave_bytes(K); }

extern "C" int oai4g_td8_batch(int n_cb, uint16_t K, const int16_t *d_llr, size_t llr_stride, uint8_t *d_out,
                               size_t out_stride, uint8_t *d_iters, uint8_t max_iterations, uint8_t crc_type, uint8_t F,
                               void *d_scratch, void *stream)
{
  NEED_INIT(-1);
  if (crc_type > OAI4G_CRC24_B) { set_err("turbo decoder8: only CRC24_A / CRC24_B are on the path"); return -1; }
  if ((K & 15) || K < 512 || oai4g_qpp_index(K) < 0) {
    set_err("turbo decoder8: K %u outside n %% 16 == 0, n >= 512 (the reference reads past its tables there)", K);
    return -1;
  }
  if ((F & 7) || F + 24 > K) { set_err("turbo decoder8: filler F=%u unsupported", F); return -1; }
  if (llr_stride < 3 * (size_t)K + 16) { set_err("turbo decoder8: llr_stride < 3K + 16"); return -1; }
  const uint16_t *pi = td8_tables(K);
  if (!pi) return -1;
  HCK(oai4g_launch_td8(n_cb, K, d_llr, llr_stride, d_out, out_stride, d_iters, max_iterations, crc_type, F, pi,
                       (uint8_t *)d_scratch, (hipStream_t)stream), -1);
  return 0;
}

/* phy_threegpplte_turbo_decoder8 drop-in: y = 3n + 12 int16 (the reference's conversion reads 4 more
 * entries; they only reach its unused tail and are taken as 0 here); decoded_bytes n/8 bytes. */
extern "C" uint8_t oai4g_phy_threegpplte_turbo_decoder8(const int16_t *y, uint8_t *decoded_bytes, uint16_t n,
                                                       uint16_t f1, uint16_t f2, uint8_t max_iterations,
                                                       uint8_t crc_type, uint8_t F)
{
  (void)f1;
  (void)f2;
  if (oai4g_init() != 0) return 255;
  if ((n & 15) || n < 512 || oai4g_qpp_index(n) < 0 || crc_type > OAI4G_CRC24_B) {
    set_err("turbo decoder8: n %u / crc %u outside the restated scope", n, crc_type);
    return 255;
  }
  const size_t ly = 3 * (size_t)n + 16, b_y = (ly * 2 + 255) & ~(size_t)255, b_o = ((size_t)n / 8 + 256) & ~(size_t)255;
  const size_t b_s = oai4g_td8_scratch_bytes(n, 1);
  uint8_t *buf = scratch(b_y + b_o + 256 + b_s);
  if (!buf) return 255;
  int16_t *dy = (int16_t *)buf;
  uint8_t *dout = buf + b_y, *dit = dout + b_o, *dscr = dit + 256;
  std::vector<int16_t> h(ly, 0);
  memcpy(h.data(), y, (3 * (size_t)n + 12) * 2);
  uint8_t itc = 255;
  if (hipMemcpyAsync(dy, h.data(), ly * 2, hipMemcpyHostToDevice, g_scr.s) != hipSuccess ||
      hipMemcpyAsync(dout, decoded_bytes, n / 8, hipMemcpyHostToDevice, g_scr.s) != hipSuccess ||
      oai4g_td8_batch(1, n, dy, ly, dout, n / 8, dit, max_iterations, crc_type, F, dscr, g_scr.s) != 0 ||
      hipMemcpyAsync(decoded_bytes, dout, n / 8, hipMemcpyDeviceToHost, g_scr.s) != hipSuccess ||
      hipMemcpyAsync(&itc, dit, 1, hipMemcpyDeviceToHost, g_scr.s) != hipSuccess ||
      hipStreamSynchronize(g_scr.s) != hipSuccess) {
    set_err("turbo decoder8: HIP error");
    return 255;
  }
  return itc;
}

/* per wave of 8 blocks (the decoder interleaves a wave's blocks in its scratch) */
extern "C" size_t oai4g_td_scratch_bytes(uint16_t K, int n_cb) { return (size_t)((n_cb + 7) & ~7) * oai4g_td_block_bytes(K); }

extern "C" int oai4g_td_batch(int n_cb, uint16_t K, const int16_t *d_llr, size_t llr_stride, uint8_t *d_out,
                              size_t out_stride, uint8_t *d_iters, uint8_t max_iterations, uint8_t crc_type, uint8_t F,
                              void *d_scratch, void *stream)
{
  NEED_INIT(-1);
  if (crc_type > OAI4G_CRC24_B) { set_err("turbo decoder: only CRC24_A / CRC24_B are on the path"); return -1; }
  if ((F & 7) || F + 24 > K) { set_err("turbo decoder: filler F=%u unsupported", F); return -1; }
  const uint16_t *pi = td_tables(K);
  if (!pi) { set_err("Illegal frame length %u", K); return -1; }
  HCK(oai4g_launch_td16(n_cb, K, d_llr, llr_stride, d_out, out_stride, d_iters, max_iterations, crc_type, F, pi,
                        (uint8_t *)d_scratch, (hipStream_t)stream), -1);
  return 0;
}

/* generate_dummy_w (lte_rate_matching.c:293-382): LTE_NULL marks of the 3 Kpi circular buffer of a
 * block of D = K + 4 bits with F filler bits; returns R (RTC) */
static uint32_t dummy_w_h(uint32_t D, uint32_t F, std::vector<uint8_t> &w)
{
  const uint32_t R = (D >> 5) + ((D & 31) ? 1 : 0), Kpi = R << 5, ND = Kpi - D;
  w.assign(3 * (size_t)Kpi, 0);
  for (uint32_t col = 0, k = 0; col < 32; col++, k += R) {
    const uint32_t index = __builtin_bitreverse32(col) >> 27;
    if (index < ND + F) { w[k] = OAI4G_LTE_NULL; w[Kpi + 2 * k] = OAI4G_LTE_NULL; }
    if (index + 32 < ND + F) { w[k + 1] = OAI4G_LTE_NULL; w[Kpi + 2 + 2 * k] = OAI4G_LTE_NULL; }
    if (index + 64 < ND + F) { w[k + 2] = OAI4G_LTE_NULL; w[Kpi + 4 + 2 * k] = OAI4G_LTE_NULL; }
    if (index + 1 < ND) w[Kpi + 1 + 2 * k] = OAI4G_LTE_NULL;
  }
  if (ND > 0) w[3 * Kpi - 1] = OAI4G_LTE_NULL;
  return R;
}

extern "C" uint32_t oai4g_generate_dummy_w(uint32_t D, uint8_t *w, uint8_t F)
{
  std::vector<uint8_t> v;
  const uint32_t R = dummy_w_h(D, F, v);
  for (size_t i = 0; i < v.size(); i++)
    if (v[i] == OAI4G_LTE_NULL) w[i] = OAI4G_LTE_NULL;   /* the reference only writes the NULL marks */
  return R;
}

/* ------------------------------------------------------------------------------------------
 * Batched UL receive chain (ulsch_decoding.c:1208-1350): n_tb transport blocks of one
 * configuration, e soft bits -> RM-rx + sub-block deinterleaving (k_ul_rm_deint) -> 16-bit turbo
 * decoding (k_td16, one launch per block size) with CRC24B / CRC24A early stop.
 * ---------------------------------------------------------------------------------------- */
struct oai4g_ul_config {
  ul_dev_t h;
  ul_dev_t *d = nullptr;
  uint32_t B, G, C, Cminus, Kminus, Kplus, F, max_it;
  std::vector<void *> dev;
  size_t d_stride = 0;
  int cap = 0;
  int16_t *d_dfull = nullptr;
  uint8_t *d_td = nullptr;
  int bits = 16;                  /* 16: phy_threegpplte_turbo_decoder16; 8: the 8-bit decoder (llr8_flag) */
};

extern "C" void oai4g_ul_config_destroy(oai4g_ul_config_t *cfg)
{
  if (!cfg) return;
  for (void *p : cfg->dev) hipFree(p);
  if (cfg->d_dfull) hipFree(cfg->d_dfull);
  if (cfg->d_td) hipFree(cfg->d_td);
  if (cfg->d) hipFree(cfg->d);
  delete cfg;
}

extern "C" oai4g_ul_config_t *oai4g_ul_config_create(uint32_t B, uint32_t G, uint8_t Qm, uint8_t rvidx, uint8_t Mdlharq,
                                                     uint32_t Nsoft, uint8_t max_iterations)
{
  NEED_INIT(nullptr);
  auto *cfg = new oai4g_ul_config();
  uint32_t Cplus, L;
  if (Qm == 0 || Mdlharq == 0 || rvidx > 3 ||
      seg_params(B, &cfg->C, &Cplus, &cfg->Cminus, &cfg->Kplus, &cfg->Kminus, &cfg->F, &L) < 0 ||
      cfg->C > OAI4G_UL_MAX_C || (cfg->F & 7) || cfg->F + 24 > cfg->Kplus) {
    set_err("ul_config: unsupported (B %u, Qm %u, rv %u, Mdlharq %u)", B, Qm, rvidx, Mdlharq);
    delete cfg;
    return nullptr;
  }
  cfg->B = B;
  cfg->G = G;
  cfg->max_it = max_iterations;
  ul_dev_t &h = cfg->h;
  memset(&h, 0, sizeof(h));
  h.C = cfg->C;
  const uint32_t C = cfg->C, Nir = Nsoft / (Mdlharq < 8 ? Mdlharq : 8), Gp = G / Qm, GpmodC = Gp % C;
  uint32_t off = 0, npat = 0, keyK[3] = {0, 0, 0}, keyF[3] = {0, 0, 0};
  for (uint32_t r = 0; r < C; r++) {
    h.E[r] = r < C - GpmodC ? Qm * (Gp / C) : Qm * ((GpmodC == 0 ? 0 : 1) + Gp / C);   /* Nl = 1 */
    h.off[r] = off;
    off += h.E[r];
    const uint32_t K = r < cfg->Cminus ? cfg->Kminus : cfg->Kplus, Fr = r == 0 ? cfg->F : 0;
    uint32_t pi = 0;
    while (pi < npat && !(keyK[pi] == K && keyF[pi] == Fr)) pi++;
    if (pi == npat) {
      keyK[npat] = K;
      keyF[npat] = Fr;
      ul_pat_t &P = h.pat[npat++];
      std::vector<uint8_t> dw;
      P.D = K + 4;
      P.R = dummy_w_h(P.D, Fr, dw);
      const uint32_t Kw = 3 * (P.R << 5);
      P.Ncb = Nir / C < Kw ? Nir / C : Kw;
      const uint32_t Ncbmod = P.Ncb % (P.R << 3);
      const uint32_t k0 = P.R * (2 + (rvidx * (((Ncbmod == 0) ? 0 : 1) + (P.Ncb / (P.R << 3))) * 2));
      std::vector<uint32_t> cidx(P.Ncb);
      uint32_t nn = 0, k0c = 0;
      for (uint32_t q = 0; q < P.Ncb; q++) {
        if (q == k0) k0c = nn;
        cidx[q] = nn;
        if (dw[q] != OAI4G_LTE_NULL) nn++;
      }
      if (k0 >= P.Ncb) k0c = 0;
      P.Nnn = nn;
      P.k0c = k0c;
      for (uint32_t rv = 0; rv < 4; rv++) {        /* every round's k0 (lte_rate_matching.c:743-745) */
        const uint32_t k0r = P.R * (2 + (rv * (((Ncbmod == 0) ? 0 : 1) + (P.Ncb / (P.R << 3))) * 2));
        uint32_t c = 0;
        for (uint32_t q = 0; q < P.Ncb && q < k0r; q++) c += dw[q] != OAI4G_LTE_NULL;
        P.k0cr[rv] = k0r >= P.Ncb ? 0 : c;
      }
      if (P.R > h.Rmax) h.Rmax = P.R;
      uint8_t *dd = nullptr;
      uint32_t *dc = nullptr;
      if (hipMalloc(&dd, dw.size()) != hipSuccess || hipMalloc(&dc, cidx.size() * 4) != hipSuccess ||
          hipMemcpy(dd, dw.data(), dw.size(), hipMemcpyHostToDevice) != hipSuccess ||
          hipMemcpy(dc, cidx.data(), cidx.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
        if (dd) cfg->dev.push_back(dd);
        if (dc) cfg->dev.push_back(dc);
        set_err("ul_config: device allocation failed");
        oai4g_ul_config_destroy(cfg);
        return nullptr;
      }
      cfg->dev.push_back(dd);
      cfg->dev.push_back(dc);
      P.dummy = dd;
      P.cidx = dc;
    }
    h.pat_of[r] = pi;
  }
  if (!td_tables(cfg->Kplus) || (cfg->Cminus && !td_tables(cfg->Kminus))) { oai4g_ul_config_destroy(cfg); return nullptr; }
  cfg->d_stride = (96 + 3 * (size_t)cfg->Kplus + 12 + 15) & ~(size_t)15;
  if (hipMalloc(&cfg->d, sizeof(ul_dev_t)) != hipSuccess ||
      hipMemcpy(cfg->d, &h, sizeof(ul_dev_t), hipMemcpyHostToDevice) != hipSuccess) {
    set_err("ul_config: upload failed");
    oai4g_ul_config_destroy(cfg);
    return nullptr;
  }
  return cfg;
}

extern "C" int oai4g_ul_config_set_decoder(oai4g_ul_config_t *cfg, int bits)
{
  if (!cfg || (bits != 8 && bits != 16)) { set_err("ul_config_set_decoder: bits must be 8 or 16"); return -1; }
  if (bits == 8 && (cfg->Cminus || (cfg->Kplus & 15) || cfg->Kplus < 512 || (cfg->C == 1 && (cfg->F & 7)))) {
    set_err("ul_config_set_decoder: the 8-bit decoder needs one block size K %% 16 == 0, K >= 512 (K %u, C- %u)",
            cfg->Kplus, cfg->Cminus);
    return -1;
  }
  if (bits != cfg->bits) {          /* the scratch size differs: reallocate on the next batch */
    if (cfg->d_dfull) hipFree(cfg->d_dfull);
    if (cfg->d_td) hipFree(cfg->d_td);
    cfg->d_dfull = nullptr;
    cfg->d_td = nullptr;
    cfg->cap = 0;
  }
  cfg->bits = bits;
  return 0;
}

extern "C" int oai4g_ul_config_C(const oai4g_ul_config_t *cfg) { return (int)cfg->C; }
extern "C" uint32_t oai4g_ul_config_G_offset(const oai4g_ul_config_t *cfg, int r) { return cfg->h.off[r]; }
extern "C" uint32_t oai4g_ul_config_E(const oai4g_ul_config_t *cfg, int r) { return cfg->h.E[r]; }

static int ul_scratch(oai4g_ul_config_t *cfg, int n_tb)
{
  if (n_tb <= cfg->cap) return 0;
  if (cfg->d_dfull) hipFree(cfg->d_dfull);
  if (cfg->d_td) hipFree(cfg->d_td);
  cfg->d_dfull = nullptr;
  cfg->d_td = nullptr;
  const size_t nb = (size_t)n_tb * cfg->C;
  const size_t td = cfg->bits == 8 ? oai4g_td8_scratch_bytes((uint16_t)cfg->Kplus, (int)nb)
                                   : oai4g_td_scratch_bytes((uint16_t)cfg->Kplus, (int)nb);
  if (hipMalloc(&cfg->d_dfull, nb * cfg->d_stride * 2) != hipSuccess || hipMalloc(&cfg->d_td, td) != hipSuccess) {
    set_err("ul_decode_batch: device allocation failed");
    cfg->cap = 0;
    return -1;
  }
  cfg->cap = n_tb;
  return 0;
}

/* the decoders over the deinterleaved rows (one launch per block size) */
static int ul_decode_rows(oai4g_ul_config_t *cfg, int n_tb, uint8_t *d_c, size_t c_stride, uint8_t *d_iters,
                          hipStream_t s)
{
  const uint32_t crc = cfg->C == 1 ? OAI4G_CRC24_A : OAI4G_CRC24_B, F = cfg->C == 1 ? cfg->F : 0;
  const int16_t *y = cfg->d_dfull + 96;
  if (cfg->bits == 8) {
    /* every block of one size (set_decoder checked), rows (tb, r) in the d_c / d_iters order */
    const uint16_t *pi = td8_tables(cfg->Kplus);
    if (!pi) return -1;
    HCK(oai4g_launch_td8(n_tb * (int)cfg->C, cfg->Kplus, y, cfg->d_stride, d_c, c_stride, d_iters, cfg->max_it, crc, F,
                         pi, cfg->d_td, s), -1);
    return 0;
  }
  if (cfg->Cminus)
    HCK(oai4g_launch_td16(n_tb * (int)cfg->Cminus, cfg->Kminus, y, cfg->d_stride, d_c, c_stride, d_iters, cfg->max_it,
                          crc, F, td_tables(cfg->Kminus), cfg->d_td, s, cfg->Cminus, cfg->C, 0), -1);
  HCK(oai4g_launch_td16(n_tb * (int)(cfg->C - cfg->Cminus), cfg->Kplus, y, cfg->d_stride, d_c, c_stride, d_iters,
                        cfg->max_it, crc, F, td_tables(cfg->Kplus), cfg->d_td, s, cfg->C - cfg->Cminus, cfg->C,
                        cfg->Cminus), -1);
  return 0;
}

extern "C" int oai4g_ul_decode_batch(oai4g_ul_config_t *cfg, int n_tb, const int16_t *d_e, size_t e_stride,
                                     uint8_t *d_c, size_t c_stride, uint8_t *d_iters, void *stream)
{
  NEED_INIT(-1);
  if (n_tb <= 0) return 0;
  if (c_stride < cfg->Kplus / 8 || e_stride < cfg->G) { set_err("ul_decode_batch: strides too small"); return -1; }
  if (ul_scratch(cfg, n_tb) != 0) return -1;
  hipStream_t s = (hipStream_t)stream;
  HCK(oai4g_launch_ul_rm_deint(cfg->d, &cfg->h, n_tb, d_e, e_stride, cfg->d_dfull, cfg->d_stride, s), -1);
  return ul_decode_rows(cfg, n_tb, d_c, c_stride, d_iters, s);
}

extern "C" size_t oai4g_ul_config_w_entries(const oai4g_ul_config_t *cfg) { return 3 * ((size_t)cfg->h.Rmax << 5); }

/* the batch with HARQ soft combining: the decoders' input comes from the caller's per-block soft
 * buffers d_w, updated in place by this round (dlsch_decoding.c:348-383, ulsch_decoding.c:1262-1294) */
extern "C" int oai4g_ul_decode_batch_harq(oai4g_ul_config_t *cfg, int n_tb, const int16_t *d_e, size_t e_stride,
                                          int16_t *d_w, size_t w_stride, uint8_t rvidx, uint8_t clear, uint8_t *d_c,
                                          size_t c_stride, uint8_t *d_iters, void *stream)
{
  NEED_INIT(-1);
  if (n_tb <= 0) return 0;
  if (rvidx > 3 || clear > 1) { set_err("ul_decode_batch_harq: rvidx 0..3, clear 0 / 1"); return -1; }
  if (c_stride < cfg->Kplus / 8 || e_stride < cfg->G || w_stride < oai4g_ul_config_w_entries(cfg)) {
    set_err("ul_decode_batch_harq: strides too small");
    return -1;
  }
  if (ul_scratch(cfg, n_tb) != 0) return -1;
  hipStream_t s = (hipStream_t)stream;
  HCK(oai4g_launch_ul_rm_harq(cfg->d, &cfg->h, n_tb, d_e, e_stride, d_w, w_stride, rvidx, clear, cfg->d_dfull,
                              cfg->d_stride, s), -1);
  return ul_decode_rows(cfg, n_tb, d_c, c_stride, d_iters, s);
}

extern "C" uint8_t oai4g_phy_threegpplte_turbo_decoder16(const int16_t *y, uint8_t *decoded_bytes, uint16_t n,
                                                         uint16_t f1, uint16_t f2, uint8_t max_iterations,
                                                         uint8_t crc_type, uint8_t F)
{
  NEED_INIT(255);
  (void)f1; (void)f2;   /* the reference also selects its tables by n (:986) */
  if (crc_type > 3) { set_err("Illegal crc length!"); return 255; }
  if (oai4g_qpp_index(n) < 0) { set_err("Illegal frame length!"); return 255; }
  if (crc_type > OAI4G_CRC24_B) { set_err("turbo decoder: CRC16 / CRC8 are not on the path"); return 255; }
  const size_t ybytes = (3 * (size_t)n + 12) * 2, sbytes = oai4g_td_scratch_bytes(n, 1);
  uint8_t *buf = scratch(ybytes + 256 + (size_t)n / 8 + 256 + sbytes + 512);
  if (!buf) return 255;
  int16_t *d_y = (int16_t *)buf;
  uint8_t *d_iter = buf + ((ybytes + 255) & ~(size_t)255);
  uint8_t *d_out = d_iter + 256;
  uint8_t *d_scr = d_out + (((size_t)n / 8 + 255) & ~(size_t)255);
  HCK(hipMemcpyAsync(d_y, y, ybytes, hipMemcpyHostToDevice, g_scr.s), 255);
  HCK(hipMemcpyAsync(d_out, decoded_bytes, n / 8, hipMemcpyHostToDevice, g_scr.s), 255);   /* untouched if never decided */
  if (oai4g_td_batch(1, n, d_y, 3 * (size_t)n + 12, d_out, n / 8, d_iter, max_iterations, crc_type, F, d_scr, g_scr.s))
    return 255;
  uint8_t it = 0;
  HCK(hipMemcpyAsync(decoded_bytes, d_out, n / 8, hipMemcpyDeviceToHost, g_scr.s), 255);
  HCK(hipMemcpyAsync(&it, d_iter, 1, hipMemcpyDeviceToHost, g_scr.s), 255);
  HCK(hipStreamSynchronize(g_scr.s), 255);
  return it;
}

extern "C" int oai4g_lte_rate_matching_turbo_rx(uint32_t RTC, uint32_t G, int16_t *w, const uint8_t *dummy_w,
                                                const int16_t *soft_input, uint8_t C, uint32_t Nsoft, uint8_t Mdlharq,
                                                uint8_t Kmimo, uint8_t rvidx, uint8_t clear, uint8_t Qm, uint8_t Nl,
                                                uint8_t r, uint32_t *E_out)
{
  NEED_INIT(-1);
  if (Kmimo == 0 || Mdlharq == 0 || C == 0 || Qm == 0 || Nl == 0) return -1;
  const uint32_t Nir = Nsoft / Kmimo / (Mdlharq < 8 ? Mdlharq : 8), Kw = 3 * (RTC << 5);
  const uint32_t Ncb = Nir / C < Kw ? Nir / C : Kw, Gp = G / Nl / Qm, GpmodC = Gp % C;
  const uint32_t E = r < C - GpmodC ? Nl * Qm * (Gp / C) : Nl * Qm * ((GpmodC == 0 ? 0 : 1) + Gp / C);
  const uint32_t Ncbmod = Ncb % (RTC << 3);
  const uint32_t k0 = RTC * (2 + (rvidx * (((Ncbmod == 0) ? 0 : 1) + (Ncb / (RTC << 3))) * 2));
  /* compact (non-NULL) index of every w position, and of k0 */
  std::vector<uint32_t> cidx(Ncb);
  uint32_t nn = 0, k0c = 0;
  for (uint32_t p = 0; p < Ncb; p++) {
    if (p == k0) k0c = nn;
    cidx[p] = nn;
    if (dummy_w[p] != OAI4G_LTE_NULL) nn++;
  }
  if (k0 >= Ncb) k0c = 0;   /* the reference's first pass is empty; selection starts at 0 */
  if (nn == 0 && E > 0) { set_err("rate_matching_rx: no non-NULL entries"); return -1; }
  const size_t b_soft = (size_t)E * 2, b_w = (size_t)Ncb * 2, b_c = (size_t)Ncb * 4;
  uint8_t *buf = scratch(b_soft + b_w + b_c + Ncb + 1024);
  if (!buf) return -1;
  int16_t *d_soft = (int16_t *)buf;
  int16_t *d_w = (int16_t *)(buf + ((b_soft + 255) & ~(size_t)255));
  uint32_t *d_c = (uint32_t *)((uint8_t *)d_w + ((b_w + 255) & ~(size_t)255));
  uint8_t *d_dummy = (uint8_t *)d_c + ((b_c + 255) & ~(size_t)255);
  HCK(hipMemcpyAsync(d_soft, soft_input, b_soft, hipMemcpyHostToDevice, g_scr.s), -1);
  HCK(hipMemcpyAsync(d_w, w, b_w, hipMemcpyHostToDevice, g_scr.s), -1);
  HCK(hipMemcpyAsync(d_c, cidx.data(), b_c, hipMemcpyHostToDevice, g_scr.s), -1);
  HCK(hipMemcpyAsync(d_dummy, dummy_w, Ncb, hipMemcpyHostToDevice, g_scr.s), -1);
  HCK(oai4g_launch_rm_rx(d_soft, E, d_w, d_dummy, d_c, Ncb, nn, k0c, clear == 1, g_scr.s), -1);
  HCK(hipMemcpyAsync(w, d_w, b_w, hipMemcpyDeviceToHost, g_scr.s), -1);
  HCK(hipStreamSynchronize(g_scr.s), -1);
  *E_out = E;
  return 0;
}

extern "C" void oai4g_sub_block_deinterleaving_turbo(uint32_t D, int16_t *d, const int16_t *w)
{
  NEED_INIT();
  const uint32_t R = (D + 31) >> 5, Kpi = R << 5;
  const size_t nd = 96 + 3 * (size_t)D + 8, b_d = nd * 2, b_w = 3 * (size_t)Kpi * 2;
  uint8_t *buf = scratch(b_d + b_w + 512);
  if (!buf) return;
  int16_t *d_d = (int16_t *)buf, *d_w = (int16_t *)(buf + ((b_d + 255) & ~(size_t)255));
  HCK(hipMemcpyAsync(d_d, d - 96, b_d, hipMemcpyHostToDevice, g_scr.s), );
  HCK(hipMemcpyAsync(d_w, w, b_w, hipMemcpyHostToDevice, g_scr.s), );
  HCK(oai4g_launch_subblock_deint(D, d_d, d_w, g_scr.s), );
  HCK(hipMemcpyAsync(d - 96, d_d, b_d, hipMemcpyDeviceToHost, g_scr.s), );
  HCK(hipStreamSynchronize(g_scr.s), );
}

extern "C" int oai4g_idft(int log2n, const int16_t *x, int16_t *y, int scale)
{
  if (!log2n_ok(log2n)) { set_err("idft: size 2^%d not supported", log2n); return -1; }
  ofdm_sym_t s = {0, 0, 0};
  return run_ofdm((const int32_t *)x, (size_t)1 << log2n, (int32_t *)y, 0, (size_t)1 << log2n, log2n, 1, &s, scale);
}

extern "C" void oai4g_idft2048(const int16_t *x, int16_t *y, int scale) { oai4g_idft(11, x, y, scale); }
extern "C" void oai4g_idft1024(const int16_t *x, int16_t *y, int scale) { oai4g_idft(10, x, y, scale); }
extern "C" void oai4g_idft512(const int16_t *x, int16_t *y, int scale) { oai4g_idft(9, x, y, scale); }
extern "C" void oai4g_idft256(const int16_t *x, int16_t *y, int scale) { oai4g_idft(8, x, y, scale); }
extern "C" void oai4g_idft128(const int16_t *x, int16_t *y, int scale) { oai4g_idft(7, x, y, scale); }
extern "C" void oai4g_idft64(const int16_t *x, int16_t *y, int scale) { oai4g_idft(6, x, y, scale); }

/* ------------------------------------------------------------------------------------------
 * UE receive front end: forward DFT drop-ins, slot_fep, batched FEP
 * ---------------------------------------------------------------------------------------- */
static int run_fep_window(const int32_t *h_in, int32_t *h_out, int log2n, int scale)
{
  NEED_INIT(-1);
  const size_t N = (size_t)1 << log2n;
  uint8_t *buf = scratch(2 * N * 4 + 256);
  if (!buf) return -1;
  int32_t *d_in = (int32_t *)buf, *d_out = (int32_t *)(buf + ((N * 4 + 255) & ~(size_t)255));
  fep_args_t a;
  memset(&a, 0, sizeof(a));
  a.n_units = 1;
  a.nsym = 1;
  a.in_stride = a.in_len = (uint32_t)N;
  a.out_stride = (uint32_t)N;
  a.scale = scale;
  HCK(hipMemcpyAsync(d_in, h_in, N * 4, hipMemcpyHostToDevice, g_scr.s), -1);
  HCK(oai4g_launch_fep(d_in, d_out, log2n, a, g_twf, g_n_cu, g_scr.s), -1);
  HCK(hipMemcpyAsync(h_out, d_out, N * 4, hipMemcpyDeviceToHost, g_scr.s), -1);
  HCK(hipStreamSynchronize(g_scr.s), -1);
  return 0;
}

extern "C" int oai4g_dft(int log2n, const int16_t *x, int16_t *y, int scale)
{
  if (!log2n_ok(log2n)) { set_err("dft: size 2^%d not supported", log2n); return -1; }
  return run_fep_window((const int32_t *)x, (int32_t *)y, log2n, scale);
}
extern "C" void oai4g_dft2048(const int16_t *x, int16_t *y, int scale) { oai4g_dft(11, x, y, scale); }
extern "C" void oai4g_dft1024(const int16_t *x, int16_t *y, int scale) { oai4g_dft(10, x, y, scale); }
extern "C" void oai4g_dft512(const int16_t *x, int16_t *y, int scale) { oai4g_dft(9, x, y, scale); }
extern "C" void oai4g_dft256(const int16_t *x, int16_t *y, int scale) { oai4g_dft(8, x, y, scale); }
extern "C" void oai4g_dft128(const int16_t *x, int16_t *y, int scale) { oai4g_dft(7, x, y, scale); }
extern "C" void oai4g_dft64(const int16_t *x, int16_t *y, int scale) { oai4g_dft(6, x, y, scale); }

/* slot_fep's DFT window (slot_fep.c:55-150), unsigned arithmetic as in the reference: returns
 * rx_offset (before the % frame_length of the read), -1 for a bad l / Ns */
extern "C" int64_t oai4g_slot_fep_offset(const oai4g_frame_parms_t *fp, uint8_t l, uint8_t Ns, int sample_offset,
                                         int no_prefix)
{
  if (l >= 7 - fp->Ncp) {
    fprintf(stderr, "slot_fep: l must be between 0 and %d\n", 7 - fp->Ncp);
    set_err("slot_fep: l must be between 0 and %d", 7 - fp->Ncp);
    return -1;
  }
  if (Ns >= 20) {
    fprintf(stderr, "slot_fep: Ns must be between 0 and 19\n");
    set_err("slot_fep: Ns must be between 0 and 19");
    return -1;
  }
  const uint32_t N = fp->ofdm_symbol_size;
  const uint32_t cp = no_prefix ? 0u : fp->nb_prefix_samples, cp0 = no_prefix ? 0u : fp->nb_prefix_samples0;
  uint32_t subframe_offset, slot_offset;
  if (no_prefix) {
    subframe_offset = N * fp->symbols_per_tti * (Ns >> 1);
    slot_offset = N * (fp->symbols_per_tti >> 1) * (Ns % 2);
  } else {
    subframe_offset = fp->samples_per_tti * (Ns >> 1);
    slot_offset = (fp->samples_per_tti >> 1) * (Ns % 2);
  }
  uint32_t rx_offset = (uint32_t)sample_offset + slot_offset + cp0 + subframe_offset;
  rx_offset = rx_offset - rx_offset % 4;                     /* "Align with 128 bit" (:118) */
  if (l > 0) rx_offset += (N + cp) + (N + cp) * (uint32_t)(l - 1);
  return (int64_t)rx_offset;
}

/* slot_fep (PHY/MODULATION/slot_fep.c:40, decl MODULATION/defs.h): CP removal + DFT of symbol l of
 * slot Ns for every receive antenna.  rxdata[aa] holds the frame (10 samples_per_tti) plus
 * ofdm_symbol_size words of wrap extension, rxdataF[aa] the frequency-domain subframe.  The
 * channel / frequency-offset estimation that follows in the reference (perfect_ce == 0) is not
 * part of this entry point. */
extern "C" int oai4g_slot_fep(int32_t *const *rxdata, int32_t *const *rxdataF, const oai4g_frame_parms_t *fp,
                              uint8_t nb_antennas_rx, uint8_t l, uint8_t Ns, int sample_offset, int no_prefix)
{
  NEED_INIT(-1);
  const int64_t off = oai4g_slot_fep_offset(fp, l, Ns, sample_offset, no_prefix);
  if (off < 0) return -1;
  const uint32_t N = fp->ofdm_symbol_size, fl = fp->samples_per_tti * 10, rx_offset = (uint32_t)off;
  const uint32_t symbol = l + (7 - fp->Ncp) * (Ns & 1);
  std::vector<int32_t> win(N);
  for (int aa = 0; aa < nb_antennas_rx; aa++) {
    if (rx_offset > fl - N) memcpy(&rxdata[aa][fl], &rxdata[aa][0], N * sizeof(int32_t));   /* :123-126, :153-156 */
    const uint32_t st = rx_offset % fl;
    memcpy(win.data(), &rxdata[aa][st], N * sizeof(int32_t));   /* the window the reference's dft reads */
    if (run_fep_window(win.data(), &rxdataF[aa][N * symbol], fp->log2_symbol_size, 1) != 0) return -1;
  }
  return 0;
}

/* Batched FEP: every symbol of n_sf subframes x n_ant antennas, device pointers
 *   d_rx  [n_sf][n_ant][samples_per_tti] int32, d_rxF [n_sf][n_ant][symbols_per_tti][N] int32;
 * each subframe is slot_fep'd (slots 0 and 1, sample_offset 0, with prefix) on its own samples. */
extern "C" int oai4g_fep_batch(const oai4g_frame_parms_t *fp, int n_sf, int n_ant, const int32_t *d_rx, int32_t *d_rxF,
                               void *stream)
{
  NEED_INIT(-1);
  if (n_sf < 0 || n_ant <= 0 || !log2n_ok(fp->log2_symbol_size) || fp->symbols_per_tti > OAI4G_FEP_MAX_SYM) {
    set_err("fep_batch: bad arguments");
    return -1;
  }
  const uint32_t N = fp->ofdm_symbol_size, spt = fp->samples_per_tti, nslot = fp->symbols_per_tti / 2;
  fep_args_t a;
  memset(&a, 0, sizeof(a));
  a.nsym = fp->symbols_per_tti;
  a.n_units = n_sf * n_ant * a.nsym;
  a.in_stride = a.in_len = spt;
  a.out_stride = N * a.nsym;
  a.scale = 1;
  for (int sym = 0; sym < a.nsym; sym++) {
    const int64_t off = oai4g_slot_fep_offset(fp, (uint8_t)(sym % nslot), (uint8_t)(sym / nslot), 0, 0);
    if (off < 0 || (uint64_t)off + N > spt) { set_err("fep_batch: symbol %d window outside its subframe", sym); return -1; }
    a.in_off[sym] = (uint32_t)off;
    a.out_off[sym] = N * (uint32_t)sym;
  }
  HCK(oai4g_launch_fep(d_rx, d_rxF, fp->log2_symbol_size, a, g_twf, g_n_cu, (hipStream_t)stream), -1);
  return 0;
}

/* ------------------------------------------------------------------------------------------
 * Control region: PCFICH (pcfich.c:48-228)
 * ---------------------------------------------------------------------------------------- */
/* generate_pcfich_reg_mapping (pcfich.c:48-84): the four REGs (units of 6 REs from the first
 * carrier) and the index of the lowest.  The silent helper serves generate_pcfich; the exported
 * drop-in prints them as the reference does (once, at init, in the reference's callers). */
static void pcfich_regs(const oai4g_frame_parms_t *fp, uint16_t pcfich_reg[4], uint8_t *pcfich_first_reg_idx)
{
  const uint32_t NRB = fp->N_RB_DL, kbar = 6 * (fp->Nid_cell % (2 * NRB));
  uint16_t first;
  pcfich_reg[0] = (uint16_t)(kbar / 6);
  first = pcfich_reg[0];
  *pcfich_first_reg_idx = 0;
  const uint32_t steps[3] = {(NRB >> 1) * 6, NRB * 6, ((3 * NRB) >> 1) * 6};
  for (int i = 1; i < 4; i++) {
    pcfich_reg[i] = (uint16_t)(((kbar + steps[i - 1]) % (NRB * 12)) / 6);
    if (pcfich_reg[i] < first) {
      *pcfich_first_reg_idx = (uint8_t)i;
      first = pcfich_reg[i];
    }
  }
}

extern "C" void oai4g_generate_pcfich_reg_mapping(const oai4g_frame_parms_t *fp, uint16_t pcfich_reg[4],
                                                  uint8_t *pcfich_first_reg_idx)
{
  pcfich_regs(fp, pcfich_reg, pcfich_first_reg_idx);
  printf("pcfich_reg : %d,%d,%d,%d\n", pcfich_reg[0], pcfich_reg[1], pcfich_reg[2], pcfich_reg[3]);
}

/* generate_pcfich (pcfich.c:144, decl proto.h:1432): overwrites the 16 PCFICH REs of symbol 0 of
 * `subframe` in the frame grids txdataF[0] (and txdataF[1] with two antennas).  The reference
 * reads frame_parms->pcfich_reg (set at init by generate_pcfich_reg_mapping); here they are
 * derived from fp.  num_pdcch_symbols outside 1..3 is rejected (-1): the reference would map an
 * uninitialised codeword (pcfich.c:164-165). */
extern "C" int oai4g_generate_pcfich(uint8_t num_pdcch_symbols, int16_t amp, const oai4g_frame_parms_t *fp,
                                     int32_t **txdataF, uint8_t subframe)
{
  NEED_INIT(-1);
  if (num_pdcch_symbols < 1 || num_pdcch_symbols > 3 || subframe > 9) {
    set_err("generate_pcfich: num_pdcch_symbols %u / subframe %u out of range", num_pdcch_symbols, subframe);
    return -1;
  }
  uint16_t reg[4];
  uint8_t first_idx;
  pcfich_regs(fp, reg, &first_idx);
  const uint32_t N = fp->ofdm_symbol_size, nsymb = fp->Ncp == 0 ? 14 : 12;
  const size_t symbol_offset = (size_t)N * subframe * nsymb;
  pcfich_args_t a;
  memset(&a, 0, sizeof(a));
  a.c_init = ((((2u * fp->Nid_cell) + 1u) * (1u + subframe)) << 9) + fp->Nid_cell;
  a.cfi = num_pdcch_symbols;
  a.gain = fp->mode1_flag == 1 ? (int16_t)((amp * 23170) >> 15) : (int16_t)(amp / 2);
  a.mode1 = fp->mode1_flag ? 1 : 0;
  a.nushift3 = (uint8_t)(fp->nushift % 3);
  for (int q = 0; q < 4; q++) {
    uint32_t ro = fp->first_carrier_offset + (uint32_t)reg[q] * 6;
    if (ro >= N) ro = 1 + ro - N;
    a.reg_off[q] = ro;
  }
  a.n_ant = fp->nb_antennas_tx > 1 ? 2 : 1;
  uint8_t *buf = scratch(2 * (size_t)N * 4 + 256);
  if (!buf) return -1;
  int32_t *d0 = (int32_t *)buf, *d1 = (int32_t *)(buf + (((size_t)N * 4 + 255) & ~(size_t)255));
  for (uint32_t aa = 0; aa < a.n_ant; aa++)
    HCK(hipMemcpyAsync(aa ? d1 : d0, txdataF[aa] + symbol_offset, (size_t)N * 4, hipMemcpyHostToDevice, g_scr.s), -1);
  HCK(oai4g_launch_pcfich(d0, d1, a, g_scr.s), -1);
  for (uint32_t aa = 0; aa < a.n_ant; aa++)
    HCK(hipMemcpyAsync(txdataF[aa] + symbol_offset, aa ? d1 : d0, (size_t)N * 4, hipMemcpyDeviceToHost, g_scr.s), -1);
  HCK(hipStreamSynchronize(g_scr.s), -1);
  return 0;
}

/* ----------------------------------------------------------------------------------------
 * Control region: PDCCH / DCI (generate_dci_top, dci.c:2024-2346) — host-side geometry
 * (the reference's init-time / scalar helpers) + the k_dci kernel for the per-subframe data.
 * ---------------------------------------------------------------------------------------- */
extern "C" uint8_t oai4g_get_mi(const oai4g_frame_parms_t *fp, uint8_t sf)
{
  if (fp->frame_type == 0) return 1;                                  /* phich.c:59-118 */
  switch (fp->tdd_config) {
  case 0: return (sf == 0 || sf == 5) ? 2 : 1;
  case 1: return (sf == 0 || sf == 5) ? 0 : 1;
  case 2: return (sf == 3 || sf == 8) ? 1 : 0;
  case 3: return (sf == 0 || sf == 8 || sf == 9) ? 1 : 0;
  case 4: return (sf == 8 || sf == 9) ? 1 : 0;
  case 5: return sf == 8 ? 1 : 0;
  case 6: return 1;
  default: return 0;
  }
}

static uint32_t phich_ngroup(const oai4g_frame_parms_t *fp)   /* Ngroup_PHICH (phich.c:292-303) */
{
  uint32_t ng = (fp->phich_resource * fp->N_RB_DL) / 48;
  if ((fp->phich_resource * fp->N_RB_DL) % 48) ng++;
  if (fp->Ncp == 1) ng <<= 1;
  return ng;
}

extern "C" uint16_t oai4g_get_nquad(uint8_t npdcch, const oai4g_frame_parms_t *fp, uint8_t mi)
{
  uint32_t Nreg = 0;                                                  /* dci.c:2499-2538 */
  uint8_t ng = (uint8_t)((fp->phich_resource * fp->N_RB_DL) / 48);    /* uint8_t, as :2502 */
  if ((fp->phich_resource * fp->N_RB_DL) % 48) ng++;
  if (fp->Ncp == 1) ng = (uint8_t)(ng << 1);
  ng = (uint8_t)(ng * mi);
  if (npdcch > 0 && npdcch < 4) {
    switch (fp->N_RB_DL) {
    case 6: Nreg = 12 + (npdcch - 1) * 18; break;
    case 25: Nreg = 50 + (npdcch - 1) * 75; break;
    case 50: Nreg = 100 + (npdcch - 1) * 150; break;
    case 100: Nreg = 200 + (npdcch - 1) * 300; break;
    default: return 0;
    }
  }
  return (uint16_t)(Nreg - 4 - 3 * ng);
}

extern "C" uint16_t oai4g_get_nCCE(uint8_t npdcch, const oai4g_frame_parms_t *fp, uint8_t mi)
{
  return (uint16_t)(oai4g_get_nquad(npdcch, fp, mi) / 9);
}

extern "C" uint8_t oai4g_get_num_pdcch_symbols(uint8_t num_dci, const oai4g_dci_alloc_t *dci,
                                               const oai4g_frame_parms_t *fp, uint8_t sf)
{
  uint16_t numCCE = 0;                                                /* dci.c:1964-2022 */
  uint8_t nmin = 0;
  if (fp->Ncp == 1)
    nmin = (fp->frame_type == 1 && (fp->tdd_config < 3 || fp->tdd_config == 6) && (sf == 1 || sf == 6)) ? 2 : 3;
  for (int i = 0; i < num_dci; i++) numCCE = (uint16_t)(numCCE + (1 << dci[i].L));
  const uint8_t mi = oai4g_get_mi(fp, sf);
  for (uint8_t n = 1; n <= 3; n++)
    if (numCCE <= oai4g_get_nCCE(n, fp, mi)) return nmin > n ? nmin : n;
  if (fp->N_RB_DL <= 10 && 9u * numCCE <= fp->N_RB_DL * (fp->nb_antennas_tx_eNB == 4 ? (fp->Ncp ? 9u : 10u)
                                                                                  : (fp->Ncp ? 10u : 11u)))
    return 4;
  return 0;
}

extern "C" int oai4g_generate_phich_reg_mapping(const oai4g_frame_parms_t *fp, uint16_t phich_reg[56][3])
{
  uint16_t pcf[4];                                                    /* phich.c:280-386 */
  uint8_t fi;
  pcfich_regs(fp, pcf, &fi);
  const uint32_t n0 = fp->N_RB_DL * 2u - 4u, ng = phich_ngroup(fp), nloop = fp->Ncp == 0 ? ng : ng >> 1;
  for (uint32_t m = 0; m < nloop && m < 56; m++) {
    const uint32_t base[3] = {(fp->Nid_cell + m) % n0, (fp->Nid_cell + m + n0 / 3) % n0,
                              (fp->Nid_cell + m + 2 * n0 / 3) % n0};
    for (int j = 0; j < 3; j++) {
      uint32_t r = base[j];
      for (int q = 0; q < 4; q++)
        if (r >= pcf[(fi + q) & 3]) r++;
      phich_reg[m][j] = (uint16_t)r;
    }
  }
  return (int)nloop;
}

static int g_cce_table[800];
extern "C" void oai4g_init_nCCE_table(void) { memset(g_cce_table, 0, sizeof(g_cce_table)); }

extern "C" int oai4g_get_nCCE_offset(uint8_t L, int nCCE, int common_dci, uint16_t rnti, uint8_t subframe)
{
  int *T = g_cce_table;                                               /* phy_procedures_lte_eNb.c:308-391 */
  if (L == 0 || nCCE / L <= 0) return -1;
  if (common_dci == 1) {
    int nb = L == 4 ? 4 : 2;
    if (nCCE / L < nb) nb = nCCE / L;
    for (int m = nb - 1; m >= 0; m--) {
      int fr = 1;
      for (int l = 0; l < L; l++) fr &= T[m * L + l] != 1;
      if (fr) {
        for (int l = 0; l < L; l++) T[m * L + l] = 1;
        return m * L;
      }
    }
    return -1;
  }
  uint32_t Yk = rnti;
  for (int i = 0; i <= subframe; i++) Yk = (Yk * 39827u) % 65537u;
  Yk %= (uint32_t)(nCCE / L);
  const int nb = (L == 1 || L == 2) ? 6 : 2;
  for (int m = 0; m < nb; m++) {
    const int s0 = (int)(((Yk + m) % (uint32_t)(nCCE / L)) * L);
    int fr = 1;
    for (int l = 0; l < L; l++) fr &= T[s0 + l] != 1;
    if (fr) {
      for (int l = 0; l < L; l++) T[s0 + l] = 1;
      return s0;
    }
  }
  return -1;
}

/* The static part of generate_dci_top for (fp, npdcch, subframe): the QPSK symbol interleaving
 * (pdcch_interleaving, dci.c:277-341: 32-column sub-block interleaver on quadruplets with the
 * <NULL>s dropped, then the cyclic shift by Nid_cell) composed with the REG allocation
 * (:2234-2340: k' outer, l' inner, PCFICH / PHICH REGs skipped (check_phich_reg :62-121), six-RE
 * REGs around the RS in symbol 0, four-RE REGs with the DC split elsewhere), cut at Msymb2
 * mapped REs.  map[r] = l * N + subcarrier, src[r] = QPSK symbol index.  Returns the RE count. */
static uint32_t pdcch_map(const oai4g_frame_parms_t *fp, uint8_t npdcch, uint8_t mi, std::vector<uint32_t> &map,
                          std::vector<uint16_t> &src)
{
  static const uint8_t bitrev_cc[32] = {1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31,
                                        0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30};
  const uint32_t N = fp->ofdm_symbol_size, Mquad = oai4g_get_nquad(npdcch, fp, mi);
  const int Msymb = ((2 * 33 + 22) * 72) / 2;
  int Msymb2;
  switch (fp->N_RB_DL) {
  case 100: Msymb2 = Msymb; break;
  case 75: Msymb2 = 3 * Msymb / 4; break;
  case 50: Msymb2 = Msymb >> 1; break;
  case 25: Msymb2 = Msymb >> 2; break;
  case 15: Msymb2 = Msymb * 15 / 100; break;
  case 6: Msymb2 = Msymb * 6 / 100; break;
  default: Msymb2 = Msymb >> 2; break;
  }
  /* quadruplet k of wtemp <- quadruplet perm[k] of y; wbar[i] = wtemp[(i + Nid) mod Mquad] */
  std::vector<uint32_t> perm;
  const uint32_t RCC = (Mquad + 31) >> 5, ND = (RCC << 5) - Mquad;
  for (uint32_t col = 0; col < 32; col++)
    for (uint32_t row = 0, idx = bitrev_cc[col]; row < RCC; row++, idx += 32)
      if (idx >= ND) perm.push_back(idx - ND);
  uint16_t pcf[4], phr[56][3];
  uint8_t fi;
  memset(phr, 0, sizeof(phr));            /* groups the mapping never writes read as REG 0 (calloc'd frame_parms) */
  pcfich_regs(fp, pcf, &fi);
  oai4g_generate_phich_reg_mapping(fp, phr);
  const uint32_t ng = phich_ngroup(fp), ns3 = fp->nushift % 3;
  const bool tx4 = fp->nb_antennas_tx_eNB == 4;
  auto phich_or_pcfich = [&](uint32_t kp, uint32_t lp) {
    if (lp > 0 && fp->Ncp == 0) return false;
    const uint32_t m = (lp == 0 || (lp == 1 && tx4)) ? kp / 6 : kp >> 2;
    if (lp == 0 && (m == pcf[0] || m == pcf[1] || m == pcf[2] || m == pcf[3])) return true;
    if (mi > 0)
      for (uint32_t i = 0; i < ng && i < 56; i++)
        if (m == phr[i][0] || m == phr[i][1] || m == phr[i][2]) return true;
    return false;
  };
  map.clear();
  src.clear();
  uint32_t mprime = 0;
  int re_offset = fp->first_carrier_offset;
  auto put = [&](uint32_t off) {
    const uint32_t q = mprime >> 2;       /* wbar quadruplet -> y symbol */
    map.push_back(off);
    src.push_back((uint16_t)(4 * perm[(q + fp->Nid_cell) % Mquad] + (mprime & 3)));
    mprime++;
  };
  for (uint32_t kp = 0; kp < (uint32_t)fp->N_RB_DL * 12; kp++) {
    for (uint32_t lp = 0; lp < npdcch; lp++) {
      const uint32_t tti = N * lp + (uint32_t)re_offset;
      if (!phich_or_pcfich(kp, lp)) {
        const uint32_t km = kp % 12;
        if (lp == 0 || (lp == 1 && tx4)) {
          if (km == 0 || km == 6)
            for (uint32_t i = 0; i < 6; i++)
              if (i != ns3 && i != ns3 + 3) put(tti + i);
        } else if (km == 0 || km == 4 || km == 8) {
          if (re_offset != (int)N - 2) {
            for (uint32_t i = 0; i < 4; i++) put(tti + i);
          } else {                        /* the REG straddles DC */
            put(tti);
            put(tti + 1);
            put(tti - N + 3);
            put(tti - N + 4);
          }
        }
        if (mprime >= (uint32_t)Msymb2) return (uint32_t)map.size();
      }
    }
    re_offset++;
    if (re_offset == (int)N) re_offset = 1;
  }
  return (uint32_t)map.size();
}

/* Fills the kernel arguments and the map of one subframe; returns npdcch (0 on error). */
static uint8_t dci_prepare(uint8_t n_ue, uint8_t n_common, const oai4g_dci_alloc_t *dci, int16_t amp,
                           const oai4g_frame_parms_t *fp, uint32_t subframe, dci_args_t &a, std::vector<uint32_t> &map,
                           std::vector<uint16_t> &src)
{
  const uint32_t n = (uint32_t)n_ue + n_common;
  if (n > OAI4G_MAX_DCI) { set_err("generate_dci_top: %u DCIs (at most %d)", n, OAI4G_MAX_DCI); return 0; }
  if (fp->phich_duration != 0 || fp->Ncp != 0) {
    set_err("generate_dci_top: only the normal cyclic prefix with normal PHICH duration is supported");
    return 0;
  }
  const uint8_t npd = oai4g_get_num_pdcch_symbols((uint8_t)n, dci, fp, (uint8_t)subframe);
  if (npd < 1 || npd > 3) {
    set_err("generate_dci_top: num_pdcch_symbols %u (too many CCEs, or no PDCCH geometry for N_RB_DL %u)", npd,
            fp->N_RB_DL);
    return npd;
  }
  const uint8_t mi = oai4g_get_mi(fp, (uint8_t)subframe);
  memset(&a, 0, sizeof(a));
  /* generate_dci_top's order: aggregation level 3 .. 0, common DCIs first within a level; the
   * encoded blocks land at their own CCEs, so only later writers over overlapping CCEs matter */
  uint32_t k = 0;
  for (int L = 3; L >= 0; L--)
    for (uint32_t i = 0; i < n; i++)
      if (dci[i].L == L && dci[i].nCCE >= 0) {
        dci_dev_t &d = a.dci[k++];
        const uint8_t *p = dci[i].dci_pdu;
        for (int b = 0; b < 8; b++) d.flip[b] = 0;
        if (dci[i].dci_length <= 32) for (int b = 0; b < 4; b++) d.flip[b] = p[3 - b];
        else for (int b = 0; b < 8; b++) d.flip[b] = p[7 - b];
        d.A = dci[i].dci_length;
        d.L = dci[i].L;
        d.nCCE = dci[i].nCCE;
        d.rnti = dci[i].rnti;
        if (d.A > 64 || d.A < 8 || d.L > 3 || 72u * (uint32_t)(d.nCCE + (1 << d.L)) > (2 * 33 + 22 + 8) * 72u) {
          set_err("generate_dci_top: DCI %u: length %u / L %u / nCCE %d out of range", i, d.A, d.L, d.nCCE);
          return 0;
        }
      }
  a.n_dci = k;
  a.nbits = 8u * oai4g_get_nquad(npd, fp, mi);
  a.c_init = (subframe << 9) + fp->Nid_cell;
  a.gain = fp->mode1_flag == 1 ? (int16_t)((amp * 23170) >> 15) : (int16_t)(amp / 2);
  a.mode1 = fp->mode1_flag ? 1 : 0;
  a.n_ant = fp->nb_antennas_tx_eNB > 1 ? 2 : 1;
  a.n_re = pdcch_map(fp, npd, mi, map, src);
  return npd;
}

extern "C" uint8_t oai4g_generate_dci_top(uint8_t num_ue_spec_dci, uint8_t num_common_dci,
                                          const oai4g_dci_alloc_t *dci_alloc, uint32_t n_rnti, int16_t amp,
                                          const oai4g_frame_parms_t *fp, int32_t **txdataF, uint32_t subframe)
{
  (void)n_rnti;
  NEED_INIT(0);
  if (subframe > 9) { set_err("generate_dci_top: subframe %u", subframe); return 0; }
  dci_args_t a;
  std::vector<uint32_t> map;
  std::vector<uint16_t> src;
  const uint8_t npd = dci_prepare(num_ue_spec_dci, num_common_dci, dci_alloc, amp, fp, subframe, a, map, src);
  if (npd < 1 || npd > 3) return npd;
  const uint32_t N = fp->ofdm_symbol_size, nsymb = 14;
  const size_t sym_off = (size_t)N * subframe * nsymb, gbytes = (size_t)npd * N * 4;
  const size_t gpad = (gbytes + 255) & ~(size_t)255, mbytes = ((size_t)a.n_re * 4 + 255) & ~(size_t)255;
  uint8_t *buf = scratch(2 * gpad + mbytes + (size_t)a.n_re * 2 + 256);
  if (!buf) return 0;
  int32_t *d0 = (int32_t *)buf, *d1 = (int32_t *)(buf + gpad);
  uint32_t *dmap = (uint32_t *)(buf + 2 * gpad);
  uint16_t *dsrc = (uint16_t *)(buf + 2 * gpad + mbytes);
  const uint32_t n_ant = a.n_ant;
  for (uint32_t aa = 0; aa < n_ant; aa++)
    HCK(hipMemcpyAsync(aa ? d1 : d0, txdataF[aa] + sym_off, gbytes, hipMemcpyHostToDevice, g_scr.s), 0);
  HCK(hipMemcpyAsync(dmap, map.data(), (size_t)a.n_re * 4, hipMemcpyHostToDevice, g_scr.s), 0);
  HCK(hipMemcpyAsync(dsrc, src.data(), (size_t)a.n_re * 2, hipMemcpyHostToDevice, g_scr.s), 0);
  /* PCFICH first (generate_dci_top :2084-2088), then the PDCCH REs */
  pcfich_args_t pa;
  memset(&pa, 0, sizeof(pa));
  {
    uint16_t reg[4];
    uint8_t fi;
    pcfich_regs(fp, reg, &fi);
    pa.c_init = ((((2u * fp->Nid_cell) + 1u) * (1u + subframe)) << 9) + fp->Nid_cell;
    pa.cfi = npd;
    pa.gain = a.gain;
    pa.mode1 = a.mode1;
    pa.nushift3 = (uint8_t)(fp->nushift % 3);
    for (int q = 0; q < 4; q++) {
      uint32_t ro = fp->first_carrier_offset + (uint32_t)reg[q] * 6;
      if (ro >= N) ro = 1 + ro - N;
      pa.reg_off[q] = ro;
    }
    pa.n_ant = n_ant;
  }
  HCK(oai4g_launch_pcfich(d0, d1, pa, g_scr.s), 0);
  HCK(oai4g_launch_dci(a, dmap, dsrc, d0, d1, 0, g_scr.s), 0);
  for (uint32_t aa = 0; aa < n_ant; aa++)
    HCK(hipMemcpyAsync(txdataF[aa] + sym_off, aa ? d1 : d0, gbytes, hipMemcpyDeviceToHost, g_scr.s), 0);
  HCK(hipStreamSynchronize(g_scr.s), 0);
  return npd;
}

/* Batched static REs: generate_dci_top's PCFICH + PDCCH (set_control) and the PSS / SSS, PBCH and
 * PHICH of the common signal procedures (set_common, phy_procedures_lte_eNb.c:1529-1760, 2585)
 * for every subframe index, computed on the GPU by the drop-in kernels into one subframe grid per
 * subframe index, gathered into a [10][14][2][N] table, marked in the RE map with OAI4G_CTL_CODE
 * and merged by the modulator. */
static void sync_args(const oai4g_frame_parms_t *fp, int16_t amp, bool pss, uint16_t slot_offset, sync_args_t &a);
static void pbch_args(const oai4g_frame_parms_t *fp, int amp, const uint8_t *pdu, uint8_t frame_mod4, pbch_args_t &a);
static int phich_item(const oai4g_frame_parms_t *fp, uint8_t nseq, uint8_t ngroup, uint8_t HI, uint8_t subframe,
                      phich_item_t &it);
static void phich_common(const oai4g_frame_parms_t *fp, int16_t amp, phich_args_t &a);

static int rebuild_static(oai4g_tx_config_t *cfg)
{
  const uint32_t N = cfg->h.N, nsymb = cfg->h.nsymb, n_ant = cfg->p.nb_antennas_tx;
  for (auto &c : cfg->h_remap)
    if ((c & 0xE000u) == OAI4G_CTL_CODE) c = 0xFFFF;
  memset(cfg->h.ctlmask, 0, sizeof(cfg->h.ctlmask));
  cfg->h.ctl_on = 0;
  if (cfg->d_ctl) hipFree(cfg->d_ctl);
  cfg->d_ctl = nullptr;
  cfg->h.ctl_tab = nullptr;
  cfg->h_ctl.clear();
  cfg->ctl_vmax = 0;
  const bool dci_on = (uint32_t)cfg->n_ue_dci + cfg->n_common_dci > 0;
  if (dci_on || cfg->common_on) {
    if (cfg->h_remap.empty()) { set_err("static REs: configuration has no RE map"); return -1; }
    const oai4g_frame_parms_t &fp = cfg->fp;
    std::vector<uint32_t> tab((size_t)10 * 14 * 2 * N, 0);
    const size_t gbytes = (size_t)14 * N * 4, gpad = (gbytes + 255) & ~(size_t)255;
    const size_t mcap = (size_t)4 * 1024;    /* >= 4 nquad REs for every geometry */
    const size_t accb = (size_t)4 * 4 * N * 4;   /* PHICH accumulators / PBCH encode grid (4 antennas x 4 symbols) */
    uint8_t *buf = scratch(4 * gpad + mcap * 4 + mcap * 2 + accb + 2048 + 256);
    if (!buf) return -1;
    int32_t *dg[4] = {(int32_t *)buf, (int32_t *)(buf + gpad), (int32_t *)(buf + 2 * gpad), (int32_t *)(buf + 3 * gpad)};
    uint32_t *dmap = (uint32_t *)(buf + 4 * gpad);
    uint16_t *dsrc = (uint16_t *)(buf + 4 * gpad + mcap * 4);
    int32_t *dacc = (int32_t *)(buf + 4 * gpad + mcap * 6);
    uint8_t *dpe = buf + 4 * gpad + mcap * 6 + accb;
    std::vector<uint32_t> g((size_t)14 * N);
    for (uint32_t sf = 0; sf < 10; sf++) {
      HCK(hipMemsetAsync(buf, 0, 4 * gpad, g_scr.s), -1);
      uint32_t n_out = n_ant > 2 ? 2 : n_ant;          /* antennas whose values the table keeps */
      if (dci_on) {
        dci_args_t a;
        std::vector<uint32_t> map;
        std::vector<uint16_t> src;
        const uint8_t npd = dci_prepare(cfg->n_ue_dci, cfg->n_common_dci, cfg->dci.data(), cfg->p.amp, &cfg->fp, sf, a,
                                        map, src);
        if (npd < 1 || npd > 3) return -1;
        if (npd > cfg->p.num_pdcch_symbols) {
          set_err("set_control: the DCIs need %u control symbols but the PDSCH starts at symbol %u (dlsim.c:2562-2565)",
                  npd, cfg->p.num_pdcch_symbols);
          return -1;
        }
        if (map.size() > mcap) { set_err("set_control: PDCCH map too large"); return -1; }
        HCK(hipMemcpyAsync(dmap, map.data(), map.size() * 4, hipMemcpyHostToDevice, g_scr.s), -1);
        HCK(hipMemcpyAsync(dsrc, src.data(), src.size() * 2, hipMemcpyHostToDevice, g_scr.s), -1);
        pcfich_args_t pa;
        memset(&pa, 0, sizeof(pa));
        uint16_t reg[4];
        uint8_t fi;
        pcfich_regs(&fp, reg, &fi);
        pa.c_init = ((((2u * fp.Nid_cell) + 1u) * (1u + sf)) << 9) + fp.Nid_cell;
        pa.cfi = npd;
        pa.gain = a.gain;
        pa.mode1 = a.mode1;
        pa.nushift3 = (uint8_t)(fp.nushift % 3);
        for (int q = 0; q < 4; q++) {
          uint32_t ro = fp.first_carrier_offset + (uint32_t)reg[q] * 6;
          if (ro >= N) ro = 1 + ro - N;
          pa.reg_off[q] = ro;
        }
        pa.n_ant = a.n_ant;
        HCK(oai4g_launch_pcfich(dg[0], dg[1], pa, g_scr.s), -1);
        HCK(oai4g_launch_dci(a, dmap, dsrc, dg[0], dg[1], 0, g_scr.s), -1);
      }
      if (cfg->common_on) {
        const oai4g_common_sig_t &cm = cfg->common;
        const uint32_t nsl = nsymb / 2;
        if (cm.pss_sss && (sf == 0 || sf == 5)) {
          sync_args_t sa;
          int32_t *sp[4];
          sync_args(&fp, cfg->p.amp, true, (uint16_t)(2 * sf), sa);
          for (uint32_t aa = 0; aa < 4; aa++) sp[aa] = dg[aa] + (size_t)(nsl - 1) * N;
          HCK(oai4g_launch_sync(sp, sa, g_scr.s), -1);
          sync_args(&fp, cfg->p.amp, false, (uint16_t)(2 * sf), sa);
          for (uint32_t aa = 0; aa < 4; aa++) sp[aa] = dg[aa] + (size_t)(nsl - 2) * N;
          HCK(oai4g_launch_sync(sp, sa, g_scr.s), -1);
        }
        if (cm.pbch && sf == 0) {
          pbch_args_t pa;
          pbch_args(&fp, cfg->p.amp, cm.pbch_pdu, 0, pa);
          int32_t *pp[4];
          for (uint32_t aa = 0; aa < 4; aa++) pp[aa] = dg[aa] + (size_t)nsl * N;
          if (cm.frame_mod4) {                          /* encode (quarter 0) into a scratch grid, then map */
            int32_t *sp[4];
            for (uint32_t aa = 0; aa < 4; aa++) sp[aa] = dacc + (size_t)aa * 4 * N;
            HCK(oai4g_launch_pbch(sp, dpe, pa, g_scr.s), -1);
            pbch_args(&fp, cfg->p.amp, cm.pbch_pdu, cm.frame_mod4, pa);
          }
          HCK(oai4g_launch_pbch(pp, dpe, pa, g_scr.s), -1);
        }
        static thread_local phich_args_t ph;
        memset(&ph, 0, sizeof(ph));
        phich_common(&fp, cfg->p.amp, ph);
        for (uint32_t i = 0; i < cm.n_phich; i++) {
          const oai4g_phich_item_t &it = cm.phich[i];
          if (it.subframe != sf) continue;
          if (phich_item(&fp, it.nseq, it.ngroup, it.hi, (uint8_t)sf, ph.it[ph.n]) != 0) return -1;
          ph.n++;
        }
        if (ph.n) {
          if (ph.n_ant > 1 && n_ant < 2) { set_err("set_common: ALAMOUTI PHICH needs two antennas"); return -1; }
          HCK(oai4g_launch_phich(dg, dacc, ph, g_scr.s), -1);
        }
        if (cm.pbch || cm.pss_sss) n_out = n_ant;
      }
      for (uint32_t ant = 0; ant < n_out && ant < 2; ant++) {
        HCK(hipMemcpyAsync(g.data(), dg[ant], gbytes, hipMemcpyDeviceToHost, g_scr.s), -1);
        HCK(hipStreamSynchronize(g_scr.s), -1);
        for (uint32_t l = 0; l < nsymb; l++)
          for (uint32_t k = 0; k < N; k++) {
            const uint32_t v = g[(size_t)l * N + k];
            if (!v) continue;
            tab[(((size_t)sf * 14 + l) * 2 + ant) * N + k] = v;
            uint16_t &code = cfg->h_remap[((size_t)sf * 14 + l) * N + k];
            if (code != 0xFFFF && code != OAI4G_CTL_CODE) {
              set_err("static REs: subframe %u symbol %u RE %u collides with a PDSCH / CRS RE", sf, l, k);
              return -1;
            }
            code = (uint16_t)OAI4G_CTL_CODE;
            cfg->h.ctlmask[sf] |= 1u << l;
          }
      }
    }
    HCK(hipMalloc(&cfg->d_ctl, tab.size() * 4), -1);
    HCK(hipMemcpy(cfg->d_ctl, tab.data(), tab.size() * 4, hipMemcpyHostToDevice), -1);
    cfg->h.ctl_tab = cfg->d_ctl;
    cfg->h.ctl_on = 1;
    cfg->h_ctl = tab;
    cfg->ctl_vmax = packed_iq_max(tab);
  }
  cfg->h.mod_nosat = mod_nosat_ok(cfg->h, std::max(packed_iq_max(cfg->h_crs), cfg->ctl_vmax));
  if (upload_remap(cfg) != 0) return -1;
  HCK(hipMemcpy(cfg->d, &cfg->h, sizeof(cfg_dev_t), hipMemcpyHostToDevice), -1);
  return 0;
}

extern "C" int oai4g_tx_config_set_control(oai4g_tx_config_t *cfg, uint8_t n_ue, uint8_t n_common,
                                           const oai4g_dci_alloc_t *dci)
{
  NEED_INIT(-1);
  cfg->dci.assign(dci, dci + ((uint32_t)n_ue + n_common));
  cfg->n_ue_dci = n_ue;
  cfg->n_common_dci = n_common;
  return rebuild_static(cfg);
}

extern "C" int oai4g_tx_config_set_common(oai4g_tx_config_t *cfg, const oai4g_common_sig_t *c)
{
  NEED_INIT(-1);
  if (c && c->n_phich > OAI4G_MAX_PHICH_ITEMS) { set_err("set_common: %u PHICHs", c->n_phich); return -1; }
  if (c && c->n_phich && cfg->p.mode1_flag == 1 && cfg->p.nb_antennas_tx > 1) {
    set_err("set_common: a SISO PHICH on antenna 0 only is not representable in the one-transform TM1 grid");
    return -1;
  }
  cfg->common_on = c != nullptr && (c->pss_sss || c->pbch || c->n_phich);
  if (c) cfg->common = *c;
  return rebuild_static(cfg);
}

/* ----------------------------------------------------------------------------------------
 * Synchronisation, broadcast and HARQ-indicator channels: host geometry and
 * tables of pss.c / sss.c / pbch.c / phich.c, the per-call data on the GPU (oai4g_ctrl.hip).
 * -------------------------------------------------------------------------------------- */
/* primary_synch0/1/2 (PHY/LTE_REFSIG/primary_synch.h): entries 10..133 of the reference table are
 * floor(32767 x) of the Zadoff-Chu sequence d_u(n), u = 25 / 29 / 34 (checked entry by entry
 * against the header in tests/test_sync_cpu.py) */
static void pss_table(uint32_t Nid2, int16_t v[62][2])
{
  static const int u[3] = {25, 29, 34};
  for (int n = 0; n < 62; n++) {
    const int m = n < 31 ? n : n + 1;
    const double ang = -M_PI * u[Nid2 % 3] * m * (m + 1) / 63.0;
    v[n][0] = (int16_t)floor(32767.0 * cos(ang));
    v[n][1] = (int16_t)floor(32767.0 * sin(ang));
  }
}

/* d0_sss / d5_sss (PHY/LTE_TRANSPORT/sss.h) restated from 36.211 6.11.2.1 */
static void sss_table(uint32_t Nid_cell, bool sf5, int16_t d[62])
{
  auto mseq = [](const int *taps, int nt, int8_t *out) {
    int x[31] = {0, 0, 0, 0, 1};
    for (int i = 0; i < 26; i++) {
      int v = 0;
      for (int t = 0; t < nt; t++) v += x[i + taps[t]];
      x[i + 5] = v & 1;
    }
    for (int i = 0; i < 31; i++) out[i] = (int8_t)(1 - 2 * x[i]);
  };
  static const int ts[2] = {2, 0}, tc[2] = {3, 0}, tz[4] = {4, 2, 1, 0};
  int8_t st[31], ct[31], zt[31];
  mseq(ts, 2, st);
  mseq(tc, 2, ct);
  mseq(tz, 4, zt);
  const int n1 = (int)Nid_cell / 3, n2 = (int)Nid_cell % 3;
  const int qp = n1 / 30, q = (n1 + qp * (qp + 1) / 2) / 30, mp = n1 + q * (q + 1) / 2;
  const int m0 = mp % 31, m1 = (m0 + mp / 31 + 1) % 31;
  for (int n = 0; n < 31; n++) {
    const int s0 = st[(n + m0) % 31], s1 = st[(n + m1) % 31], c0 = ct[(n + n2) % 31], c1 = ct[(n + n2 + 3) % 31];
    const int z0 = zt[(n + m0 % 8) % 31], z1 = zt[(n + m1 % 8) % 31];
    d[2 * n] = (int16_t)(sf5 ? s1 * c0 : s0 * c0);
    d[2 * n + 1] = (int16_t)(sf5 ? s0 * c1 * z1 : s1 * c1 * z0);
  }
}

static void sync_args(const oai4g_frame_parms_t *fp, int16_t amp, bool pss, uint16_t slot_offset, sync_args_t &a)
{
  memset(&a, 0, sizeof(a));
  if (pss) {
    pss_table(fp->Nid_cell % 3, a.val);
  } else {
    int16_t d[62];
    sss_table(fp->Nid_cell, slot_offset >= 3, d);
    for (int i = 0; i < 62; i++) a.val[i][0] = d[i];
  }
  a.a = fp->nb_antennas_tx == 1 ? amp : (int16_t)((amp * 23170) >> 15);
  a.pss = pss ? 1 : 0;
  a.n_ant = fp->nb_antennas_tx;
  a.N = fp->ofdm_symbol_size;
}

/* one symbol of every antenna: upload, kernel, download */
static int sync_dropin(int32_t **txdataF, int16_t amp, const oai4g_frame_parms_t *fp, uint16_t symbol,
                       uint16_t slot_offset, bool pss)
{
  NEED_INIT(-1);
  const uint32_t N = fp->ofdm_symbol_size, Nsymb = fp->Ncp == 0 ? 14 : 12, n_ant = fp->nb_antennas_tx;
  if (n_ant < 1 || n_ant > 4) { set_err("generate_%s: nb_antennas_tx %u", pss ? "pss" : "sss", n_ant); return -1; }
  const size_t off = (size_t)slot_offset * Nsymb / 2 * N + (size_t)symbol * N, sb = ((size_t)N * 4 + 255) & ~(size_t)255;
  sync_args_t a;
  sync_args(fp, amp, pss, slot_offset, a);
  uint8_t *buf = scratch(4 * sb);
  if (!buf) return -1;
  int32_t *d[4];
  for (uint32_t aa = 0; aa < n_ant; aa++) {
    d[aa] = (int32_t *)(buf + aa * sb);
    HCK(hipMemcpyAsync(d[aa], txdataF[aa] + off, (size_t)N * 4, hipMemcpyHostToDevice, g_scr.s), -1);
  }
  HCK(oai4g_launch_sync(d, a, g_scr.s), -1);
  for (uint32_t aa = 0; aa < n_ant; aa++)
    HCK(hipMemcpyAsync(txdataF[aa] + off, d[aa], (size_t)N * 4, hipMemcpyDeviceToHost, g_scr.s), -1);
  HCK(hipStreamSynchronize(g_scr.s), -1);
  return 0;
}

extern "C" int oai4g_generate_pss(int32_t **txdataF, int16_t amp, const oai4g_frame_parms_t *fp, uint16_t symbol,
                                  uint16_t slot_offset)
{
  return sync_dropin(txdataF, amp, fp, symbol, slot_offset, true);
}

extern "C" int oai4g_generate_sss(int32_t **txdataF, int16_t amp, const oai4g_frame_parms_t *fp, uint16_t symbol,
                                  uint16_t slot_offset)
{
  return sync_dropin(txdataF, amp, fp, symbol, slot_offset, false);
}

static void pbch_args(const oai4g_frame_parms_t *fp, int amp, const uint8_t *pdu, uint8_t frame_mod4, pbch_args_t &a)
{
  memset(&a, 0, sizeof(a));
  for (int i = 0; i < 3; i++) a.a[3 - i - 1] = pdu[i];       /* pbch.c:214-215 */
  a.encode = frame_mod4 == 0 ? 1 : 0;
  a.amask = fp->mode1_flag == 1 ? 0 : (fp->nb_antennas_tx_eNB == 2 ? 0xffff : (fp->nb_antennas_tx_eNB == 4 ? 0x5555 : 0));
  a.E = fp->Ncp == 0 ? 1920 : 1728;
  a.Nid = fp->Nid_cell;
  a.quarter = frame_mod4 & 3u;
  a.N = fp->ofdm_symbol_size;
  const uint32_t nsymb = fp->Ncp == 0 ? 14 : 12, second = fp->Ncp == 0 ? 4 : 3;
  for (uint32_t i = 0; i < 4; i++) {                          /* pbch.c:345-362 */
    const uint32_t l = (nsymb >> 1) + i;
    if (l == 0 || l == (nsymb >> 1) || l == 1 || l == (nsymb >> 1) + 1 || l == second || l == second + (nsymb >> 1))
      a.pil_mask |= 1u << i;
  }
  a.nushift3 = fp->nushift % 3;
  a.gain = (int16_t)((amp * 23170) >> 15);
  a.mode1 = fp->mode1_flag == 1 ? 1 : 0;
  a.n_ant = fp->nb_antennas_tx;
}

extern "C" int oai4g_generate_pbch(oai4g_pbch_t *st, int32_t **txdataF, int amp, const oai4g_frame_parms_t *fp,
                                   const uint8_t *pbch_pdu, uint8_t frame_mod4)
{
  NEED_INIT(-1);
  const uint32_t N = fp->ofdm_symbol_size, nsymb = fp->Ncp == 0 ? 14 : 12, n_ant = fp->nb_antennas_tx;
  if (n_ant < 1 || n_ant > 4 || (fp->mode1_flag != 1 && n_ant != 2) || frame_mod4 > 3) {
    set_err("generate_pbch: %u antennas (mode1 %u), frame_mod4 %u", n_ant, fp->mode1_flag, frame_mod4);
    return -1;
  }
  pbch_args_t a;
  pbch_args(fp, amp, pbch_pdu, frame_mod4, a);
  const size_t gb = (size_t)4 * N * 4, gs = (gb + 255) & ~(size_t)255, off = (size_t)(nsymb >> 1) * N;
  uint8_t *buf = scratch(4 * gs + 2048);
  if (!buf) return -1;
  int32_t *d[4];
  uint8_t *de = buf + 4 * gs;
  for (uint32_t aa = 0; aa < n_ant; aa++) {
    d[aa] = (int32_t *)(buf + aa * gs);
    HCK(hipMemcpyAsync(d[aa], txdataF[aa] + off, gb, hipMemcpyHostToDevice, g_scr.s), -1);
  }
  if (!a.encode) HCK(hipMemcpyAsync(de, st->pbch_e, a.E, hipMemcpyHostToDevice, g_scr.s), -1);
  HCK(oai4g_launch_pbch(d, de, a, g_scr.s), -1);
  if (a.encode) HCK(hipMemcpyAsync(st->pbch_e, de, a.E, hipMemcpyDeviceToHost, g_scr.s), -1);
  for (uint32_t aa = 0; aa < n_ant; aa++)
    HCK(hipMemcpyAsync(txdataF[aa] + off, d[aa], gb, hipMemcpyDeviceToHost, g_scr.s), -1);
  HCK(hipStreamSynchronize(g_scr.s), -1);
  return 0;
}

static uint32_t ngroup_phich_h(const oai4g_frame_parms_t *fp)
{
  uint32_t n = ((uint32_t)fp->phich_resource * fp->N_RB_DL) / 48;
  if (((uint32_t)fp->phich_resource * fp->N_RB_DL) % 48) n++;
  return n;
}

/* phich_item_t of one generate_phich call; offsets relative to symbol 0 of the subframe */
static int phich_item(const oai4g_frame_parms_t *fp, uint8_t nseq, uint8_t ngroup, uint8_t HI, uint8_t subframe,
                      phich_item_t &it)
{
  if (fp->Ncp != 0 || fp->phich_duration != 0 || fp->nushift >= 3) {
    set_err("generate_phich: only normal CP, normal duration and nushift < 3 are defined (phich.c:540-580)");
    return -1;
  }
  uint16_t reg[56][3];
  const int ng = oai4g_generate_phich_reg_mapping(fp, reg);
  if (ngroup >= ng || nseq > 7 || subframe > 9) { set_err("generate_phich: group %u / seq %u", ngroup, nseq); return -1; }
  it.c_init = ((((uint32_t)subframe + 1u) * (fp->Nid_cell + 1u)) << 9) + fp->Nid_cell;
  const uint32_t N = fp->ofdm_symbol_size;
  for (int q = 0; q < 3; q++) {
    uint32_t ro = fp->first_carrier_offset + (uint32_t)reg[ngroup][q] * 6;
    if (ro > N) ro -= N - 1;                                   /* '>' as phich.c:560 */
    it.reg_off[q] = ro;
  }
  it.nseq = nseq;
  it.hi = HI ? 1 : 0;
  return 0;
}

static void phich_common(const oai4g_frame_parms_t *fp, int16_t amp, phich_args_t &a)
{
  a.gain = fp->mode1_flag == 1 ? (int16_t)(((int32_t)amp * 23170) >> 15) : (int16_t)(amp / 2);
  a.mode1 = fp->mode1_flag == 1 ? 1 : 0;
  a.n_ant = fp->mode1_flag == 1 ? 1 : 2;                      /* SISO writes y[0] only (phich.c:696-760) */
  a.nushift = fp->nushift;
  a.win = 2u * fp->ofdm_symbol_size;
}

extern "C" int oai4g_generate_phich(const oai4g_frame_parms_t *fp, int16_t amp, uint8_t nseq_PHICH, uint8_t ngroup_PHICH,
                                    uint8_t HI, uint8_t subframe, int32_t **y)
{
  NEED_INIT(-1);
  static thread_local phich_args_t a;
  memset(&a, 0, sizeof(a));
  if (phich_item(fp, nseq_PHICH, ngroup_PHICH, HI, subframe, a.it[0]) != 0) return -1;
  a.n = 1;
  phich_common(fp, amp, a);
  if (a.n_ant > 1 && fp->nb_antennas_tx < 2) { set_err("generate_phich: ALAMOUTI needs two grids"); return -1; }
  const uint32_t N = fp->ofdm_symbol_size;
  const size_t wb = (size_t)a.win * 4, ws = (wb + 255) & ~(size_t)255, off = (size_t)14 * N * subframe;
  uint8_t *buf = scratch(2 * ws + 4 * ws);
  if (!buf) return -1;
  int32_t *d[2] = {(int32_t *)buf, (int32_t *)(buf + ws)};
  int32_t *acc = (int32_t *)(buf + 2 * ws);
  for (uint32_t aa = 0; aa < a.n_ant; aa++) HCK(hipMemcpyAsync(d[aa], y[aa] + off, wb, hipMemcpyHostToDevice, g_scr.s), -1);
  HCK(oai4g_launch_phich(d, acc, a, g_scr.s), -1);
  for (uint32_t aa = 0; aa < a.n_ant; aa++) HCK(hipMemcpyAsync(y[aa] + off, d[aa], wb, hipMemcpyDeviceToHost, g_scr.s), -1);
  HCK(hipStreamSynchronize(g_scr.s), -1);
  return 0;
}

extern "C" int oai4g_phich_group_seq(const oai4g_frame_parms_t *fp, uint16_t first_rb, uint8_t n_DMRS, uint8_t *ngroup,
                                     uint8_t *nseq)
{
  const uint32_t Ng = ngroup_phich_h(fp), NSF = fp->Ncp == 1 ? 2 : 4;
  if (!Ng) { set_err("phich_group_seq: no PHICH groups"); return -1; }
  *ngroup = (uint8_t)((first_rb + n_DMRS) % Ng);
  *nseq = (uint8_t)((first_rb / Ng + n_DMRS) % (2 * NSF));
  return 0;
}

/* ----------------------------------------------------------------------------------------
 * UE PDSCH demodulation (second half): host geometry of rx_pdsch's
 * extraction / LLR lengths (dlsch_demodulation.c:3167-3300, dlsch_llr_computation.c:636-930,
 * adjust_G2 lte_mcs.c:157-245) and the scrambling words; the per-RE work on the GPU
 * (oai4g_rx.hip).  TM1, one receive antenna, even N_RB_DL.
 * -------------------------------------------------------------------------------------- */
struct oai4g_rx_config {
  oai4g_frame_parms_t fp;
  rx_dev_t h;
  rx_dev_t *d = nullptr;
  uint32_t *d_map = nullptr, *d_gold = nullptr;
  uint8_t *d_shift = nullptr;
  int shift_cap = 0;
  uint32_t llr_count[10];
  bool bad[10];                   /* subframe index whose LLR stream would read unwritten ext slots */
};

static int rx_alloc_bit(const uint32_t rb_alloc[4], int rb)
{
  if (rb < 32) return (rb_alloc[0] >> rb) & 1;
  if (rb < 64) return (rb_alloc[1] >> (rb - 32)) & 1;
  if (rb < 96) return (rb_alloc[2] >> (rb - 64)) & 1;
  if (rb < 100) return (rb_alloc[3] >> (rb - 96)) & 1;
  return 0;
}

/* adjust_G2 (lte_mcs.c:157-245) */
static int rx_adjust_G2(const oai4g_frame_parms_t *fp, const uint32_t rb_alloc[4], uint32_t subframe, uint32_t symbol)
{
  const uint32_t nsymb = fp->Ncp == 0 ? 14 : 12;
  int re = 0;
  if (subframe != 0 && subframe != 5 && subframe != 6) return 0;
  if (symbol < (nsymb >> 1) && fp->frame_type == 1 && subframe != 6) return 0;
  if (fp->frame_type == 1) {
    if (symbol > (nsymb >> 1) + 3 && symbol != nsymb - 1) return 0;
    if (subframe == 5 && symbol != nsymb - 1) return 0;
    if (subframe == 6 && symbol != 2) return 0;
  } else {
    if (symbol > (nsymb >> 1) + 3 || symbol < (nsymb >> 1) - 2) return 0;
    if (subframe == 5 && symbol != (nsymb >> 1) - 1 && symbol != (nsymb >> 1) - 2) return 0;
    if (subframe == 6) return 0;
  }
  const int half = fp->N_RB_DL >> 1;
  if (fp->N_RB_DL & 1) {
    for (int rb = half - 3; rb <= half + 3; rb++)
      if (rx_alloc_bit(rb_alloc, rb)) re += (rb == half - 3 || rb == half + 3) ? 6 : 12;
  } else {
    for (int rb = half - 3; rb < half + 3; rb++)
      if (rx_alloc_bit(rb_alloc, rb)) re += 12;
  }
  return re;
}

/* dlsch_extract_rbs_single (dlsch_demodulation.c:3167-3681) of one symbol as an extraction map:
 * the ext slots the call leaves written, each FFT bin | (estimate column 5 + 12 rb + i) << 16, with
 * the reference's pointer steps (the odd-N_RB RB around DC can write one slot past the step it then
 * takes; the next RB overwrites it).  n = slots written; nb_rb as the reference counts it. */
static void rx_extract_map(const oai4g_frame_parms_t *fp, const uint32_t rb_alloc[4], uint32_t subframe, uint32_t l,
                           std::vector<uint32_t> &map, uint32_t &nb_rb, uint32_t &n)
{
  const uint32_t smod = l >= 7u - fp->Ncp ? l - (7u - fp->Ncp) : l;
  const bool pil = smod == 0 || smod == 4u - fp->Ncp;
  const uint32_t poff = smod == 4u - fp->Ncp ? 3 : 0, ns = fp->nushift;
  const int nsymb = fp->Ncp == 0 ? 14 : 12, half = fp->N_RB_DL >> 1;
  uint32_t slot[12 * 110 + 12];
  uint32_t ptr = 0, hw = 0;
  nb_rb = 0;
  auto put = [&](uint32_t pos, uint32_t bin, uint32_t col) {
    slot[pos] = bin | (col << 16);
    hw = pos + 1 > hw ? pos + 1 : hw;
  };
  if ((fp->N_RB_DL & 1) == 0) {
    uint32_t bin = fp->first_carrier_offset;
    for (int rb = 0; rb < fp->N_RB_DL; rb++) {
      if (rb == half) bin = 1;
      if (rx_alloc_bit(rb_alloc, rb)) {
        for (uint32_t i = 0; i < 12; i++)
          if (!pil || (i != ns + poff && i != (ns + poff + 6) % 12)) put(ptr++, bin + i, 5 + 12 * rb + i);
        nb_rb++;
      }
      bin += 12;
    }
  } else {
    const int sss_symb = fp->frame_type == 1 ? nsymb - 1 : (nsymb >> 1) - 2;
    const int pss_symb = fp->frame_type == 1 ? 2 : (nsymb >> 1) - 1;
    const int li = (int)l;
    const bool pbch = subframe == 0 && li >= (nsymb >> 1) && li < (nsymb >> 1) + 4;
    const bool sss = (subframe == 0 || subframe == 5) && li == sss_symb;
    const bool pss = (fp->frame_type == 0 && (subframe == 0 || subframe == 5) && li == pss_symb) ||
                     (fp->frame_type == 1 && subframe == 6 && li == pss_symb);
    const bool excl = pbch || sss || pss;
    uint32_t bin = fp->first_carrier_offset;
    for (int rb = 0; rb < fp->N_RB_DL; rb++) {
      int ind = rx_alloc_bit(rb_alloc, rb);
      const uint32_t col = 5 + 12 * rb;
      if (rb == half) {                                       /* :3434-3525, split at bin 0 */
        if (excl) ind = 0;
        if (ind) {
          uint32_t j = 0;
          for (uint32_t i = 0; i < 12; i++) {
            const uint32_t b = i < 6 ? bin + i : 1 + i - 6;
            if (!pil) put(ptr + i, b, col + i);
            else if (i < 6 ? i != (ns + poff) % 6 : i != (ns + 6 + poff) % 12) put(ptr + j++, b, col + i);
          }
          ptr += pil ? 10 : 12;
          nb_rb++;
        }
        bin = 7;
        continue;
      }
      int skip_half = 0;
      if (excl && rb > half - 3 && rb < half + 3) ind = 0;
      if (excl) skip_half = rb == half - 3 ? 1 : (rb == half + 3 ? 2 : 0);
      if (ind) {
        uint32_t j = 0;
        if (skip_half) {
          const uint32_t o = skip_half == 2 ? 6 : 0;
          for (uint32_t i = 0; i < 6; i++)
            if (!pil || i != (ns + poff) % 6) put(ptr + j++, bin + i + o, col + i + o);
          ptr += pil ? 5 : 6;
        } else {
          for (uint32_t i = 0; i < 12; i++)
            if (!pil || (i != ns + poff && i != (ns + poff + 6) % 12)) put(ptr + j++, bin + i, col + i);
          ptr += pil ? 10 : 12;
        }
        nb_rb++;
      }
      bin += 12;
    }
  }
  n = hw;
  map.insert(map.end(), slot, slot + hw);
}

/* dlsch_extract_rbs_dual (dlsch_demodulation.c:3683-4056) of one symbol as an extraction map of
 * the slots one receive antenna's call leaves written (every antenna and both ports share it): the
 * PBCH / PSS / SSS RBs are dropped; 8 REs per RB in pilot symbols; odd N_RB_DL as written there —
 * the RB around DC reads bins 0..5 for its upper half in non-pilot symbols, the skip_half = 2
 * pilot branch advances the pointers inside its RE loop, and the full-RB non-pilot branch
 * (:3932-3936) is `for (i=0;i<12;i++) dl_ch0_ext+=12;` (its loop body was a printf, now commented
 * out), so the port-0 estimate pointer moves 144 slots per RB while rxF_ext / dl_ch1_ext move 12.
 * The port-0 writes are tracked with that drift; n = the prefix of slots where the received RE and
 * both estimates come from the same column (past it the reference reads stale or unwritten port-0
 * slots, and its writes run past dl_ch_estimates_ext: a stream reaching there is refused). */
static void rx_extract_map_dual(const oai4g_frame_parms_t *fp, const uint32_t rb_alloc[4], uint32_t subframe, uint32_t l,
                                std::vector<uint32_t> &map, uint32_t &nb_rb, uint32_t &n)
{
  const uint32_t smod = l >= 7u - fp->Ncp ? l - (7u - fp->Ncp) : l;
  const bool pil = smod == 0 || smod == 4u - fp->Ncp;
  const int nsymb = fp->Ncp == 0 ? 14 : 12, half = fp->N_RB_DL >> 1, li = (int)l;
  const uint32_t ns = fp->nushift;
  const int sss_symb = fp->frame_type == 1 ? nsymb - 1 : (nsymb >> 1) - 2;
  const int pss_symb = fp->frame_type == 1 ? 2 : (nsymb >> 1) - 1;
  std::vector<uint32_t> slot(12 * 110 + 256, 0);
  std::vector<uint8_t> wr(12 * 110 + 256, 0);
  std::vector<int32_t> col_rx(12 * 110 + 256, -1), col_c0(12 * 110 + 256, -1);
  uint32_t p = 0, hw = 0, drift = 0;                         /* drift = dl_ch0_ext - rxF_ext (slots) */
  nb_rb = 0;
  auto put = [&](uint32_t pos, uint32_t bin, uint32_t col) {
    slot[pos] = bin | ((5 + col) << 16);
    wr[pos] = 1;
    col_rx[pos] = (int32_t)col;
    if (pos + drift < col_c0.size()) col_c0[pos + drift] = (int32_t)col;
    hw = pos + 1 > hw ? pos + 1 : hw;
  };
  auto data_re = [&](uint32_t i) { return i != ns && i != ns + 3 && i != ns + 6 && i != (ns + 9) % 12; };
  for (int prb = 0; prb < fp->N_RB_DL; prb++) {
    int ind = rx_alloc_bit(rb_alloc, prb), skip_half = 0;
    if (subframe == 0 && prb > half - 3 && prb < half + 3 && li >= (nsymb >> 1) && li < (nsymb >> 1) + 4) ind = 0;
    if ((subframe == 0 || subframe == 5) && prb > half - 3 && prb < half + 3 && li == sss_symb) ind = 0;
    if (fp->frame_type == 0 && (subframe == 0 || subframe == 5) && prb > half - 3 && prb < half + 3 && li == pss_symb) ind = 0;
    if (fp->frame_type == 1 && subframe == 6 && prb >= half - 3 && prb <= half + 3 && li == pss_symb) ind = 0;
    if (!ind) continue;
    const uint32_t col0 = 12 * prb;
    if ((fp->N_RB_DL & 1) == 0) {
      const uint32_t b0 = prb < half ? fp->first_carrier_offset + 12 * prb : 1 + 12 * (prb - half);
      uint32_t j = 0;
      for (uint32_t i = 0; i < 12; i++)
        if (!pil || data_re(i)) put(p + j++, b0 + i, col0 + i);
      p += pil ? 8 : 12;
      nb_rb++;
      continue;
    }
    if (subframe == 0 && prb == half - 3 && li >= (nsymb >> 1) && li < (nsymb >> 1) + 4) skip_half = 1;
    else if (subframe == 0 && prb == half + 3 && li >= (nsymb >> 1) && li < (nsymb >> 1) + 4) skip_half = 2;
    if ((subframe == 0 || subframe == 5) && prb == half - 3 && li == sss_symb) skip_half = 1;
    else if ((subframe == 0 || subframe == 5) && prb == half + 3 && li == sss_symb) skip_half = 2;
    if ((fp->frame_type == 0 && (subframe == 0 || subframe == 5)) || (fp->frame_type == 1 && (subframe == 2 || subframe == 6))) {
      if (prb == half - 3 && li == pss_symb) skip_half = 1;
      else if ((subframe == 0 || subframe == 5) && prb == half + 3 && li == pss_symb) skip_half = 2;
    }
    const uint32_t b0 = prb <= half ? fp->first_carrier_offset + 12 * prb : 7 + 12 * (prb - half - 1);
    if (prb != half) {
      if (!pil) {
        const uint32_t o = skip_half == 2 ? 6 : 0, cnt = skip_half ? 6 : 12;
        for (uint32_t i = 0; i < cnt; i++) put(p + i, b0 + o + i, col0 + o + i);
        p += cnt;
        if (!skip_half) drift += 132;                        /* dl_ch0_ext += 144 (:3932-3934) */
      } else if (skip_half == 1) {
        uint32_t j = 0;
        for (uint32_t i = 0; i < 6; i++)
          if (i != ns && i != (ns + 3) % 6) put(p + j++, b0 + i, col0 + i);
        p += 4;
      } else if (skip_half == 2) {
        uint32_t j = 0;
        for (uint32_t i = 0; i < 6; i++) {
          if (i != ns && i != (ns + 3) % 6) put(p + j++, b0 + i + 6, col0 + i + 6);
          p += 4;                                            /* inside the loop, as written */
        }
      } else {
        uint32_t j = 0;
        for (uint32_t i = 0; i < 12; i++)
          if (data_re(i)) put(p + j++, b0 + i, col0 + i);
        p += 8;
      }
    } else {                                                 /* the RB around DC */
      if (!pil) {
        for (uint32_t i = 0; i < 6; i++) put(p + i, b0 + i, col0 + i);
        for (uint32_t i = 0; i < 6; i++) put(p + 6 + i, i, col0 + 6 + i);
        p += 12;
      } else {
        uint32_t j = 0, i = 0;
        for (; i < 6; i++)
          if (i != ns && i != (ns + 3) % 6) put(p + j++, b0 + i, col0 + i);
        for (; i < 12; i++)
          if (i != (ns + 6) % 12 && i != (ns + 9) % 12) put(p + j++, 1 + i - 6, col0 + i);
        p += 8;
      }
    }
    nb_rb++;
  }
  /* n = the written prefix: the skip_half = 2 pilot branch leaves holes, which the reference would
   * fill from earlier symbols' ext data (a stream reaching one is refused) */
  n = 0;
  while (n < hw && wr[n] && col_c0[n] == col_rx[n]) n++;
  map.insert(map.end(), slot.begin(), slot.begin() + hw);
}

/* offset_mumimo_llr_drange (dlsch_demodulation.c:76, the active table) [MCS][Qm1 / 2 - 1] */
static const uint8_t k_mumimo_off[29][3] = {{0, 6, 5}, {0, 4, 5}, {0, 4, 5}, {0, 5, 4}, {0, 5, 6}, {0, 5, 3}, {0, 4, 4},
                                            {0, 4, 4}, {0, 3, 3}, {0, 1, 2}, {1, 1, 0}, {1, 3, 2}, {3, 4, 1}, {2, 0, 0},
                                            {2, 2, 2}, {1, 1, 1}, {2, 1, 0}, {2, 1, 1}, {1, 0, 1}, {1, 0, 1}, {0, 0, 0},
                                            {1, 0, 0}, {0, 0, 0}, {0, 1, 0}, {1, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0},
                                            {0, 0, 0}};

static oai4g_rx_config_t *rx_config_build(const oai4g_frame_parms_t *fp, const uint32_t rb_alloc[4], uint8_t Qm,
                                          uint8_t num_pdcch_symbols, uint16_t rnti, uint8_t first_subframe,
                                          uint8_t subframe_step, int tm3, uint8_t Qm1, uint8_t mcs0, uint8_t nb_rx,
                                          int tm2 = 0)
{
  NEED_INIT(nullptr);
  const bool dual = tm3 || tm2;
  if (tm2 && (fp->nb_antennas_tx != 2 || fp->mode1_flag != 0 || (Qm != 2 && Qm != 4 && Qm != 6) || nb_rx < 1 ||
              nb_rx > 2 || num_pdcch_symbols < 1 || num_pdcch_symbols > 3)) {
    set_err("rx_config_tm2: two TX ports (mode1_flag 0), Qm 2/4/6, 1-2 RX antennas, 1..3 PDCCH symbols");
    return nullptr;
  }
  if (!dual && (fp->nb_antennas_tx != 1 || fp->mode1_flag != 1 || (Qm != 2 && Qm != 4 && Qm != 6) ||
               num_pdcch_symbols < 1 || num_pdcch_symbols > 3)) {
    set_err("rx_config: TM1 (one TX port), Qm 2/4/6, 1..3 PDCCH symbols only");
    return nullptr;
  }
  if (tm3 && (fp->nb_antennas_tx != 2 || fp->mode1_flag != 0 || (Qm != 2 && Qm != 4 && Qm != 6) ||
              (Qm1 != 2 && Qm1 != 4 && Qm1 != 6) || mcs0 > 28 || nb_rx < 1 || nb_rx > 2 || num_pdcch_symbols < 1 ||
              num_pdcch_symbols > 3)) {
    set_err("rx_config_tm3: two TX ports, Qm0 and Qm1 2/4/6, 1-2 RX antennas, 1..3 PDCCH symbols");
    return nullptr;
  }
  const uint32_t nsymb = fp->Ncp == 0 ? 14 : 12, N = fp->ofdm_symbol_size;
  const uint32_t first_mod = num_pdcch_symbols >= 7u - fp->Ncp ? num_pdcch_symbols - (7u - fp->Ncp) : num_pdcch_symbols;
  if (first_mod == 0 || first_mod == 4u - fp->Ncp) {
    set_err("rx_config: the first PDSCH symbol carries pilots (dlsch_channel_level would read past the extracted REs)");
    return nullptr;
  }
  auto *cfg = new oai4g_rx_config();
  cfg->fp = *fp;
  rx_dev_t &h = cfg->h;
  memset(&h, 0, sizeof(h));
  h.N = N;
  h.nsymb = nsymb;
  h.Qm = Qm;
  h.npdcch = num_pdcch_symbols;
  h.n_sym = nsymb - num_pdcch_symbols;
  h.first_sf = first_subframe % 10;
  h.sf_step = subframe_step;
  h.a1 = Qm == 4 ? 20724 : (Qm == 6 ? 20225 : 0);          /* QAM16_n1 / QAM64_n1 (impl_defs_top.h:215-224) */
  h.a2 = Qm == 6 ? 10112 : 0;                               /* QAM64_n2 */
  h.tm3 = tm3 ? 1u : 0u;
  h.tm2 = tm2 ? 1u : 0u;
  h.nb_rx = dual ? nb_rx : 1u;
  h.mu_off = tm3 ? k_mumimo_off[mcs0][(Qm1 >> 1) - 1] : 0;
  h.qm1 = tm3 ? Qm1 : 0u;
  /* estimate rows from the 5 pilot rows (P0 .. P3 = symbols 0, p1, p2, p3; P4 = the next subframe's
   * symbol 0): lte_dl_channel_estimation.c:639-698 as k_chest's ce_interp applies it */
  {
    const uint32_t p1 = fp->Ncp ? 3 : 4, p2 = fp->Ncp ? 6 : 7, p3 = fp->Ncp ? 9 : 11;
    auto row = [&](uint32_t l, uint8_t a, int16_t wa, uint8_t b, int16_t wb) {
      h.ea[l] = a; h.ewa[l] = wa; h.eb[l] = b; h.ewb[l] = wb;
    };
    row(0, 0, 0, 0, 0); row(p1, 1, 0, 0, 0); row(p2, 2, 0, 0, 0); row(p3, 3, 0, 0, 0);
    row(p3 + 1, 3, 21845, 4, 10923); row(p3 + 2, 3, 10923, 4, 21845);
    row(p1 + 1, 1, 21845, 2, 10923); row(p1 + 2, 1, 10923, 2, 21845);
    if (fp->Ncp == 0) {
      row(1, 0, 24576, 1, 8192); row(2, 0, 16384, 1, 16384); row(3, 0, 8192, 1, 24576);
      row(p2 + 1, 2, 24576, 3, 8192); row(p2 + 2, 2, 16384, 3, 16384); row(p2 + 3, 2, 8192, 3, 24576);
    } else {                                                 /* the reference's 1/3, 2/3 order, as written */
      row(1, 0, 10923, 1, 21845); row(2, 0, 21845, 1, 10923);
      row(p2 + 1, 2, 10923, 3, 21845); row(p2 + 2, 2, 21845, 3, 10923);
    }
  }
  std::vector<uint32_t> map;
  uint32_t max_llr = 0;
  for (uint32_t sf = 0; sf < 10; sf++) {
    uint32_t off = 0;
    for (uint32_t k = 0; k < h.n_sym; k++) {
      const uint32_t l = num_pdcch_symbols + k;
      const uint32_t smod = l >= 7u - fp->Ncp ? l - (7u - fp->Ncp) : l;
      const bool pil = smod == 0 || smod == 4u - fp->Ncp;
      h.map_off[sf][k] = (uint32_t)map.size();
      uint32_t nb_rb = 0, n = 0;
      if (dual)
        rx_extract_map_dual(fp, rb_alloc, sf, l, map, nb_rb, n);
      else
        rx_extract_map(fp, rb_alloc, sf, l, map, nb_rb, n);
      h.n_ext[sf][k] = n;
      const int adj = Qm == 2 ? 0 : rx_adjust_G2(fp, rb_alloc, sf, l);
      /* dlsch_*_llr: pilot symbols carry 10 (one port) or 8 (two ports, mode1_flag 0) REs per RB */
      const int len = pil ? (dual ? (int)nb_rb * 8 - 2 * adj / 3 : (int)nb_rb * 10 - 5 * adj / 6) : (int)nb_rb * 12 - adj;
      h.len[sf][k] = (uint32_t)(len > 0 ? len : 0);
      /* channel_level_TM3 takes 8 REs per RB only where symbol_mod == 0 (its 4-Ncp test reads
       * Ncp-1, :2917-2922); the SISO level reads 12 per RB */
      const uint32_t lvl_nre = dual && smod == 0 ? 8u : 12u;
      /* TM2 combines RE pairs: the partner of an odd last RE must have been extracted too */
      const uint32_t need = tm2 ? (h.len[sf][k] + 1) & ~1u : h.len[sf][k];
      if (need > n || (k == 0 && lvl_nre * nb_rb > n)) {
        /* the reference would read ext slots this symbol did not write (odd N_RB_DL with a
         * PBCH / sync half RB and the unadjusted QPSK length, :3354-3427): a batch that runs
         * this subframe index is refused */
        cfg->bad[sf] = true;
        h.len[sf][k] = h.len[sf][k] < n ? h.len[sf][k] : n;
      }
      if (h.len[sf][k] > 1280) { set_err("rx_config: > 1280 REs in a symbol (k_rx_llr covers 256 x 5)"); delete cfg; return nullptr; }
      h.llr_off[sf][k] = off;
      off += h.len[sf][k] * Qm;
      if (k == 0) {
        h.lvl_n[sf] = lvl_nre * nb_rb;
        h.lvl_div[sf] = dual ? lvl_nre * nb_rb : (pil ? 10 : 12) * nb_rb;
      }
      if (nb_rb == 0) cfg->bad[sf] = true;                   /* empty allocation in this symbol */
    }
    cfg->llr_count[sf] = off;
    max_llr = off > max_llr ? off : max_llr;
  }
  h.llr_stride = (max_llr + 63) & ~63u;
  /* scrambling words per subframe index: c_init = rnti 2^14 + q 2^13 + (Ns/2) 2^9 + Nid, q = 0,
   * Ns = 2 subframe (dlsch_scrambling.c:116), word w = lte_gold_generic output 50 + w */
  h.gold_words = (max_llr + 31) / 32 + 1;
  std::vector<uint32_t> gold((size_t)10 * h.gold_words);
  for (uint32_t sf = 0; sf < 10; sf++) {
    uint32_t x1 = 1u + (1u << 31), x2 = ((uint32_t)rnti << 14) + (sf << 9) + fp->Nid_cell;
    x2 = x2 ^ ((x2 ^ (x2 >> 1) ^ (x2 >> 2) ^ (x2 >> 3)) << 31);
    auto step = [&]() {
      x1 = (x1 >> 1) ^ (x1 >> 4);
      x1 = x1 ^ (x1 << 31) ^ (x1 << 28);
      x2 = (x2 >> 1) ^ (x2 >> 2) ^ (x2 >> 3) ^ (x2 >> 4);
      x2 = x2 ^ (x2 << 31) ^ (x2 << 30) ^ (x2 << 29) ^ (x2 << 28);
    };
    for (int n = 1; n < 50; n++) step();
    for (uint32_t w = 0; w < h.gold_words; w++) {
      step();
      gold[(size_t)sf * h.gold_words + w] = x1 ^ x2;
    }
  }
  if (hipMalloc(&cfg->d_map, map.size() * 4) != hipSuccess || hipMalloc(&cfg->d_gold, gold.size() * 4) != hipSuccess ||
      hipMalloc(&cfg->d, sizeof(rx_dev_t)) != hipSuccess) {
    set_err("rx_config: device allocation failed");
    oai4g_rx_config_destroy(cfg);
    return nullptr;
  }
  h.map = cfg->d_map;
  h.gold = cfg->d_gold;
  if (hipMemcpy(cfg->d_map, map.data(), map.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(cfg->d_gold, gold.data(), gold.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(cfg->d, &h, sizeof(rx_dev_t), hipMemcpyHostToDevice) != hipSuccess) {
    set_err("rx_config: upload failed");
    oai4g_rx_config_destroy(cfg);
    return nullptr;
  }
  return cfg;
}

extern "C" oai4g_rx_config_t *oai4g_rx_config_create(const oai4g_frame_parms_t *fp, const uint32_t rb_alloc[4], uint8_t Qm,
                                                     uint8_t num_pdcch_symbols, uint16_t rnti, uint8_t first_subframe,
                                                     uint8_t subframe_step)
{
  return rx_config_build(fp, rb_alloc, Qm, num_pdcch_symbols, rnti, first_subframe, subframe_step, 0, 0, 0, 1);
}

extern "C" oai4g_rx_config_t *oai4g_rx_config_create_tm3(const oai4g_frame_parms_t *fp, const uint32_t rb_alloc[4],
                                                         uint8_t Qm0, uint8_t Qm1, uint8_t mcs0,
                                                         uint8_t num_pdcch_symbols, uint16_t rnti,
                                                         uint8_t first_subframe, uint8_t subframe_step, uint8_t nb_rx)
{
  return rx_config_build(fp, rb_alloc, Qm0, num_pdcch_symbols, rnti, first_subframe, subframe_step, 1, Qm1, mcs0, nb_rx);
}

extern "C" oai4g_rx_config_t *oai4g_rx_config_create_tm2(const oai4g_frame_parms_t *fp, const uint32_t rb_alloc[4],
                                                         uint8_t Qm, uint8_t num_pdcch_symbols, uint16_t rnti,
                                                         uint8_t first_subframe, uint8_t subframe_step, uint8_t nb_rx)
{
  return rx_config_build(fp, rb_alloc, Qm, num_pdcch_symbols, rnti, first_subframe, subframe_step, 0, 0, 0, nb_rx, 1);
}

extern "C" void oai4g_rx_config_destroy(oai4g_rx_config_t *cfg)
{
  if (!cfg) return;
  if (cfg->d) hipFree(cfg->d);
  if (cfg->d_map) hipFree(cfg->d_map);
  if (cfg->d_gold) hipFree(cfg->d_gold);
  if (cfg->d_shift) hipFree(cfg->d_shift);
  delete cfg;
}

extern "C" int oai4g_rx_llr_count(const oai4g_rx_config_t *cfg, int subframe_index)
{
  return (subframe_index < 0 || subframe_index > 9) ? -1 : (int)cfg->llr_count[subframe_index];
}

extern "C" size_t oai4g_rx_llr_stride(const oai4g_rx_config_t *cfg) { return cfg->h.llr_stride; }

/* a batch of n_sf elements must not run a subframe index whose stream the reference would build
 * from ext slots it did not write (rx_config's bad[]) */
static int rx_check_batch(const oai4g_rx_config_t *cfg, int n_sf)
{
  for (int i = 0; i < n_sf && i < 10; i++) {
    const uint32_t sfi = (cfg->h.first_sf + (uint32_t)i * cfg->h.sf_step) % 10;
    if (cfg->bad[sfi]) {
      set_err("rx_batch: subframe index %u reads extracted REs the reference does not write (odd N_RB_DL with "
              "PBCH / sync half RBs, or an empty symbol)", sfi);
      return -1;
    }
  }
  return 0;
}

extern "C" int oai4g_rx_batch(oai4g_rx_config_t *cfg, int n_sf, const int32_t *d_rxdataF, const int32_t *d_ch,
                              int16_t *d_llr, int unscramble, void *stream)
{
  NEED_INIT(-1);
  if (n_sf <= 0) return 0;
  if (rx_check_batch(cfg, n_sf) != 0) return -1;
  if (n_sf > cfg->shift_cap) {
    if (cfg->d_shift) hipFree(cfg->d_shift);
    HCK(hipMalloc(&cfg->d_shift, (size_t)n_sf), -1);
    cfg->shift_cap = n_sf;
  }
  HCK(oai4g_launch_rx(cfg->d, &cfg->h, n_sf, d_rxdataF, d_ch, d_llr, cfg->d_shift, unscramble, (hipStream_t)stream), -1);
  return 0;
}

/* rx_pdsch over the PDSCH symbols of one subframe (dlsim.c:3188-3260) on host buffers:
 * rxdataF / dl_ch_estimates = [nsymb][N] of the subframe; writes the LLR stream (not unscrambled)
 * and log2_maxh; returns the stream length or -1. */
extern "C" int oai4g_rx_batch_tm3(oai4g_rx_config_t *cfg, int n_sf, const int32_t *d_rxdataF, const int32_t *d_est,
                                  int16_t *d_llr, int unscramble, void *stream)
{
  NEED_INIT(-1);
  if (!cfg || !cfg->h.tm3) { set_err("rx_batch_tm3: not a TM3 configuration (oai4g_rx_config_create_tm3)"); return -1; }
  if (n_sf <= 0) return 0;
  if (rx_check_batch(cfg, n_sf) != 0) return -1;
  if (n_sf > cfg->shift_cap) {
    if (cfg->d_shift) hipFree(cfg->d_shift);
    HCK(hipMalloc(&cfg->d_shift, (size_t)n_sf), -1);
    cfg->shift_cap = n_sf;
  }
  const size_t plane = (size_t)n_sf * cfg->h.nsymb * cfg->h.N;
  if (cfg->h.Qm == 2)   /* codeword 0 QPSK: the interference-aware qpsk_qpsk / qpsk_16qam / qpsk_64qam LLRs */
    HCK(oai4g_launch_rx_tm3qq(cfg->d, &cfg->h, n_sf, d_rxdataF, d_est, plane, d_llr, nullptr, cfg->d_shift, unscramble,
                              (hipStream_t)stream), -1);
  else
    HCK(oai4g_launch_rx_tm3(cfg->d, &cfg->h, n_sf, d_rxdataF, d_est, plane, d_llr, cfg->d_shift, unscramble,
                            (hipStream_t)stream), -1);
  return 0;
}

/* The TM3 batch from the pilot rows only: oai4g_chest_batch_pilots wrote [p * 2 + a][n_sf][5][N]
 * (the 5 frequency-interpolated pilot rows per subframe); the demodulator forms every other row
 * with the estimator's temporal interpolation, so the 14-row estimate planes never reach HBM.
 * LLRs bit-identical to oai4g_chest_batch x 4 + oai4g_rx_batch_tm3 / _tm3_2cw. */
static int rx_batch_tm3_pil(oai4g_rx_config_t *cfg, int n_sf, const int32_t *d_rxdataF, const int32_t *d_pil,
                            int16_t *d_llr0, int16_t *d_llr1, int unscramble, void *stream, bool two_cw)
{
  NEED_INIT(-1);
  if (!cfg || !cfg->h.tm3) { set_err("rx_batch_tm3_pilots: not a TM3 configuration"); return -1; }
  if (two_cw && (cfg->h.Qm != 2 || cfg->h.qm1 != 2)) {
    set_err("rx_batch_tm3_2cw_pilots: not a TM3 configuration with both codewords QPSK");
    return -1;
  }
  if (n_sf <= 0) return 0;
  if (rx_check_batch(cfg, n_sf) != 0) return -1;
  if (n_sf > cfg->shift_cap) {
    if (cfg->d_shift) hipFree(cfg->d_shift);
    HCK(hipMalloc(&cfg->d_shift, (size_t)n_sf), -1);
    cfg->shift_cap = n_sf;
  }
  const size_t plane = (size_t)n_sf * 4 * cfg->h.N * 2;        /* words: 4 pilot-row pairs per subframe */
  if (cfg->h.Qm == 2)
    HCK(oai4g_launch_rx_tm3qq(cfg->d, &cfg->h, n_sf, d_rxdataF, d_pil, plane, d_llr0, two_cw ? d_llr1 : nullptr,
                              cfg->d_shift, unscramble, (hipStream_t)stream, 1), -1);
  else
    HCK(oai4g_launch_rx_tm3(cfg->d, &cfg->h, n_sf, d_rxdataF, d_pil, plane, d_llr0, cfg->d_shift, unscramble,
                            (hipStream_t)stream, 1), -1);
  return 0;
}
extern "C" int oai4g_rx_batch_tm3_pilots(oai4g_rx_config_t *cfg, int n_sf, const int32_t *d_rxdataF, const int32_t *d_pil,
                                         int16_t *d_llr, int unscramble, void *stream)
{
  return rx_batch_tm3_pil(cfg, n_sf, d_rxdataF, d_pil, d_llr, nullptr, unscramble, stream, false);
}
extern "C" int oai4g_rx_batch_tm3_2cw_pilots(oai4g_rx_config_t *cfg, int n_sf, const int32_t *d_rxdataF,
                                             const int32_t *d_pil, int16_t *d_llr0, int16_t *d_llr1, int unscramble,
                                             void *stream)
{
  return rx_batch_tm3_pil(cfg, n_sf, d_rxdataF, d_pil, d_llr0, d_llr1, unscramble, stream, true);
}

extern "C" int oai4g_rx_batch_tm3_2cw(oai4g_rx_config_t *cfg, int n_sf, const int32_t *d_rxdataF, const int32_t *d_est,
                                      int16_t *d_llr0, int16_t *d_llr1, int unscramble, void *stream)
{
  NEED_INIT(-1);
  if (!cfg || !cfg->h.tm3 || cfg->h.Qm != 2 || cfg->h.qm1 != 2) {
    set_err("rx_batch_tm3_2cw: not a TM3 configuration with both codewords QPSK");
    return -1;
  }
  if (n_sf <= 0) return 0;
  if (rx_check_batch(cfg, n_sf) != 0) return -1;
  if (n_sf > cfg->shift_cap) {
    if (cfg->d_shift) hipFree(cfg->d_shift);
    HCK(hipMalloc(&cfg->d_shift, (size_t)n_sf), -1);
    cfg->shift_cap = n_sf;
  }
  const size_t plane = (size_t)n_sf * cfg->h.nsymb * cfg->h.N;
  HCK(oai4g_launch_rx_tm3qq(cfg->d, &cfg->h, n_sf, d_rxdataF, d_est, plane, d_llr0, d_llr1, cfg->d_shift, unscramble,
                            (hipStream_t)stream), -1);
  return 0;
}

extern "C" int oai4g_rx_batch_tm2(oai4g_rx_config_t *cfg, int n_sf, const int32_t *d_rxdataF, const int32_t *d_est,
                                  int16_t *d_llr, int unscramble, void *stream)
{
  NEED_INIT(-1);
  if (!cfg || !cfg->h.tm2) { set_err("rx_batch_tm2: not a TM2 configuration (oai4g_rx_config_create_tm2)"); return -1; }
  if (n_sf <= 0) return 0;
  if (rx_check_batch(cfg, n_sf) != 0) return -1;
  if (n_sf > cfg->shift_cap) {
    if (cfg->d_shift) hipFree(cfg->d_shift);
    HCK(hipMalloc(&cfg->d_shift, (size_t)n_sf), -1);
    cfg->shift_cap = n_sf;
  }
  const size_t plane = (size_t)n_sf * cfg->h.nsymb * cfg->h.N;
  HCK(oai4g_launch_rx_tm2(cfg->d, &cfg->h, n_sf, d_rxdataF, d_est, plane, d_llr, cfg->d_shift, unscramble,
                          (hipStream_t)stream), -1);
  return 0;
}

/* The rx_pdsch drop-ins' configurations, cached per calling thread (the UE calls rx_pdsch once per
 * subframe with a handful of distinct (frame, allocation, modulation, subframe) keys; building one
 * costs Gold generation, allocations and copies).  Round-robin over 32 entries; an evicted entry
 * is destroyed.  Entries of an exiting thread are not reclaimed (the UE's threads live as long as
 * the process, and tearing down device memory in thread-exit handlers can run after the HIP
 * runtime is gone). */
namespace {
struct rx_key_t {
  oai4g_frame_parms_t fp;
  uint32_t rb_alloc[4];
  uint8_t Qm, Qm1, mcs0, npdcch, subframe, tm3, nb_rx, pad;
};
struct rx_cache_t {
  rx_key_t key[32];
  oai4g_rx_config_t *cfg[32] = {};
  int next = 0;
};
thread_local rx_cache_t t_rx_cache;

oai4g_rx_config_t *rx_cached(const oai4g_frame_parms_t *fp, const uint32_t rb_alloc[4], uint8_t Qm, uint8_t Qm1,
                             uint8_t mcs0, uint8_t npdcch, uint8_t subframe, int tm3, int nb_rx)
{
  rx_key_t k;
  memset(&k, 0, sizeof(k));
  k.fp = *fp;
  memcpy(k.rb_alloc, rb_alloc, sizeof(k.rb_alloc));
  k.Qm = Qm; k.Qm1 = Qm1; k.mcs0 = mcs0; k.npdcch = npdcch; k.subframe = subframe;
  k.tm3 = (uint8_t)tm3; k.nb_rx = (uint8_t)nb_rx;
  rx_cache_t &c = t_rx_cache;
  for (int i = 0; i < 32; i++)
    if (c.cfg[i] && memcmp(&c.key[i], &k, sizeof(k)) == 0) return c.cfg[i];
  oai4g_rx_config_t *cfg = tm3 == 2 ? oai4g_rx_config_create_tm2(fp, rb_alloc, Qm, npdcch, 0, subframe, 1, (uint8_t)nb_rx)
                          : tm3 ? oai4g_rx_config_create_tm3(fp, rb_alloc, Qm, Qm1, mcs0, npdcch, 0, subframe, 1,
                                                             (uint8_t)nb_rx)
                                : oai4g_rx_config_create(fp, rb_alloc, Qm, npdcch, 0, subframe, 1);
  if (!cfg) return nullptr;
  const int slot = c.next;
  c.next = (c.next + 1) % 32;
  if (c.cfg[slot]) {
    hipStreamSynchronize(g_scr.s);
    oai4g_rx_config_destroy(c.cfg[slot]);
  }
  c.cfg[slot] = cfg;
  c.key[slot] = k;
  return cfg;
}
}  // namespace

extern "C" int oai4g_rx_pdsch_tm3(const oai4g_frame_parms_t *fp, int nb_rx, const int32_t *const *rxdataF,
                                  const int32_t *const *dl_ch_estimates, const uint32_t rb_alloc[4], uint8_t Qm0,
                                  uint8_t Qm1, uint8_t mcs0, uint8_t num_pdcch_symbols, uint8_t subframe, int16_t *llr,
                                  uint8_t *log2_maxh)
{
  NEED_INIT(-1);
  oai4g_rx_config_t *cfg = rx_cached(fp, rb_alloc, Qm0, Qm1, mcs0, num_pdcch_symbols, subframe, 1, nb_rx);
  if (!cfg) return -1;
  if (rx_check_batch(cfg, 1) != 0) return -1;
  const size_t gb = (size_t)cfg->h.nsymb * cfg->h.N * 4, gs = (gb + 255) & ~(size_t)255;
  const int n = (int)cfg->llr_count[subframe % 10];
  uint8_t *buf = scratch(6 * gs + (size_t)cfg->h.llr_stride * 2 + 256);
  if (!buf) return -1;
  int32_t *dy = (int32_t *)buf, *de = (int32_t *)(buf + 2 * gs);   /* [nb_rx][grid], planes [p * 2 + a] */
  int16_t *dl = (int16_t *)(buf + 6 * gs);
  bool ok = true;
  for (int a = 0; a < nb_rx && ok; a++) ok = hipMemcpyAsync((uint8_t *)dy + a * gb, rxdataF[a], gb, hipMemcpyHostToDevice, g_scr.s) == hipSuccess;
  for (int pa = 0; pa < 4 && ok; pa++)
    if ((pa & 1) < nb_rx)
      ok = hipMemcpyAsync((uint8_t *)de + pa * gb, dl_ch_estimates[pa], gb, hipMemcpyHostToDevice, g_scr.s) == hipSuccess;
  int rc = -1;
  if (ok && oai4g_rx_batch_tm3(cfg, 1, dy, de, dl, 0, g_scr.s) == 0 &&
      hipMemcpyAsync(llr, dl, (size_t)n * 2, hipMemcpyDeviceToHost, g_scr.s) == hipSuccess &&
      (!log2_maxh || hipMemcpyAsync(log2_maxh, cfg->d_shift, 1, hipMemcpyDeviceToHost, g_scr.s) == hipSuccess) &&
      hipStreamSynchronize(g_scr.s) == hipSuccess)
    rc = n;
  else
    set_err("rx_pdsch_tm3: HIP error");
  return rc;
}

extern "C" int oai4g_rx_pdsch_tm3_2cw(const oai4g_frame_parms_t *fp, int nb_rx, const int32_t *const *rxdataF,
                                      const int32_t *const *dl_ch_estimates, const uint32_t rb_alloc[4], uint8_t mcs0,
                                      uint8_t num_pdcch_symbols, uint8_t subframe, int16_t *llr0, int16_t *llr1,
                                      uint8_t *log2_maxh)
{
  NEED_INIT(-1);
  oai4g_rx_config_t *cfg = rx_cached(fp, rb_alloc, 2, 2, mcs0, num_pdcch_symbols, subframe, 1, nb_rx);
  if (!cfg) return -1;
  if (rx_check_batch(cfg, 1) != 0) return -1;
  const size_t gb = (size_t)cfg->h.nsymb * cfg->h.N * 4, gs = (gb + 255) & ~(size_t)255;
  const int n = (int)cfg->llr_count[subframe % 10];
  uint8_t *buf = scratch(6 * gs + (size_t)cfg->h.llr_stride * 4 + 256);
  if (!buf) return -1;
  int32_t *dy = (int32_t *)buf, *de = (int32_t *)(buf + 2 * gs);   /* [nb_rx][grid], planes [p * 2 + a] */
  int16_t *dl = (int16_t *)(buf + 6 * gs), *dl1 = dl + cfg->h.llr_stride;
  bool ok = true;
  for (int a = 0; a < nb_rx && ok; a++) ok = hipMemcpyAsync((uint8_t *)dy + a * gb, rxdataF[a], gb, hipMemcpyHostToDevice, g_scr.s) == hipSuccess;
  for (int pa = 0; pa < 4 && ok; pa++)
    if ((pa & 1) < nb_rx)
      ok = hipMemcpyAsync((uint8_t *)de + pa * gb, dl_ch_estimates[pa], gb, hipMemcpyHostToDevice, g_scr.s) == hipSuccess;
  int rc = -1;
  if (ok && oai4g_rx_batch_tm3_2cw(cfg, 1, dy, de, dl, dl1, 0, g_scr.s) == 0 &&
      hipMemcpyAsync(llr0, dl, (size_t)n * 2, hipMemcpyDeviceToHost, g_scr.s) == hipSuccess &&
      hipMemcpyAsync(llr1, dl1, (size_t)n * 2, hipMemcpyDeviceToHost, g_scr.s) == hipSuccess &&
      (!log2_maxh || hipMemcpyAsync(log2_maxh, cfg->d_shift, 1, hipMemcpyDeviceToHost, g_scr.s) == hipSuccess) &&
      hipStreamSynchronize(g_scr.s) == hipSuccess)
    rc = n;
  else
    set_err("rx_pdsch_tm3_2cw: HIP error");
  return rc;
}

extern "C" int oai4g_rx_pdsch_tm2(const oai4g_frame_parms_t *fp, int nb_rx, const int32_t *const *rxdataF,
                                  const int32_t *const *dl_ch_estimates, const uint32_t rb_alloc[4], uint8_t Qm,
                                  uint8_t num_pdcch_symbols, uint8_t subframe, int16_t *llr, uint8_t *log2_maxh)
{
  NEED_INIT(-1);
  oai4g_rx_config_t *cfg = rx_cached(fp, rb_alloc, Qm, 0, 0, num_pdcch_symbols, subframe, 2, nb_rx);
  if (!cfg) return -1;
  if (rx_check_batch(cfg, 1) != 0) return -1;
  const size_t gb = (size_t)cfg->h.nsymb * cfg->h.N * 4, gs = (gb + 255) & ~(size_t)255;
  const int n = (int)cfg->llr_count[subframe % 10];
  uint8_t *buf = scratch(6 * gs + (size_t)cfg->h.llr_stride * 2 + 256);
  if (!buf) return -1;
  int32_t *dy = (int32_t *)buf, *de = (int32_t *)(buf + 2 * gs);   /* [nb_rx][grid], planes [p * 2 + a] */
  int16_t *dl = (int16_t *)(buf + 6 * gs);
  bool ok = true;
  for (int a = 0; a < nb_rx && ok; a++) ok = hipMemcpyAsync((uint8_t *)dy + a * gb, rxdataF[a], gb, hipMemcpyHostToDevice, g_scr.s) == hipSuccess;
  for (int pa = 0; pa < 4 && ok; pa++)
    if ((pa & 1) < nb_rx)
      ok = hipMemcpyAsync((uint8_t *)de + pa * gb, dl_ch_estimates[pa], gb, hipMemcpyHostToDevice, g_scr.s) == hipSuccess;
  int rc = -1;
  if (ok && oai4g_rx_batch_tm2(cfg, 1, dy, de, dl, 0, g_scr.s) == 0 &&
      hipMemcpyAsync(llr, dl, (size_t)n * 2, hipMemcpyDeviceToHost, g_scr.s) == hipSuccess &&
      (!log2_maxh || hipMemcpyAsync(log2_maxh, cfg->d_shift, 1, hipMemcpyDeviceToHost, g_scr.s) == hipSuccess) &&
      hipStreamSynchronize(g_scr.s) == hipSuccess)
    rc = n;
  else
    set_err("rx_pdsch_tm2: HIP error");
  return rc;
}

extern "C" int oai4g_rx_pdsch_siso(const oai4g_frame_parms_t *fp, const int32_t *rxdataF, const int32_t *dl_ch_estimates,
                                   const uint32_t rb_alloc[4], uint8_t Qm, uint8_t num_pdcch_symbols, uint8_t subframe,
                                   int16_t *llr, uint8_t *log2_maxh)
{
  NEED_INIT(-1);
  oai4g_rx_config_t *cfg = rx_cached(fp, rb_alloc, Qm, 0, 0, num_pdcch_symbols, subframe, 0, 1);
  if (!cfg) return -1;
  if (rx_check_batch(cfg, 1) != 0) return -1;
  const size_t gb = (size_t)cfg->h.nsymb * cfg->h.N * 4, gs = (gb + 255) & ~(size_t)255;
  const int n = (int)cfg->llr_count[subframe % 10];
  uint8_t *buf = scratch(2 * gs + (size_t)cfg->h.llr_stride * 2 + 256);
  if (!buf) return -1;
  int32_t *dy = (int32_t *)buf, *dh = (int32_t *)(buf + gs);
  int16_t *dl = (int16_t *)(buf + 2 * gs);
  int rc = -1;
  if (hipMemcpyAsync(dy, rxdataF, gb, hipMemcpyHostToDevice, g_scr.s) == hipSuccess &&
      hipMemcpyAsync(dh, dl_ch_estimates, gb, hipMemcpyHostToDevice, g_scr.s) == hipSuccess &&
      oai4g_rx_batch(cfg, 1, dy, dh, dl, 0, g_scr.s) == 0 &&
      hipMemcpyAsync(llr, dl, (size_t)n * 2, hipMemcpyDeviceToHost, g_scr.s) == hipSuccess &&
      (!log2_maxh || hipMemcpyAsync(log2_maxh, cfg->d_shift, 1, hipMemcpyDeviceToHost, g_scr.s) == hipSuccess) &&
      hipStreamSynchronize(g_scr.s) == hipSuccess)
    rc = n;
  else
    set_err("rx_pdsch_siso: HIP error");
  return rc;
}

/* dlsch_unscrambling (dlsch_scrambling.c:99-137): llr[k] *= 2 c(k) - 1 for k < 32 (1 + G / 32),
 * c_init = rnti 2^14 + q 2^13 + (Ns / 2) 2^9 + Nid_cell (mbsfn_flag = 0), on a host buffer: the
 * sequence words are set up here, the sign flips run on the GPU (k_rx_unscramble) */
extern "C" void oai4g_dlsch_unscrambling(const oai4g_frame_parms_t *fp, int mbsfn_flag, uint16_t rnti, int G,
                                         int16_t *llr, uint8_t q, uint8_t Ns)
{
  NEED_INIT();
  if (G < 0) return;
  /* dlsch_scrambling.c:115-118: the PMCH (mbsfn_flag) sequence depends on the MBSFN area only */
  uint32_t x1 = 1u + (1u << 31),
           x2 = mbsfn_flag ? ((uint32_t)(Ns >> 1) << 9) + fp->Nid_cell_mbsfn
                           : ((uint32_t)rnti << 14) + ((uint32_t)q << 13) + ((uint32_t)(Ns >> 1) << 9) + fp->Nid_cell;
  x2 = x2 ^ ((x2 ^ (x2 >> 1) ^ (x2 >> 2) ^ (x2 >> 3)) << 31);
  auto step = [&]() {
    x1 = (x1 >> 1) ^ (x1 >> 4);
    x1 = x1 ^ (x1 << 31) ^ (x1 << 28);
    x2 = (x2 >> 1) ^ (x2 >> 2) ^ (x2 >> 3) ^ (x2 >> 4);
    x2 = x2 ^ (x2 << 31) ^ (x2 << 30) ^ (x2 << 29) ^ (x2 << 28);
  };
  for (int n = 1; n < 50; n++) step();
  const int words = 1 + (G >> 5);
  std::vector<uint32_t> c(words);
  for (int i = 0; i < words; i++) {
    step();
    c[i] = x1 ^ x2;
  }
  const size_t lb = (size_t)words * 64, lbs = (lb + 255) & ~(size_t)255;
  uint8_t *buf = scratch(lbs + (size_t)words * 4);
  if (!buf) return;
  int16_t *dl = (int16_t *)buf;
  uint32_t *dc = (uint32_t *)(buf + lbs);
  if (hipMemcpyAsync(dl, llr, lb, hipMemcpyHostToDevice, g_scr.s) != hipSuccess ||
      hipMemcpyAsync(dc, c.data(), (size_t)words * 4, hipMemcpyHostToDevice, g_scr.s) != hipSuccess ||
      oai4g_launch_unscramble(dl, dc, words * 32, g_scr.s) != hipSuccess ||
      hipMemcpyAsync(llr, dl, lb, hipMemcpyDeviceToHost, g_scr.s) != hipSuccess ||
      hipStreamSynchronize(g_scr.s) != hipSuccess)
    set_err("dlsch_unscrambling: HIP error");
}

/* ------------------------------------------------------------------------------------------
 * Downlink channel estimation (lte_dl_channel_estimation.c:37-701 with high_speed_flag = 1;
 * one RX antenna; the 6 / 50 / 100, 25 and 15 PRB interpolators).
 * ---------------------------------------------------------------------------------------- */
/* filt96_32.h by formula: ramp levels floor(16384 v / 6); the six filters of pilot offset k
 * (lte_dl_channel_estimation.c:105-180) as fl, f2l2, f, f2, fr, f2r2 */
extern "C" void oai4g_chest_filters(uint8_t k, int16_t out[6][24])
{
  auto lv = [](int v) { return (int16_t)((16384 * v) / 6); };
  const int s1 = k, s2 = k + 2;
  for (int t = 0; t < 24; t++) {
    const int u1 = t - s1, u2 = t - s2;
    const int16_t tri1 = (u1 >= 0 && u1 <= 10) ? lv(6 - std::abs(u1 - 5)) : 0;
    const int16_t tri2 = (u2 >= 0 && u2 <= 10) ? lv(6 - std::abs(u2 - 5)) : 0;
    out[2][t] = tri1;                                                           /* filt24_k */
    out[3][t] = tri2;                                                           /* filt24_(k+2) */
    out[4][t] = (u1 >= 11 && u1 <= 16) ? (int16_t)-lv(u1 - 11) : tri1;          /* filt24_kr2 */
    out[5][t] = (u2 >= 0 && u2 <= 10) ? lv(u2 + 1) : 0;                         /* filt24_(k+2)r */
    if (k == 0) {                                                               /* filt24_0, filt24_2 */
      out[0][t] = tri1;
      out[1][t] = tri2;
    } else {
      out[0][t] = (u1 >= 0 && u1 <= 10 && !(k == 3 && (t == 3 || t == 4))) ? lv(11 - u1) : 0;   /* filt24_kl */
      out[1][t] = (u2 >= -6 && u2 <= -1) ? (int16_t)(k == 3 && t == 0 ? 0 : -lv(-u2 - 1)) : tri2; /* _(k+2)l2 */
    }
  }
}

/* The DC-pair filters of the 25-PRB interpolator, filt24_k_dcr (last pilot below DC) and
 * filt24_(k+2)_dcl (first pilot above it), k = 0..5 (filt96_32.h:35-113; used at
 * lte_dl_channel_estimation.c:431-454).  Their slopes round irregularly, so they are table data. */
static const int16_t chest_dcr[6][24] = {
    {2730, 5461, 8192, 10922, 13653, 16384, 14043, 11703, 9362, 7022, 4681},
    {0, 2730, 5461, 8192, 10922, 13653, 16384, 14043, 11703, 9362, 7022, 4681},
    {0, 0, 2730, 5461, 8192, 10922, 13653, 16384, 14043, 11703, 9362, 4681, 2341},
    {0, 0, 0, 2730, 5461, 8192, 10922, 13653, 16384, 14043, 11703, 7022, 4681, 2341},
    {0, 0, 0, 0, 2730, 5461, 8192, 10922, 13653, 16384, 14043, 11703, 7022, 4681, 2341},
    {0, 0, 0, 0, 0, 2730, 5461, 8192, 10922, 13653, 16384, 11703, 9362, 7022, 4681, 2730}};
static const int16_t chest_dcl[6][24] = {
    {0, 0, 2341, 4681, 7022, 9362, 11703, 16384, 13653, 10922, 8192, 5461, 2730},
    {0, 0, 0, 2341, 4681, 7022, 9362, 14043, 16384, 13653, 10922, 8192, 5461, 2730},
    {0, 0, 0, 0, 2341, 7022, 9362, 11703, 14043, 16384, 13653, 10922, 8192, 5461, 2730},
    {0, 0, 0, 0, 0, 2341, 4681, 9362, 11703, 14043, 16384, 13653, 10922, 8192, 5461, 2730},
    {0, 0, 0, 0, 0, 0, 4681, 7022, 9362, 11703, 14043, 16384, 13653, 10922, 8192, 5461, 2730},
    {0, 0, 0, 0, 0, 0, 0, 4681, 7022, 9362, 11703, 14043, 16384, 13653, 10922, 8192, 5461, 2730}};

extern "C" void oai4g_chest_dc_filters(uint8_t k, int16_t out[2][24])
{
  memcpy(out[0], chest_dcr[k % 6], sizeof(out[0]));
  memcpy(out[1], chest_dcl[k % 6], sizeof(out[1]));
}

struct oai4g_chest_config {
  chest_dev_t h;
  chest_dev_t *d = nullptr;
};

static int chest_fill(const oai4g_frame_parms_t *fp, uint8_t p, chest_dev_t &h)
{
  const uint32_t N_RB = fp->N_RB_DL;
  if (p > 1) { set_err("lte_dl_channel_estimation: p %d (ports 0 / 1 only)", p); return -1; }
  memset(&h, 0, sizeof(h));
  h.N = fp->ofdm_symbol_size;
  h.N_RB = N_RB;
  h.nsymb = fp->Ncp == 0 ? 14 : 12;
  h.elem_syms = h.nsymb;
  h.next_syms = h.nsymb;
  h.Ncp = fp->Ncp;
  h.fco = fp->first_carrier_offset;
  h.p = p;
  h.branch = (N_RB == 6 || N_RB == 15 || N_RB == 25 || N_RB == 50 || N_RB == 100) ? 1 : 0;   /* others: "not implemented" */
  for (int l01 = 0; l01 < 2; l01++) {
    const uint32_t nu = p == 0 ? (l01 ? 3 : 0) : (l01 ? 0 : 3);
    h.k[l01] = (nu + fp->nushift) % 6;
    /* the pilots above DC start at bin 1 + k; the 15-PRB branch uses 1 + nushift + 3 p whatever
     * nu is (lte_dl_channel_estimation.c:582) */
    h.off2[l01] = N_RB == 15 ? 1 + fp->nushift + 3 * p : 1 + h.k[l01];
    oai4g_chest_filters((uint8_t)h.k[l01], h.filt[l01]);
    memcpy(h.filt[l01][6], chest_dcr[h.k[l01]], sizeof(h.filt[l01][6]));
    memcpy(h.filt[l01][7], chest_dcl[h.k[l01]], sizeof(h.filt[l01][7]));
  }
  lte_gold_table_h(fp, h.gold);
  return 0;
}

extern "C" oai4g_chest_config_t *oai4g_chest_config_create(const oai4g_frame_parms_t *fp, uint8_t p,
                                                           uint8_t first_subframe, uint8_t subframe_step)
{
  NEED_INIT(nullptr);
  auto *cfg = new oai4g_chest_config();
  if (chest_fill(fp, p, cfg->h) != 0) { delete cfg; return nullptr; }
  cfg->h.first_sf = first_subframe % 10;
  cfg->h.sf_step = subframe_step;
  if (hipMalloc(&cfg->d, sizeof(chest_dev_t)) != hipSuccess ||
      hipMemcpy(cfg->d, &cfg->h, sizeof(chest_dev_t), hipMemcpyHostToDevice) != hipSuccess) {
    set_err("chest_config: device allocation / upload failed");
    oai4g_chest_config_destroy(cfg);
    return nullptr;
  }
  return cfg;
}

extern "C" int oai4g_chest_config_set_stride(oai4g_chest_config_t *cfg, uint32_t subframes_per_element,
                                             uint32_t next_subframes)
{
  NEED_INIT(-1);
  if (!cfg || subframes_per_element < 1 || next_subframes < 1) { set_err("chest_config_set_stride: bad arguments"); return -1; }
  cfg->h.elem_syms = cfg->h.nsymb * subframes_per_element;
  cfg->h.next_syms = cfg->h.nsymb * next_subframes;
  if (hipMemcpy(cfg->d, &cfg->h, sizeof(chest_dev_t), hipMemcpyHostToDevice) != hipSuccess) {
    set_err("chest_config_set_stride: upload failed");
    return -1;
  }
  return 0;
}

extern "C" void oai4g_chest_config_destroy(oai4g_chest_config_t *cfg)
{
  if (!cfg) return;
  if (cfg->d) hipFree(cfg->d);
  delete cfg;
}

extern "C" int oai4g_chest_batch(oai4g_chest_config_t *cfg, int n_sf, const int32_t *d_rxdataF, int32_t *d_est,
                                 void *stream)
{
  NEED_INIT(-1);
  if (!cfg || n_sf < 0) { set_err("chest_batch: bad arguments"); return -1; }
  HCK(oai4g_launch_chest(cfg->d, &cfg->h, n_sf, d_rxdataF, d_est, (hipStream_t)stream), -1);
  return 0;
}

extern "C" int oai4g_chest_batch_pilots(oai4g_chest_config_t *cfg, int n_sf, const int32_t *d_rxdataF, int32_t *d_pil,
                                        void *stream)
{
  NEED_INIT(-1);
  if (!cfg || n_sf < 0) { set_err("chest_batch_pilots: bad arguments"); return -1; }
  HCK(oai4g_launch_chest_pilots(cfg->d, &cfg->h, n_sf, d_rxdataF, d_pil, (hipStream_t)stream), -1);
  return 0;
}

/* Fused batch: estimation + demodulation without the estimate buffer (k_rx_chest); the two
 * configurations must describe the same frame and subframe sequence. */
extern "C" int oai4g_rx_batch_estimated(oai4g_rx_config_t *rx, oai4g_chest_config_t *ce, int n_sf,
                                        const int32_t *d_rxdataF, int16_t *d_llr, int unscramble, void *stream)
{
  NEED_INIT(-1);
  if (!rx || !ce || n_sf < 0) { set_err("rx_batch_estimated: bad arguments"); return -1; }
  if (rx_check_batch(rx, n_sf) != 0) return -1;
  if (rx->h.N != ce->h.N || rx->h.nsymb != ce->h.nsymb || rx->h.first_sf != ce->h.first_sf ||
      rx->h.sf_step != ce->h.sf_step || ce->h.p != 0 || ce->h.N_RB > 100) {
    set_err("rx_batch_estimated: the demodulation and estimation configurations differ (frame, subframes, port 0)");
    return -1;
  }
  if (n_sf > rx->shift_cap) {
    if (rx->d_shift) hipFree(rx->d_shift);
    HCK(hipMalloc(&rx->d_shift, (size_t)n_sf), -1);
    rx->shift_cap = n_sf;
  }
  HCK(oai4g_launch_rx_chest(ce->d, rx->d, &rx->h, n_sf, d_rxdataF, d_llr, rx->d_shift, unscramble,
                            (hipStream_t)stream), -1);
  return 0;
}

/* lte_dl_channel_estimation drop-in on host buffers: rxdataF / dl_ch_estimates = [nsymb][N] of the
 * subframe (the UE's rxdataF and dl_ch_estimates[eNB_offset 0][(p << 1) + 0]); Ns, p, l, symbol as
 * slot_fep passes them (slot_fep.c:188-192) */
extern "C" int oai4g_lte_dl_channel_estimation(const oai4g_frame_parms_t *fp, const int32_t *rxdataF,
                                               int32_t *dl_ch_estimates, uint8_t Ns, uint8_t p, uint8_t l,
                                               uint8_t symbol)
{
  NEED_INIT(-1);
  const uint32_t nsymb = fp->Ncp == 0 ? 14 : 12, p1 = fp->Ncp ? 3 : 4, p2 = fp->Ncp ? 6 : 7, p3 = fp->Ncp ? 9 : 11;
  if (Ns >= 20 || (symbol != 0 && symbol != p1 && symbol != p2 && symbol != p3)) {
    set_err("lte_dl_channel_estimation: Ns %d / symbol %d is not a pilot symbol", Ns, symbol);
    return -1;
  }
  chest_dev_t h;
  if (chest_fill(fp, p, h) != 0) return -1;
  const size_t N = fp->ofdm_symbol_size, eb = (size_t)nsymb * N * 4, cs = (sizeof(chest_dev_t) + 255) & ~(size_t)255;
  uint8_t *buf = scratch(cs + eb + N * 4);
  if (!buf) return -1;
  chest_dev_t *dc = (chest_dev_t *)buf;
  int32_t *de = (int32_t *)(buf + cs), *dr = (int32_t *)(buf + cs + eb);
  /* the call reads the previous pilot row and writes its own row plus the rows between the two
   * (k_chest_symbol / ce_interp): only those rows cross PCIe */
  const uint32_t prev_row = symbol == 0 ? p3 : symbol == p1 ? 0 : symbol == p2 ? p1 : p2;
  const size_t rb = N * 4;
  auto rows_d2h = [&](uint32_t r0, uint32_t n) {
    return hipMemcpyAsync(dl_ch_estimates + (size_t)r0 * N, de + (size_t)r0 * N, n * rb, hipMemcpyDeviceToHost,
                          g_scr.s) == hipSuccess;
  };
  if (hipMemcpyAsync(dc, &h, sizeof(h), hipMemcpyHostToDevice, g_scr.s) != hipSuccess ||
      hipMemcpyAsync(de + (size_t)prev_row * N, dl_ch_estimates + (size_t)prev_row * N, rb, hipMemcpyHostToDevice,
                     g_scr.s) != hipSuccess ||
      hipMemcpyAsync(dr, rxdataF + (size_t)symbol * N, N * 4, hipMemcpyHostToDevice, g_scr.s) != hipSuccess ||
      oai4g_launch_chest_symbol(dc, &h, dr, de, Ns, l, symbol, g_scr.s) != hipSuccess ||
      !(symbol == 0 ? rows_d2h(p3 + 1, nsymb - 1 - p3) && rows_d2h(0, 1) : rows_d2h(prev_row + 1, symbol - prev_row)) ||
      hipStreamSynchronize(g_scr.s) != hipSuccess) {
    set_err("lte_dl_channel_estimation: HIP error");
    return -1;
  }
  return 0;
}

/* ------------------------------------------------------------------------------------------
 * lte_est_freq_offset (PHY/LTE_ESTIMATION/lte_est_freq_offset.c:104-193) and dl_ch_estimates_time
 * (lte_dl_channel_estimation.c:704-738)
 * ---------------------------------------------------------------------------------------- */
static int fo_rows(const oai4g_frame_parms_t *fp, int l, uint32_t *row_off, uint32_t *prev_off)
{
  const int lp = 4 - fp->Ncp;
  if (l != 0 && l != lp) {
    set_err("lte_est_freq_offset: l (%d) must be 0 or %d", l, lp);   /* :127-130 */
    return -1;
  }
  if (fp->N_RB_DL < 4 || (size_t)fp->N_RB_DL * 12 + 12 > fp->ofdm_symbol_size) {
    set_err("lte_est_freq_offset: N_RB_DL %d not supported", fp->N_RB_DL);
    return -1;
  }
  *row_off = (uint32_t)l * fp->ofdm_symbol_size;
  *prev_off = (uint32_t)(l == 0 ? lp : 0) * fp->ofdm_symbol_size;
  return 0;
}

extern "C" int oai4g_freq_offset_omega_batch(const oai4g_frame_parms_t *fp, int n_jobs, const int32_t *d_est,
                                             size_t est_stride, int l, int32_t *d_omega, void *stream)
{
  NEED_INIT(-1);
  uint32_t ro, po;
  if (fo_rows(fp, l, &ro, &po) != 0) return -1;
  if (n_jobs < 0 || (n_jobs > 0 && (!d_est || !d_omega))) { set_err("freq_offset_omega_batch: bad arguments"); return -1; }
  HCK(oai4g_launch_freq_offset(d_est, est_stride, n_jobs, fp->N_RB_DL, ro, po, d_omega, (hipStream_t)stream), -1);
  return 0;
}

extern "C" int oai4g_freq_offset_update(const oai4g_frame_parms_t *fp, int32_t omega, int *freq_offset, int *first_run)
{
  if (!fp || !freq_offset || !first_run) { set_err("freq_offset_update: bad arguments"); return -1; }
  const double phase = atan2((double)(int16_t)((uint32_t)omega >> 16), (double)(int16_t)omega);   /* :168 */
  const int est = (int)(phase / (2 * M_PI) / (fp->Ncp == 0 ? 285.8e-6 : 2.5e-4));              /* :174 */
  if (*first_run == 1) {                                                                          /* :178-182 */
    *freq_offset = est;
    *first_run = 0;
  } else
    *freq_offset = (est * (1 << 10) + *freq_offset * (32767 - (1 << 10))) >> 15;
  return 0;
}

/* the reference's function-static first_run (:117), shared by every caller as there */
static int g_fo_first_run = 1;
static std::mutex g_fo_mu;

extern "C" int oai4g_lte_est_freq_offset(int32_t *const *dl_ch_estimates, const oai4g_frame_parms_t *fp, int l,
                                         int *freq_offset, int reset)
{
  NEED_INIT(-1);
  if (!dl_ch_estimates || !dl_ch_estimates[0] || !fp || !freq_offset) { set_err("lte_est_freq_offset: bad arguments"); return -1; }
  std::lock_guard<std::mutex> lk(g_fo_mu);
  if (reset != 0) g_fo_first_run = 1;                                                             /* :122-123 */
  uint32_t ro, po;
  if (fo_rows(fp, l, &ro, &po) != 0) return -1;
  const size_t words = (size_t)(4 - fp->Ncp + 1) * fp->ofdm_symbol_size;   /* rows 0 .. 4 - Ncp */
  uint8_t *buf = scratch(words * 4 + 256);
  if (!buf) return -1;
  int32_t *d_est = (int32_t *)buf, *d_om = (int32_t *)(buf + ((words * 4 + 255) & ~(size_t)255));
  int32_t om = 0;
  HCK(hipMemcpyAsync(d_est, dl_ch_estimates[0], words * 4, hipMemcpyHostToDevice, g_scr.s), -1);
  HCK(oai4g_launch_freq_offset(d_est, 0, 1, fp->N_RB_DL, ro, po, d_om, g_scr.s), -1);
  HCK(hipMemcpyAsync(&om, d_om, 4, hipMemcpyDeviceToHost, g_scr.s), -1);
  HCK(hipStreamSynchronize(g_scr.s), -1);
  return oai4g_freq_offset_update(fp, om, freq_offset, &g_fo_first_run);
}

static int chest_time_log2n(const oai4g_frame_parms_t *fp)
{
  const int l2 = fp->log2_symbol_size;
  return (l2 >= 7 && l2 <= 11) ? l2 : 9;   /* the switch's default: idft512 (:713-735) */
}

extern "C" int oai4g_chest_time_batch(const oai4g_frame_parms_t *fp, int n_jobs, const int32_t *d_est,
                                      size_t est_stride, int32_t *d_time, size_t time_stride, void *stream)
{
  NEED_INIT(-1);
  const int l2 = chest_time_log2n(fp);
  if (!fp || n_jobs < 0 || (n_jobs > 0 && (!d_est || !d_time)) || est_stride < ((size_t)1 << l2) + 8 ||
      time_stride < ((size_t)1 << l2)) {
    set_err("chest_time_batch: bad arguments (an estimate plane must hold N + 8 words)");
    return -1;
  }
  HCK(oai4g_launch_idft_strided(d_est, d_time, l2, n_jobs, est_stride, 8, time_stride, 1, g_tw, (hipStream_t)stream), -1);
  return 0;
}

extern "C" int oai4g_dl_ch_estimates_time(const oai4g_frame_parms_t *fp, int nb_antennas_rx,
                                          const int32_t *const *dl_ch_estimates, int32_t *const *dl_ch_estimates_time)
{
  NEED_INIT(-1);
  if (!fp || !dl_ch_estimates || !dl_ch_estimates_time || nb_antennas_rx < 1 || nb_antennas_rx > 2) {
    set_err("dl_ch_estimates_time: bad arguments");
    return -1;
  }
  const int l2 = chest_time_log2n(fp);
  const size_t n = (size_t)1 << l2, in_w = n + 8;
  const int ntx = fp->nb_antennas_tx_eNB ? fp->nb_antennas_tx_eNB : fp->nb_antennas_tx;
  int planes[8], np = 0;
  for (int aarx = 0; aarx < nb_antennas_rx; aarx++)        /* :731-737, NULL planes skipped */
    for (int p = 0; p < ntx && p < 4; p++)
      if (dl_ch_estimates[(p << 1) + aarx]) planes[np++] = (p << 1) + aarx;
  if (np == 0) return 0;
  const size_t ib = (size_t)np * in_w * 4, ob = (size_t)np * n * 4;
  uint8_t *buf = scratch(ib + ob + 256);
  if (!buf) return -1;
  int32_t *d_in = (int32_t *)buf, *d_out = (int32_t *)(buf + ((ib + 255) & ~(size_t)255));
  for (int i = 0; i < np; i++)
    HCK(hipMemcpyAsync(d_in + i * in_w, dl_ch_estimates[planes[i]], in_w * 4, hipMemcpyHostToDevice, g_scr.s), -1);
  HCK(oai4g_launch_idft_strided(d_in, d_out, l2, np, in_w, 8, n, 1, g_tw, g_scr.s), -1);   /* words 8 .. N + 7 */
  for (int i = 0; i < np; i++)
    HCK(hipMemcpyAsync(dl_ch_estimates_time[planes[i]], d_out + i * n, n * 4, hipMemcpyDeviceToHost, g_scr.s), -1);
  HCK(hipStreamSynchronize(g_scr.s), -1);
  return 0;
}
