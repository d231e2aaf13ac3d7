/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle of the control region of the downlink grid (PDCCH /
 * DCI).  A plain-C restatement of the reference's algorithm, loop for
 * loop, used by tests/ and __graft_entry__.smoke() as the checker of the GPU path; never linked
 * into the product library.
 *
 *   crc16                       PHY/CODING/crc_byte.c:155-171 (incl. its partial-byte step)
 *   ccodelte_encode             PHY/CODING/ccoding_byte_lte.c:55-230 (+ ccodelte_init :243-262)
 *   sub_block_interleaving_cc   PHY/CODING/lte_rate_matching.c:133-190
 *   lte_rate_matching_cc        PHY/CODING/lte_rate_matching.c:637-680
 *   get_mi                      PHY/LTE_TRANSPORT/phich.c:59-118
 *   generate_phich_reg_mapping  PHY/LTE_TRANSPORT/phich.c:280-386 (normal PHICH duration)
 *   check_phich_reg             PHY/LTE_TRANSPORT/dci.c:62-121
 *   generate_dci0/dci_encoding  PHY/LTE_TRANSPORT/dci.c:170-270
 *   pdcch_interleaving          PHY/LTE_TRANSPORT/dci.c:277-341
 *   pdcch_scrambling            PHY/LTE_TRANSPORT/dci.c:1905-1930
 *   get_num_pdcch_symbols       PHY/LTE_TRANSPORT/dci.c:1964-2022
 *   generate_dci_top            PHY/LTE_TRANSPORT/dci.c:2024-2346
 *   get_nCCE / get_nquad        PHY/LTE_TRANSPORT/dci.c:2494-2538
 *   get_nCCE_offset             SCHED/phy_procedures_lte_eNb.c:308-391
 *
 * Pinned: crc16 and ccodelte_encode against the reference's own crc_byte.c / ccoding_byte_lte.c
 * (oracle/_ref/libref_coding.so, tests/test_ctrl_cpu.py); the whole PDCCH chain against the
 * 36.211 §6.8 / 36.212 §5.3.3 spec model (tests/spec_model.py: pdcch_grid).
 */
#include <stdlib.h>
#include <string.h>

#include "oai_oracle.h"

#define CCEBITS 72
#define DCI_BITS_MAX ((2 * 33 + 22) * CCEBITS)   /* dci.c:264-267 */
#define MSYMB (DCI_BITS_MAX / 2)

static const uint8_t bitrev_cc[32] = {1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31,
                                      0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30};

/* ---------------------------------------------------------------- CRC16 */
static uint16_t crc16_tab[256];
static void crc16_init(void)
{
  if (crc16_tab[1]) return;
  for (int v = 0; v < 256; v++) {          /* crcbit(&v, 1, 0x10210000) >> 16 (crc_byte.c:66-83,95) */
    uint32_t crc = 0, c = (uint32_t)v << 24;
    for (int i = 0; i < 8; i++) {
      crc = ((c ^ crc) & 0x80000000u) ? (crc << 1) ^ 0x10210000u : crc << 1;
      c <<= 1;
    }
    crc16_tab[v] = (uint16_t)(crc >> 16);
  }
}

uint32_t orc_crc16(const uint8_t *in, int bitlen)
{
  crc16_init();
  int octetlen = bitlen / 8, resbit = bitlen % 8;
  uint32_t crc = 0;
  while (octetlen-- > 0) crc = (crc << 8) ^ ((uint32_t)crc16_tab[(*in++) ^ (crc >> 24)] << 16);
  if (resbit > 0)        /* the reference's partial-byte step, as written (:167-168) */
    crc = (crc << resbit) ^ ((uint32_t)crc16_tab[((*in) >> (8 - resbit)) ^ (crc >> (32 - resbit))] << 16);
  return crc;
}

/* ---------------------------------------------------------------- tail-biting convolutional code */
static uint8_t cc_tab[128];
static void cc_init(void)
{
  static const uint16_t g[3] = {0133, 0171, 0165};       /* glte (:37) */
  if (cc_tab[127] || cc_tab[1]) return;
  for (int i = 0; i < 128; i++) {
    uint8_t o = 0;
    for (int j = 0; j < 3; j++) o |= (uint8_t)((__builtin_popcount((unsigned)i & g[j]) & 1) << j);
    cc_tab[i] = o;
  }
}

void orc_ccodelte_encode(int32_t numbits, uint8_t add_crc, const uint8_t *in, uint8_t *out, uint16_t rnti)
{
  cc_init();
  uint32_t state = 0, crc = 0;
  uint8_t c, first_bit;
  uint32_t next_last_byte = 0;
  if (add_crc == 1) {                       /* UCI CRC8: not used on this path */
    return;
  } else if (add_crc == 2) {
    crc = orc_crc16(in, numbits) ^ ((uint32_t)rnti << 16);
    first_bit = 2;
    c = (uint8_t)((crc >> 16) & 0xff);
  } else {
    next_last_byte = (uint32_t)numbits >> 3;
    first_bit = (uint8_t)((numbits - 6) & 7);
    c = in[next_last_byte - 1];
  }
  for (int sb = 0; sb < 8 - first_bit; sb++)              /* tail-biting start state (:107-118) */
    if (c & (1 << (7 - first_bit - sb))) state |= 1u << sb;
  if (add_crc == 0 && (numbits & 7) > 0) {
    c = in[next_last_byte];
    for (int sb = (numbits & 7) - 1; sb >= 0; sb--) {
      state >>= 1;
      if (c & (1 << sb)) state |= 64;
    }
  }
  state = (state & 0x3f) << 1;
  while (numbits > 0) {                                   /* :147-176 */
    c = *in++;
    for (int sb = 7; sb >= 0 && numbits > 0; sb--, numbits--) {
      state >>= 1;
      if (c & (1 << sb)) state |= 64;
      const uint8_t o = cc_tab[state];
      *out++ = o & 1;
      *out++ = (o >> 1) & 1;
      *out++ = (o >> 2) & 1;
    }
  }
  if (add_crc == 2) {                                     /* :208-230 */
    const uint16_t c16 = (uint16_t)(crc >> 16);
    for (int sb = 15; sb >= 0; sb--) {
      state >>= 1;
      if (c16 & (1 << sb)) state |= 64;
      const uint8_t o = cc_tab[state];
      *out++ = o & 1;
      *out++ = (o >> 1) & 1;
      *out++ = (o >> 2) & 1;
    }
  }
}

uint32_t orc_sub_block_interleaving_cc(uint32_t D, const uint8_t *d, uint8_t *w)
{
  uint32_t RCC = D >> 5;
  if (D & 0x1f) RCC++;
  const uint32_t Kpi = RCC << 5, ND3 = (Kpi - D) * 3;
  uint32_t k = 0;
  for (uint32_t col = 0; col < 32; col++) {
    uint32_t index3 = 3 * bitrev_cc[col];
    for (uint32_t row = 0; row < RCC; row++) {             /* d[-3 ND ...] reads the NULL prefix */
      w[k] = d[(int32_t)index3 - (int32_t)ND3];
      w[Kpi + k] = d[(int32_t)index3 - (int32_t)ND3 + 1];
      w[2 * Kpi + k] = d[(int32_t)index3 - (int32_t)ND3 + 2];
      index3 += 96;
      k++;
    }
  }
  return RCC;
}

uint32_t orc_lte_rate_matching_cc(uint32_t RCC, uint16_t E, const uint8_t *w, uint8_t *e)
{
  uint32_t ind = 0;
  const uint16_t Kw = (uint16_t)(3 * (RCC << 5));
  for (uint32_t k = 0; k < E; k++) {
    while (w[ind] == 2) {
      ind++;
      if (ind == Kw) ind = 0;
    }
    e[k] = w[ind];
    ind++;
    if (ind == Kw) ind = 0;
  }
  return E;
}

/* ---------------------------------------------------------------- geometry */
uint8_t orc_get_mi(const orc_frame_t *fp, uint8_t sf)
{
  if (fp->frame_type == 0) return 1;
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

static uint32_t ngroup_phich(const orc_frame_t *fp)
{
  uint32_t ng = (fp->phich_resource * fp->N_RB_DL) / 48;
  if ((fp->phich_resource * fp->N_RB_DL) % 48) ng++;
  if (fp->Ncp == 1) ng <<= 1;
  return ng;
}

uint16_t orc_get_nquad(uint8_t npdcch, const orc_frame_t *fp, uint8_t mi)
{
  uint32_t Nreg = 0;
  /* get_nquad truncates Ngroup_PHICH to uint8_t before the doubling and the mi product (:2502) */
  uint8_t ng = (uint8_t)((fp->phich_resource * fp->N_RB_DL) / 48);
  if ((fp->phich_resource * fp->N_RB_DL) % 48) ng++;
  if (fp->Ncp == 1) ng <<= 1;
  ng *= mi;
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

uint16_t orc_get_nCCE(uint8_t npdcch, const orc_frame_t *fp, uint8_t mi)
{
  return orc_get_nquad(npdcch, fp, mi) / 9;
}

uint8_t orc_get_num_pdcch_symbols(uint8_t num_dci, const orc_dci_alloc_t *dci_alloc, const orc_frame_t *fp,
                                  uint8_t sf)
{
  uint16_t numCCE = 0;
  uint8_t nCCEmin = 0;
  if (fp->Ncp == 1) {
    if (fp->frame_type == 1 && (fp->tdd_config < 3 || fp->tdd_config == 6) && (sf == 1 || sf == 6))
      nCCEmin = 2;
    else
      nCCEmin = 3;
  }
  for (int i = 0; i < num_dci; i++) numCCE += (uint16_t)(1 << dci_alloc[i].L);
  const uint8_t mi = orc_get_mi(fp, sf);
  if (numCCE <= orc_get_nCCE(1, fp, mi)) return nCCEmin > 1 ? nCCEmin : 1;
  if (numCCE <= orc_get_nCCE(2, fp, mi)) return nCCEmin > 2 ? nCCEmin : 2;
  if (numCCE <= orc_get_nCCE(3, fp, mi)) return nCCEmin > 3 ? nCCEmin : 3;
  if (fp->N_RB_DL <= 10) {
    if (fp->Ncp == 0) {
      if (9 * numCCE <= fp->N_RB_DL * (fp->nb_antennas_tx_eNB == 4 ? 10 : 11)) return 4;
    } else {
      if (9 * numCCE <= fp->N_RB_DL * (fp->nb_antennas_tx_eNB == 4 ? 9 : 10)) return 4;
    }
  }
  return 0;
}

int orc_phich_reg_mapping(const orc_frame_t *fp, uint16_t phich_reg[56][3])
{
  uint16_t pcfich_reg[4];
  uint8_t fi;
  orc_pcfich_reg_mapping(fp, pcfich_reg, &fi);
  const uint16_t n0 = (uint16_t)(fp->N_RB_DL * 2 - 4);
  uint32_t ng = ngroup_phich(fp);
  const uint32_t nloop = fp->Ncp == 0 ? ng : ng >> 1;
  for (uint32_t m = 0; m < nloop; m++) {
    const uint32_t base[3] = {(fp->Nid_cell + m) % n0, (fp->Nid_cell + m + n0 / 3) % n0,
                              (fp->Nid_cell + m + 2 * n0 / 3) % n0};
    for (int j = 0; j < 3; j++) {
      uint32_t r = base[j];
      for (int q = 0; q < 4; q++)     /* skip the PCFICH REGs in increasing order (:319-363) */
        if (r >= pcfich_reg[(fi + q) & 3]) r++;
      phich_reg[m][j] = (uint16_t)r;
    }
  }
  return (int)nloop;
}

static int check_phich_reg(const orc_frame_t *fp, const uint16_t pcfich_reg[4], const uint16_t phich_reg[56][3],
                           uint32_t kprime, uint8_t lprime, uint8_t mi)
{
  if (lprime > 0 && fp->Ncp == 0) return 0;
  const uint32_t mprime = (lprime == 0 || (lprime == 1 && fp->nb_antennas_tx_eNB == 4)) ? kprime / 6 : kprime >> 2;
  if (lprime == 0 && (mprime == pcfich_reg[0] || mprime == pcfich_reg[1] || mprime == pcfich_reg[2] ||
                      mprime == pcfich_reg[3]))
    return 1;
  if (mi > 0) {
    const uint32_t ng = ngroup_phich(fp);
    for (uint32_t i = 0; i < ng; i++)
      if (mprime == phich_reg[i][0] || mprime == phich_reg[i][1] || mprime == phich_reg[i][2]) return 1;
  }
  return 0;
}

int orc_get_nCCE_offset(int *CCE_table, uint8_t L, int nCCE, int common_dci, uint16_t rnti, uint8_t subframe)
{
  if (common_dci == 1) {
    int nb = L == 4 ? 4 : 2;
    if (nCCE / L < nb) nb = nCCE / L;
    for (int m = nb - 1; m >= 0; m--) {
      int fr = 1;
      for (int l = 0; l < L; l++)
        if (CCE_table[m * L + l] == 1) { fr = 0; break; }
      if (fr) {
        for (int l = 0; l < L; l++) CCE_table[m * L + l] = 1;
        return m * L;
      }
    }
    return -1;
  }
  uint32_t Yk = rnti;
  for (int i = 0; i <= subframe; i++) Yk = (Yk * 39827u) % 65537u;
  Yk = Yk % (uint32_t)(nCCE / L);
  const int nb = (L == 1 || L == 2) ? 6 : 2;
  for (int m = 0; m < nb; m++) {
    const int s = (int)(((Yk + m) % (uint32_t)(nCCE / L)) * L);
    int fr = 1;
    for (int l = 0; l < L; l++)
      if (CCE_table[s + l] == 1) { fr = 0; break; }
    if (fr) {
      for (int l = 0; l < L; l++) CCE_table[s + l] = 1;
      return s;
    }
  }
  return -1;
}

/* ---------------------------------------------------------------- generate_dci_top */
static uint8_t dci_e[DCI_BITS_MAX + 8 * 72];
static uint32_t dci_e_len;

const uint8_t *orc_last_dci_e(uint32_t *len)
{
  *len = dci_e_len;
  return dci_e;
}

static void dci_encode_one(const orc_dci_alloc_t *a, uint8_t *e)
{
  uint8_t flip[8] = {0}, d[3 * (64 + 16) + 96], w[3 * 3 * (64 + 16) + 96];
  const uint8_t *p = a->dci_pdu;
  if (a->dci_length <= 32) {                            /* generate_dci0 byte flip (:233-251) */
    for (int i = 0; i < 4; i++) flip[i] = p[3 - i];
  } else {
    for (int i = 0; i < 8; i++) flip[i] = p[7 - i];
  }
  const uint32_t D = a->dci_length + 16u, E = 72u << a->L;
  memset(d, 2, 96);
  orc_ccodelte_encode(a->dci_length, 2, flip, d + 96, a->rnti);
  const uint32_t RCC = orc_sub_block_interleaving_cc(D, d + 96, w);
  orc_lte_rate_matching_cc(RCC, (uint16_t)E, w, e);
}

uint8_t orc_generate_dci_top(uint8_t num_ue_spec_dci, uint8_t num_common_dci, const orc_dci_alloc_t *dci_alloc,
                             uint32_t n_rnti, int16_t amp, const orc_frame_t *fp, int32_t **txdataF,
                             uint32_t subframe)
{
  (void)n_rnti;
  const uint8_t mi = orc_get_mi(fp, (uint8_t)subframe);
  const uint32_t nushiftmod3 = fp->nushift % 3, N = fp->ofdm_symbol_size;
  int Msymb2;
  switch (fp->N_RB_DL) {                                /* :2050-2074 */
  case 100: Msymb2 = MSYMB; break;
  case 75: Msymb2 = 3 * MSYMB / 4; break;
  case 50: Msymb2 = MSYMB >> 1; break;
  case 25: Msymb2 = MSYMB >> 2; break;
  case 15: Msymb2 = MSYMB * 15 / 100; break;
  case 6: Msymb2 = MSYMB * 6 / 100; break;
  default: Msymb2 = MSYMB >> 2; break;
  }
  const uint8_t npdcch = orc_get_num_pdcch_symbols(num_ue_spec_dci + num_common_dci, dci_alloc, fp, (uint8_t)subframe);
  if (npdcch < 1 || npdcch > 3) return npdcch;         /* the reference maps an undefined CFI codeword here */
  orc_generate_pcfich(npdcch, amp, fp, txdataF, (uint8_t)subframe);

  memset(dci_e, 2, sizeof(dci_e));
  for (int L = 3; L >= 0; L--) {                        /* :2108-2156 */
    int i;
    for (i = 0; i < num_common_dci; i++)
      if (dci_alloc[i].L == L && dci_alloc[i].nCCE >= 0) dci_encode_one(&dci_alloc[i], dci_e + 72 * dci_alloc[i].nCCE);
    for (; i < num_ue_spec_dci + num_common_dci; i++)
      if (dci_alloc[i].L == L && dci_alloc[i].nCCE >= 0) dci_encode_one(&dci_alloc[i], dci_e + 72 * dci_alloc[i].nCCE);
  }
  const uint32_t nquad = orc_get_nquad(npdcch, fp, mi);
  {                                                      /* pdcch_scrambling (:1905-1930) */
    uint32_t x1, x2 = (subframe << 9) + fp->Nid_cell, s = 0;
    for (uint32_t i = 0; i < 8 * nquad; i++) {
      if ((i & 0x1f) == 0) s = orc_gold_generic(&x1, &x2, i == 0);
      if (dci_e[i] != 2) dci_e[i] = (dci_e[i] & 1) ^ ((s >> (i & 0x1f)) & 1);
    }
  }
  dci_e_len = 8 * nquad;

  static int16_t y[2][4096][2], wt[2][4096][2], wbar[2][4096][2];   /* >= 4 Mquad for every N_RB */
  memset(y, 0, sizeof(y));
  memset(wt, 0, sizeof(wt));
  memset(wbar, 0, sizeof(wbar));
  const int16_t g = fp->mode1_flag == 1 ? (int16_t)((amp * 23170) >> 15) : (int16_t)(amp / 2);
  const uint8_t *ep = dci_e;
  if (fp->mode1_flag) {                                  /* :2182-2198: <NIL> -> 0 */
    for (int i = 0; i < Msymb2; i++) {
      for (int c = 0; c < 2; c++, ep++) {
        const int16_t v = *ep == 2 ? 0 : (*ep == 1 ? -g : g);
        y[0][i][c] = y[1][i][c] = v;
      }
    }
  } else {                                               /* :2200-2224: ALAMOUTI, <NIL> -> +g */
    for (int i = 0; i < Msymb2; i += 2) {
      y[0][i][0] = ep[0] == 1 ? -g : g;
      y[0][i][1] = ep[1] == 1 ? -g : g;
      y[1][i][0] = ep[2] == 1 ? g : -g;
      y[1][i][1] = ep[3] == 1 ? -g : g;
      ep += 4;
      y[0][i + 1][0] = -y[1][i][0];
      y[0][i + 1][1] = y[1][i][1];
      y[1][i + 1][0] = y[0][i][0];
      y[1][i + 1][1] = -y[0][i][1];
    }
  }
  {                                                      /* pdcch_interleaving (:277-341) */
    const uint32_t Mquad = nquad;
    uint32_t RCC = Mquad >> 5;
    if (Mquad & 0x1f) RCC++;
    const uint32_t ND = (RCC << 5) - Mquad;
    uint32_t k = 0;
    for (uint32_t col = 0; col < 32; col++) {
      uint32_t index = bitrev_cc[col];
      for (uint32_t row = 0; row < RCC; row++) {
        if (index >= ND) {
          for (int a = 0; a < fp->nb_antennas_tx_eNB && a < 2; a++)
            memcpy(wt[a][k << 2], y[a][(index - ND) << 2], 16);
          k++;
        }
        index += 32;
      }
    }
    for (uint32_t i = 0; i < Mquad; i++)
      for (int a = 0; a < fp->nb_antennas_tx_eNB && a < 2; a++)
        memcpy(wbar[a][i << 2], wt[a][((i + fp->Nid_cell) % Mquad) << 2], 16);
  }
  uint16_t pcfich_reg[4], phich_reg[56][3];
  uint8_t fi;
  memset(phich_reg, 0, sizeof(phich_reg));              /* entries the mapping never writes stay 0 */
  orc_pcfich_reg_mapping(fp, pcfich_reg, &fi);
  orc_phich_reg_mapping(fp, phich_reg);
  const uint32_t nsymb = fp->Ncp == 0 ? 14 : 12;
  uint32_t mprime = 0;
  int re_offset = fp->first_carrier_offset;
#define PUT(off)                                                                  \
  do {                                                                            \
    memcpy(&txdataF[0][(off)], wbar[0][mprime], 4);                               \
    if (fp->nb_antennas_tx_eNB > 1) memcpy(&txdataF[1][(off)], wbar[1][mprime], 4); \
    mprime++;                                                                     \
  } while (0)
  for (uint32_t kprime = 0; kprime < (uint32_t)fp->N_RB_DL * 12; kprime++) {   /* :2240-2340 */
    for (uint8_t lprime = 0; lprime < npdcch; lprime++) {
      const uint32_t symbol_offset = N * (lprime + subframe * nsymb), tti = symbol_offset + (uint32_t)re_offset;
      const int split = re_offset == (int)N - 2;
      if (!check_phich_reg(fp, pcfich_reg, (const uint16_t(*)[3])phich_reg, kprime, lprime, mi)) {
        const uint32_t km = kprime % 12;
        if (lprime == 0 || (lprime == 1 && fp->nb_antennas_tx_eNB == 4)) {
          if (km == 0 || km == 6)
            for (uint32_t i = 0; i < 6; i++)
              if (i != nushiftmod3 && i != nushiftmod3 + 3) PUT(tti + i);
        } else if (km == 0 || km == 4 || km == 8) {
          if (!split) {
            for (uint32_t i = 0; i < 4; i++) PUT(tti + i);
          } else {
            PUT(tti);
            PUT(tti + 1);
            PUT(tti - N + 3);
            PUT(tti - N + 4);
          }
        }
      }
      if (mprime >= (uint32_t)Msymb2) return npdcch;
    }
    re_offset++;
    if (re_offset == (int)N) re_offset = 1;
  }
#undef PUT
  return npdcch;
}
