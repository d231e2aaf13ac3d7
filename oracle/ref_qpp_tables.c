/*
 * TEST INFRASTRUCTURE ONLY — link-time data for the reference build in oracle/_ref.
 *
 * The reference's turbo encoder and decoders (PHY/CODING/3gpplte_sse.c:398-405,
 * 3gpplte_turbo_decoder_sse_16bit.c:906-907,1013, 3gpplte_turbo_decoder_sse_8bit.c:854-855,976)
 * read the QPP interleaver through two extern tables declared in the reference's own
 * PHY/CODING/extern_3GPPinterleaver.h:36-37 (`f1f2mat[]`, `il_tb[]`).  Their definitions live in
 * PHY/CODING/lte_interleaver.h, which is listed in the reference's .MISSING_LARGE_BLOBS and is not
 * in the tree.  The data is fully determined by 36.212 Table 5.1.3-3 (the (f1, f2) pairs are also
 * in the reference's lte_interleaver2.h:29 `f1f2mat_old`) and by the QPP rule the reference itself
 * states at 3gpplte.c:50-74: il_tb[beg + i] = (f1 i + f2 i^2) mod K.  This file defines those
 * two objects from include/oai4g_qpp.c; no reference header is replaced and no reference source
 * is modified.  ref_qpp_init() must run before the first encoder/decoder call.
 */
#include "../include/oai4g_qpp.h"

typedef struct interleaver_codebook {   /* layout of extern_3GPPinterleaver.h:28-34 */
  unsigned long nb_bits;
  unsigned short f1;
  unsigned short f2;
  unsigned int beg_index;
} t_interleaver_codebook;

t_interleaver_codebook f1f2mat[OAI4G_QPP_ROWS];
short il_tb[188 * 6144];                 /* >= sum of all K (1.1e6 entries is a loose bound) */
short reverse_il_tl[1];                  /* declared by extern_3GPPinterleaver.h:38; unused by the built TUs */

void ref_qpp_init(void)
{
  unsigned int beg = 0;
  for (int r = 0; r < OAI4G_QPP_ROWS; r++) {
    const unsigned int K = oai4g_qpp_table[r].K, f1 = oai4g_qpp_table[r].f1, f2 = oai4g_qpp_table[r].f2;
    f1f2mat[r].nb_bits = K;
    f1f2mat[r].f1 = (unsigned short)f1;
    f1f2mat[r].f2 = (unsigned short)f2;
    f1f2mat[r].beg_index = beg;
    for (unsigned int i = 0; i < K; i++)
      il_tb[beg + i] = (short)((f1 * (unsigned long long)i + f2 * (unsigned long long)i * i) % K);
    beg += K;
  }
}
