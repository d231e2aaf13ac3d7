/* QPP interleaver parameter table (3GPP TS 36.212 Table 5.1.3-3). */
#ifndef OAI4G_QPP_H
#define OAI4G_QPP_H
#ifdef __cplusplus
extern "C" {
#endif

#define OAI4G_QPP_ROWS 188

typedef struct {
  unsigned short K;
  unsigned short f1;
  unsigned short f2;
} oai4g_qpp_row_t;

extern const oai4g_qpp_row_t oai4g_qpp_table[OAI4G_QPP_ROWS];

/* Row index for code-block size K (bits), or -1 if K is not a legal turbo size.
 * Same selection rule as the reference (dlsch_coding.c:327-338). */
int oai4g_qpp_index(unsigned int K);

#ifdef __cplusplus
}
#endif
#endif
