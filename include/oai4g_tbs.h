/* 36.213 Table 7.1.7.2.1-1 (transport block sizes), see oai4g_tbs.c. */
#ifndef OAI4G_TBS_H
#define OAI4G_TBS_H
#ifdef __cplusplus
extern "C" {
#endif

extern const unsigned int oai4g_tbs_by_prb[110][27];   /* [N_PRB - 1][I_TBS], bits */

#ifdef __cplusplus
}
#endif
#endif
