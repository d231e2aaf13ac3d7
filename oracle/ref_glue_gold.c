/* TEST INFRASTRUCTURE ONLY — linked into oracle/_ref/libref_gold.so next to the reference's own
 * PHY/LTE_REFSIG/lte_gold.c (compiled unmodified).  Not a stand-in for any reference file: it is the
 * caller a ctypes test needs, because lte_gold (lte_gold.c:52) takes the reference's
 * LTE_DL_FRAME_PARMS (PHY/impl_defs_lte.h:470-572) and reads its Ncp field only. */
#include <stdint.h>
#include <string.h>
#include "PHY/impl_defs_lte.h"

void lte_gold(LTE_DL_FRAME_PARMS *frame_parms, uint32_t lte_gold_table[20][2][14], uint16_t Nid_cell);

void ref_glue_lte_gold(int Ncp, uint16_t Nid_cell, uint32_t table[20][2][14])
{
  LTE_DL_FRAME_PARMS fp;
  memset(&fp, 0, sizeof(fp));
  fp.Ncp = (lte_prefix_type_t)Ncp;
  fp.Nid_cell = Nid_cell;
  lte_gold(&fp, table, Nid_cell);
}
