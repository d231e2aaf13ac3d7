/* oai4g_shim_fp.h — LTE_DL_FRAME_PARMS (PHY/impl_defs_lte.h:470-572) -> the library's
 * oai4g_frame_parms_t, shared by oai4g_shim.c and oai4g_shim_ue.c. */
#ifndef OAI4G_SHIM_FP_H
#define OAI4G_SHIM_FP_H
static void fp_to(const LTE_DL_FRAME_PARMS *f, oai4g_frame_parms_t *o)
{
  memset(o, 0, sizeof(*o));
  o->N_RB_DL = f->N_RB_DL;            o->Nid_cell = f->Nid_cell;
  o->Ncp = f->Ncp;                    o->nushift = f->nushift;
  o->mode1_flag = f->mode1_flag;      o->nb_antennas_tx = f->nb_antennas_tx;
  o->frame_type = f->frame_type;      o->symbols_per_tti = f->symbols_per_tti;
  o->log2_symbol_size = f->log2_symbol_size;
  o->ofdm_symbol_size = f->ofdm_symbol_size;
  o->first_carrier_offset = f->first_carrier_offset;
  o->nb_prefix_samples = f->nb_prefix_samples;
  o->nb_prefix_samples0 = f->nb_prefix_samples0;
  o->samples_per_tti = f->samples_per_tti;
  o->phich_resource = f->phich_config_common.phich_resource;
  o->phich_duration = f->phich_config_common.phich_duration;
  o->tdd_config = f->tdd_config;      o->nb_antennas_tx_eNB = f->nb_antennas_tx_eNB;
  o->Nid_cell_mbsfn = (uint8_t)f->Nid_cell_mbsfn;   /* 0..255 (36.211 N_ID^MBSFN) */
}

#endif
