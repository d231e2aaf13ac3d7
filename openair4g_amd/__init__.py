"""openair4g_amd — MI355X-native LTE PDSCH transmit path (host side).

This module is the Python mirror of the C ABI in ``include/oai4g.h``: ctypes bindings for
the drop-in entry points (``dlsch_encoding``, ``dlsch_scrambling``, ``dlsch_modulation``,
``PHY_ofdm_mod`` and their callees, named as in openair1/PHY) and for the batched,
device-resident transmit path (``TxPipeline``).  All arithmetic runs in the gfx950 kernels
of ``lib/libopenair4g_amd.so``; if that library or a gfx950 device is missing every compute
entry point raises ``OAI4GError`` — there is no CPU fallback.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libopenair4g_amd.so")

LTE_NULL = 2
NSOFT = 1827072
MAX_SEGMENTS = 16
MAX_CHANNEL_BITS = 14 * 1200 * 6
D_BYTES = 96 + 12 + 3 + 3 * 6144
W_BYTES = 3 * 6144 + 96
SISO, ALAMOUTI, LARGE_CDD = 0, 1, 2
CYCLIC_PREFIX = 0


class OAI4GError(RuntimeError):
    pass


u8p = ctypes.POINTER(ctypes.c_uint8)


class FrameParms(ctypes.Structure):
    """oai4g_frame_parms_t — LTE_DL_FRAME_PARMS subset (PHY/impl_defs_lte.h:470-572)."""
    _fields_ = [("N_RB_DL", ctypes.c_uint16), ("Nid_cell", ctypes.c_uint16), ("Ncp", ctypes.c_uint8),
                ("nushift", ctypes.c_uint8), ("mode1_flag", ctypes.c_uint8), ("nb_antennas_tx", ctypes.c_uint8),
                ("frame_type", ctypes.c_uint8), ("symbols_per_tti", ctypes.c_uint8),
                ("log2_symbol_size", ctypes.c_uint8), ("Nid_cell_mbsfn", ctypes.c_uint8),
                ("ofdm_symbol_size", ctypes.c_uint16), ("first_carrier_offset", ctypes.c_uint16),
                ("nb_prefix_samples", ctypes.c_uint16), ("nb_prefix_samples0", ctypes.c_uint16),
                ("samples_per_tti", ctypes.c_uint32), ("phich_resource", ctypes.c_uint8),
                ("phich_duration", ctypes.c_uint8), ("tdd_config", ctypes.c_uint8),
                ("nb_antennas_tx_eNB", ctypes.c_uint8)]


class DciAlloc(ctypes.Structure):
    """oai4g_dci_alloc_t — DCI_ALLOC_t (PHY/LTE_TRANSPORT/defs.h:734-749)."""
    _fields_ = [("dci_length", ctypes.c_uint8), ("L", ctypes.c_uint8), ("nCCE", ctypes.c_int32),
                ("ra_flag", ctypes.c_uint8), ("rnti", ctypes.c_uint16), ("format", ctypes.c_uint32),
                ("dci_pdu", ctypes.c_uint8 * 8)]


class DlHarq(ctypes.Structure):
    """oai4g_dl_harq_t — LTE_DL_eNB_HARQ_t subset (PHY/LTE_TRANSPORT/defs.h:104-169)."""
    _fields_ = [("TBS", ctypes.c_uint32), ("B", ctypes.c_uint32), ("b", u8p), ("c", u8p * MAX_SEGMENTS),
                ("RTC", ctypes.c_uint32 * MAX_SEGMENTS), ("round", ctypes.c_uint8), ("mcs", ctypes.c_uint8),
                ("rvidx", ctypes.c_uint8), ("mimo_mode", ctypes.c_uint8), ("rb_alloc", ctypes.c_uint32 * 4),
                ("nb_rb", ctypes.c_uint16), ("e", u8p), ("d", u8p * MAX_SEGMENTS), ("w", u8p * MAX_SEGMENTS),
                ("C", ctypes.c_uint32), ("Cminus", ctypes.c_uint32), ("Cplus", ctypes.c_uint32),
                ("Kminus", ctypes.c_uint32), ("Kplus", ctypes.c_uint32), ("F", ctypes.c_uint32),
                ("Nl", ctypes.c_uint8), ("Nlayers", ctypes.c_uint8), ("first_layer", ctypes.c_uint8)]


class Dlsch(ctypes.Structure):
    """oai4g_dlsch_t — LTE_eNB_DLSCH_t subset (PHY/LTE_TRANSPORT/defs.h:240-274)."""
    _fields_ = [("rnti", ctypes.c_uint16), ("current_harq_pid", ctypes.c_uint8), ("Mdlharq", ctypes.c_uint8),
                ("Kmimo", ctypes.c_uint8), ("sqrt_rho_a", ctypes.c_int16), ("sqrt_rho_b", ctypes.c_int16),
                ("harq_processes", ctypes.POINTER(DlHarq) * 8)]


class TxParams(ctypes.Structure):
    """oai4g_tx_params_t — the POD parameter block rank 0 broadcasts to the other ranks."""
    _fields_ = [("N_RB_DL", ctypes.c_uint16), ("Nid_cell", ctypes.c_uint16), ("Ncp", ctypes.c_uint8),
                ("nb_antennas_tx", ctypes.c_uint8), ("mode1_flag", ctypes.c_uint8), ("frame_type", ctypes.c_uint8),
                ("n_cw", ctypes.c_uint8), ("mimo_mode", ctypes.c_uint8), ("num_pdcch_symbols", ctypes.c_uint8),
                ("Kmimo", ctypes.c_uint8), ("Mdlharq", ctypes.c_uint8), ("first_subframe", ctypes.c_uint8),
                ("subframe_step", ctypes.c_uint8), ("with_crs", ctypes.c_uint8), ("rnti", ctypes.c_uint16),
                ("amp", ctypes.c_int16), ("sqrt_rho_a", ctypes.c_int16), ("sqrt_rho_b", ctypes.c_int16),
                ("rb_alloc", ctypes.c_uint32 * 4), ("nb_rb", ctypes.c_uint16), ("mcs", ctypes.c_uint8 * 2),
                ("rvidx", ctypes.c_uint8 * 2), ("q", ctypes.c_uint8 * 2), ("TBS", ctypes.c_uint32 * 2),
                ("payload_stride", ctypes.c_uint32), ("rm_limited_buffer", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32 * 7)]

    def to_bytes(self):
        return bytes(ctypes.string_at(ctypes.addressof(self), ctypes.sizeof(self)))

    @classmethod
    def from_bytes(cls, b):
        p = cls()
        ctypes.memmove(ctypes.addressof(p), bytes(b), ctypes.sizeof(cls))
        return p


_lib = None

_SIGS = {
    "oai4g_init": (ctypes.c_int, []),
    "oai4g_last_error": (ctypes.c_char_p, []),
    "oai4g_device_name": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int]),
    "oai4g_init_frame_parms": (ctypes.c_int, [ctypes.POINTER(FrameParms), ctypes.c_uint16, ctypes.c_uint16,
                                              ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8]),
    "oai4g_get_Qm": (ctypes.c_uint8, [ctypes.c_uint8]),
    "oai4g_get_Qm_ul": (ctypes.c_uint8, [ctypes.c_uint8]),
    "oai4g_get_I_TBS": (ctypes.c_uint8, [ctypes.c_uint8]),
    "oai4g_get_I_TBS_UL": (ctypes.c_uint8, [ctypes.c_uint8]),
    "oai4g_tbs_bits": (ctypes.c_uint32, [ctypes.c_uint8, ctypes.c_uint16]),
    "oai4g_get_TBS_DL": (ctypes.c_uint32, [ctypes.c_uint8, ctypes.c_uint16]),
    "oai4g_get_TBS_UL": (ctypes.c_uint32, [ctypes.c_uint8, ctypes.c_uint16]),
    "oai4g_get_G": (ctypes.c_int, [ctypes.POINTER(FrameParms), ctypes.c_uint16, ctypes.POINTER(ctypes.c_uint32),
                                   ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_int, ctypes.c_uint8]),
    "oai4g_new_dlsch": (ctypes.POINTER(Dlsch), [ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8]),
    "oai4g_free_dlsch": (None, [ctypes.POINTER(Dlsch)]),
    "oai4g_lte_gold_generic": (ctypes.c_uint32, [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                                 ctypes.c_uint8]),
    "oai4g_crc24a": (ctypes.c_uint32, [ctypes.c_void_p, ctypes.c_int]),
    "oai4g_crc24b": (ctypes.c_uint32, [ctypes.c_void_p, ctypes.c_int]),
    "oai4g_lte_segmentation": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(u8p), ctypes.c_uint32]
                               + [ctypes.POINTER(ctypes.c_uint32)] * 6),
    "oai4g_threegpplte_turbo_encoder": (None, [ctypes.c_void_p, ctypes.c_uint16, ctypes.c_void_p, ctypes.c_uint8,
                                               ctypes.c_uint16, ctypes.c_uint16]),
    "oai4g_sub_block_interleaving_turbo": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    "oai4g_lte_rate_matching_turbo": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                                        ctypes.c_void_p] + [ctypes.c_uint8] + [ctypes.c_uint32]
                                      + [ctypes.c_uint8] * 8),
    "oai4g_dlsch_encoding": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(FrameParms), ctypes.c_uint8,
                                            ctypes.POINTER(Dlsch), ctypes.c_int, ctypes.c_uint8]),
    "oai4g_dlsch_scrambling": (None, [ctypes.POINTER(FrameParms), ctypes.c_int, ctypes.POINTER(Dlsch), ctypes.c_int,
                                      ctypes.c_uint8, ctypes.c_uint8]),
    "oai4g_dlsch_modulation": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int16, ctypes.c_uint32,
                                              ctypes.POINTER(FrameParms), ctypes.c_uint8, ctypes.POINTER(Dlsch),
                                              ctypes.POINTER(Dlsch)]),
    "oai4g_PHY_ofdm_mod": (None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint16,
                                  ctypes.c_int]),
    "oai4g_normal_prefix_mod": (None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint8, ctypes.POINTER(FrameParms)]),
    "oai4g_do_OFDM_mod": (None, [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                 ctypes.c_uint16, ctypes.POINTER(FrameParms)]),
    "oai4g_generate_pilots": (None, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int16, ctypes.POINTER(FrameParms),
                                     ctypes.c_uint16]),
    "oai4g_lte_dl_cell_spec": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int16, ctypes.POINTER(FrameParms),
                                              ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8]),
    "oai4g_phy_threegpplte_turbo_decoder16": (ctypes.c_uint8, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint16,
                                                               ctypes.c_uint16, ctypes.c_uint16, ctypes.c_uint8,
                                                               ctypes.c_uint8, ctypes.c_uint8]),
    "oai4g_lte_rate_matching_turbo_rx": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint8,
                                                        ctypes.c_uint32] + [ctypes.c_uint8] * 7 +
                                         [ctypes.POINTER(ctypes.c_uint32)]),
    "oai4g_sub_block_deinterleaving_turbo": (None, [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    "oai4g_td_scratch_bytes": (ctypes.c_size_t, [ctypes.c_uint16, ctypes.c_int]),
    "oai4g_td_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint16, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                      ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint8,
                                      ctypes.c_uint8, ctypes.c_void_p, ctypes.c_void_p]),
    "oai4g_idft": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "oai4g_idft2048": (None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "oai4g_idft1024": (None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "oai4g_idft512": (None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "oai4g_idft256": (None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "oai4g_idft128": (None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "oai4g_idft64": (None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "oai4g_generate_pcfich_reg_mapping": (None, [ctypes.POINTER(FrameParms), ctypes.POINTER(ctypes.c_uint16),
                                                  ctypes.POINTER(ctypes.c_uint8)]),
    "oai4g_get_mi": (ctypes.c_uint8, [ctypes.POINTER(FrameParms), ctypes.c_uint8]),
    "oai4g_get_nquad": (ctypes.c_uint16, [ctypes.c_uint8, ctypes.POINTER(FrameParms), ctypes.c_uint8]),
    "oai4g_get_nCCE": (ctypes.c_uint16, [ctypes.c_uint8, ctypes.POINTER(FrameParms), ctypes.c_uint8]),
    "oai4g_get_num_pdcch_symbols": (ctypes.c_uint8, [ctypes.c_uint8, ctypes.POINTER(DciAlloc),
                                                     ctypes.POINTER(FrameParms), ctypes.c_uint8]),
    "oai4g_generate_phich_reg_mapping": (ctypes.c_int, [ctypes.POINTER(FrameParms), ctypes.POINTER(ctypes.c_uint16)]),
    "oai4g_init_nCCE_table": (None, []),
    "oai4g_get_nCCE_offset": (ctypes.c_int, [ctypes.c_uint8, ctypes.c_int, ctypes.c_int, ctypes.c_uint16,
                                             ctypes.c_uint8]),
    "oai4g_generate_dci_top": (ctypes.c_uint8, [ctypes.c_uint8, ctypes.c_uint8, ctypes.POINTER(DciAlloc),
                                                ctypes.c_uint32, ctypes.c_int16, ctypes.POINTER(FrameParms),
                                                ctypes.c_void_p, ctypes.c_uint32]),
    "oai4g_tx_config_set_control": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint8,
                                                    ctypes.POINTER(DciAlloc)]),
    "oai4g_generate_pcfich": (ctypes.c_int, [ctypes.c_uint8, ctypes.c_int16, ctypes.POINTER(FrameParms),
                                             ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint8]),
    "oai4g_generate_pss": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int16, ctypes.POINTER(FrameParms),
                                          ctypes.c_uint16, ctypes.c_uint16]),
    "oai4g_generate_sss": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int16, ctypes.POINTER(FrameParms),
                                          ctypes.c_uint16, ctypes.c_uint16]),
    "oai4g_generate_pbch": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                                           ctypes.POINTER(FrameParms), ctypes.c_void_p, ctypes.c_uint8]),
    "oai4g_generate_phich": (ctypes.c_int, [ctypes.POINTER(FrameParms), ctypes.c_int16, ctypes.c_uint8, ctypes.c_uint8,
                                            ctypes.c_uint8, ctypes.c_uint8, ctypes.POINTER(ctypes.c_void_p)]),
    "oai4g_phich_group_seq": (ctypes.c_int, [ctypes.POINTER(FrameParms), ctypes.c_uint16, ctypes.c_uint8,
                                             ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_uint8)]),
    "oai4g_tx_config_set_common": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "oai4g_rx_pdsch_siso": (ctypes.c_int, [ctypes.POINTER(FrameParms), ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint8, ctypes.c_uint8,
                                           ctypes.c_uint8, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8)]),
    "oai4g_dlsch_unscrambling": (None, [ctypes.POINTER(FrameParms), ctypes.c_int, ctypes.c_uint16, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint8]),
    "oai4g_rx_config_create": (ctypes.c_void_p, [ctypes.POINTER(FrameParms), ctypes.POINTER(ctypes.c_uint32),
                                                 ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint16, ctypes.c_uint8,
                                                 ctypes.c_uint8]),
    "oai4g_rx_config_destroy": (None, [ctypes.c_void_p]),
    "oai4g_rx_llr_count": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "oai4g_rx_llr_stride": (ctypes.c_size_t, [ctypes.c_void_p]),
    "oai4g_rx_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_int, ctypes.c_void_p]),
    "oai4g_lte_dl_channel_estimation": (ctypes.c_int, [ctypes.POINTER(FrameParms), ctypes.c_void_p, ctypes.c_void_p,
                                                       ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8]),
    "oai4g_chest_filters": (None, [ctypes.c_uint8, ctypes.c_void_p]),
    "oai4g_chest_dc_filters": (None, [ctypes.c_uint8, ctypes.c_void_p]),
    "oai4g_ul_config_set_decoder": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "oai4g_set_device": (ctypes.c_int, [ctypes.c_int]),
    "oai4g_dist_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
    "oai4g_dist_init": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    "oai4g_dist_broadcast_params": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "oai4g_dist_allreduce_sum_u64": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "oai4g_dist_allreduce_max_f64": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "oai4g_dist_barrier": (ctypes.c_int, []),
    "oai4g_dist_rank": (ctypes.c_int, []),
    "oai4g_dist_world": (ctypes.c_int, []),
    "oai4g_dist_finalize": (ctypes.c_int, []),
    "oai4g_shard_range": (None, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                 ctypes.POINTER(ctypes.c_int)]),
    "oai4g_payload_seed": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32]),
    "oai4g_chest_config_set_stride": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]),
    "oai4g_rx_pdsch_tm3": (ctypes.c_int, [ctypes.POINTER(FrameParms), ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8,
                                          ctypes.c_uint8, ctypes.c_uint8, ctypes.c_void_p, ctypes.c_void_p]),
    "oai4g_rx_config_create_tm3": (ctypes.c_void_p, [ctypes.POINTER(FrameParms), ctypes.c_void_p, ctypes.c_uint8,
                                                     ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint16,
                                                     ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8]),
    "oai4g_rx_batch_tm3": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "oai4g_rx_pdsch_tm3_2cw": (ctypes.c_int, [ctypes.POINTER(FrameParms), ctypes.c_int, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint8,
                                              ctypes.c_uint8, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "oai4g_rx_batch_tm3_2cw": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "oai4g_rx_pdsch_tm2": (ctypes.c_int, [ctypes.POINTER(FrameParms), ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8,
                                          ctypes.c_void_p, ctypes.c_void_p]),
    "oai4g_rx_config_create_tm2": (ctypes.c_void_p, [ctypes.POINTER(FrameParms), ctypes.c_void_p, ctypes.c_uint8,
                                                     ctypes.c_uint8, ctypes.c_uint16, ctypes.c_uint8, ctypes.c_uint8,
                                                     ctypes.c_uint8]),
    "oai4g_rx_batch_tm2": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "oai4g_dl_ch_estimates_time": (ctypes.c_int, [ctypes.POINTER(FrameParms), ctypes.c_int, ctypes.c_void_p,
                                                  ctypes.c_void_p]),
    "oai4g_chest_time_batch": (ctypes.c_int, [ctypes.POINTER(FrameParms), ctypes.c_int, ctypes.c_void_p,
                                              ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "oai4g_lte_est_freq_offset": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(FrameParms), ctypes.c_int,
                                                 ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    "oai4g_freq_offset_omega_batch": (ctypes.c_int, [ctypes.POINTER(FrameParms), ctypes.c_int, ctypes.c_void_p,
                                                     ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "oai4g_freq_offset_update": (ctypes.c_int, [ctypes.POINTER(FrameParms), ctypes.c_int32,
                                                ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "oai4g_signal_energy": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_uint32]),
    "oai4g_signal_energy_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_uint32,
                                                 ctypes.c_void_p, ctypes.c_void_p]),
    "oai4g_awgn_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_void_p,
                                        ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_double, ctypes.c_uint64, ctypes.c_uint32,
                                        ctypes.c_void_p]),
    "oai4g_chest_config_create": (ctypes.c_void_p, [ctypes.POINTER(FrameParms), ctypes.c_uint8, ctypes.c_uint8,
                                                    ctypes.c_uint8]),
    "oai4g_chest_config_destroy": (None, [ctypes.c_void_p]),
    "oai4g_rx_batch_estimated": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "oai4g_chest_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p]),
    "oai4g_chest_batch_pilots": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_void_p]),
    "oai4g_rx_batch_tm3_pilots": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "oai4g_rx_batch_tm3_2cw_pilots": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "oai4g_phy_threegpplte_turbo_decoder8": (ctypes.c_uint8, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint16,
                                                              ctypes.c_uint16, ctypes.c_uint16, ctypes.c_uint8,
                                                              ctypes.c_uint8, ctypes.c_uint8]),
    "oai4g_td8_scratch_bytes": (ctypes.c_size_t, [ctypes.c_uint16, ctypes.c_int]),
    "oai4g_td8_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint16, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                       ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8,
                                       ctypes.c_void_p, ctypes.c_void_p]),
    "oai4g_generate_dummy_w": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint8]),
    "oai4g_ul_config_create": (ctypes.c_void_p, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint8, ctypes.c_uint8,
                                                 ctypes.c_uint8, ctypes.c_uint32, ctypes.c_uint8]),
    "oai4g_ul_config_destroy": (None, [ctypes.c_void_p]),
    "oai4g_ul_config_C": (ctypes.c_int, [ctypes.c_void_p]),
    "oai4g_ul_config_E": (ctypes.c_uint32, [ctypes.c_void_p, ctypes.c_int]),
    "oai4g_ul_config_G_offset": (ctypes.c_uint32, [ctypes.c_void_p, ctypes.c_int]),
    "oai4g_ul_decode_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                             ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]),
    "oai4g_ul_config_w_entries": (ctypes.c_size_t, [ctypes.c_void_p]),
    "oai4g_ul_decode_batch_harq": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                                  ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint8, ctypes.c_uint8,
                                                  ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]),
    "oai4g_dft": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "oai4g_dft2048": (None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "oai4g_dft1024": (None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "oai4g_dft512": (None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "oai4g_dft256": (None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "oai4g_dft128": (None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "oai4g_dft64": (None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "oai4g_slot_fep_offset": (ctypes.c_int64, [ctypes.POINTER(FrameParms), ctypes.c_uint8, ctypes.c_uint8,
                                               ctypes.c_int, ctypes.c_int]),
    "oai4g_slot_fep": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                      ctypes.POINTER(FrameParms), ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8,
                                      ctypes.c_int, ctypes.c_int]),
    "oai4g_fep_batch": (ctypes.c_int, [ctypes.POINTER(FrameParms), ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p]),
    "oai4g_tx_config_create": (ctypes.c_void_p, [ctypes.POINTER(TxParams)]),
    "oai4g_tx_config_destroy": (None, [ctypes.c_void_p]),
    "oai4g_tx_G": (ctypes.c_uint32, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "oai4g_tx_ebits_words": (ctypes.c_uint32, [ctypes.c_void_p]),
    "oai4g_tx_iq_samples": (ctypes.c_uint32, [ctypes.c_void_p]),
    "oai4g_tx_workspace_bytes": (ctypes.c_size_t, [ctypes.c_void_p, ctypes.c_int]),
    "oai4g_tx_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p]),
    "oai4g_tx_batch_timed": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]),
    "oai4g_tx_encode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p]),
    "oai4g_tx_modulate": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p]),
    "oai4g_tx_mod_nosat": (ctypes.c_int, [ctypes.c_void_p]),
    "oai4g_diag_encode_phase_ms": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]),
    "oai4g_diag_encode_occupancy": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                                   ctypes.POINTER(ctypes.c_size_t)]),
    "oai4g_diag_stream": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                         ctypes.c_void_p]),
    "oai4g_dev_alloc": (ctypes.c_void_p, [ctypes.c_size_t]),
    "oai4g_dev_free": (None, [ctypes.c_void_p]),
    "oai4g_memcpy_h2d": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    "oai4g_memcpy_d2h": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    "oai4g_memset_d": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]),
    "oai4g_sync": (ctypes.c_int, []),
    "oai4g_fill_payload": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_void_p]),
}


def load_library(path=None):
    """Load the HIP library (raises OAI4GError if it is not built).  OAI4G_LIB selects an
    alternative in-tree build (kernel variants for A/B measurements)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("OAI4G_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise OAI4GError(f"HIP library not built: {path} (run __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def exported_symbols():
    return sorted(_SIGS)


def lib():
    return load_library()


def init():
    """Initialise the device (raises if no gfx950 GPU: no CPU fallback)."""
    L = lib()
    if L.oai4g_init() != 0:
        raise OAI4GError(L.oai4g_last_error().decode())
    return L


def _check(ok):
    if not ok:
        raise OAI4GError(lib().oai4g_last_error().decode())


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def device_name():
    L = init()
    buf = ctypes.create_string_buffer(256)
    _check(L.oai4g_device_name(buf, 256) == 0)
    return buf.value.decode()


# ------------------------------------------------------------------------------------------
# drop-in entry points (host numpy buffers in/out, GPU compute)
# ------------------------------------------------------------------------------------------
def frame_parms(N_RB_DL, Nid_cell=0, Ncp=0, nb_antennas_tx=1, mode1_flag=1, frame_type=0):
    fp = FrameParms()
    _check(lib().oai4g_init_frame_parms(ctypes.byref(fp), N_RB_DL, Nid_cell, Ncp, nb_antennas_tx, mode1_flag,
                                        frame_type) == 0)
    return fp


def get_G(fp, nb_rb, rb_alloc, Qm, Nl, num_pdcch, subframe):
    ra = (ctypes.c_uint32 * 4)(*rb_alloc)
    return lib().oai4g_get_G(ctypes.byref(fp), nb_rb, ra, Qm, Nl, num_pdcch, 0, subframe)


def crc24a(data, bitlen):
    init()
    a = np.ascontiguousarray(data, dtype=np.uint8)
    return int(lib().oai4g_crc24a(_ptr(a), bitlen))


def crc24b(data, bitlen):
    init()
    a = np.ascontiguousarray(data, dtype=np.uint8)
    return int(lib().oai4g_crc24b(_ptr(a), bitlen))


def turbo_encode(c, f1, f2):
    """threegpplte_turbo_encoder: c (K/8 bytes) -> d (3K+12 bytes)."""
    init()
    c = np.ascontiguousarray(c, dtype=np.uint8)
    K = 8 * len(c)
    d = np.zeros(3 * K + 12, dtype=np.uint8)
    lib().oai4g_threegpplte_turbo_encoder(_ptr(c), len(c), _ptr(d), 0, f1, f2)
    _check(True)
    return d


def subblock_interleave(d_full, D):
    """sub_block_interleaving_turbo: d_full = 96-byte NULL prefix + d.  Returns (R, w)."""
    init()
    d_full = np.ascontiguousarray(d_full, dtype=np.uint8)
    R = (D + 31) >> 5
    w = np.zeros(3 * 32 * R, dtype=np.uint8)
    dptr = ctypes.c_void_p(d_full.ctypes.data + 96)
    rtc = lib().oai4g_sub_block_interleaving_turbo(D, dptr, _ptr(w))
    if rtc == 0:
        _check(False)
    return rtc, w


def rate_match(RTC, G, w, C, r, Qm, rvidx=0, Nl=1, Kmimo=1, Mdlharq=8, Nsoft=NSOFT):
    init()
    w = np.ascontiguousarray(w, dtype=np.uint8)
    e = np.zeros(G + 64, dtype=np.uint8)
    E = lib().oai4g_lte_rate_matching_turbo(RTC, G, _ptr(w), _ptr(e), C, Nsoft, Mdlharq, Kmimo, rvidx, Qm, Nl, r,
                                            0, 0)
    return e[:E]


def idft(x, scale=1):
    """x: complex int16 pairs as int16 array of length 2N."""
    init()
    x = np.ascontiguousarray(x, dtype=np.int16)
    n = len(x) // 2
    y = np.zeros_like(x)
    _check(lib().oai4g_idft(int(n).bit_length() - 1, _ptr(x), _ptr(y), scale) == 0)
    return y


def generate_pcfich(cfi, amp, fp, grids, subframe):
    """generate_pcfich drop-in on a list of frame grids (int32 arrays, modified in place)."""
    init()
    n = len(grids)
    gp = (ctypes.c_void_p * n)(*[g.ctypes.data for g in grids])
    return lib().oai4g_generate_pcfich(cfi, amp, ctypes.byref(fp), gp, subframe)


def _grid_ptrs(grids):
    return (ctypes.c_void_p * len(grids))(*[g.ctypes.data for g in grids])


def generate_pss(grids, amp, fp, symbol, slot_offset):
    """generate_pss drop-in (pss.c:50) on frame grids (int32 arrays, modified in place)."""
    init()
    return lib().oai4g_generate_pss(_grid_ptrs(grids), amp, ctypes.byref(fp), symbol, slot_offset)


def generate_sss(grids, amp, fp, symbol, slot_offset):
    """generate_sss drop-in (sss.c:47)."""
    init()
    return lib().oai4g_generate_sss(_grid_ptrs(grids), amp, ctypes.byref(fp), symbol, slot_offset)


class PhichItem(ctypes.Structure):
    _fields_ = [("subframe", ctypes.c_uint8), ("ngroup", ctypes.c_uint8), ("nseq", ctypes.c_uint8), ("hi", ctypes.c_uint8)]


class CommonSig(ctypes.Structure):
    """oai4g_common_sig_t"""
    _fields_ = [("pss_sss", ctypes.c_uint8), ("pbch", ctypes.c_uint8), ("pbch_pdu", ctypes.c_uint8 * 3),
                ("frame_mod4", ctypes.c_uint8), ("n_phich", ctypes.c_uint8), ("phich", PhichItem * 64)]


class Pbch(ctypes.Structure):
    """oai4g_pbch_t (LTE_eNB_PBCH): the scrambled coded bits kept across frame_mod4."""
    _fields_ = [("pbch_e", ctypes.c_uint8 * 1920)]


def generate_pbch(state, grids, amp, fp, pdu, frame_mod4):
    """generate_pbch drop-in (pbch.c:161) on the subframe-0 grids."""
    init()
    pdu = np.ascontiguousarray(pdu, dtype=np.uint8)
    return lib().oai4g_generate_pbch(ctypes.byref(state), _grid_ptrs(grids), amp, ctypes.byref(fp), _ptr(pdu), frame_mod4)


def generate_phich(fp, amp, nseq, ngroup, hi, subframe, grids):
    """generate_phich drop-in (phich.c:401) on frame grids."""
    init()
    return lib().oai4g_generate_phich(ctypes.byref(fp), amp, nseq, ngroup, hi, subframe, _grid_ptrs(grids))


def phich_group_seq(fp, first_rb, n_dmrs):
    g, q = ctypes.c_uint8(), ctypes.c_uint8()
    _check(lib().oai4g_phich_group_seq(ctypes.byref(fp), first_rb, n_dmrs, ctypes.byref(g), ctypes.byref(q)) == 0)
    return g.value, q.value


def dft(x, scale=1):
    """Forward DFT (lte_dfts.c dft64..dft2048): complex int16 pairs, int16 array of length 2N."""
    init()
    x = np.ascontiguousarray(x, dtype=np.int16)
    n = len(x) // 2
    y = np.zeros_like(x)
    _check(lib().oai4g_dft(int(n).bit_length() - 1, _ptr(x), _ptr(y), scale) == 0)
    return y


def slot_fep(rxdata, rxdataF, fp, l, Ns, sample_offset=0, no_prefix=0):
    """slot_fep drop-in: rxdata / rxdataF are lists (one per RX antenna) of int32 arrays, modified
    in place (rxdata: 10 subframes + N words of wrap extension).  Returns the entry point's code."""
    init()
    n = len(rxdata)
    rp = (ctypes.c_void_p * n)(*[a.ctypes.data for a in rxdata])
    fpp = (ctypes.c_void_p * n)(*[a.ctypes.data for a in rxdataF])
    return lib().oai4g_slot_fep(rp, fpp, ctypes.byref(fp), n, l, Ns, sample_offset, no_prefix)


def rx_pdsch_siso(fp, rxdataF, dl_ch, rb_alloc, Qm, num_pdcch, subframe):
    """rx_pdsch over one subframe's PDSCH symbols (TM1, one RX antenna): rxdataF / dl_ch are
    int32 [nsymb*N].  Returns (LLR stream int16, log2_maxh)."""
    init()
    rxdataF = np.ascontiguousarray(rxdataF, dtype=np.int32)
    dl_ch = np.ascontiguousarray(dl_ch, dtype=np.int32)
    out = np.zeros(14 * 1200 * 6 + 64, dtype=np.int16)
    sh = ctypes.c_uint8()
    ra = (ctypes.c_uint32 * 4)(*rb_alloc)
    n = lib().oai4g_rx_pdsch_siso(ctypes.byref(fp), _ptr(rxdataF), _ptr(dl_ch), ra, Qm, num_pdcch, subframe,
                                  _ptr(out), ctypes.byref(sh))
    _check(n >= 0)
    return out[:n], sh.value


def rx_pdsch_tm3(fp, rxF, est, rb_alloc, Qm0, Qm1, mcs0, num_pdcch, subframe):
    """rx_pdsch for TM3 (dual_stream_flag = 0): rxF = [nb_rx][nsymb*N], est[(p, a)] = [nsymb*N].
    Returns (codeword-0 LLRs, log2_maxh)."""
    init()
    nb_rx = len(rxF)
    rx = [np.ascontiguousarray(r, dtype=np.int32) for r in rxF]
    keep = {k: np.ascontiguousarray(v, dtype=np.int32) for k, v in est.items()}
    ep = (ctypes.c_void_p * 4)()
    for (p_, a), arr in keep.items():
        if a < nb_rx:
            ep[2 * p_ + a] = arr.ctypes.data
    rp = (ctypes.c_void_p * 2)(*[r.ctypes.data for r in rx] + [None] * (2 - nb_rx))
    out = np.zeros(14 * 1200 * 6 + 64, dtype=np.int16)
    sh = ctypes.c_uint8()
    ra = (ctypes.c_uint32 * 4)(*rb_alloc)
    n = lib().oai4g_rx_pdsch_tm3(ctypes.byref(fp), nb_rx, rp, ep, ra, Qm0, Qm1, mcs0, num_pdcch, subframe, _ptr(out),
                                 ctypes.byref(sh))
    _check(n >= 0)
    return out[:n], sh.value


def rx_pdsch_tm3_2cw(fp, rxF, est, rb_alloc, mcs0, num_pdcch, subframe):
    """rx_pdsch for TM3 with both codewords QPSK: rxF = [nb_rx][nsymb*N], est[(p, a)] = [nsymb*N].
    Returns (codeword-0 LLRs, codeword-1 LLRs, log2_maxh)."""
    init()
    nb_rx = len(rxF)
    rx = [np.ascontiguousarray(r, dtype=np.int32) for r in rxF]
    keep = {k: np.ascontiguousarray(v, dtype=np.int32) for k, v in est.items()}
    ep = (ctypes.c_void_p * 4)()
    for (p_, a), arr in keep.items():
        if a < nb_rx:
            ep[2 * p_ + a] = arr.ctypes.data
    rp = (ctypes.c_void_p * 2)(*[r.ctypes.data for r in rx] + [None] * (2 - nb_rx))
    o0 = np.zeros(14 * 1200 * 2 + 64, dtype=np.int16)
    o1 = np.zeros_like(o0)
    sh = ctypes.c_uint8()
    ra = (ctypes.c_uint32 * 4)(*rb_alloc)
    n = lib().oai4g_rx_pdsch_tm3_2cw(ctypes.byref(fp), nb_rx, rp, ep, ra, mcs0, num_pdcch, subframe, _ptr(o0),
                                     _ptr(o1), ctypes.byref(sh))
    _check(n >= 0)
    return o0[:n], o1[:n], sh.value


def rx_pdsch_tm2(fp, rxF, est, rb_alloc, Qm, num_pdcch, subframe):
    """rx_pdsch for TM2 (ALAMOUTI): rxF = [nb_rx][nsymb*N], est[(p, a)] = [nsymb*N].
    Returns (LLRs, log2_maxh)."""
    init()
    nb_rx = len(rxF)
    rx = [np.ascontiguousarray(r, dtype=np.int32) for r in rxF]
    keep = {k: np.ascontiguousarray(v, dtype=np.int32) for k, v in est.items()}
    ep = (ctypes.c_void_p * 4)()
    for (p_, a), arr in keep.items():
        if a < nb_rx:
            ep[2 * p_ + a] = arr.ctypes.data
    rp = (ctypes.c_void_p * 2)(*[r.ctypes.data for r in rx] + [None] * (2 - nb_rx))
    out = np.zeros(14 * 1200 * 6 + 64, dtype=np.int16)
    sh = ctypes.c_uint8()
    ra = (ctypes.c_uint32 * 4)(*rb_alloc)
    n = lib().oai4g_rx_pdsch_tm2(ctypes.byref(fp), nb_rx, rp, ep, ra, Qm, num_pdcch, subframe, _ptr(out),
                                 ctypes.byref(sh))
    _check(n >= 0)
    return out[:n], sh.value


class RxBatchTM3:
    """Device-resident batched TM3 demodulation (oai4g_rx_batch_tm3): codeword 0's LLRs from the FEP
    output of nb_rx antennas and the four estimate planes (ports 0 / 1 per antenna)."""

    def __init__(self, fp, rb_alloc, Qm0, Qm1, mcs0, num_pdcch, rnti, n_sf, nb_rx=2, first_subframe=0,
                 subframe_step=1):
        init()
        self.L = lib()
        ra = (ctypes.c_uint32 * 4)(*rb_alloc)
        self.cfg = self.L.oai4g_rx_config_create_tm3(ctypes.byref(fp), ra, Qm0, Qm1, mcs0, num_pdcch, rnti,
                                                     first_subframe, subframe_step, nb_rx)
        _check(bool(self.cfg))
        self._setup(fp, n_sf, nb_rx)

    def _setup(self, fp, n_sf, nb_rx):
        self.fp, self.n_sf, self.nb_rx = fp, n_sf, nb_rx
        self.stride = self.L.oai4g_rx_llr_stride(self.cfg)
        self.plane = n_sf * fp.symbols_per_tti * fp.ofdm_symbol_size
        self.d_est = self.L.oai4g_dev_alloc(4 * self.plane * 4)
        self.d_llr = self.L.oai4g_dev_alloc(n_sf * self.stride * 2)
        _check(bool(self.d_est) and bool(self.d_llr))
        self._chest = {}

    def llr_count(self, sfi):
        return self.L.oai4g_rx_llr_count(self.cfg, sfi)

    def est_plane(self, p, a):
        """device pointer of the estimate plane of port p at receive antenna a"""
        return ctypes.c_void_p(self.d_est + (2 * p + a) * self.plane * 4)

    def _chest_cfgs(self, first_subframe, subframe_step):
        """the ports' 0 / 1 estimation configurations (element stride nb_rx subframes), cached"""
        key = (first_subframe, subframe_step)
        if key not in self._chest:
            cfgs = []
            for p in (0, 1):
                cfg = self.L.oai4g_chest_config_create(ctypes.byref(self.fp), p, first_subframe, subframe_step)
                _check(bool(cfg))
                cfgs.append(cfg)
                _check(self.L.oai4g_chest_config_set_stride(cfg, self.nb_rx, self.nb_rx) == 0)
            self._chest[key] = cfgs
        return self._chest[key]

    def estimate(self, d_rxF, first_subframe=0, subframe_step=1, stream=None):
        """The four channel-estimation batches over the FEP output [n_sf + 1][nb_rx][nsymb][N]
        (the extra element's symbol 0 closes the last subframe's rows 12 / 13)."""
        N, nsymb = self.fp.ofdm_symbol_size, self.fp.symbols_per_tti
        for p, cfg in enumerate(self._chest_cfgs(first_subframe, subframe_step)):
            for a in range(self.nb_rx):
                _check(self.L.oai4g_chest_batch(cfg, self.n_sf, ctypes.c_void_p(d_rxF + a * nsymb * N * 4),
                                                self.est_plane(p, a), stream) == 0)

    def launch(self, d_rxF, unscramble=1, stream=None):
        _check(self.L.oai4g_rx_batch_tm3(self.cfg, self.n_sf, d_rxF, self.d_est, self.d_llr, unscramble, stream) == 0)

    def _pil(self):
        if not getattr(self, "d_pil", None):
            self.pil_plane = self.n_sf * 4 * self.fp.ofdm_symbol_size * 2
            self.d_pil = self.L.oai4g_dev_alloc(4 * self.pil_plane * 4)
            _check(bool(self.d_pil))
        return self.d_pil

    def estimate_pilots(self, d_rxF, first_subframe=0, subframe_step=1, stream=None):
        """The four pilot-row estimations (oai4g_chest_batch_pilots): 5 rows per subframe instead of 14."""
        N, nsymb = self.fp.ofdm_symbol_size, self.fp.symbols_per_tti
        d_pil = self._pil()
        for p, cfg in enumerate(self._chest_cfgs(first_subframe, subframe_step)):
            for a in range(self.nb_rx):
                _check(self.L.oai4g_chest_batch_pilots(cfg, self.n_sf, ctypes.c_void_p(d_rxF + a * nsymb * N * 4),
                                                       ctypes.c_void_p(d_pil + (2 * p + a) * self.pil_plane * 4),
                                                       stream) == 0)

    def launch_pilots(self, d_rxF, unscramble=1, stream=None):
        """oai4g_rx_batch_tm3_pilots: the demodulation from the pilot rows (estimate_pilots)"""
        _check(self.L.oai4g_rx_batch_tm3_pilots(self.cfg, self.n_sf, d_rxF, self._pil(), self.d_llr, unscramble,
                                                stream) == 0)

    def launch_2cw_pilots(self, d_rxF, unscramble=1, stream=None):
        if not getattr(self, "d_llr1", None):
            self.d_llr1 = self.L.oai4g_dev_alloc(self.n_sf * self.stride * 2)
            _check(bool(self.d_llr1))
        _check(self.L.oai4g_rx_batch_tm3_2cw_pilots(self.cfg, self.n_sf, d_rxF, self._pil(), self.d_llr, self.d_llr1,
                                                    unscramble, stream) == 0)

    def launch_2cw(self, d_rxF, unscramble=1, stream=None):
        """both codewords QPSK: codeword 0 into d_llr, codeword 1 into d_llr1 (llrs1())"""
        if not getattr(self, "d_llr1", None):
            self.d_llr1 = self.L.oai4g_dev_alloc(self.n_sf * self.stride * 2)
            _check(bool(self.d_llr1))
        _check(self.L.oai4g_rx_batch_tm3_2cw(self.cfg, self.n_sf, d_rxF, self.d_est, self.d_llr, self.d_llr1,
                                             unscramble, stream) == 0)

    def llrs1(self):
        _check(self.L.oai4g_sync() == 0)
        out = np.empty((self.n_sf, self.stride), dtype=np.int16)
        _check(self.L.oai4g_memcpy_d2h(_ptr(out), self.d_llr1, out.nbytes) == 0)
        return out

    def llrs(self):
        _check(self.L.oai4g_sync() == 0)
        out = np.empty((self.n_sf, self.stride), dtype=np.int16)
        _check(self.L.oai4g_memcpy_d2h(_ptr(out), self.d_llr, out.nbytes) == 0)
        return out

    def estimates(self):
        _check(self.L.oai4g_sync() == 0)
        out = np.empty((4, self.n_sf, self.plane // self.n_sf), dtype=np.int32)
        _check(self.L.oai4g_memcpy_d2h(_ptr(out), self.d_est, out.nbytes) == 0)
        return out

    def close(self):
        self.L.oai4g_sync()
        for cfgs in self._chest.values():
            for cfg in cfgs:
                self.L.oai4g_chest_config_destroy(cfg)
        self._chest = {}
        self.L.oai4g_dev_free(self.d_est)
        self.L.oai4g_dev_free(self.d_llr)
        if getattr(self, "d_llr1", None):
            self.L.oai4g_dev_free(self.d_llr1)
            self.d_llr1 = None
        if getattr(self, "d_pil", None):
            self.L.oai4g_dev_free(self.d_pil)
            self.d_pil = None
        self.L.oai4g_rx_config_destroy(self.cfg)

class RxBatchTM2(RxBatchTM3):
    """Device-resident batched TM2 demodulation (oai4g_rx_batch_tm2): the ALAMOUTI-combined stream's
    LLRs from the FEP output of nb_rx antennas and the four estimate planes (ports 0 / 1 per antenna)."""

    def __init__(self, fp, rb_alloc, Qm, num_pdcch, rnti, n_sf, nb_rx=2, first_subframe=0, subframe_step=1):
        init()
        self.L = lib()
        ra = (ctypes.c_uint32 * 4)(*rb_alloc)
        self.cfg = self.L.oai4g_rx_config_create_tm2(ctypes.byref(fp), ra, Qm, num_pdcch, rnti, first_subframe,
                                                     subframe_step, nb_rx)
        _check(bool(self.cfg))
        self._setup(fp, n_sf, nb_rx)

    def launch(self, d_rxF, unscramble=1, stream=None):
        _check(self.L.oai4g_rx_batch_tm2(self.cfg, self.n_sf, d_rxF, self.d_est, self.d_llr, unscramble, stream) == 0)


def dlsch_unscrambling(fp, rnti, G, llr, q, Ns, mbsfn_flag=0):
    """dlsch_unscrambling drop-in (in place on an int16 array of >= 32 (1 + G/32) entries)."""
    init()
    lib().oai4g_dlsch_unscrambling(ctypes.byref(fp), mbsfn_flag, rnti, G, _ptr(llr), q, Ns)
    return llr


def lte_dl_channel_estimation(fp, rxdataF, est, Ns, p, l, symbol):
    """lte_dl_channel_estimation drop-in (high_speed_flag 1): rxdataF / est int32 [nsymb*N]; est in place."""
    init()
    rxdataF = np.ascontiguousarray(rxdataF, dtype=np.int32)
    assert est.dtype == np.int32 and est.flags.c_contiguous
    _check(lib().oai4g_lte_dl_channel_estimation(ctypes.byref(fp), _ptr(rxdataF), _ptr(est), Ns, p, l, symbol) == 0)
    return est


def _plane_ptrs(planes):
    arr = (ctypes.c_void_p * 8)()
    for i, a in enumerate(planes):
        if a is not None:
            assert a.dtype == np.int32 and a.flags.c_contiguous
            arr[i] = a.ctypes.data
    return arr


def dl_ch_estimates_time(fp, nb_antennas_rx, planes, out_planes):
    """lte_dl_channel_estimation's idft tail (:704-738): out_planes[(p << 1) + aarx] = idft_N of the
    estimate plane from word 8 (scale 1), for every non-None plane; lists of 8 int32 arrays / None."""
    init()
    _check(lib().oai4g_dl_ch_estimates_time(ctypes.byref(fp), nb_antennas_rx, _plane_ptrs(planes),
                                             _plane_ptrs(out_planes)) == 0)
    return out_planes


def lte_est_freq_offset(planes, fp, l, freq_offset, reset=0):
    """lte_est_freq_offset drop-in: planes[0] = antenna 0's estimate plane (int32 [nsymb*N]);
    freq_offset = a ctypes.c_int updated in place (process-wide first_run, as the reference's static)."""
    init()
    _check(lib().oai4g_lte_est_freq_offset(_plane_ptrs(planes), ctypes.byref(fp), l, ctypes.byref(freq_offset),
                                            reset) == 0)
    return freq_offset.value


def freq_offset_update(fp, omega, freq_offset, first_run):
    """The scalar tail of one lte_est_freq_offset call (ctypes.c_int state in place)."""
    _check(lib().oai4g_freq_offset_update(ctypes.byref(fp), int(np.int32(omega)), ctypes.byref(freq_offset),
                                           ctypes.byref(first_run)) == 0)
    return freq_offset.value


def chest_dc_filters(k):
    """The 25-PRB DC-pair filters (filt24_k_dcr, filt24_(k+2)_dcl) of pilot offset k."""
    out = np.zeros((2, 24), dtype=np.int16)
    lib().oai4g_chest_dc_filters(k, _ptr(out))
    return out


def chest_filters(k):
    """The six filt96_32.h filters (fl, f2l2, f, f2, fr, f2r2) of pilot offset k, as the library builds them."""
    out = np.zeros((6, 24), dtype=np.int16)
    lib().oai4g_chest_filters(k, _ptr(out))
    return out


class ChestBatch:
    """Device-resident batched channel estimation (oai4g_chest_batch) of n_sf consecutive subframes."""

    def __init__(self, fp, n_sf, p=0, first_subframe=0, subframe_step=1):
        init()
        self.L = lib()
        self.cfg = self.L.oai4g_chest_config_create(ctypes.byref(fp), p, first_subframe, subframe_step)
        _check(bool(self.cfg))
        self.fp, self.n_sf = fp, n_sf
        self.n_grid = n_sf * fp.symbols_per_tti * fp.ofdm_symbol_size
        self.d_rx = self.L.oai4g_dev_alloc((self.n_grid + fp.ofdm_symbol_size) * 4)
        self.d_est = self.L.oai4g_dev_alloc(self.n_grid * 4)
        _check(bool(self.d_rx) and bool(self.d_est))

    def run(self, rxdataF, next_symbol0, d_rxdataF=None):
        """rxdataF [n_sf][nsymb*N] and the N words of the following subframe's symbol 0."""
        if d_rxdataF is None:
            y = np.concatenate([np.ascontiguousarray(rxdataF, dtype=np.int32).ravel(),
                                np.ascontiguousarray(next_symbol0, dtype=np.int32).ravel()])
            assert y.size == self.n_grid + self.fp.ofdm_symbol_size
            _check(self.L.oai4g_memcpy_h2d(self.d_rx, _ptr(y), y.nbytes) == 0)
        self.launch(d_rxdataF or self.d_rx)
        _check(self.L.oai4g_sync() == 0)
        out = np.empty((self.n_sf, self.n_grid // self.n_sf), dtype=np.int32)
        _check(self.L.oai4g_memcpy_d2h(_ptr(out), self.d_est, out.nbytes) == 0)
        return out

    def launch(self, d_rxdataF, stream=None):
        """Device-only: estimates of d_rxdataF (n_sf grids + the next symbol 0) into self.d_est."""
        _check(self.L.oai4g_chest_batch(self.cfg, self.n_sf, d_rxdataF, self.d_est, stream) == 0)

    def time_estimates(self, stream=None):
        """dl_ch_estimates_time of every subframe's estimate plane in self.d_est: [n_sf][N] int32."""
        N, stride = self.fp.ofdm_symbol_size, self.n_grid // self.n_sf
        d_t = self.L.oai4g_dev_alloc(self.n_sf * N * 4)
        _check(bool(d_t))
        try:
            _check(self.L.oai4g_chest_time_batch(ctypes.byref(self.fp), self.n_sf, self.d_est, stride, d_t, N,
                                                 stream) == 0)
            _check(self.L.oai4g_sync() == 0)
            out = np.empty((self.n_sf, N), dtype=np.int32)
            _check(self.L.oai4g_memcpy_d2h(_ptr(out), d_t, out.nbytes) == 0)
        finally:
            self.L.oai4g_dev_free(d_t)
        return out

    def freq_offset_omegas(self, l, stream=None):
        """lte_est_freq_offset's integer part (omega, re | im << 16) of every subframe's plane."""
        d_o = self.L.oai4g_dev_alloc(max(4, self.n_sf * 4))
        _check(bool(d_o))
        try:
            _check(self.L.oai4g_freq_offset_omega_batch(ctypes.byref(self.fp), self.n_sf, self.d_est,
                                                        self.n_grid // self.n_sf, l, d_o, stream) == 0)
            _check(self.L.oai4g_sync() == 0)
            out = np.empty(self.n_sf, dtype=np.int32)
            _check(self.L.oai4g_memcpy_d2h(_ptr(out), d_o, out.nbytes) == 0)
        finally:
            self.L.oai4g_dev_free(d_o)
        return out

    def close(self):
        self.L.oai4g_dev_free(self.d_rx)
        self.L.oai4g_dev_free(self.d_est)
        self.L.oai4g_chest_config_destroy(self.cfg)


class RxBatch:
    """Device-resident batched PDSCH demodulation (oai4g_rx_batch)."""

    def __init__(self, fp, rb_alloc, Qm, num_pdcch, rnti, n_sf, first_subframe=0, subframe_step=1):
        init()
        self.L = lib()
        ra = (ctypes.c_uint32 * 4)(*rb_alloc)
        self.cfg = self.L.oai4g_rx_config_create(ctypes.byref(fp), ra, Qm, num_pdcch, rnti, first_subframe,
                                                 subframe_step)
        _check(bool(self.cfg))
        self.fp, self.n_sf = fp, n_sf
        self.stride = self.L.oai4g_rx_llr_stride(self.cfg)
        n_in = n_sf * fp.symbols_per_tti * fp.ofdm_symbol_size
        self.d_y = self.L.oai4g_dev_alloc(n_in * 4)
        self.d_h = self.L.oai4g_dev_alloc(n_in * 4)
        self.d_llr = self.L.oai4g_dev_alloc(n_sf * self.stride * 2)
        _check(bool(self.d_y) and bool(self.d_h) and bool(self.d_llr))

    def llr_count(self, sfi):
        return self.L.oai4g_rx_llr_count(self.cfg, sfi)

    def run(self, rxdataF, dl_ch, unscramble=1, d_rxdataF=None):
        if d_rxdataF is None:
            y = np.ascontiguousarray(rxdataF, dtype=np.int32)
            _check(self.L.oai4g_memcpy_h2d(self.d_y, _ptr(y), y.nbytes) == 0)
        h = np.ascontiguousarray(dl_ch, dtype=np.int32)
        _check(self.L.oai4g_memcpy_h2d(self.d_h, _ptr(h), h.nbytes) == 0)
        self.launch(d_rxdataF or self.d_y, self.d_h, unscramble)
        _check(self.L.oai4g_sync() == 0)
        out = np.empty((self.n_sf, self.stride), dtype=np.int16)
        _check(self.L.oai4g_memcpy_d2h(_ptr(out), self.d_llr, out.nbytes) == 0)
        return out

    def launch_estimated(self, chest, d_rxdataF, unscramble=1, stream=None):
        """Device-only, fused with the channel estimation of `chest` (a ChestBatch of the same
        subframes): LLRs of d_rxdataF into self.d_llr, no estimate buffer."""
        _check(self.L.oai4g_rx_batch_estimated(self.cfg, chest.cfg, self.n_sf, d_rxdataF, self.d_llr, unscramble,
                                               stream) == 0)

    def llrs(self):
        _check(self.L.oai4g_sync() == 0)
        out = np.empty((self.n_sf, self.stride), dtype=np.int16)
        _check(self.L.oai4g_memcpy_d2h(_ptr(out), self.d_llr, out.nbytes) == 0)
        return out

    def launch(self, d_rxdataF, d_est, unscramble=1, stream=None):
        """Device-only: LLRs of d_rxdataF / d_est into self.d_llr."""
        _check(self.L.oai4g_rx_batch(self.cfg, self.n_sf, d_rxdataF, d_est, self.d_llr, unscramble, stream) == 0)

    def close(self):
        for p in (self.d_y, self.d_h, self.d_llr):
            self.L.oai4g_dev_free(p)
        self.L.oai4g_rx_config_destroy(self.cfg)


class FepBatch:
    """Device-resident batched FEP (oai4g_fep_batch): n_sf subframes x n_ant antennas."""

    def __init__(self, fp, n_sf, n_ant):
        init()
        self.L = lib()
        self.fp, self.n_sf, self.n_ant = fp, n_sf, n_ant
        self.n_in = n_sf * n_ant * fp.samples_per_tti
        self.n_out = n_sf * n_ant * fp.symbols_per_tti * fp.ofdm_symbol_size
        self.d_rx = self.L.oai4g_dev_alloc(self.n_in * 4)
        self.d_rxF = self.L.oai4g_dev_alloc(self.n_out * 4)
        _check(bool(self.d_rx) and bool(self.d_rxF))

    def upload(self, rx):
        rx = np.ascontiguousarray(rx, dtype=np.int32)
        assert rx.size == self.n_in
        _check(self.L.oai4g_memcpy_h2d(self.d_rx, _ptr(rx), rx.nbytes) == 0)

    def run(self, stream=None):
        _check(self.L.oai4g_fep_batch(ctypes.byref(self.fp), self.n_sf, self.n_ant, self.d_rx, self.d_rxF,
                                      stream) == 0)

    def result(self):
        _check(self.L.oai4g_sync() == 0)
        out = np.empty((self.n_sf, self.n_ant, self.fp.symbols_per_tti, self.fp.ofdm_symbol_size), dtype=np.int32)
        _check(self.L.oai4g_memcpy_d2h(_ptr(out), self.d_rxF, out.nbytes) == 0)
        return out

    def close(self):
        self.L.oai4g_dev_free(self.d_rx)
        self.L.oai4g_dev_free(self.d_rxF)


def ofdm_mod(grid, log2n, nb_symbols, cp):
    """PHY_ofdm_mod (CYCLIC_PREFIX): grid int32[nb_symbols*N] -> int32[nb_symbols*(N+cp)]."""
    init()
    grid = np.ascontiguousarray(grid, dtype=np.int32)
    N = 1 << log2n
    out = np.zeros(nb_symbols * (N + cp), dtype=np.int32)
    lib().oai4g_PHY_ofdm_mod(_ptr(grid), _ptr(out), log2n, nb_symbols, cp, CYCLIC_PREFIX)
    return out


def generate_pilots(grids, amp, fp, ntti=10):
    """generate_pilots (pilots.c:43): CRS into the frame grids (list of int32 arrays, in place)."""
    init()
    ptrs = (ctypes.c_void_p * 2)(*[g.ctypes.data for g in grids] + [None] * (2 - len(grids)))
    lib().oai4g_generate_pilots(ptrs, amp, ctypes.byref(fp), ntti)
    return grids


def lte_dl_cell_spec(symbol, amp, fp, Ns, l, p):
    """lte_dl_cell_spec (lte_dl_cell_spec.c:123): CRS into one OFDM symbol (int32 array, in place)."""
    init()
    _check(lib().oai4g_lte_dl_cell_spec(_ptr(symbol), amp, ctypes.byref(fp), Ns, l, p) == 0)
    return symbol


def turbo_decoder16(y, n, max_iterations=8, crc_type=0, F=0):
    """phy_threegpplte_turbo_decoder16: y = 3n+12 int16 LLRs.  Returns (iterations, decoded bytes)."""
    init()
    y = np.ascontiguousarray(y, dtype=np.int16)
    out = np.zeros(n // 8, dtype=np.uint8)
    it = lib().oai4g_phy_threegpplte_turbo_decoder16(_ptr(y), _ptr(out), n, 0, 0, max_iterations, crc_type, F)
    _check(it != 255)
    return it, out


def rate_matching_turbo_rx(RTC, G, w, dummy_w, soft, C, r, Qm, rvidx=0, clear=1, Nl=1, Kmimo=1, Mdlharq=8,
                           Nsoft=1827072):
    """lte_rate_matching_turbo_rx (in place on w int16).  Returns E."""
    init()
    E = ctypes.c_uint32()
    soft = np.ascontiguousarray(soft, dtype=np.int16)
    _check(lib().oai4g_lte_rate_matching_turbo_rx(RTC, G, _ptr(w), _ptr(dummy_w), _ptr(soft), C, Nsoft, Mdlharq,
                                                  Kmimo, rvidx, clear, Qm, Nl, r, ctypes.byref(E)) == 0)
    return E.value


def sub_block_deinterleaving_turbo(D, w):
    """sub_block_deinterleaving_turbo: returns the d buffer (96 + 3D + 8 int16, d = buf[96:])."""
    init()
    buf = np.zeros(96 + 3 * D + 8, dtype=np.int16)
    lib().oai4g_sub_block_deinterleaving_turbo(D, ctypes.c_void_p(buf.ctypes.data + 2 * 96),
                                               _ptr(np.ascontiguousarray(w, dtype=np.int16)))
    return buf


def turbo_decoder8(y, n, max_iterations=8, crc_type=0, F=0):
    """phy_threegpplte_turbo_decoder8 drop-in: y = 3n+12 int16 LLRs.  Returns (iterations, bytes)."""
    init()
    y = np.ascontiguousarray(y, dtype=np.int16)
    out = np.zeros(n // 8, dtype=np.uint8)
    it = lib().oai4g_phy_threegpplte_turbo_decoder8(_ptr(y), _ptr(out), n, 0, 0, max_iterations, crc_type, F)
    _check(it != 255)
    return it, out


def _upload_tiled(dec, base, chunk_bytes=64 << 20):
    """Block i of a decoder batch gets base[i % len(base)], without a host copy of the whole batch
    (the C5 bench's 393 216-block batch would be 13 GB): one host chunk of whole base periods,
    copied over the device LLR buffer piece by piece."""
    base = np.asarray(base, dtype=np.int16)
    nb = len(base)
    per = max(1, chunk_bytes // (nb * dec.llr_stride * 2)) * nb       # rows per chunk, a multiple of nb
    per = min(per, ((dec.n_cb + nb - 1) // nb) * nb)
    buf = np.zeros((per, dec.llr_stride), dtype=np.int16)
    buf[:, :base.shape[1]] = np.tile(base, (per // nb, 1))
    for r0 in range(0, dec.n_cb, per):
        n = min(per, dec.n_cb - r0)
        _check(dec.L.oai4g_memcpy_h2d(dec.d_llr + r0 * dec.llr_stride * 2, _ptr(buf), n * dec.llr_stride * 2) == 0)


class TurboDecoder8Batch:
    """Device-resident batch of n_cb blocks of size K through the 8-bit decoder (oai4g_td8_batch)."""

    def __init__(self, K, n_cb):
        init()
        self.L = lib()
        self.K, self.n_cb = K, n_cb
        self.llr_stride = 3 * K + 16
        self.d_llr = self.L.oai4g_dev_alloc(n_cb * self.llr_stride * 2)
        self.d_out = self.L.oai4g_dev_alloc(n_cb * (K // 8))
        self.d_it = self.L.oai4g_dev_alloc(n_cb)
        self.d_scr = self.L.oai4g_dev_alloc(self.L.oai4g_td8_scratch_bytes(K, n_cb))
        _check(all(bool(p) for p in (self.d_llr, self.d_out, self.d_it, self.d_scr)))

    def upload(self, llr):
        buf = np.zeros((self.n_cb, self.llr_stride), dtype=np.int16)
        llr = np.asarray(llr, dtype=np.int16)
        buf[:, :llr.shape[1]] = llr
        _check(self.L.oai4g_memcpy_h2d(self.d_llr, _ptr(buf), buf.nbytes) == 0)

    def upload_tiled(self, base):
        _upload_tiled(self, base)

    def run(self, max_iterations=8, crc_type=0, F=0, stream=None):
        _check(self.L.oai4g_td8_batch(self.n_cb, self.K, self.d_llr, self.llr_stride, self.d_out, self.K // 8,
                                      self.d_it, max_iterations, crc_type, F, self.d_scr, stream) == 0)

    def results(self):
        _check(self.L.oai4g_sync() == 0)
        out = np.empty((self.n_cb, self.K // 8), dtype=np.uint8)
        it = np.empty(self.n_cb, dtype=np.uint8)
        _check(self.L.oai4g_memcpy_d2h(_ptr(out), self.d_out, out.nbytes) == 0)
        _check(self.L.oai4g_memcpy_d2h(_ptr(it), self.d_it, it.nbytes) == 0)
        return it, out

    def close(self):
        for p in (self.d_llr, self.d_out, self.d_it, self.d_scr):
            self.L.oai4g_dev_free(p)


def generate_dummy_w(D, F=0):
    """generate_dummy_w: the uint8 NULL-mark buffer (3 Kpi) of a block of D = K + 4 with F fillers."""
    R = (D + 31) >> 5
    w = np.zeros(3 * 32 * R + 64, dtype=np.uint8)
    lib().oai4g_generate_dummy_w(D, _ptr(w), F)
    return w


class UlDecodeBatch:
    """Batched ulsch_decoding chain (oai4g_ul_decode_batch): n_tb transport blocks of B = TBS + 24
    bits, G soft bits each -> RM-rx + deinterleaving + 16-bit turbo decoding per code block."""

    def __init__(self, B, G, Qm, n_tb, rvidx=0, max_iterations=8, Mdlharq=8, Nsoft=1827072):
        init()
        self.L = lib()
        self.cfg = self.L.oai4g_ul_config_create(B, G, Qm, rvidx, Mdlharq, Nsoft, max_iterations)
        _check(bool(self.cfg))
        self.C = self.L.oai4g_ul_config_C(self.cfg)
        self.n_tb, self.G = n_tb, G
        self.e_stride = (G + 63) & ~63
        self.c_stride = 6144 // 8 + 8
        self.d_e = self.L.oai4g_dev_alloc(n_tb * self.e_stride * 2)
        self.d_c = self.L.oai4g_dev_alloc(n_tb * self.C * self.c_stride)
        self.d_it = self.L.oai4g_dev_alloc(n_tb * self.C)
        _check(bool(self.d_e) and bool(self.d_c) and bool(self.d_it))

    def E(self, r):
        return self.L.oai4g_ul_config_E(self.cfg, r)

    def offset(self, r):
        return self.L.oai4g_ul_config_G_offset(self.cfg, r)

    def upload(self, e):
        buf = np.zeros((self.n_tb, self.e_stride), dtype=np.int16)
        buf[:, :self.G] = np.asarray(e, dtype=np.int16).reshape(self.n_tb, -1)[:, :self.G]
        _check(self.L.oai4g_memcpy_h2d(self.d_e, _ptr(buf), buf.nbytes) == 0)

    def launch(self, stream=None):
        _check(self.L.oai4g_ul_decode_batch(self.cfg, self.n_tb, self.d_e, self.e_stride, self.d_c, self.c_stride,
                                            self.d_it, stream) == 0)

    def launch_harq(self, rvidx, clear, stream=None):
        """One HARQ round (oai4g_ul_decode_batch_harq) on the uploaded soft bits: the per-block soft
        buffers (allocated zeroed on first use) combine this round's rvidx; clear = 1 on round 0."""
        if getattr(self, "d_w", None) is None:
            self.w_stride = (self.L.oai4g_ul_config_w_entries(self.cfg) + 63) & ~63
            nbytes = self.n_tb * self.C * self.w_stride * 2
            self.d_w = self.L.oai4g_dev_alloc(nbytes)
            _check(bool(self.d_w))
            z = np.zeros(nbytes // 2, np.int16)
            _check(self.L.oai4g_memcpy_h2d(self.d_w, _ptr(z), nbytes) == 0)
        _check(self.L.oai4g_ul_decode_batch_harq(self.cfg, self.n_tb, self.d_e, self.e_stride, self.d_w, self.w_stride,
                                                 rvidx, clear, self.d_c, self.c_stride, self.d_it, stream) == 0)

    def soft_buffers(self):
        """[n_tb][C][w_stride] int16 HARQ soft buffers (after launch_harq)."""
        _check(self.L.oai4g_sync() == 0)
        w = np.empty((self.n_tb, self.C, self.w_stride), dtype=np.int16)
        _check(self.L.oai4g_memcpy_d2h(_ptr(w), self.d_w, w.nbytes) == 0)
        return w

    def results(self):
        _check(self.L.oai4g_sync() == 0)
        c = np.empty((self.n_tb, self.C, self.c_stride), dtype=np.uint8)
        it = np.empty((self.n_tb, self.C), dtype=np.uint8)
        _check(self.L.oai4g_memcpy_d2h(_ptr(c), self.d_c, c.nbytes) == 0)
        _check(self.L.oai4g_memcpy_d2h(_ptr(it), self.d_it, it.nbytes) == 0)
        return it, c

    def close(self):
        for p in (self.d_e, self.d_c, self.d_it, getattr(self, "d_w", None)):
            if p:
                self.L.oai4g_dev_free(p)
        self.L.oai4g_ul_config_destroy(self.cfg)


class TurboDecoderBatch:
    """Device-resident batch of n_cb code blocks of size K (oai4g_td_batch)."""

    def __init__(self, K, n_cb):
        init()
        self.L = lib()
        self.K, self.n_cb = K, n_cb
        self.llr_stride = 3 * K + 16
        self.d_llr = self.L.oai4g_dev_alloc(n_cb * self.llr_stride * 2)
        self.d_out = self.L.oai4g_dev_alloc(n_cb * (K // 8))
        self.d_it = self.L.oai4g_dev_alloc(max(256, n_cb))
        self.d_scr = self.L.oai4g_dev_alloc(self.L.oai4g_td_scratch_bytes(K, n_cb))
        _check(all([self.d_llr, self.d_out, self.d_it, self.d_scr]))
        # the decoder writes d_out only once a hard decision is made (iteration >= 2), as the
        # reference leaves decoded_bytes untouched at max_iterations = 1: start from a zeroed buffer
        z = np.zeros(n_cb * (K // 8), dtype=np.uint8)
        _check(self.L.oai4g_memcpy_h2d(self.d_out, _ptr(z), z.nbytes) == 0)

    def upload(self, llr):
        buf = np.zeros((self.n_cb, self.llr_stride), dtype=np.int16)
        buf[:, :3 * self.K + 12] = llr
        _check(self.L.oai4g_memcpy_h2d(self.d_llr, _ptr(buf), buf.nbytes) == 0)

    def upload_tiled(self, base):
        _upload_tiled(self, base)

    def run(self, max_iterations=8, crc_type=0, F=0, stream=None):
        _check(self.L.oai4g_td_batch(self.n_cb, self.K, self.d_llr, self.llr_stride, self.d_out, self.K // 8,
                                     self.d_it, max_iterations, crc_type, F, self.d_scr, stream) == 0)

    def results(self):
        _check(self.L.oai4g_sync() == 0)
        out = np.empty((self.n_cb, self.K // 8), dtype=np.uint8)
        it = np.empty(self.n_cb, dtype=np.uint8)
        _check(self.L.oai4g_memcpy_d2h(_ptr(out), self.d_out, out.nbytes) == 0)
        _check(self.L.oai4g_memcpy_d2h(_ptr(it), self.d_it, it.nbytes) == 0)
        return it, out

    def close(self):
        for p in (self.d_llr, self.d_out, self.d_it, self.d_scr):
            self.L.oai4g_dev_free(p)


def dci_allocs(items):
    """items: (dci_length, L, nCCE, rnti, pdu bytes) -> ctypes array of DciAlloc"""
    arr = (DciAlloc * max(1, len(items)))()
    for a, (ln, L, ncce, rnti, pdu) in zip(arr, items):
        a.dci_length, a.L, a.nCCE, a.rnti = ln, L, ncce, rnti
        for i, b in enumerate(list(pdu)[:8]):
            a.dci_pdu[i] = int(b)
    return arr


def generate_dci_top(items, n_common, amp, fp, txdataF, subframe):
    """generate_dci_top on frame grids (int32 arrays, modified in place): num_pdcch_symbols"""
    init()
    arr = dci_allocs(items)
    gp = (ctypes.c_void_p * len(txdataF))(*[g.ctypes.data for g in txdataF])
    return lib().oai4g_generate_dci_top(len(items) - n_common, n_common, arr, 0, amp, ctypes.byref(fp), gp, subframe)


def normal_prefix_mod(txdataF, fp, nsymb=7, out=None):
    init()
    txdataF = np.ascontiguousarray(txdataF, dtype=np.int32)
    if out is None:
        out = np.zeros(fp.samples_per_tti, dtype=np.int32)
    lib().oai4g_normal_prefix_mod(_ptr(txdataF), _ptr(out), nsymb, ctypes.byref(fp))
    return out


class DlschHandle:
    """Owns an oai4g_dlsch_t (new_eNB_dlsch) and exposes its HARQ-0 buffers as numpy views."""

    def __init__(self, Kmimo=1, Mdlharq=8, N_RB_DL=100):
        init()
        self.ptr = lib().oai4g_new_dlsch(Kmimo, Mdlharq, N_RB_DL)
        if not self.ptr:
            raise OAI4GError("new_dlsch failed")
        self.d = self.ptr.contents
        self.h = self.d.harq_processes[0].contents

    def close(self):
        if self.ptr:
            lib().oai4g_free_dlsch(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def view(self, field, n, r=None):
        p = getattr(self.h, field) if r is None else getattr(self.h, field)[r]
        return np.ctypeslib.as_array(p, shape=(n,))


def dlsch_encoding(a, fp, num_pdcch, dl, subframe):
    return lib().oai4g_dlsch_encoding(_ptr(a), ctypes.byref(fp), num_pdcch, dl.ptr, 0, subframe)


def dlsch_scrambling(fp, dl, G, q, Ns, mbsfn_flag=0):
    lib().oai4g_dlsch_scrambling(ctypes.byref(fp), mbsfn_flag, dl.ptr, G, q, Ns)


def dlsch_modulation(txdataF, amp, subframe, fp, num_pdcch, dl0, dl1=None):
    """txdataF: list of int32 arrays (one per antenna), modified in place."""
    arr = (ctypes.c_void_p * len(txdataF))(*[a.ctypes.data for a in txdataF])
    return lib().oai4g_dlsch_modulation(arr, amp, subframe, ctypes.byref(fp), num_pdcch, dl0.ptr,
                                        dl1.ptr if dl1 is not None else None)


# ------------------------------------------------------------------------------------------
# configurations (BASELINE.json configs) and the batched pipeline
# ------------------------------------------------------------------------------------------
FULL_ALLOC_100 = (0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xF)
FULL_ALLOC_6 = (0x3F, 0, 0, 0)
FULL_ALLOC_15 = (0x7FFF, 0, 0, 0)
FULL_ALLOC_50 = (0xFFFFFFFF, 0x3FFFF, 0, 0)
FULL_ALLOC_25 = (0x1FFFFFF, 0, 0, 0)

def get_TBS_DL(mcs, nb_rb):
    """get_TBS_DL (lte_mcs.c:118): transport block size in BYTES, from the library's TBStable."""
    return lib().oai4g_get_TBS_DL(mcs, nb_rb)


def tbs_bits(mcs, nb_rb):
    """TBS in bits for (mcs, nb_rb) as dlsim uses it (get_TBS_DL << 3; dci_tools.c)."""
    return get_TBS_DL(mcs, nb_rb) << 3

CONFIGS = {
    # C1: dlsim 1.4 MHz SISO QPSK (MCS 9), 3 PDCCH symbols
    "C1": dict(N_RB_DL=6, nb_antennas_tx=1, mode1_flag=1, n_cw=1, mimo_mode=SISO, num_pdcch_symbols=3,
               mcs=(9, 0), rb_alloc=FULL_ALLOC_6, nb_rb=6, Kmimo=1),
    # C2: dlsim 20 MHz SISO 16-QAM (MCS 16)
    "C2": dict(N_RB_DL=100, nb_antennas_tx=1, mode1_flag=1, n_cw=1, mimo_mode=SISO, num_pdcch_symbols=1,
               mcs=(16, 0), rb_alloc=FULL_ALLOC_100, nb_rb=100, Kmimo=1),
    # C3: dlsim 20 MHz 2x2 TM3 (LARGE_CDD) 64-QAM, MCS 19 on both codewords (highest the reference encodes)
    "C3": dict(N_RB_DL=100, nb_antennas_tx=2, mode1_flag=0, n_cw=2, mimo_mode=LARGE_CDD, num_pdcch_symbols=1,
               mcs=(19, 19), rb_alloc=FULL_ALLOC_100, nb_rb=100, Kmimo=2),
    # C4: C3 on 4 TX antennas (build-defined extension: 4-port CRS exclusions, 36.211 6.3.4.2.2
    # large-delay CDD precoding over the rank-2 codebook entries 12-15)
    "C4": dict(N_RB_DL=100, nb_antennas_tx=4, mode1_flag=0, n_cw=2, mimo_mode=LARGE_CDD, num_pdcch_symbols=1,
               mcs=(19, 19), rb_alloc=FULL_ALLOC_100, nb_rb=100, Kmimo=2),
    # TM2: dlsim 20 MHz 2 TX transmit diversity (ALAMOUTI, DCI format 1: one codeword, Nl = 1), 16-QAM
    "TM2": dict(N_RB_DL=100, nb_antennas_tx=2, mode1_flag=0, n_cw=1, mimo_mode=ALAMOUTI, num_pdcch_symbols=1,
                mcs=(16, 0), rb_alloc=FULL_ALLOC_100, nb_rb=100, Kmimo=1),
    # TM2 at 1.4 MHz, QPSK (MCS 9), 3 PDCCH symbols
    "TM2S": dict(N_RB_DL=6, nb_antennas_tx=2, mode1_flag=0, n_cw=1, mimo_mode=ALAMOUTI, num_pdcch_symbols=3,
                 mcs=(9, 0), rb_alloc=FULL_ALLOC_6, nb_rb=6, Kmimo=1),
}


def make_params(name="C3", subframe=7, subframe_step=0, rnti=0x1234, Nid_cell=0, with_crs=0, **over):
    c = dict(CONFIGS[name])
    c.update(over)
    p = TxParams()
    p.N_RB_DL = c["N_RB_DL"]
    p.Nid_cell = Nid_cell
    p.Ncp = c.get("Ncp", 0)
    p.nb_antennas_tx = c["nb_antennas_tx"]
    p.mode1_flag = c["mode1_flag"]
    p.frame_type = 0
    p.n_cw = c["n_cw"]
    p.mimo_mode = c["mimo_mode"]
    p.num_pdcch_symbols = c["num_pdcch_symbols"]
    p.Kmimo = c["Kmimo"]
    p.Mdlharq = 8
    p.first_subframe = subframe
    p.subframe_step = subframe_step
    p.with_crs = with_crs
    p.rnti = rnti
    p.amp = 512
    p.sqrt_rho_a = 8192
    p.sqrt_rho_b = 8192
    for i in range(4):
        p.rb_alloc[i] = c["rb_alloc"][i]
    p.nb_rb = c["nb_rb"]
    tbs = c.get("TBS")
    for cw in range(p.n_cw):
        p.mcs[cw] = c["mcs"][cw]
        p.rvidx[cw] = 0
        p.q[cw] = 0
        p.TBS[cw] = tbs[cw] if tbs else tbs_bits(c["mcs"][cw], c["nb_rb"])
    maxA = max(p.TBS[cw] // 8 for cw in range(p.n_cw))
    p.payload_stride = (maxA + 3 + 15) & ~15
    return p


class TxPipeline:
    """Batched device-resident transmit path for one configuration (oai4g_tx_*)."""

    def __init__(self, params, n_sf, alloc=True):
        self.L = init()
        self.params = params
        self.n_sf = n_sf
        self.cfg = self.L.oai4g_tx_config_create(ctypes.byref(params))
        if not self.cfg:
            raise OAI4GError(self.L.oai4g_last_error().decode())
        self.n_cw = params.n_cw
        self.n_ant = params.nb_antennas_tx
        self.spt = self.L.oai4g_tx_iq_samples(self.cfg)
        self.ebits_words = self.L.oai4g_tx_ebits_words(self.cfg)
        self.payload_bytes = n_sf * self.n_cw * params.payload_stride
        self.work_bytes = self.L.oai4g_tx_workspace_bytes(self.cfg, n_sf)
        self.iq_samples = n_sf * self.n_ant * self.spt
        self.d_payload = self.d_work = self.d_iq = None
        if alloc:
            self.d_payload = self._alloc(self.payload_bytes)
            self.d_work = self._alloc(self.work_bytes)
            self.d_iq = self._alloc(self.iq_samples * 4)

    def _alloc(self, n):
        p = self.L.oai4g_dev_alloc(n)
        if not p:
            raise OAI4GError(self.L.oai4g_last_error().decode())
        return p

    def G(self, cw, subframe):
        return self.L.oai4g_tx_G(self.cfg, cw, subframe)

    def set_control(self, items, n_common=0):
        """oai4g_tx_config_set_control: generate_dci_top's PCFICH + PDCCH for these DCIs in every
        batch element (items as for generate_dci_top; [] switches it off)."""
        arr = dci_allocs(items)
        _check(self.L.oai4g_tx_config_set_control(self.cfg, len(items) - n_common, n_common, arr) == 0)

    def set_common(self, pss_sss=False, pbch_pdu=None, frame_mod4=0, phich=()):
        """oai4g_tx_config_set_common: PSS + SSS (subframe indices 0 / 5), the PBCH quarter
        frame_mod4 of pbch_pdu (subframe index 0) and PHICHs (subframe, ngroup, nseq, hi);
        with no argument it switches them off."""
        c = CommonSig()
        c.pss_sss = 1 if pss_sss else 0
        if pbch_pdu is not None:
            c.pbch = 1
            for i in range(3):
                c.pbch_pdu[i] = int(pbch_pdu[i])
        c.frame_mod4 = frame_mod4
        c.n_phich = len(phich)
        for i, (sf, g, q, h) in enumerate(phich):
            c.phich[i].subframe, c.phich[i].ngroup, c.phich[i].nseq, c.phich[i].hi = sf, g, q, h
        on = c.pss_sss or c.pbch or c.n_phich
        _check(self.L.oai4g_tx_config_set_common(self.cfg, ctypes.byref(c) if on else None) == 0)

    def fill_payload(self, seed):
        _check(self.L.oai4g_fill_payload(self.d_payload, self.payload_bytes, seed, None) == 0)

    def upload_payload(self, payload):
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        assert payload.nbytes == self.payload_bytes
        _check(self.L.oai4g_memcpy_h2d(self.d_payload, _ptr(payload), payload.nbytes) == 0)

    def download_payload(self):
        out = np.empty(self.payload_bytes, dtype=np.uint8)
        _check(self.L.oai4g_memcpy_d2h(_ptr(out), self.d_payload, out.nbytes) == 0)
        return out.reshape(self.n_sf, self.n_cw, self.params.payload_stride)

    def run(self, stream=None):
        _check(self.L.oai4g_tx_batch(self.cfg, self.n_sf, self.d_payload, self.d_work, self.d_iq, stream) == 0)

    def run_timed(self, stream=None):
        ms = (ctypes.c_float * 2)()
        _check(self.L.oai4g_tx_batch_timed(self.cfg, self.n_sf, self.d_payload, self.d_work, self.d_iq, stream,
                                           ms) == 0)
        return ms[0], ms[1]

    def encode_only(self, stream=None):
        _check(self.L.oai4g_tx_encode(self.cfg, self.n_sf, self.d_payload, self.d_work, stream) == 0)

    def diag_encode_phase_ms(self, stop_phase, reps=5):
        ms = ctypes.c_float()
        _check(self.L.oai4g_diag_encode_phase_ms(self.cfg, self.n_sf, self.d_payload, self.d_work, stop_phase, reps,
                                                 ctypes.byref(ms)) == 0)
        return ms.value

    def modulate_only(self, stream=None):
        """oai4g_tx_modulate: the modulator kernel alone, from the e-bit words in the workspace."""
        _check(self.L.oai4g_tx_modulate(self.cfg, self.n_sf, self.d_work, self.d_iq, stream) == 0)

    def upload_ebits(self, words):
        """Packed scrambled e-bit words [n_sf][n_cw][ebits_words] into the workspace."""
        words = np.ascontiguousarray(words, dtype=np.uint32)
        assert words.nbytes <= self.work_bytes
        _check(self.L.oai4g_memcpy_h2d(self.d_work, _ptr(words), words.nbytes) == 0)

    @property
    def mod_nosat(self):
        return bool(self.L.oai4g_tx_mod_nosat(self.cfg))

    def sync(self):
        _check(self.L.oai4g_sync() == 0)

    def ebits(self):
        out = np.empty(self.work_bytes // 4, dtype=np.uint32)
        _check(self.L.oai4g_memcpy_d2h(_ptr(out), self.d_work, out.nbytes) == 0)
        return out.reshape(self.n_sf, self.n_cw, self.ebits_words)

    def iq(self):
        out = np.empty(self.iq_samples, dtype=np.int32)
        _check(self.L.oai4g_memcpy_d2h(_ptr(out), self.d_iq, out.nbytes) == 0)
        return out.reshape(self.n_sf, self.n_ant, self.spt)

    def close(self):
        for p in (self.d_payload, self.d_work, self.d_iq):
            if p:
                self.L.oai4g_dev_free(p)
        self.d_payload = self.d_work = self.d_iq = None
        if self.cfg:
            self.L.oai4g_tx_config_destroy(self.cfg)
            self.cfg = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def unpack_bits(words, nbits):
    """Packed LSB-first uint32 words -> uint8 bit array."""
    b = np.unpackbits(np.ascontiguousarray(words, dtype="<u4").view(np.uint8), bitorder="little")
    return b[:nbits]
