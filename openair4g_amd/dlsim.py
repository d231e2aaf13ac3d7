"""dlsim's BLER loop on the GPU (openair1/SIMULATION/LTE_PHY/dlsim.c:2065-3545), batched over trials.

One trial of the reference, TM1 / SISO / one receive antenna / AWGN (`-gN`: channel_model = AWGN, value
18 of SCM_t in SIMULATION/TOOLS/defs.h:158-178, applied through multipath_channel, a single unit tap at
Ricean factor 0 -- `-gL` would be Rice8 = 14), the configuration the reference's
AWGN_results/bler_tx1_chan18_nrx1_mcs*.csv name in their file names (the reference also holds a second
set for it, AWGN/Perf_Curves_Abs/awgn_bler_tx1_mcs*.csv, 0.05-0.3 dB apart; the GPU chain follows that
one, tests/test_gpu_dlsim.py):
  - transmit (:2553-2704): generate_dci_top's PCFICH + PDCCH for one format-1 DCI (L = 1, RNTI
    0x1234; dlsim.c:1154-1157), dlsch_encoding / dlsch_scrambling / dlsch_modulation of a random
    transport block, generate_pilots, do_OFDM_mod_l of the subframe's two slots, and of the next
    subframe's first slot (which carries only its CRS, the grid being cleared each trial :2161);
  - tx_lev = signal_energy of the subframe (:2714-2719);
  - AWGN over the two subframes with sigma2_dB = 10 log10(tx_lev) + 10 log10(N / (12 NB_RB)) - SNR
    - pa_dB (:2852-2866), pa = 0 dB;
  - the UE (:2907-3260): slot_fep of both slots plus symbol 0 of the next, lte_dl_channel_estimation
    (perfect_ce = 0, high_speed_flag = 1), rx_pdsch, dlsch_unscrambling, dlsch_decoding with the
    16-bit decoder (dlsim's default, llr8_flag = 0 at dlsim.c:339; `-L` selects the 8-bit one, llr8
    here) and MAX_TURBO_ITERATIONS = 4 (PHY/CODING/defs.h:51);
  - a trial errs when dlsch_decoding returns more than max_turbo_iterations (:3330-3350); one round
    (the CSVs hold no retransmission counts).
On the GPU: TxPipeline (k_encode + k_modofdm with CRS + control) -> k_signal_energy -> k_awgn ->
k_fep over [trial][2 subframes] -> k_rx_chest (estimation + demodulation + unscrambling, elements two
subframes apart) -> k_ul_rm_deint + k_td16.  Nothing here runs on the CPU but bookkeeping."""
import ctypes
import math

import numpy as np

from . import (FULL_ALLOC_25, ChestBatch, FepBatch, OAI4GError, RxBatch, TxPipeline, _check, _ptr, frame_parms,
               init, lib, make_params, normal_prefix_mod, generate_pilots, UlDecodeBatch)

DCI1_LEN = {6: 23, 15: 25, 25: 27, 50: 27, 100: 39}      # sizeof_DCI1_xMHz_FDD_t (PHY/LTE_TRANSPORT/dci.h)
FULL_ALLOC = {6: (0x3F, 0, 0, 0), 15: (0x7FFF, 0, 0, 0), 25: FULL_ALLOC_25, 50: (0xFFFFFFFF, 0x3FFFF, 0, 0),
              100: (0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xF)}


def qm_of(mcs):
    """get_Qm (lte_mcs.c:31)"""
    return 2 if mcs < 10 else (4 if mcs < 17 else 6)


class DlsimBler:
    """Batched BLER trials of one (N_RB_DL, MCS) configuration; see the module docstring."""

    def __init__(self, mcs, N_RB_DL=25, batch=4096, subframe=7, num_pdcch_symbols=1, Nid_cell=0, rnti=0x1234,
                 max_iterations=4, with_dci=True, llr8=False):
        self.L = init()
        self.mcs, self.N_RB, self.B, self.sf = mcs, N_RB_DL, batch, subframe
        self.max_it = max_iterations
        self.Qm = qm_of(mcs)
        self.p = make_params("C2", subframe=subframe, subframe_step=0, rnti=rnti, Nid_cell=Nid_cell, with_crs=1,
                             N_RB_DL=N_RB_DL, nb_rb=N_RB_DL, rb_alloc=FULL_ALLOC[N_RB_DL], mcs=[mcs], TBS=None,
                             num_pdcch_symbols=num_pdcch_symbols)
        self.fp = frame_parms(N_RB_DL, Nid_cell=Nid_cell)
        self.spt, self.N = self.fp.samples_per_tti, self.fp.ofdm_symbol_size
        self.tx = TxPipeline(self.p, batch)
        if with_dci:
            self.L.oai4g_init_nCCE_table()
            nCCE = self.L.oai4g_get_nCCE(num_pdcch_symbols, ctypes.byref(self.fp), 1)
            ncce = self.L.oai4g_get_nCCE_offset(2, nCCE, 0, rnti, subframe)
            pdu = np.zeros(8, np.uint8)       # DCI1 content (rah 0, rballoc, mcs, ndi 1, rv 0): bits only move QPSK signs
            self.tx.set_control([(DCI1_LEN[N_RB_DL], 1, ncce, rnti, pdu)])
        # the next subframe's first slot: its CRS only (generate_pilots over the cleared grid), the
        # second slot never modulated (zeros)
        nsymb = self.fp.symbols_per_tti
        grid = np.zeros(10 * nsymb * self.N, np.int32)
        generate_pilots([grid], 512, self.fp)
        nxt = (subframe + 1) % 10
        tail = np.zeros(self.spt, np.int32)
        normal_prefix_mod(grid[nxt * nsymb * self.N:], self.fp, nsymb // 2, tail)
        self.tail = tail
        L = self.L
        self.d_tail = L.oai4g_dev_alloc(tail.nbytes)
        self.d_lev = L.oai4g_dev_alloc(4 * batch)
        self.fep = FepBatch(self.fp, 2 * batch, 1)
        _check(bool(self.d_tail) and bool(self.d_lev))
        _check(L.oai4g_memcpy_h2d(self.d_tail, _ptr(tail), tail.nbytes) == 0)
        self.ce = ChestBatch(self.fp, batch, first_subframe=subframe, subframe_step=0)
        _check(L.oai4g_chest_config_set_stride(self.ce.cfg, 2, 1) == 0)
        self.rx = RxBatch(self.fp, list(FULL_ALLOC[N_RB_DL]), self.Qm, num_pdcch_symbols, rnti, batch,
                          first_subframe=subframe, subframe_step=0)
        self.G = self.rx.llr_count(subframe)
        self.TBS = self.p.TBS[0]
        self.dec = UlDecodeBatch(self.TBS + 24, self.G, self.Qm, batch, max_iterations=max_iterations)
        if llr8:                              # dlsim -L: dlsch_decoding with the 8-bit decoder
            _check(self.L.oai4g_ul_config_set_decoder(self.dec.cfg, 8) == 0)
        self.C = self.dec.C
        self.offset_fac = 10 * math.log10(self.N / (12.0 * N_RB_DL))

    def sigma_offset(self, snr_db, pa_db=0.0):
        return self.offset_fac - snr_db - pa_db

    def run_batch(self, snr_db, seed, first_trial=0, want_bits=False):
        """One batch of trials; returns the per-trial error flags (and decoded / sent bytes)."""
        L, B = self.L, self.B
        self.tx.fill_payload(seed)
        self.tx.run()
        d_iq = self.tx.d_iq
        _check(L.oai4g_signal_energy_batch(d_iq, B, self.spt, self.spt, self.d_lev, None) == 0)
        _check(L.oai4g_awgn_batch(d_iq, self.spt, self.spt, self.d_tail, self.spt, self.fep.d_rx, 2 * self.spt, B,
                                  self.d_lev, self.sigma_offset(snr_db), seed, first_trial, None) == 0)
        self.fep.run()
        self.rx.launch_estimated(self.ce, self.fep.d_rxF, 1)
        _check(L.oai4g_ul_decode_batch(self.dec.cfg, B, self.rx.d_llr, self.rx.stride, self.dec.d_c,
                                       self.dec.c_stride, self.dec.d_it, None) == 0)
        it, c = self.dec.results()
        err = np.any(it > self.max_it, axis=1)
        if not want_bits:
            return err
        return err, c, self.tx.download_payload()

    def tx_lev(self):
        out = np.empty(self.B, np.int32)
        _check(self.L.oai4g_sync() == 0)
        _check(self.L.oai4g_memcpy_d2h(_ptr(out), self.d_lev, out.nbytes) == 0)
        return out

    def run_point(self, snr_db, n_trials, seed=1):
        """(errors, trials) at one SNR over ceil(n_trials / batch) batches."""
        errs = trials = 0
        b = 0
        while trials < n_trials:
            e = self.run_batch(snr_db, seed * 1000003 + b, first_trial=b * self.B)
            take = min(self.B, n_trials - trials)
            errs += int(e[:take].sum())
            trials += take
            b += 1
        return errs, trials

    def close(self):
        for o in (self.tx, self.fep, self.ce, self.rx, self.dec):
            o.close()
        self.L.oai4g_dev_free(self.d_tail)
        self.L.oai4g_dev_free(self.d_lev)


def tb_bytes_from_blocks(c, TBS, C, K_list, F):
    """Reassemble a TB from the decoded code blocks c[r] (dlsch_decoding.c:455-490)."""
    out = []
    for r in range(C):
        kb = K_list[r] // 8
        start = (F >> 3) if r == 0 else 0
        out.append(c[r, start:kb - (3 if C > 1 else 0)])
    return np.concatenate(out)[:TBS // 8]


def wilson(k, n, z=1.96):
    """95 % binomial (Wilson) interval of k errors in n trials."""
    if n == 0:
        return 0.0, 1.0
    ph = k / n
    d = 1 + z * z / n
    c = (ph + z * z / (2 * n)) / d
    h = z * math.sqrt(ph * (1 - ph) / n + z * z / (4 * n * n)) / d
    return max(0.0, c - h), min(1.0, c + h)


__all__ = ["DlsimBler", "qm_of", "wilson", "OAI4GError", "lib"]
