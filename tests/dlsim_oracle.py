"""TEST INFRASTRUCTURE: one dlsim BLER trial on the CPU oracle (TM1, SISO, one RX antenna, AWGN),
the reference's loop restated step by step (SIMULATION/LTE_PHY/dlsim.c:2131-3545):

  transmit    orc_tx_subframe_dci: generate_dci_top (one format-1 DCI, L = 1), dlsch_encoding,
              dlsch_scrambling, dlsch_modulation, generate_pilots, do_OFDM_mod_l (:2553-2704); the
              next subframe's first slot carries its CRS only (:2701-2704 over the grid cleared at :2161)
  tx_lev      signal_energy of the subframe (:2714-2719; orc_signal_energy, pinned to the reference TU)
  AWGN        (:2852-2866) with the reference's own generator (rangen_double.c, restated; seeded)
  UE          slot_fep x 14 + symbol 0 of the next slot, lte_dl_channel_estimation (perfect_ce = 0),
              rx_pdsch, dlsch_unscrambling, dlsch_decoding (16-bit decoder, MAX_TURBO_ITERATIONS 4)

Used by tests/test_dlsim_cpu.py (statistical pin of the whole chain to the reference-held
AWGN_results/bler_tx1_chan18_nrx1_mcs*.csv) and tests/test_gpu_dlsim.py (the GPU chain bit-exact
against this one on the same noisy samples)."""
import ctypes
import math
import os

import numpy as np

import oracle_lib as O

CSV_DIR = "openair1/SIMULATION/LTE_PHY/BLER_SIMULATIONS/AWGN/AWGN_results"
HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN_CSV = os.path.join(HERE, "golden", "bler_awgn_tx1_nrx1.json")
DCI1_LEN = {6: 23, 15: 25, 25: 27, 50: 27, 100: 39}


def qm_of(mcs):
    return 2 if mcs < 10 else (4 if mcs < 17 else 6)


def wilson(k, n, z=1.96):
    if n == 0:
        return 0.0, 1.0
    ph = k / n
    d = 1 + z * z / n
    c = (ph + z * z / (2 * n)) / d
    h = z * math.sqrt(ph * (1 - ph) / n + z * z / (4 * n * n)) / d
    return max(0.0, c - h), min(1.0, c + h)


def load_curves(which="awgn_results"):
    """{mcs: [(snr, err0, trials0)]} from the committed fixture (tests/golden/make_bler_fixture.py):
    which = "awgn_results" (AWGN_results/bler_tx1_chan18_nrx1_mcs*.csv) or "perf_curves_abs" (the
    reference's second set for the same configuration, Perf_Curves_Abs/awgn_bler_tx1_mcs*.csv)."""
    import json
    d = json.load(open(GOLDEN_CSV))
    c = d["curves"] if which == "awgn_results" else d["curves_" + which]
    return {int(k): [tuple(r) for r in v["rows"]] for k, v in c.items()}


class OracleTrial:
    """Per-configuration state of the oracle's dlsim loop (25 PRB by default)."""

    def __init__(self, mcs, N_RB=25, subframe=7, npdcch=1, Nid_cell=0, rnti=0x1234, max_it=4, with_dci=True,
                 llr8=False):
        from test_rx_cpu import alloc, params
        self.p = params("C2", N_RB, mcs, npdcch, subframe, Nid_cell=Nid_cell, rnti=rnti)
        self.cfg = O.tx_cfg_from_params(self.p, subframe)
        self.fp = self.cfg.fp
        self.mcs, self.sf, self.npdcch, self.rnti, self.max_it = mcs, subframe, npdcch, rnti, max_it
        self.llr8 = llr8                       # dlsim -L: dlsch_decoding with phy_threegpplte_turbo_decoder8
        self.Qm = qm_of(mcs)
        self.alloc = alloc(N_RB)
        self.TBS = self.p.TBS[0]
        fp = self.fp
        self.N, self.spt, self.nsymb = fp.ofdm_symbol_size, fp.samples_per_tti, fp.symbols_per_tti
        self.dci = None
        if with_dci:
            table = np.zeros(800, np.int32)
            nCCE = O.get_nCCE(npdcch, fp)
            self.dci = [(DCI1_LEN[N_RB], 1, O.get_nCCE_offset(table, 2, nCCE, 0, rnti, subframe), rnti,
                         np.zeros(8, np.uint8))]
        grid = O.generate_pilots(fp, 512)[0]
        nxt = (subframe + 1) % 10
        self.tail = np.zeros(self.spt, np.int32)
        O.orc().orc_normal_prefix_mod(O.P(np.ascontiguousarray(grid[nxt * self.nsymb * self.N:])), O.P(self.tail),
                                      self.nsymb // 2, ctypes.byref(fp))
        self.offset_fac = 10 * math.log10(self.N / (12.0 * N_RB))

    def transmit(self, pay):
        txd, _, _ = O.tx_subframe(self.cfg, [pay], dci=self.dci)
        return txd[0]

    def tx_lev(self, txd):
        O.orc().orc_signal_energy.restype = ctypes.c_int32
        return O.orc().orc_signal_energy(O.P(np.ascontiguousarray(txd, np.int32)), self.spt)

    def channel(self, txd, snr_db):
        """dlsim's AWGN over [subframe | next subframe] with the restated reference generator."""
        L = O.orc()
        L.orc_awgn_sigma2.restype = ctypes.c_double
        sigma2 = L.orc_awgn_sigma2(self.tx_lev(txd), ctypes.c_double(self.offset_fac - snr_db))
        s = np.concatenate([txd, self.tail]).astype(np.int32)
        r = np.zeros_like(s)
        L.orc_awgn(O.P(s), O.P(r), len(s), ctypes.c_double(sigma2))
        return r

    def receive(self, rx2):
        """The UE on [subframe | next subframe] samples: unscrambled LLRs (G of them)."""
        fp, N, spt = self.fp, self.N, self.spt
        frame = np.zeros(10 * spt + N, np.int32)
        s = self.sf
        frame[s * spt:(s + 2) * spt] = rx2
        rxF = np.zeros(15 * N, np.int32)
        for Ns in (2 * s, 2 * s + 1):
            for l in range(7):
                assert O.slot_fep([frame], [rxF], fp, l, Ns) == 0
        nxt = np.zeros(15 * N, np.int32)
        assert O.slot_fep([frame], [nxt], fp, 0, (2 * s + 2) % 20) == 0
        est = O.chest_subframe(fp, rxF[:14 * N].copy(), nxt[:N].copy(), s)
        llr, _ = O.rx_pdsch_siso(fp, rxF[:14 * N], est, self.alloc, self.Qm, self.npdcch, s)
        G = len(llr)
        u = np.zeros(32 * (1 + G // 32), np.int16)
        u[:G] = llr
        O.dlsch_unscrambling(u, G, (self.rnti << 14) + (s << 9) + fp.Nid_cell)
        return u[:G]

    def decode(self, llr):
        from test_rx_cpu import decode_tb
        ops = None
        if self.llr8:
            ops = (O.rate_match_rx, O.subblock_deinterleave,
                   lambda d, K, ct, F: O.turbo_decode8(d, K, max_it=self.max_it, crc_type=ct, F=F))
        res, tb = decode_tb(llr, len(llr), self.TBS, self.Qm, C_ops=ops, max_it=self.max_it)
        return res, tb

    def trial(self, pay, snr_db):
        txd = self.transmit(pay)
        res, tb = self.decode(self.receive(self.channel(txd, snr_db)))
        err = any(it > self.max_it for it, _ in res)
        return err, res, tb


def randominit(seed):
    O.orc().orc_randominit(ctypes.c_uint32(seed))
