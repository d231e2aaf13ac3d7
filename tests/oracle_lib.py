"""ctypes bindings to the CPU oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this; the product
package (openair4g_amd) never does.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle.so")
REF_SO = os.path.join(ORACLE_DIR, "_ref", "libref_dfts.so")
REF_CODING_SO = os.path.join(ORACLE_DIR, "_ref", "libref_coding.so")

_orc = None


class OrcFrame(ctypes.Structure):
    _fields_ = [("N_RB_DL", ctypes.c_uint16), ("Nid_cell", ctypes.c_uint16), ("Ncp", ctypes.c_uint8),
                ("nushift", ctypes.c_uint8), ("mode1_flag", ctypes.c_uint8), ("nb_antennas_tx", ctypes.c_uint8),
                ("frame_type", ctypes.c_uint8), ("symbols_per_tti", ctypes.c_uint8),
                ("log2_symbol_size", ctypes.c_uint8), ("ofdm_symbol_size", ctypes.c_uint16),
                ("first_carrier_offset", ctypes.c_uint16), ("nb_prefix_samples", ctypes.c_uint16),
                ("nb_prefix_samples0", ctypes.c_uint16), ("samples_per_tti", ctypes.c_uint32),
                ("phich_resource", ctypes.c_uint8), ("phich_duration", ctypes.c_uint8), ("tdd_config", ctypes.c_uint8),
                ("nb_antennas_tx_eNB", ctypes.c_uint8)]


class OrcCw(ctypes.Structure):
    _fields_ = [("e", ctypes.c_void_p), ("mcs", ctypes.c_uint8), ("mimo_mode", ctypes.c_uint8),
                ("Nlayers", ctypes.c_uint8), ("rb_alloc", ctypes.c_uint32 * 4)]


class OrcTxCfg(ctypes.Structure):
    _fields_ = [("fp", OrcFrame), ("n_cw", ctypes.c_uint8), ("mimo_mode", ctypes.c_uint8),
                ("num_pdcch_symbols", ctypes.c_uint8), ("subframe", ctypes.c_uint8), ("rnti", ctypes.c_uint16),
                ("amp", ctypes.c_int16), ("sqrt_rho_a", ctypes.c_int16), ("sqrt_rho_b", ctypes.c_int16),
                ("Kmimo", ctypes.c_uint8), ("Mdlharq", ctypes.c_uint8), ("rb_alloc", ctypes.c_uint32 * 4),
                ("nb_rb", ctypes.c_uint16), ("mcs", ctypes.c_uint8 * 2), ("rvidx", ctypes.c_uint8 * 2),
                ("q", ctypes.c_uint8 * 2), ("TBS", ctypes.c_uint32 * 2), ("with_crs", ctypes.c_uint8)]


def build():
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR, "liboracle.so"], check=True)


def orc():
    global _orc
    if _orc is None:
        build()
        L = ctypes.CDLL(ORACLE_SO)
        L.orc_crc24a.restype = ctypes.c_uint32
        L.orc_crc24b.restype = ctypes.c_uint32
        L.orc_subblock_interleave.restype = ctypes.c_uint32
        L.orc_rate_match.restype = ctypes.c_uint32
        L.orc_rate_match.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_uint8, ctypes.c_uint32] + [ctypes.c_uint8] * 6
        L.orc_gold_generic.restype = ctypes.c_uint32
        L.orc_get_G.restype = ctypes.c_int
        L.orc_get_G.argtypes = [ctypes.c_uint16, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint16,
                                ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8]
        L.orc_modulation.restype = ctypes.c_int
        L.orc_modulation.argtypes = [ctypes.c_void_p, ctypes.c_int16, ctypes.c_uint32, ctypes.POINTER(OrcFrame),
                                     ctypes.c_uint8, ctypes.POINTER(OrcCw), ctypes.POINTER(OrcCw), ctypes.c_int16,
                                     ctypes.c_int16]
        L.orc_tx_subframe.restype = ctypes.c_int
        L.orc_turbo_encode.argtypes = [ctypes.c_void_p, ctypes.c_uint16, ctypes.c_void_p, ctypes.c_uint16,
                                       ctypes.c_uint16]
        L.orc_scramble.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32]
        L.orc_idft.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.orc_dft.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.orc_dft_twiddle_ab.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_slot_fep.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                   ctypes.POINTER(OrcFrame), ctypes.c_int, ctypes.c_uint8, ctypes.c_uint8,
                                   ctypes.c_int, ctypes.c_int]
        L.orc_ofdm_mod.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint16]
        L.orc_normal_prefix_mod.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint8, ctypes.POINTER(OrcFrame)]
        L.orc_generate_pilots.argtypes = [ctypes.c_void_p, ctypes.c_int16, ctypes.POINTER(OrcFrame), ctypes.c_uint16]
        L.orc_generate_pilots_subframe.argtypes = [ctypes.c_void_p, ctypes.c_int16, ctypes.POINTER(OrcFrame),
                                                   ctypes.c_uint8]
        L.orc_turbo_decoder16.restype = ctypes.c_uint8
        L.orc_turbo_decoder16.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint16, ctypes.c_uint8,
                                          ctypes.c_uint8, ctypes.c_uint8]
        L.orc_generate_dummy_w.restype = ctypes.c_uint32
        L.orc_rate_matching_turbo_rx.restype = ctypes.c_int
        L.orc_rate_matching_turbo_rx.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint32] + \
            [ctypes.c_uint8] * 7 + [ctypes.POINTER(ctypes.c_uint32)]
        L.orc_sub_block_deinterleaving_turbo.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
        _orc = L
    return _orc


def ref_dfts():
    """The reference's own lte_dfts.c (oracle/_ref), or None if it was not built here."""
    if not os.path.exists(REF_SO):
        return None
    return ctypes.CDLL(REF_SO)


_refc = None


def ref_coding():
    """The reference's own CRC and tail-biting convolutional coder (oracle/_ref/libref_coding.so:
    PHY/CODING/crc_byte.c, ccoding_byte_lte.c, compiled unmodified), initialised as the reference's
    phy_init_lte_top does (lte_init.c: crcTableInit, ccodelte_init), or None when it was not built
    here (the GPU box never has it)."""
    global _refc
    if _refc is None:
        if not os.path.exists(REF_CODING_SO):
            return None
        L = ctypes.CDLL(REF_CODING_SO)
        L.crcTableInit()
        L.ccodelte_init()
        L.crc24a.restype = ctypes.c_uint32
        L.crc24b.restype = ctypes.c_uint32
        L.crc16.restype = ctypes.c_uint32
        L.crc8.restype = ctypes.c_uint32
        L.ccodelte_encode.argtypes = [ctypes.c_int32, ctypes.c_uint8, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_uint16]
        _refc = L
    return _refc


def _aligned(n, dtype, align=64):
    itemsize = np.dtype(dtype).itemsize
    raw = np.zeros(n + align // itemsize, dtype=dtype)
    off = (-raw.ctypes.data % align) // itemsize
    return raw[off:off + n]


def ref_crc(data, bitlen, kind="24a"):
    L = ref_coding()
    a = _aligned(len(data) + 16, np.uint8)
    a[:len(data)] = data
    return {"24a": L.crc24a, "24b": L.crc24b, "16": L.crc16, "8": L.crc8}[kind](P(a), bitlen)


def P(a):
    return ctypes.c_void_p(a.ctypes.data)


def frame(N_RB_DL, Nid_cell=0, Ncp=0, nb_antennas_tx=1, mode1_flag=1, frame_type=0):
    fp = OrcFrame()
    assert orc().orc_init_frame(ctypes.byref(fp), N_RB_DL, Nid_cell, Ncp, nb_antennas_tx, mode1_flag,
                                frame_type) == 0
    return fp


def crc24a(data, bitlen):
    a = np.ascontiguousarray(data, dtype=np.uint8)
    return orc().orc_crc24a(P(a), bitlen)


def crc24b(data, bitlen):
    a = np.ascontiguousarray(data, dtype=np.uint8)
    return orc().orc_crc24b(P(a), bitlen)


def turbo_encode(c, f1, f2):
    c = np.ascontiguousarray(c, dtype=np.uint8)
    d = np.zeros(3 * 8 * len(c) + 12, dtype=np.uint8)
    orc().orc_turbo_encode(P(c), len(c), P(d), f1, f2)
    return d


def subblock(d, D):
    """d = d^(i) interleaved bytes (3D entries, no prefix).  Returns (R, w, d_with_side_effect)."""
    buf = np.full(96 + 3 * D + 16, 2, dtype=np.uint8)
    buf[96:96 + len(d)] = d
    R = (D + 31) >> 5
    w = np.zeros(3 * 32 * R, dtype=np.uint8)
    rtc = orc().orc_subblock_interleave(D, ctypes.c_void_p(buf.ctypes.data + 96), P(w))
    return rtc, w, buf


def rate_match(RTC, G, w, C, r, Qm, rvidx=0, Nl=1, Kmimo=1, Mdlharq=8, Nsoft=1827072):
    w = np.ascontiguousarray(w, dtype=np.uint8)
    e = np.zeros(G + 64, dtype=np.uint8)
    E = orc().orc_rate_match(RTC, G, P(w), P(e), C, Nsoft, Mdlharq, Kmimo, rvidx, Qm, Nl, r)
    return e[:E]


def generate_pcfich(cfi, amp, fp, grids, subframe):
    """orc_generate_pcfich on a list of frame grids (int32 arrays, modified in place)"""
    n = len(grids)
    gp = (ctypes.c_void_p * n)(*[g.ctypes.data for g in grids])
    return orc().orc_generate_pcfich(cfi, amp, ctypes.byref(fp), gp, subframe)


def pcfich_reg_mapping(fp):
    reg = (ctypes.c_uint16 * 4)()
    first = ctypes.c_uint8()
    orc().orc_pcfich_reg_mapping(ctypes.byref(fp), reg, ctypes.byref(first))
    return list(reg), first.value


def set_rm_limited(on):
    orc().orc_set_rm_limited(1 if on else 0)


def scramble(e, G, c_init):
    buf = np.zeros((1 + (G >> 5)) * 32 + 32, dtype=np.uint8)
    buf[:len(e)] = e
    orc().orc_scramble(P(buf), G, c_init)
    return buf


def idft(x, scale=1):
    x = np.ascontiguousarray(x, dtype=np.int16)
    y = np.zeros_like(x)
    orc().orc_idft(int(len(x) // 2).bit_length() - 1, P(x), P(y), scale)
    return y


def dft(x, scale=1):
    x = np.ascontiguousarray(x, dtype=np.int16)
    y = np.zeros_like(x)
    orc().orc_dft(int(len(x) // 2).bit_length() - 1, P(x), P(y), scale)
    return y


def dft_twiddle_ab(N, m):
    a = np.zeros(2, np.int16)
    b = np.zeros(2, np.int16)
    orc().orc_dft_twiddle_ab(N, m, P(a), P(b))
    return a, b


def slot_fep(rxdata, rxdataF, fp, l, Ns, sample_offset=0, no_prefix=0):
    """orc_slot_fep on lists of int32 arrays (modified in place); returns its code."""
    n = len(rxdata)
    rp = (ctypes.c_void_p * n)(*[a.ctypes.data for a in rxdata])
    fpp = (ctypes.c_void_p * n)(*[a.ctypes.data for a in rxdataF])
    return orc().orc_slot_fep(rp, fpp, ctypes.byref(fp), n, l, Ns, sample_offset, no_prefix)


def get_G(N_RB_DL, Ncp, mode1_flag, frame_type, nb_rb, rb_alloc, Qm, Nl, num_pdcch, subframe):
    ra = (ctypes.c_uint32 * 4)(*rb_alloc)
    return orc().orc_get_G(N_RB_DL, Ncp, mode1_flag, frame_type, nb_rb, ra, Qm, Nl, num_pdcch, subframe)


def tx_cfg_from_params(p, subframe):
    """Oracle config mirroring an openair4g_amd.TxParams (same semantics)."""
    c = OrcTxCfg()
    c.fp = frame(p.N_RB_DL, p.Nid_cell, p.Ncp, p.nb_antennas_tx, p.mode1_flag, p.frame_type)
    c.n_cw = p.n_cw
    c.mimo_mode = p.mimo_mode
    c.num_pdcch_symbols = p.num_pdcch_symbols
    c.subframe = subframe
    c.rnti = p.rnti
    c.amp = p.amp
    c.sqrt_rho_a = p.sqrt_rho_a
    c.sqrt_rho_b = p.sqrt_rho_b
    c.Kmimo = p.Kmimo
    c.Mdlharq = p.Mdlharq
    for i in range(4):
        c.rb_alloc[i] = p.rb_alloc[i]
    c.nb_rb = p.nb_rb
    for cw in range(2):
        c.mcs[cw] = p.mcs[cw]
        c.rvidx[cw] = p.rvidx[cw]
        c.q[cw] = p.q[cw]
        c.TBS[cw] = p.TBS[cw]
    c.with_crs = getattr(p, "with_crs", 0)
    return c


def tx_subframe(cfg, payloads, want_e=False, dci=None, n_common=0):
    """Run the oracle on one subframe.  payloads: list of byte arrays (TBS/8 each); dci: optional
    generate_dci_top items (dci_length, L, nCCE, rnti, pdu) for the control region.
    Returns (txdata [n_ant][spt] int32, txdataF [n_ant][14*N], e list)."""
    fp = cfg.fp
    n_ant = fp.nb_antennas_tx
    N = fp.ofdm_symbol_size
    bufs = []
    for cw in range(cfg.n_cw):
        b = np.zeros(cfg.TBS[cw] // 8 + 8, dtype=np.uint8)
        b[:cfg.TBS[cw] // 8] = payloads[cw][:cfg.TBS[cw] // 8]
        bufs.append(b)
    pay = (ctypes.c_void_p * 2)(*[P(b).value for b in bufs] + [None] * (2 - len(bufs)))
    txF = [np.zeros(14 * N, dtype=np.int32) for _ in range(n_ant)]
    txd = [np.zeros(fp.samples_per_tti, dtype=np.int32) for _ in range(n_ant)]
    fptrs = (ctypes.c_void_p * n_ant)(*[a.ctypes.data for a in txF])
    dptrs = (ctypes.c_void_p * n_ant)(*[a.ctypes.data for a in txd])
    es = [np.zeros(14 * 1200 * 6 + 64, dtype=np.uint8) for _ in range(cfg.n_cw)]
    eptrs = (ctypes.c_void_p * 2)(*[e.ctypes.data for e in es] + [None] * (2 - len(es)))
    if dci:
        rc = orc().orc_tx_subframe_dci(ctypes.byref(cfg), pay, fptrs, dptrs, eptrs if want_e else None,
                                       len(dci) - n_common, n_common, dci_allocs(dci))
    else:
        rc = orc().orc_tx_subframe(ctypes.byref(cfg), pay, fptrs, dptrs, eptrs if want_e else None)
    assert rc == 0
    return np.stack(txd), np.stack(txF), es


def modulation_count(cfg):
    """dlsch_modulation's return value (re_allocated) for the subframe of cfg."""
    tx_subframe(cfg, [np.zeros(cfg.TBS[cw] // 8 + 8, dtype=np.uint8) for cw in range(cfg.n_cw)])
    return orc().orc_last_re_allocated()


def generate_pilots(fp, amp, ntti=10):
    """Reference-layout frame grid(s) with CRS (pilots.c:43-168): [n_ant][ntti * 14 * N] int32."""
    N = fp.ofdm_symbol_size
    grids = [np.zeros(ntti * fp.symbols_per_tti * N, dtype=np.int32) for _ in range(fp.nb_antennas_tx)]
    ptrs = (ctypes.c_void_p * 2)(*[g.ctypes.data for g in grids] + [None] * (2 - len(grids)))
    orc().orc_generate_pilots(ptrs, amp, ctypes.byref(fp), ntti)
    return grids


def turbo_decode(y, K, max_it=8, crc_type=0, F=0):
    """phy_threegpplte_turbo_decoder16: y = 3K+12 int16 LLRs (positive = bit 1).
    Returns (iterations, decoded bytes)."""
    y = np.ascontiguousarray(y, dtype=np.int16)
    out = np.zeros(K // 8 + 8, dtype=np.uint8)
    it = orc().orc_turbo_decoder16(P(y), P(out), K, max_it, crc_type, F)
    return it, out[:K // 8]


def dummy_w(D):
    R = (D + 31) >> 5
    w = np.zeros(3 * 32 * R + 64, dtype=np.uint8)
    orc().orc_generate_dummy_w(D, P(w))
    return w


def dummy_w_F(D, F):
    """generate_dummy_w(D, w, F) of lte_rate_matching.c:293 (filler-aware NULL marks)."""
    R = (D + 31) >> 5
    w = np.zeros(3 * 32 * R + 64, dtype=np.uint8)
    orc().orc_generate_dummy_w_F(D, P(w), F)
    return w


def rate_match_rx(soft, K, G, C, r, Qm, rvidx=0, Nl=1, Kmimo=1, Mdlharq=8, w=None, clear=1, Nsoft=1827072, dw=None):
    """lte_rate_matching_turbo_rx: returns (w int16, E)."""
    D = K + 4
    R = (D + 31) >> 5
    dw = dummy_w(D) if dw is None else dw
    if w is None:
        w = np.zeros(3 * 32 * R + 64, dtype=np.int16)
    soft = np.ascontiguousarray(soft, dtype=np.int16)
    E = ctypes.c_uint32()
    rc = orc().orc_rate_matching_turbo_rx(R, G, P(w), P(dw), P(soft), C, Nsoft, Mdlharq, Kmimo, rvidx, clear, Qm, Nl,
                                          r, ctypes.byref(E))
    assert rc == 0
    return w, E.value


def subblock_deinterleave(w, K):
    """sub_block_deinterleaving_turbo: returns d (3K+12 int16, the decoder input)."""
    D = K + 4
    buf = np.zeros(96 + 3 * D + 64, dtype=np.int16)
    orc().orc_sub_block_deinterleaving_turbo(D, ctypes.c_void_p(buf.ctypes.data + 2 * 96),
                                             P(np.ascontiguousarray(w, dtype=np.int16)))
    return buf[96:96 + 3 * K + 12].copy()



# ------------------------------------------------------------------ control region (oai_oracle_ctrl.c)
class OrcDciAlloc(ctypes.Structure):
    """orc_dci_alloc_t = DCI_ALLOC_t (LTE_TRANSPORT/defs.h:734-749)"""
    _fields_ = [("dci_length", ctypes.c_uint8), ("L", ctypes.c_uint8), ("nCCE", ctypes.c_int32),
                ("ra_flag", ctypes.c_uint8), ("rnti", ctypes.c_uint16), ("format", ctypes.c_uint32),
                ("dci_pdu", ctypes.c_uint8 * 8)]


def dci_allocs(items, cls=OrcDciAlloc):
    """items: list of (dci_length, L, nCCE, rnti, pdu bytes) -> ctypes array"""
    arr = (cls * max(1, len(items)))()
    for a, (ln, L, ncce, rnti, pdu) in zip(arr, items):
        a.dci_length, a.L, a.nCCE, a.rnti = ln, L, ncce, rnti
        for i, b in enumerate(pdu[:8]):
            a.dci_pdu[i] = int(b)
    return arr


def crc16(data, bitlen):
    a = np.zeros(len(data) + 8, np.uint8)
    a[:len(data)] = data
    orc().orc_crc16.restype = ctypes.c_uint32
    return orc().orc_crc16(P(a), bitlen)


def ccode_encode(data, numbits, add_crc, rnti):
    a = np.zeros(len(data) + 8, np.uint8)
    a[:len(data)] = data
    out = np.zeros(3 * (numbits + 16) + 16, np.uint8)
    orc().orc_ccodelte_encode(numbits, add_crc, P(a), P(out), ctypes.c_uint16(rnti))
    return out[:3 * (numbits + (16 if add_crc == 2 else 0))]


def ref_ccode_encode(data, numbits, add_crc, rnti):
    L = ref_coding()
    a = np.zeros(len(data) + 8, np.uint8)
    a[:len(data)] = data
    out = np.zeros(3 * (numbits + 16) + 16, np.uint8)
    L.ccodelte_encode(numbits, add_crc, P(a), P(out), rnti)
    return out[:3 * (numbits + (16 if add_crc == 2 else 0))]


def generate_dci_top(items, n_common, amp, fp, grids, subframe):
    """orc_generate_dci_top on frame grids (int32 arrays, modified in place); returns num_pdcch_symbols"""
    L = orc()
    L.orc_generate_dci_top.restype = ctypes.c_uint8
    arr = dci_allocs(items)
    gp = (ctypes.c_void_p * len(grids))(*[g.ctypes.data for g in grids])
    return L.orc_generate_dci_top(len(items) - n_common, n_common, arr, 0, ctypes.c_int16(amp), ctypes.byref(fp),
                                  gp, subframe)


def last_dci_e():
    L = orc()
    L.orc_last_dci_e.restype = ctypes.POINTER(ctypes.c_uint8)
    n = ctypes.c_uint32()
    p = L.orc_last_dci_e(ctypes.byref(n))
    return np.ctypeslib.as_array(p, shape=(n.value,)).copy() if n.value else np.zeros(0, np.uint8)


def get_nCCE(npdcch, fp, mi=1):
    orc().orc_get_nCCE.restype = ctypes.c_uint16
    return orc().orc_get_nCCE(npdcch, ctypes.byref(fp), mi)


def get_nquad(npdcch, fp, mi=1):
    orc().orc_get_nquad.restype = ctypes.c_uint16
    return orc().orc_get_nquad(npdcch, ctypes.byref(fp), mi)


def phich_reg_mapping(fp):
    reg = (ctypes.c_uint16 * (56 * 3))()
    n = orc().orc_phich_reg_mapping(ctypes.byref(fp), reg)
    return [tuple(reg[3 * i:3 * i + 3]) for i in range(n)]


def get_nCCE_offset(table, L, nCCE, common, rnti, subframe):
    return orc().orc_get_nCCE_offset(table.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), L, nCCE, common, rnti,
                                     subframe)


# ---- synchronisation / broadcast / HARQ-indicator channels (oracle/oai_oracle_sync.c) ----
class OrcPbch(ctypes.Structure):
    _fields_ = [("pbch_d", ctypes.c_uint8 * (96 + 120)), ("pbch_w", ctypes.c_uint8 * 360),
                ("pbch_e", ctypes.c_uint8 * 1920)]


def _grid_ptrs(grids):
    return (ctypes.c_void_p * len(grids))(*[g.ctypes.data for g in grids])


def primary_synch(nid2):
    out = np.zeros(144, dtype=np.int16)
    orc().orc_primary_synch(nid2, P(out))
    return out


def sss_seq(nid_cell, sf5):
    d = np.zeros(62, dtype=np.int16)
    orc().orc_sss_seq(nid_cell, int(sf5), P(d))
    return d


def generate_pss(grids, amp, fp, symbol, slot_offset):
    return orc().orc_generate_pss(_grid_ptrs(grids), ctypes.c_int16(amp), ctypes.byref(fp), symbol, slot_offset)


def generate_sss(grids, amp, fp, symbol, slot_offset):
    return orc().orc_generate_sss(_grid_ptrs(grids), ctypes.c_int16(amp), ctypes.byref(fp), symbol, slot_offset)


def generate_pbch(state, grids, amp, fp, pdu, frame_mod4):
    """orc_generate_pbch on the subframe-0 grids (state: OrcPbch kept across frame_mod4, as eNB_pbch)"""
    pdu = np.ascontiguousarray(pdu, dtype=np.uint8)
    return orc().orc_generate_pbch(ctypes.byref(state), _grid_ptrs(grids), amp, ctypes.byref(fp), P(pdu), frame_mod4)


def generate_phich(fp, amp, nseq, ngroup, hi, subframe, grids):
    return orc().orc_generate_phich(ctypes.byref(fp), ctypes.c_int16(amp), nseq, ngroup, hi, subframe,
                                    _grid_ptrs(grids))


# ---- UE PDSCH demodulation (oracle/oai_oracle_rx.c) ----
def rx_pdsch_siso(fp, rxdataF, dl_ch, rb_alloc, Qm, num_pdcch, subframe):
    L = orc()
    rxdataF = np.ascontiguousarray(rxdataF, dtype=np.int32)
    dl_ch = np.ascontiguousarray(dl_ch, dtype=np.int32)
    out = np.zeros(14 * 1200 * 6 + 64, dtype=np.int16)
    sh = ctypes.c_uint8()
    ra = (ctypes.c_uint32 * 4)(*rb_alloc)
    n = L.orc_rx_pdsch_siso(ctypes.byref(fp), P(rxdataF), P(dl_ch), ra, Qm, num_pdcch, subframe, P(out),
                            ctypes.byref(sh))
    assert n >= 0
    return out[:n], sh.value


def dlsch_unscrambling(llr, G, c_init):
    orc().orc_dlsch_unscrambling(P(llr), G, ctypes.c_uint32(c_init))
    return llr


def adjust_G2(fp, rb_alloc, subframe, symbol):
    ra = (ctypes.c_uint32 * 4)(*rb_alloc)
    return orc().orc_adjust_G2(ctypes.byref(fp), ra, subframe, symbol)


def chest_filters(k):
    out = np.zeros((6, 24), np.int16)
    orc().orc_chest_filters(k, P(out))
    return out


def chest_dc_filters(k):
    out = np.zeros((2, 24), np.int16)
    orc().orc_chest_dc_filters(k, P(out))
    return out


def gold_table(fp):
    t = np.zeros((20, 2, 14), np.uint32)
    orc().orc_lte_gold_table(ctypes.byref(fp), P(t))
    return t


def dl_channel_estimation(fp, gold, rxdataF, est, Ns, p, l, symbol):
    """lte_dl_channel_estimation on one subframe grid rxdataF [nsymb*N] into est [nsymb*N] (in place)."""
    rc = orc().orc_lte_dl_channel_estimation(ctypes.byref(fp), P(gold), P(np.ascontiguousarray(rxdataF, np.int32)),
                                             P(est), Ns, p, l, symbol)
    assert rc == 0
    return est


def chest_subframe(fp, rxF, rxF_next0, sf, p=0):
    """The estimates rx_pdsch reads for every symbol of subframe sf, in dlsim's call order
    (dlsim.c:2907-2931 -> slot_fep.c:180-199): pilot symbols 0, 4, 7, 11 of slots 2 sf, 2 sf + 1
    and then symbol 0 of slot 2 sf + 2, which interpolates rows 12 / 13 (and overwrites row 0 with
    the next subframe's estimate, so the current row 0 is kept).  Extended prefix: 0, 3, 6, 9."""
    N = fp.ofdm_symbol_size
    nsymb = 14 if fp.Ncp == 0 else 12
    lp = 4 if fp.Ncp == 0 else 3
    est = np.zeros(nsymb * N, np.int32)
    g = gold_table(fp)
    for Ns, l, sym in ((2 * sf, 0, 0), (2 * sf, lp, lp), (2 * sf + 1, 0, nsymb // 2), (2 * sf + 1, lp, nsymb // 2 + lp)):
        dl_channel_estimation(fp, g, rxF, est, Ns, p, l, sym)
    row0 = est[:N].copy()
    nxt = np.zeros(nsymb * N, np.int32)
    nxt[:N] = rxF_next0
    dl_channel_estimation(fp, g, nxt, est, (2 * sf + 2) % 20, p, 0, 0)
    est[:N] = row0
    return est


def ulsch_decode(e, B, G, Qm, rvidx=0, max_it=8, Mdlharq=8):
    """ulsch_decoding.c:1208-1350 on one TB's soft bits e (first round): per code block r,
    generate_dummy_w(4 + K_r, F if r == 0), lte_rate_matching_turbo_rx (clear), sub-block
    deinterleaving, phy_threegpplte_turbo_decoder16 (CRC24_B if C > 1 else CRC24_A with F).
    Returns [(iterations, bytes K_r / 8)] per block."""
    import spec_model as S
    blocks, F = S.segment([0] * B)
    C = len(blocks)
    e = np.ascontiguousarray(e, dtype=np.int16)
    off, out = 0, []
    for r, blk in enumerate(blocks):
        K = len(blk)
        dw = dummy_w_F(K + 4, F if r == 0 else 0)
        w, E = rate_match_rx(e[off:], K, G, C, r, Qm, rvidx=rvidx, Mdlharq=Mdlharq, dw=dw)
        off += E
        d = subblock_deinterleave(w, K)
        out.append(turbo_decode(d, K, max_it=max_it, crc_type=1 if C > 1 else 0, F=(F if C == 1 else 0)))
    return out


def ulsch_decode_harq(e, B, G, Qm, rvidx, clear, w_state, max_it=8, Mdlharq=8):
    """One HARQ round of the per-block chain (dlsch_decoding.c:348-383): lte_rate_matching_turbo_rx
    into the kept soft buffers w_state[r] (int16 arrays, updated in place; clear = 1 on round 0),
    sub-block deinterleaving, turbo decoding.  Returns [(iterations, bytes)] per block."""
    import spec_model as S
    blocks, F = S.segment([0] * B)
    C = len(blocks)
    e = np.ascontiguousarray(e, dtype=np.int16)
    off, out = 0, []
    for r, blk in enumerate(blocks):
        K = len(blk)
        dw = dummy_w_F(K + 4, F if r == 0 else 0)
        w, E = rate_match_rx(e[off:], K, G, C, r, Qm, rvidx=rvidx, Mdlharq=Mdlharq, dw=dw, w=w_state[r], clear=clear)
        off += E
        d = subblock_deinterleave(w, K)
        out.append(turbo_decode(d, K, max_it=max_it, crc_type=1 if C > 1 else 0, F=(F if C == 1 else 0)))
    return out


def turbo_decode8(y, K, max_it=8, crc_type=0, F=0):
    """phy_threegpplte_turbo_decoder8 (oracle/oai_oracle_td8.c): y = 3K+12 int16 LLRs (4 more
    entries are read, zero here).  Returns (iterations, decoded bytes)."""
    buf = np.zeros(3 * K + 64, dtype=np.int16)
    y = np.asarray(y, dtype=np.int16)
    buf[:len(y)] = y
    out = np.zeros(K // 8 + 8, dtype=np.uint8)
    orc().orc_turbo_decoder8.restype = ctypes.c_uint8
    it = orc().orc_turbo_decoder8(P(buf), P(out), K, max_it, crc_type, F)
    return it, out[:K // 8]


def rx_pdsch_tm3(fp, rxF, est, rb_alloc, Qm0, Qm1, mcs0, num_pdcch, subframe):
    """orc_rx_pdsch_tm3: rxF = [nb_rx][nsymb*N], est[(p, a)] = [nsymb*N] estimates of port p at RX a.
    Returns (codeword-0 LLRs, log2_maxh)."""
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
    n = orc().orc_rx_pdsch_tm3(ctypes.byref(fp), nb_rx, rp, ep, ra, Qm0, Qm1, mcs0, num_pdcch, subframe, P(out),
                               ctypes.byref(sh))
    assert n >= 0
    return out[:n], sh.value


def rx_pdsch_tm2(fp, rxF, est, rb_alloc, Qm, num_pdcch, subframe, check=True):
    """orc_rx_pdsch_tm2 (ALAMOUTI): rxF = [nb_rx][nsymb*N], est[(p, a)] = [nsymb*N] estimates of port p
    at RX a.  Returns (LLRs, log2_maxh); with check=False a refusal returns (None, 0)."""
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
    n = orc().orc_rx_pdsch_tm2(ctypes.byref(fp), nb_rx, rp, ep, ra, Qm, num_pdcch, subframe, P(out), ctypes.byref(sh))
    if not check and n < 0:
        return None, 0
    assert n >= 0
    return out[:n], sh.value


def rx_pdsch_tm3_qq(fp, rxF, est, rb_alloc, mcs0, num_pdcch, subframe, check=True):
    """orc_rx_pdsch_tm3_qq: TM3 with both codewords QPSK (the interference-aware qpsk_qpsk LLRs of
    both streams).  Returns (LLRs of codeword 0, LLRs of codeword 1, log2_maxh)."""
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
    n = orc().orc_rx_pdsch_tm3_qq(ctypes.byref(fp), nb_rx, rp, ep, ra, mcs0, num_pdcch, subframe, P(o0), P(o1),
                                  ctypes.byref(sh))
    if not check and n < 0:
        return None, None, 0
    assert n >= 0
    return o0[:n], o1[:n], sh.value


# ---- lte_est_freq_offset (lte_est_freq_offset.c:45-193), dot_product (cdot_prod.c:40-118),
#      dl_ch_estimates_time (lte_dl_channel_estimation.c:704-738) ----
REF_TOOLS_SO = os.path.join(ORACLE_DIR, "_ref", "libref_tools.so")


def ref_tools():
    """The reference's PHY/TOOLS signal_energy.c / cdot_prod.c / log2_approx.c compiled unmodified
    (oracle/_ref/libref_tools.so), or None when it was not built here."""
    if not os.path.exists(REF_TOOLS_SO):
        return None
    L = ctypes.CDLL(REF_TOOLS_SO)
    if hasattr(L, "dot_product"):
        L.dot_product.restype = ctypes.c_int32
        L.dot_product.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint8]
        L.log2_approx.restype = ctypes.c_uint8
        L.log2_approx.argtypes = [ctypes.c_uint32]
    return L


def dot_product(x, y, N, shift):
    L = orc()
    L.orc_dot_product.restype = ctypes.c_int32
    L.orc_dot_product.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint8]
    return L.orc_dot_product(P(np.ascontiguousarray(x, np.int16)), P(np.ascontiguousarray(y, np.int16)), N, shift)


def fo_omega(fp, plane0, l):
    L = orc()
    L.orc_fo_omega.restype = ctypes.c_int32
    return L.orc_fo_omega(ctypes.byref(fp), P(np.ascontiguousarray(plane0, np.int32)), l)


class FreqOffsetState:
    """The reference's *freq_offset and static first_run for a sequence of lte_est_freq_offset calls."""

    def __init__(self):
        self.f = ctypes.c_int(0)
        self.first = ctypes.c_int(1)

    def call(self, fp, plane0, l, reset=0):
        if reset:
            self.first.value = 1
        om = fo_omega(fp, plane0, l)
        orc().orc_fo_update(fp.Ncp, ctypes.c_int32(om), ctypes.byref(self.f), ctypes.byref(self.first))
        return self.f.value


def chest_time(fp, plane):
    """dl_ch_estimates_time of one estimate plane (int32 [>= N + 8])."""
    out = np.zeros(fp.ofdm_symbol_size if 7 <= fp.log2_symbol_size <= 11 else 512, np.int32)
    a = _aligned(plane.size, np.int32)
    a[:] = plane
    orc().orc_chest_time(ctypes.byref(fp), P(a), P(out))
    return out


# ---- the reference's own rate matcher and Gold generator (oracle/_ref/libref_rm.so: PHY/CODING/
#      lte_rate_matching.c, oracle/_ref/libref_gold.so: PHY/LTE_REFSIG/lte_gold.c, both compiled
#      unmodified; present only in the build container) ----
REF_RM_SO = os.path.join(ORACLE_DIR, "_ref", "libref_rm.so")
REF_GOLD_SO = os.path.join(ORACLE_DIR, "_ref", "libref_gold.so")
_refrm = None
_refgold = None
U8, U16, U32 = ctypes.c_uint8, ctypes.c_uint16, ctypes.c_uint32
VP = ctypes.c_void_p


def ref_rm():
    """lte_rate_matching.c compiled unmodified, or None when it was not built here."""
    global _refrm
    if _refrm is None:
        if not os.path.exists(REF_RM_SO):
            return None
        L = ctypes.CDLL(REF_RM_SO)
        L.sub_block_interleaving_turbo.restype = U32
        L.sub_block_interleaving_turbo.argtypes = [U32, VP, VP]
        L.sub_block_deinterleaving_turbo.restype = None
        L.sub_block_deinterleaving_turbo.argtypes = [U32, VP, VP]
        L.generate_dummy_w.restype = U32
        L.generate_dummy_w.argtypes = [U32, VP, U8]
        L.lte_rate_matching_turbo.restype = U32
        L.lte_rate_matching_turbo.argtypes = [U32, U32, VP, VP, U8, U32, U8, U8, U8, U8, U8, U8, U8, U8]
        L.lte_rate_matching_turbo_rx.restype = ctypes.c_int
        L.lte_rate_matching_turbo_rx.argtypes = [U32, U32, VP, VP, VP, U8, U32, U8, U8, U8, U8, U8, U8, U8,
                                                 ctypes.POINTER(U32)]
        L.sub_block_interleaving_cc.restype = U32
        L.sub_block_interleaving_cc.argtypes = [U32, VP, VP]
        L.lte_rate_matching_cc.restype = U32
        L.lte_rate_matching_cc.argtypes = [U32, U16, VP, VP]
        _refrm = L
    return _refrm


def ref_gold():
    """lte_gold.c compiled unmodified (+ the ctypes glue ref_glue_gold.c), or None."""
    global _refgold
    if _refgold is None:
        if not os.path.exists(REF_GOLD_SO):
            return None
        L = ctypes.CDLL(REF_GOLD_SO)
        L.lte_gold_generic.restype = U32
        L.lte_gold_generic.argtypes = [ctypes.POINTER(U32), ctypes.POINTER(U32), U8]
        L.ref_glue_lte_gold.argtypes = [ctypes.c_int, U16, VP]
        _refgold = L
    return _refgold


def _dbuf(d, D, prefix=96):
    """d (3D stream entries, no prefix) behind a `prefix`-byte LTE_NULL prefix, as new_eNB_dlsch lays
    out harq->d (dlsch_coding.c:202-206), with slack after it for the d[3D+2] side effect."""
    buf = _aligned(prefix + 3 * D + 64, np.uint8)
    buf[:] = 2
    buf[prefix:prefix + len(d)] = d
    return buf


def ref_subblock(d, D):
    """sub_block_interleaving_turbo on d (3D entries).  Returns (R, w, d buffer after the call)."""
    buf = _dbuf(d, D)
    R = (D + 31) >> 5
    w = _aligned(3 * 32 * R + 64, np.uint8)
    rtc = ref_rm().sub_block_interleaving_turbo(D, VP(buf.ctypes.data + 96), P(w))
    return rtc, w[:3 * 32 * R].copy(), buf


def ref_rate_match(RTC, G, w, C, r, Qm, rvidx=0, Nl=1, Kmimo=1, Mdlharq=8, Nsoft=1827072):
    wa = _aligned(len(w) + 64, np.uint8)
    wa[:len(w)] = w
    e = _aligned(G + 64, np.uint8)
    E = ref_rm().lte_rate_matching_turbo(RTC, G, P(wa), P(e), C, Nsoft, Mdlharq, Kmimo, rvidx, Qm, Nl, r, 0, 0)
    return e[:E].copy()


def ref_dummy_w(D, F=0):
    R = (D + 31) >> 5
    w = _aligned(3 * 32 * R + 64, np.uint8)
    rtc = ref_rm().generate_dummy_w(D, P(w), F)
    return rtc, w[:3 * 32 * R].copy()


def ref_rate_match_rx(RTC, G, w, dummy_w, soft, C, r, Qm, rvidx=0, clear=1, Nl=1, Kmimo=1, Mdlharq=8,
                      Nsoft=1827072):
    """lte_rate_matching_turbo_rx: w (int16, modified copy returned), returns (ret, E, w)."""
    wa = _aligned(len(w) + 32, np.int16)
    wa[:len(w)] = w
    dw = _aligned(len(dummy_w) + 64, np.uint8)
    dw[:len(dummy_w)] = dummy_w
    sa = _aligned(len(soft) + 32, np.int16)
    sa[:len(soft)] = soft
    E = U32()
    ret = ref_rm().lte_rate_matching_turbo_rx(RTC, G, P(wa), P(dw), P(sa), C, Nsoft, Mdlharq, Kmimo, rvidx, clear,
                                              Qm, Nl, r, ctypes.byref(E))
    return ret, E.value, wa[:len(w)].copy()


def ref_deinterleave(D, w, pad=96):
    """sub_block_deinterleaving_turbo: writes d - 3 ND .. (the caller's d has room in front)."""
    d = _aligned(pad + 3 * D + 64, np.int16)
    wa = _aligned(len(w) + 32, np.int16)
    wa[:len(w)] = w
    ref_rm().sub_block_deinterleaving_turbo(D, VP(d.ctypes.data + 2 * pad), P(wa))
    return d


def ref_gold_words(c_init, n):
    """n words of lte_gold_generic from c_init (reset on the first call, as dlsch_scrambling does)."""
    L = ref_gold()
    x1, x2 = U32(0), U32(c_init)
    out = np.empty(n, np.uint32)
    for i in range(n):
        out[i] = L.lte_gold_generic(ctypes.byref(x1), ctypes.byref(x2), 1 if i == 0 else 0)
    return out


def ref_gold_table(Ncp, Nid_cell):
    t = np.zeros((20, 2, 14), np.uint32)
    ref_gold().ref_glue_lte_gold(Ncp, Nid_cell, P(t))
    return t


# ---- the reference's own segmentation and OFDM modulator (oracle/_ref/libref_seg.so: PHY/CODING/
#      lte_segmentation.c, oracle/_ref/libref_ofdm.so: PHY/MODULATION/ofdm_mod.c, both compiled
#      unmodified; present only in the build container) ----
REF_SEG_SO = os.path.join(ORACLE_DIR, "_ref", "libref_seg.so")
REF_OFDM_SO = os.path.join(ORACLE_DIR, "_ref", "libref_ofdm.so")
_refseg = None
_refofdm = None


def ref_seg():
    """lte_segmentation.c compiled unmodified (its crc24b from libref_coding.so, whose table
    ref_coding() initialises), or None when it was not built here."""
    global _refseg
    if _refseg is None:
        if not os.path.exists(REF_SEG_SO) or ref_coding() is None:
            return None
        L = ctypes.CDLL(REF_SEG_SO)
        L.lte_segmentation.restype = ctypes.c_int
        L.lte_segmentation.argtypes = [VP, ctypes.POINTER(VP), U32] + [ctypes.POINTER(U32)] * 6
        _refseg = L
    return _refseg


def ref_ofdm():
    """ofdm_mod.c compiled unmodified (+ the ctypes glue ref_glue_ofdm.c), or None."""
    global _refofdm
    if _refofdm is None:
        if not os.path.exists(REF_OFDM_SO):
            return None
        # RTLD_LAZY: logRecord (LOG_D on the PMCH branch, ofdm_mod.c:244/260) stays unbound; no
        # case here reaches that branch (ref_glue_ofdm.c)
        L = ctypes.CDLL(REF_OFDM_SO, mode=os.RTLD_LAZY | os.RTLD_LOCAL)
        L.PHY_ofdm_mod.restype = None
        L.PHY_ofdm_mod.argtypes = [VP, VP, ctypes.c_ubyte, ctypes.c_ubyte, ctypes.c_ushort, ctypes.c_int]
        L.ref_glue_normal_prefix_mod.argtypes = [VP, VP, U8, VP]
        L.ref_glue_do_OFDM_mod.argtypes = [ctypes.POINTER(VP), ctypes.POINTER(VP), U32, U16, VP]
        _refofdm = L
    return _refofdm


def seg_out_buffers(C, fill=0xA5, size=768 + 8 + 3):
    """output_buffers for lte_segmentation: C (>= 1) byte buffers pre-filled with `fill`, so bytes the
    function does not write stay visible."""
    bufs = [_aligned(size, np.uint8) for _ in range(max(C, 1))]
    for b in bufs:
        b[:] = fill
    return bufs


def ref_segmentation(B, data=None, C_hint=16):
    """lte_segmentation(input, outputs, B, ...): (ret, (C, Cplus, Cminus, Kplus, Kminus, F), buffers).
    Without `data` both pointers are NULL (the parameter-only call of dlsch_coding.c)."""
    vals = [U32(0) for _ in range(6)]
    if data is None:
        ret = ref_seg().lte_segmentation(None, None, B, *[ctypes.byref(v) for v in vals])
        return ret, tuple(v.value for v in vals), None
    inp = _aligned(len(data) + 16, np.uint8)
    inp[:len(data)] = data
    bufs = seg_out_buffers(C_hint)
    ptrs = (VP * len(bufs))(*[b.ctypes.data for b in bufs])
    ret = ref_seg().lte_segmentation(P(inp), ptrs, B, *[ctypes.byref(v) for v in vals])
    return ret, tuple(v.value for v in vals), bufs


def frame_geometry(fp):
    """The ofdm_mod.c glue's geometry vector from an OrcFrame / FrameParms."""
    return np.array([fp.N_RB_DL, fp.Ncp, fp.nb_antennas_tx, fp.ofdm_symbol_size, fp.log2_symbol_size,
                     fp.nb_prefix_samples, fp.nb_prefix_samples0, fp.symbols_per_tti, fp.samples_per_tti], np.int32)


# ---- dlsch_modulation.c / dlsch_scrambling.c compiled unmodified (oracle/_ref/libref_mod.so) ----
REF_MOD_SO = os.path.join(ORACLE_DIR, "_ref", "libref_mod.so")
_refmod = None


class RefCw(ctypes.Structure):
    """ref_cw_t of oracle/ref_glue_mod.c"""
    _fields_ = [("e", VP), ("G", ctypes.c_int32), ("mcs", U8), ("mimo_mode", U8), ("Nlayers", U8),
                ("first_layer", U8), ("rb_alloc", U32 * 4), ("nb_rb", U16), ("pmi_alloc", U16)]


def ref_mod():
    """dlsch_modulation.c + dlsch_scrambling.c compiled unmodified (+ the ctypes glue ref_glue_mod.c),
    or None when they were not built here."""
    global _refmod
    if _refmod is None:
        if not os.path.exists(REF_MOD_SO) or ref_gold() is None:
            return None
        # RTLD_LAZY: logRecord (LOG_E / LOG_W on the unsupported-mode branches) stays unbound
        L = ctypes.CDLL(REF_MOD_SO, mode=os.RTLD_LAZY | os.RTLD_LOCAL)
        L.ref_glue_dlsch_modulation.restype = ctypes.c_int
        L.ref_glue_dlsch_modulation.argtypes = [ctypes.POINTER(VP), ctypes.c_int16, U32, VP, U8,
                                                ctypes.POINTER(RefCw), ctypes.POINTER(RefCw), ctypes.c_int16,
                                                ctypes.c_int16]
        L.ref_glue_dlsch_scrambling.argtypes = [VP, ctypes.c_int, U16, U16, U8, U8]
        L.ref_glue_qam_tables.argtypes = [VP, VP]
        L.ref_glue_pcfich.argtypes = [U8, ctypes.c_int16, VP, ctypes.POINTER(VP), U8, VP, VP]
        _refmod = L
    return _refmod


def mod_frame_words(fp):
    """ref_glue_mod.c's frame vector from an OrcFrame"""
    return np.array([fp.N_RB_DL, fp.Ncp, fp.nb_antennas_tx, fp.ofdm_symbol_size, fp.first_carrier_offset,
                     fp.nushift, fp.mode1_flag, fp.frame_type, fp.Nid_cell], dtype=np.int32)


def _grids(fp):
    n = 10 * fp.symbols_per_tti * fp.ofdm_symbol_size
    grids = [np.zeros(n, dtype=np.int32) for _ in range(fp.nb_antennas_tx)]
    ptrs = (VP * max(2, len(grids)))(*([g.ctypes.data for g in grids] + [None] * max(0, 2 - len(grids))))
    return grids, ptrs


def ref_modulation(fp, amp, subframe, num_pdcch, cws, sqrt_rho_a=8192, sqrt_rho_b=8192):
    """The reference's dlsch_modulation over frame grids: (return value, [grid per TX antenna]).
    cws: 1 or 2 dicts {e (uint8 0/1, >= the bits consumed), mcs, mimo_mode, rb_alloc (4 words)}."""
    grids, ptrs = _grids(fp)
    keep = []
    rc = []
    for cw in cws:
        e = np.ascontiguousarray(cw["e"][:14 * 1200 * 6], dtype=np.uint8)   # MAX_NUM_CHANNEL_BITS
        keep.append(e)
        ra = cw["rb_alloc"]
        c = RefCw(e=e.ctypes.data, G=len(e), mcs=cw["mcs"], mimo_mode=cw["mimo_mode"], Nlayers=cw.get("Nlayers", 1),
                  first_layer=0, nb_rb=sum(bin(int(w)).count("1") for w in ra), pmi_alloc=0)
        for i in range(4):
            c.rb_alloc[i] = int(ra[i])
        rc.append(c)
    f = mod_frame_words(fp)
    ret = ref_mod().ref_glue_dlsch_modulation(ptrs, amp, subframe, f.ctypes.data, num_pdcch, ctypes.byref(rc[0]),
                                              ctypes.byref(rc[1]) if len(rc) > 1 else None, sqrt_rho_a,
                                              sqrt_rho_b)
    return ret, grids


def orc_modulation_grids(fp, amp, subframe, num_pdcch, cws, sqrt_rho_a=8192, sqrt_rho_b=8192):
    """The oracle's orc_modulation with the same arguments as ref_modulation."""
    grids, ptrs = _grids(fp)
    keep = []
    oc = []
    for cw in cws:
        e = np.ascontiguousarray(cw["e"], dtype=np.uint8)
        keep.append(e)
        c = OrcCw(e=e.ctypes.data, mcs=cw["mcs"], mimo_mode=cw["mimo_mode"], Nlayers=cw.get("Nlayers", 1))
        for i in range(4):
            c.rb_alloc[i] = int(cw["rb_alloc"][i])
        oc.append(c)
    ret = orc().orc_modulation(ptrs, amp, subframe, ctypes.byref(fp), num_pdcch, ctypes.byref(oc[0]),
                               ctypes.byref(oc[1]) if len(oc) > 1 else None, sqrt_rho_a, sqrt_rho_b)
    return ret, grids


def ref_scrambling(e, G, rnti, Nid_cell, q, Ns):
    """The reference's dlsch_scrambling of e[0 .. G) (returns the 32 (1 + G / 32) entries it writes)."""
    n = 32 * (1 + (G >> 5))
    buf = np.zeros(n, dtype=np.uint8)
    src = np.asarray(e, dtype=np.uint8)
    buf[:min(n, len(src))] = src[:n]
    ref_mod().ref_glue_dlsch_scrambling(buf.ctypes.data, G, rnti, Nid_cell, q, Ns)
    return buf


def ref_pcfich(cfi, amp, fp, subframe):
    """The reference's generate_pcfich_reg_mapping + generate_pcfich (pcfich.c, compiled unmodified into
    libref_mod.so) over zeroed frame grids: (grids, reg[4], first_idx)."""
    grids, ptrs = _grids(fp)
    reg = np.zeros(4, np.uint16)
    first = np.zeros(1, np.uint8)
    f = mod_frame_words(fp)
    ref_mod().ref_glue_pcfich(cfi, amp, f.ctypes.data, ptrs, subframe, reg.ctypes.data, first.ctypes.data)
    return grids, [int(r) for r in reg], int(first[0])


# ---- dlsch_llr_computation.c compiled unmodified (oracle/_ref/libref_llr.so) ----
REF_LLR_SO = os.path.join(ORACLE_DIR, "_ref", "libref_llr.so")
_refllr = None


def ref_llr():
    """dlsch_llr_computation.c compiled unmodified (+ ref_glue_llr.c), or None when not built here."""
    global _refllr
    if _refllr is None:
        if not os.path.exists(REF_LLR_SO):
            return None
        L = ctypes.CDLL(REF_LLR_SO, mode=os.RTLD_LAZY | os.RTLD_LOCAL)
        L.ref_glue_qam_llr.restype = ctypes.c_int
        L.ref_glue_qam_llr.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, VP, VP, VP, VP, U8, U16,
                                       U16]
        for f in ("qpsk_qpsk", "qpsk_qam16", "qpsk_qam64"):
            getattr(L, f).restype = None
        L.qpsk_qpsk.argtypes = [VP, VP, VP, VP, ctypes.c_int]
        L.qpsk_qam16.argtypes = [VP, VP, VP, VP, VP, ctypes.c_int32]
        L.qpsk_qam64.argtypes = [VP, VP, VP, VP, VP, ctypes.c_int32]
        _refllr = L
    return _refllr


def aligned(a, align=64):
    """a copy of array a whose data starts on an `align`-byte boundary (the reference's SSE loads are
    aligned ones)"""
    a = np.ascontiguousarray(a)
    raw = np.zeros(a.nbytes + align, np.uint8)
    off = (-raw.ctypes.data) % align
    out = raw[off:off + a.nbytes].view(a.dtype).reshape(a.shape)
    out[...] = a
    return out


def _orc_llr_types():
    L = orc()
    if not getattr(L, "_llr_typed", False):
        L.orc_llr_qam.argtypes = [ctypes.c_int, VP, VP, VP, ctypes.c_int, VP]
        L.orc_llr_qpsk_qpsk.argtypes = [VP, VP, VP, ctypes.c_int, VP]
        L.orc_llr_qpsk_qamx.argtypes = [ctypes.c_int, VP, VP, VP, VP, ctypes.c_int, VP]
        L.orc_llr_qpsk_qpsk.restype = L.orc_llr_qpsk_qamx.restype = None
        L._llr_typed = True
    return L


def orc_llr_qam(Qm, comp, mag, magb, n):
    """the oracle's per-RE LLR stage (orc_llr_qam) over n REs of flat int16 streams"""
    _orc_llr_types()
    out = np.zeros(6 * n + 8, np.int16)
    comp = np.ascontiguousarray(comp, np.int16)
    mag = np.ascontiguousarray(mag, np.int16)
    magb = np.ascontiguousarray(magb, np.int16)
    orc().orc_llr_qam(Qm, comp.ctypes.data, mag.ctypes.data, magb.ctypes.data, n, out.ctypes.data)
    return out[:Qm * n]


def orc_llr_ia(qm1, s0, s1, mag1, rho, n):
    """the oracle's interference-aware LLRs of stream 0 (orc_llr_qpsk_qpsk / orc_llr_qpsk_qamx)"""
    _orc_llr_types()
    out = np.zeros(2 * n, np.int16)
    s0, s1, rho = (np.ascontiguousarray(x, np.int16) for x in (s0, s1, rho))
    if qm1 == 2:
        orc().orc_llr_qpsk_qpsk(s0.ctypes.data, s1.ctypes.data, rho.ctypes.data, n, out.ctypes.data)
    else:
        mag1 = np.ascontiguousarray(mag1, np.int16)
        orc().orc_llr_qpsk_qamx(qm1, s0.ctypes.data, s1.ctypes.data, mag1.ctypes.data, rho.ctypes.data, n,
                                out.ctypes.data)
    return out


# ---- lte_est_freq_offset.c compiled unmodified (oracle/_ref/libref_fo.so) ----
REF_FO_SO = os.path.join(ORACLE_DIR, "_ref", "libref_fo.so")
_reffo = None


def ref_fo():
    """lte_est_freq_offset.c compiled unmodified (+ ref_glue_fo.c over libref_tools.so), or None."""
    global _reffo
    if _reffo is None:
        if not os.path.exists(REF_FO_SO) or ref_tools() is None:
            return None
        L = ctypes.CDLL(REF_FO_SO, mode=os.RTLD_LAZY | os.RTLD_LOCAL)
        L.ref_glue_est_freq_offset.restype = ctypes.c_int
        L.ref_glue_est_freq_offset.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, VP, ctypes.c_int,
                                               ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        _reffo = L
    return _reffo


REF_TD_SO = os.path.join(ORACLE_DIR, "_ref", "libref_td.so")
_reftd = None


def ref_td():
    """PHY/CODING/3gpplte_turbo_decoder.c compiled unmodified (the reference's scalar max-log-MAP
    decoder, phy_threegpplte_turbo_decoder_scalar :883), its CRCs from libref_coding.so (initialised
    by ref_coding()), or None when it was not built here."""
    global _reftd
    if _reftd is None:
        if not os.path.exists(REF_TD_SO) or ref_coding() is None:
            return None
        L = ctypes.CDLL(REF_TD_SO)
        L.phy_threegpplte_turbo_decoder_scalar.restype = U8
        L.phy_threegpplte_turbo_decoder_scalar.argtypes = [VP, VP, U16, U16, U16, U8, U8, U8, U8]
        _reftd = L
    return _reftd


def ref_turbo_decode_scalar(y, K, f1, f2, max_it=8, crc_type=1, F=0):
    """phy_threegpplte_turbo_decoder_scalar(y, decoded, n = K, f1, f2, max_it, crc_type, F, 0).
    y: int16 LLRs in the order the decoder reads them (:929-960): (x, z, z') for k < K, then (x, z) x 3
    and (x', z') x 3 -- the d[96 ...] layout, positive = bit 1 (:1019).  Returns (iterations, K/8 bytes);
    iterations = max_it + 1 means the CRC never matched (:1075)."""
    n = 3 * K + 12
    ya = _aligned(n + 64, np.int16)
    ya[:n] = np.asarray(y, np.int16)[:n]
    out = _aligned(K // 8 + 16, np.uint8)       # the CRC test reads an unsigned int at K/8 - 3 (:1028)
    it = ref_td().phy_threegpplte_turbo_decoder_scalar(P(ya), P(out), K, f1, f2, max_it, crc_type, F, 0)
    return int(it), out[:K // 8].copy()
