"""The cases behind tests/golden/rm_ref.{json,npz}: the reference's own lte_rate_matching.c and
lte_gold.c (compiled unmodified into oracle/_ref, build container only) run on inputs this module
generates deterministically, and their outputs kept as digests (sweeps) and as data (the bench
geometries).  TEST INFRASTRUCTURE ONLY.

One `run_*` function per reference function; each takes the implementation to run as a dict of
callables (`impl`) with the reference's argument meaning, so the fixture generator
(tests/golden/gen_rm_ref.py, impl = the reference), the CPU fixture check (impl = the oracle) and
the GPU check (impl = the product library's drop-ins) share one definition of every case.
"""
import hashlib

import numpy as np

from ref_cases import QPP

KS = sorted(QPP)


def splitmix64(seed, n):
    """n outputs of splitmix64 from `seed` (uint64, wrapping), the fixture input generator."""
    with np.errstate(over="ignore"):
        i = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def gen_bits(seed, n):
    return (splitmix64(seed, n) >> np.uint64(63)).astype(np.uint8)


def gen_int16(seed, n):
    return (splitmix64(seed, n) >> np.uint64(48)).astype(np.uint16).view(np.int16)


def digest(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()[:24]


def rm_geometries(K):
    """(G, C, r, Qm, Nl) per K for the sweep: E = floor and ceil, Nl = 2, one code block with
    repetition (E > Kw), and a large C."""
    return [(2 * (3 * K + 100), 1, 0, 2, 1),            # C = 1, E > Kw: wraps the circular buffer
            (6 * (3 * (K // 2) + 1), 3, 2, 6, 1),       # G' mod C != 0, last block
            (2 * 4 * (5 * (K // 3) + 2), 5, 1, 4, 2),   # Nl = 2
            (6 * (13 * (K // 4) + 7), 13, 12, 6, 1)]    # large C (RM condition at Kmimo 2, big K)


def run_sbi(impl, K):
    """sub_block_interleaving_turbo on d = gen_bits(K, 3K+12): (R, w)."""
    return impl["sbi"](gen_bits(K, 3 * K + 12), K + 4)


def run_rm_sweep(impl, K):
    """lte_rate_matching_turbo over rm_geometries x Kmimo 1/2 x rv 0-3 on run_sbi's w:
    (list of E, concatenated e)."""
    R, w = run_sbi(impl, K)
    Es, es = [], []
    for (G, C, r, Qm, Nl) in rm_geometries(K):
        for Kmimo in (1, 2):
            for rv in range(4):
                e = impl["rm"](R, G, w, C, r, Qm, rv, Nl, Kmimo)
                Es.append(len(e))
                es.append(np.asarray(e, np.uint8))
    return Es, np.concatenate(es)


DUMMY_F = (0, 8, 16, 24, 40, 64)


def run_dummy_w(impl, K):
    """NULL masks of generate_dummy_w(K + 4, w, F) for F in DUMMY_F (F < K)."""
    return np.concatenate([(np.asarray(impl["dummy_w"](K + 4, F)) == 2).astype(np.uint8)
                           for F in DUMMY_F if F < K])


RX_KS = (40, 512, 960, 1056, 2112, 4032, 5504, 6144)


def rx_geometries(K):
    return [(3 * K + 300, 1, 0, 2, 1, 1), (6 * (3 * K) + 24, 2, 1, 6, 1, 2), (4 * 2 * K, 2, 0, 4, 2, 1)]


def run_rm_rx(impl, K):
    """lte_rate_matching_turbo_rx HARQ sequences (rv 0 clear = 1, then rv 2, 3, 1 with clear = 0)
    over int16 soft bits that wrap: (list of E, concatenated w after every round)."""
    D = K + 4
    R = (D + 31) >> 5
    dw = np.asarray(impl["dummy_w"](D, 0), np.uint8)
    Es, ws = [], []
    for gi, (G, C, r, Qm, Nl, Kmimo) in enumerate(rx_geometries(K)):
        w = np.zeros(3 * 32 * R, np.int16)
        for rnd, rv in enumerate((0, 2, 3, 1)):
            soft = gen_int16((K << 8) + (gi << 4) + rnd, G)
            E, w = impl["rm_rx"](R, G, w, dw, soft, C, r, Qm, rv, 1 if rnd == 0 else 0, Nl, Kmimo)
            Es.append(E)
            ws.append(np.asarray(w, np.int16).copy())
    return Es, np.concatenate(ws)


DEINT_KS = tuple(KS[::11]) + (5504, 6144)


def run_deint(impl, K):
    """sub_block_deinterleaving_turbo of w = gen_int16: d[-3 ND .. 3D + 3), every entry it writes
    (d3 = d1 + 5 reaches d[3D + 2]).  impl["deint"] returns the int16 buffer whose entry 96 is d[0]."""
    D = K + 4
    R = (D + 31) >> 5
    ND = 32 * R - D
    buf = np.asarray(impl["deint"](D, gen_int16(K + 77, 3 * 32 * R)), np.int16)
    return buf[96 - 3 * ND:96 + 3 * D + 3]


GOLD_CINITS = (0, 1, 0x1234 << 14, (0x1234 << 14) + (1 << 13) + (7 << 9) + 503, 0x7FFFFFFF, 0x48D1C00, 0x3D << 14)


def run_gold(impl):
    """lte_gold_generic: 2701 words (one C3 codeword's G = 86400 bits) from each c_init."""
    return np.concatenate([np.asarray(impl["gold"](c, 2701), np.uint32) for c in GOLD_CINITS])


# ---- bench geometries as data: the composed sub-block interleaver + rate matcher as a map from e
#      position to the d entry (index into the 96 + 3D entry buffer, prefix included) whose value it
#      carries; -1 never occurs (NULLs are skipped).  (K, G, C, Qm, Kmimo, Nl)
MAP_GEOMS = {"C1": (960, 1512, 1, 2, 1, 1), "C2": (6144, 60000, 5, 4, 1, 1), "C3": (6144, 86400, 6, 6, 2, 1)}


def rm_map(impl, K, G, C, r, Qm, Kmimo, Nl, rv=0):
    """Provenance map of lte_rate_matching_turbo(sub_block_interleaving_turbo(d)) for block r: run
    both on bit planes of the d index (d[i] = bit b of i for the 3D data entries) and read the index
    back from e."""
    D = K + 4
    n = 3 * D
    nb = int(n + 96).bit_length()
    acc = None
    for b in range(nb):
        d = ((np.arange(96, 96 + n) >> b) & 1).astype(np.uint8)
        R, w = impl["sbi"](d, D)
        e = np.asarray(impl["rm"](R, G, w, C, r, Qm, rv, Nl, Kmimo), np.int64)
        acc = e << b if acc is None else acc | (e << b)
    return acc.astype(np.int32)


def gold_bits(words, G):
    return ((np.asarray(words, np.uint32)[:, None] >> np.arange(32, dtype=np.uint32)) & 1).astype(np.uint8).ravel()[:G]


def c_init(rnti, q, subframe, Nid_cell):
    """dlsch_scrambling.c:69 with Ns = 2 subframe (dlsim.c:2642-2647)."""
    return (rnti << 14) + (q << 13) + (subframe << 9) + Nid_cell


# ---- implementations with the reference's argument meaning ----
def ref_impl(O):
    """The reference compiled here (oracle/_ref/libref_rm.so, libref_gold.so)."""
    return {
        "sbi": lambda d, D: O.ref_subblock(d, D)[:2],
        "rm": lambda R, G, w, C, r, Qm, rv, Nl, Kmimo: O.ref_rate_match(R, G, w, C, r, Qm, rvidx=rv, Nl=Nl,
                                                                          Kmimo=Kmimo),
        "dummy_w": lambda D, F: O.ref_dummy_w(D, F)[1],
        "rm_rx": lambda R, G, w, dw, soft, C, r, Qm, rv, clear, Nl, Kmimo: O.ref_rate_match_rx(
            R, G, w, dw, soft, C, r, Qm, rvidx=rv, clear=clear, Nl=Nl, Kmimo=Kmimo)[1:],
        "deint": lambda D, w: O.ref_deinterleave(D, w),
        "gold": lambda c, n: O.ref_gold_words(c, n),
    }


def oracle_impl(O):
    """The CPU restatement (oracle/liboracle.so)."""
    import ctypes

    def sbi(d, D):
        R, w, _ = O.subblock(d, D)
        return R, w[:3 * 32 * R]

    def dummy_w(D, F):
        R = (D + 31) >> 5
        return O.dummy_w_F(D, F)[:3 * 32 * R]

    def rm_rx(R, G, w, dw, soft, C, r, Qm, rv, clear, Nl, Kmimo):
        wb = np.zeros(len(w) + 64, np.int16)
        wb[:len(w)] = w
        E = ctypes.c_uint32()
        dwb = np.zeros(len(dw) + 64, np.uint8)
        dwb[:len(dw)] = dw
        s = np.ascontiguousarray(soft, np.int16)
        rc = O.orc().orc_rate_matching_turbo_rx(R, G, O.P(wb), O.P(dwb), O.P(s), C, 1827072, 8, Kmimo, rv, clear,
                                                Qm, Nl, r, ctypes.byref(E))
        assert rc == 0
        return E.value, wb[:len(w)]

    def deint(D, w):
        buf = np.zeros(96 + 3 * D + 64, np.int16)
        O.orc().orc_sub_block_deinterleaving_turbo(D, ctypes.c_void_p(buf.ctypes.data + 2 * 96),
                                                   O.P(np.ascontiguousarray(w, np.int16)))
        return buf

    def gold(c, n):
        x1, x2 = ctypes.c_uint32(0), ctypes.c_uint32(c)
        L = O.orc()
        return np.array([L.orc_gold_generic(ctypes.byref(x1), ctypes.byref(x2), 1 if i == 0 else 0)
                         for i in range(n)], np.uint32)

    return {"sbi": sbi,
            "rm": lambda R, G, w, C, r, Qm, rv, Nl, Kmimo: O.rate_match(R, G, w, C, r, Qm, rvidx=rv, Nl=Nl,
                                                                          Kmimo=Kmimo),
            "dummy_w": dummy_w, "rm_rx": rm_rx, "deint": deint, "gold": gold}


def gpu_impl(gpu):
    """The product library's drop-in entry points (include/oai4g.h), through openair4g_amd."""
    import ctypes

    def sbi(d, D):
        dfull = np.full(96 + 3 * D + 16, 2, dtype=np.uint8)
        dfull[96:96 + len(d)] = d
        return gpu.subblock_interleave(dfull, D)

    def dummy_w(D, F):
        R = (D + 31) >> 5
        return gpu.generate_dummy_w(D, F)[:3 * 32 * R]

    def rm_rx(R, G, w, dw, soft, C, r, Qm, rv, clear, Nl, Kmimo):
        wb = np.zeros(len(w) + 64, np.int16)
        wb[:len(w)] = w
        dwb = np.zeros(len(dw) + 64, np.uint8)
        dwb[:len(dw)] = dw
        E = gpu.rate_matching_turbo_rx(R, G, wb, dwb, soft, C, r, Qm, rvidx=rv, clear=clear, Nl=Nl, Kmimo=Kmimo)
        return E, wb[:len(w)]

    def gold(c, n):
        x1, x2 = ctypes.c_uint32(0), ctypes.c_uint32(c)
        L = gpu.lib()
        return np.array([L.oai4g_lte_gold_generic(ctypes.byref(x1), ctypes.byref(x2), 1 if i == 0 else 0)
                         for i in range(n)], np.uint32)

    return {"sbi": sbi,
            "rm": lambda R, G, w, C, r, Qm, rv, Nl, Kmimo: gpu.rate_match(R, G, w, C, r, Qm, rvidx=rv, Nl=Nl,
                                                                            Kmimo=Kmimo),
            "dummy_w": dummy_w, "rm_rx": rm_rx,
            "deint": lambda D, w: gpu.sub_block_deinterleaving_turbo(D, w), "gold": gold}
