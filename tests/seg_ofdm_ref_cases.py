"""The cases behind tests/golden/seg_ofdm_ref.{json,npz}: the reference's own lte_segmentation.c and
ofdm_mod.c (compiled unmodified into oracle/_ref, build container only) run on inputs this module
generates deterministically; their outputs are kept as data (segmentation parameters) and digests
(code-block buffers, OFDM output).  TEST INFRASTRUCTURE ONLY.

As in tests/rm_ref_cases.py, every `run_*` takes the implementation as a dict of callables with the
reference's argument meaning, so the fixture generator (tests/golden/gen_seg_ofdm_ref.py, impl = the
reference), the CPU fixture check (impl = the oracle) and the GPU check (impl = the product's
drop-ins, include/oai4g.h) share one definition of every case.

Cases:
  segmentation (lte_segmentation.c:39-176)
    seg_params  every B of the parameter sweep (all B < 20000, B = TBS + 24 for every entry of the
                reference's TBS table dlsch_tbs_full.h:34, and the C > 16 refusal) with NULL
                buffers: (ret, C, Cplus, Cminus, Kplus, Kminus, F)
    seg_data    a subset of byte-aligned B with buffers: the C code-block buffers (filler bytes,
                payload, CRC-24B per block when C > 1), pre-filled with 0xA5 so every byte the
                function does not write is compared too
  OFDM modulation (ofdm_mod.c:47-284)
    ofdm_mod    PHY_ofdm_mod for N = 128..2048 (the N = 128 static-temp path :94/:142-165 included),
                1..14 symbols, several prefix lengths, in a sentinel-filled output
    npm         normal_prefix_mod for N_RB 6/15/25/50/100 x normal/extended prefix (15 PRB extended
                only: see OFDM_CASES) x nsymb 1, 2, 3,
                6, 7, 12, 14 (the short_offset branch :53-54, one and two slots)
    do_ofdm     do_OFDM_mod over whole-frame grids for 1, 2 and 4 antennas, slots 0, 1, 9, 14, 19
"""
import numpy as np

from rm_ref_cases import digest, gen_int16, splitmix64

CYCLIC_PREFIX = 0

# ---------------------------------------------------------------- segmentation
SEG_EXTRA_B = (0, 1, 7, 39, 40, 41, 6144, 6145, 6152, 6168, 6169, 12240, 12241, 12288, 18360, 18361, 36720,
               36721, 61200, 61201, 97920, 97921, 97928, 100000, 150000)


def seg_B_values(tbs_values):
    """Parameter sweep: every B below 20000, B = TBS + 24 for the TBS table, and SEG_EXTRA_B."""
    s = set(range(20000)) | {int(t) + 24 for t in tbs_values} | set(SEG_EXTRA_B)
    return np.array(sorted(s), np.int64)


def run_seg_params(impl, Bs):
    """(ret, C, Cplus, Cminus, Kplus, Kminus, F) per B, NULL buffers.  Fields the function leaves
    unset on its early return (C > MAX_NUM_DLSCH_SEGMENTS, :69-72) read as 0."""
    out = np.zeros((len(Bs), 7), np.int64)
    for i, B in enumerate(Bs):
        ret, vals = impl["seg"](int(B), None)[:2]
        out[i, 0] = ret
        out[i, 1:] = vals if ret == 0 else (vals[0], 0, 0, 0, 0, 0)
    return out


def seg_data_B(Bs):
    """The byte-aligned B with buffers: every 17th byte-aligned B of the sweep that segments into at
    most 16 blocks, plus all the multi-block and filler edge cases of SEG_EXTRA_B."""
    al = [int(b) for b in Bs if b % 8 == 0 and 0 < b <= 97920]
    pick = set(al[::17]) | {b for b in SEG_EXTRA_B if b % 8 == 0 and 0 < b <= 97920}
    return sorted(pick)


def seg_payload(B):
    return (splitmix64(0x5E6 + B, (B + 7) // 8 + 8) >> np.uint64(56)).astype(np.uint8)


def run_seg_data(impl, B):
    """(ret, params, the C output buffers concatenated, 779 bytes each)."""
    ret, vals, bufs = impl["seg"](B, seg_payload(B))
    assert ret == 0
    return vals, np.concatenate([np.asarray(b, np.uint8)[:779] for b in bufs[:vals[0]]])


# ---------------------------------------------------------------- OFDM modulation
# The reference's idft256..idft2048 store through aligned SSE stores, so PHY_ofdm_mod faults unless
# every symbol start (i << log2n) + (1 + i) * cp is a multiple of 4 samples (16 bytes); only N = 128
# goes through the aligned static temp (ofdm_mod.c:94, :142-165) and takes any prefix.  Hence cp % 4 == 0
# for N >= 256 below, and no 15-PRB normal-prefix case (CP 20/18 at N = 256: the reference faults on
# the second symbol; the oracle and the GPU path compute it, tests/test_gpu_parity.py covers it).
OFDM_CASES = [(7, 1, 9), (7, 6, 9), (7, 7, 10), (7, 6, 32), (7, 14, 0), (8, 6, 20), (8, 7, 20), (8, 6, 64),
              (9, 6, 36), (9, 7, 40), (9, 6, 128), (10, 6, 72), (10, 7, 80), (10, 6, 256), (10, 3, 1020),
              (11, 1, 160), (11, 6, 144), (11, 7, 160), (11, 6, 512), (11, 12, 512), (11, 2, 0)]


def ofdm_grid(seed, n, lim=4096):
    """int32 grid of n complex int16 samples in [-lim, lim)."""
    v = gen_int16(seed, 2 * n).astype(np.int32)
    return ((v % (2 * lim)) - lim).astype(np.int16).view(np.int32)


def sentinel(seed, n):
    return gen_int16(seed, 2 * n).view(np.int32).copy()


def run_ofdm_mod(impl, case):
    log2n, nsym, cp = case
    N = 1 << log2n
    grid = ofdm_grid(0x0F + 31 * log2n + nsym + 1000 * cp, nsym * N, 32768 if cp == 0 else 4096)
    out = sentinel(0xF0 + log2n, nsym * (N + cp) + 64)
    return impl["ofdm_mod"](grid, out, log2n, nsym, cp)


NPM_FRAMES = [(n, ncp) for n in (6, 15, 25, 50, 100) for ncp in (0, 1) if (n, ncp) != (15, 0)]
NPM_NSYMB = (1, 2, 3, 6, 7, 12, 14)


def run_npm(impl, fp, nsymb):
    """normal_prefix_mod(txdataF, txdata, nsymb, fp) on a 14-symbol grid into a sentinel-filled
    subframe (+64 samples of guard)."""
    N, spt = fp.ofdm_symbol_size, fp.samples_per_tti
    grid = ofdm_grid(0x4E + N + 7 * fp.Ncp + nsymb, 14 * N)
    out = sentinel(0x77 + N + fp.Ncp, spt + 64)
    return impl["npm"](grid, out, nsymb, fp)


DO_OFDM_SLOTS = (0, 1, 9, 14, 19)
DO_OFDM_FRAMES = [(6, 0, 1), (25, 1, 2), (50, 0, 4), (100, 0, 2), (100, 1, 1), (15, 1, 2)]


def run_do_ofdm(impl, fp, frame, next_slot):
    """do_OFDM_mod(txdataF, txdata, frame, next_slot, fp) over whole-frame buffers, one per antenna
    (txdataF: 10 subframes of symbols_per_tti symbols; txdata: 10 subframes of samples)."""
    N, spt, nsymb = fp.ofdm_symbol_size, fp.samples_per_tti, fp.symbols_per_tti
    na = fp.nb_antennas_tx
    grids = [ofdm_grid(0xD0 + 13 * a + N + fp.Ncp, 10 * nsymb * N) for a in range(na)]
    outs = [sentinel(0xD7 + a + N, 10 * spt + 64) for a in range(na)]
    return impl["do_ofdm"](grids, outs, frame, next_slot, fp)


# ---------------------------------------------------------------- the C3 bench batch
BENCH_SEED = 0x5EED0000                   # bench.py: payload_seed(0x5EED0000, rank 0)
BENCH_N_SF = 8192
BENCH_C3_SAMPLES = (0, 1, 2, 777, 4095, 4096, 6000, 8190, 8191)


def bench_payload(seed, n_sf, n_cw, stride):
    """The device payload generator (oai4g_fill_payload, k_fill in oai4g_encode.hip): little-endian
    64-bit words of splitmix64 from `seed`, over n_sf x n_cw x stride bytes."""
    nbytes = n_sf * n_cw * stride
    w = splitmix64(seed, (nbytes + 7) // 8)
    return w.view(np.uint8)[:nbytes].reshape(n_sf, n_cw, stride)


def bench_c3_params():
    """C3 as bench.py runs it (openair4g_amd.make_params("C3", subframe=7): host-side helpers only)."""
    import openair4g_amd as oai
    return oai.make_params("C3", subframe=7)


def bench_c3_digests(impl, O, i):
    """Per-antenna digests of subframe i of the C3 bench batch: the scrambled e bits of that
    subframe (the oracle's encoder + rate matching + scrambling, RM / Gold pinned to the reference,
    tests/golden/rm_ref.json) through impl["mod"] (dlsch_modulation, when impl has it; else the
    oracle's grid) and impl["do_ofdm"] for slots 14 and 15 of a frame grid (subframe 7)."""
    p = bench_c3_params()
    pay = bench_payload(BENCH_SEED, BENCH_N_SF, p.n_cw, p.payload_stride)[i]
    cfg = O.tx_cfg_from_params(p, 7)
    _, txF, es = O.tx_subframe(cfg, [pay[cw] for cw in range(p.n_cw)], want_e=True)
    fp = cfg.fp
    N, spt, na = fp.ofdm_symbol_size, fp.samples_per_tti, fp.nb_antennas_tx
    if "mod" in impl:
        assert not cfg.with_crs                  # the bench batch is the PDSCH alone
        cws = [dict(e=es[cw], mcs=cfg.mcs[cw], mimo_mode=cfg.mimo_mode, rb_alloc=list(cfg.rb_alloc))
               for cw in range(cfg.n_cw)]
        ret, grids = impl["mod"](fp, cfg.amp, 7, cfg.num_pdcch_symbols, cws, cfg.sqrt_rho_a, cfg.sqrt_rho_b)
        assert ret > 0
    else:
        grids = [np.zeros(10 * 14 * N, np.int32) for _ in range(na)]
        for a in range(na):
            grids[a][7 * 14 * N:8 * 14 * N] = txF[a]
    outs = [np.zeros(10 * spt + 64, np.int32) for _ in range(na)]
    for slot in (14, 15):
        frame = impl["do_ofdm"](grids, outs, 0, slot, fp).reshape(na, -1)
        outs = [frame[a].copy() for a in range(na)]
    return [digest(outs[a][7 * spt:8 * spt]) for a in range(na)]


# ---------------------------------------------------------------- implementations
def _ptrs(arrs):
    import ctypes
    return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


def ref_impl(O):
    """The reference compiled here (oracle/_ref/libref_seg.so, libref_ofdm.so)."""

    def seg(B, data):
        return O.ref_segmentation(B, data)

    def ofdm_mod(grid, out, log2n, nsym, cp):
        g, o = np.ascontiguousarray(grid).copy(), np.ascontiguousarray(out).copy()
        O.ref_ofdm().PHY_ofdm_mod(O.P(g), O.P(o), log2n, nsym, cp, CYCLIC_PREFIX)
        return o

    def npm(grid, out, nsymb, fp):
        g, o = np.ascontiguousarray(grid).copy(), np.ascontiguousarray(out).copy()
        O.ref_ofdm().ref_glue_normal_prefix_mod(O.P(g), O.P(o), nsymb, O.P(O.frame_geometry(fp)))
        return o

    def do_ofdm(grids, outs, frame, slot, fp):
        gs, os_ = [g.copy() for g in grids], [o.copy() for o in outs]
        O.ref_ofdm().ref_glue_do_OFDM_mod(_ptrs(gs), _ptrs(os_), frame, slot, O.P(O.frame_geometry(fp)))
        return np.concatenate(os_)

    impl = {"seg": seg, "ofdm_mod": ofdm_mod, "npm": npm, "do_ofdm": do_ofdm}
    if O.ref_mod() is not None:                  # dlsch_modulation.c (oracle/_ref/libref_mod.so)
        impl["mod"] = O.ref_modulation
    return impl


def oracle_impl(O):
    """The CPU restatement (oracle/liboracle.so)."""
    import ctypes
    L = O.orc()
    L.orc_segmentation.restype = ctypes.c_int
    L.orc_segmentation.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32] + \
        [ctypes.POINTER(ctypes.c_uint32)] * 6
    L.orc_do_OFDM_mod.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                  ctypes.c_uint16, ctypes.POINTER(O.OrcFrame)]

    def seg(B, data):
        vals = [ctypes.c_uint32(0) for _ in range(6)]
        if data is None:
            ret = L.orc_segmentation(None, None, B, *[ctypes.byref(v) for v in vals])
            return ret, tuple(v.value for v in vals), None
        inp = np.zeros(len(data) + 16, np.uint8)
        inp[:len(data)] = data
        bufs = O.seg_out_buffers(16)
        ret = L.orc_segmentation(O.P(inp), _ptrs(bufs), B, *[ctypes.byref(v) for v in vals])
        return ret, tuple(v.value for v in vals), bufs

    def ofdm_mod(grid, out, log2n, nsym, cp):
        o = np.ascontiguousarray(out).copy()
        L.orc_ofdm_mod(O.P(np.ascontiguousarray(grid)), O.P(o), log2n, nsym, cp)
        return o

    def npm(grid, out, nsymb, fp):
        o = np.ascontiguousarray(out).copy()
        L.orc_normal_prefix_mod(O.P(np.ascontiguousarray(grid)), O.P(o), nsymb, ctypes.byref(fp))
        return o

    def do_ofdm(grids, outs, frame, slot, fp):
        os_ = [o.copy() for o in outs]
        L.orc_do_OFDM_mod(_ptrs(grids), _ptrs(os_), frame, slot, ctypes.byref(fp))
        return np.concatenate(os_)

    return {"seg": seg, "ofdm_mod": ofdm_mod, "npm": npm, "do_ofdm": do_ofdm}


def gpu_impl(gpu):
    """The product library's drop-in entry points (oai4g_lte_segmentation, oai4g_PHY_ofdm_mod,
    oai4g_normal_prefix_mod, oai4g_do_OFDM_mod), called through the C ABI."""
    import ctypes
    gpu.init()
    L = gpu.lib()

    def seg(B, data):
        vals = [ctypes.c_uint32(0) for _ in range(6)]
        if data is None:
            ret = L.oai4g_lte_segmentation(None, None, B, *[ctypes.byref(v) for v in vals])
            return ret, tuple(v.value for v in vals), None
        inp = np.zeros(len(data) + 16, np.uint8)
        inp[:len(data)] = data
        bufs = [np.full(779, 0xA5, np.uint8) for _ in range(16)]
        ptrs = (ctypes.POINTER(ctypes.c_uint8) * 16)(*[b.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
                                                       for b in bufs])
        ret = L.oai4g_lte_segmentation(inp.ctypes.data, ptrs, B, *[ctypes.byref(v) for v in vals])
        return ret, tuple(v.value for v in vals), bufs

    def ofdm_mod(grid, out, log2n, nsym, cp):
        o = np.ascontiguousarray(out).copy()
        L.oai4g_PHY_ofdm_mod(gpu._ptr(np.ascontiguousarray(grid)), gpu._ptr(o), log2n, nsym, cp, CYCLIC_PREFIX)
        return o

    def _fp(fp):
        return gpu.frame_parms(fp.N_RB_DL, 0, fp.Ncp, fp.nb_antennas_tx, 1 if fp.nb_antennas_tx == 1 else 0)

    def npm(grid, out, nsymb, fp):
        o = np.ascontiguousarray(out).copy()
        L.oai4g_normal_prefix_mod(gpu._ptr(np.ascontiguousarray(grid)), gpu._ptr(o), nsymb, ctypes.byref(_fp(fp)))
        return o

    def do_ofdm(grids, outs, frame, slot, fp):
        os_ = [o.copy() for o in outs]
        g = [np.ascontiguousarray(x) for x in grids]
        L.oai4g_do_OFDM_mod(_ptrs(g), _ptrs(os_), frame, slot, ctypes.byref(_fp(fp)))
        return np.concatenate(os_)

    return {"seg": seg, "ofdm_mod": ofdm_mod, "npm": npm, "do_ofdm": do_ofdm}
