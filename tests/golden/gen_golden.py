#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (run in the dev container).

  dft_ref.npz       inputs and outputs of the REFERENCE's own fixed-point forward DFTs
                    (lte_dfts.c dft64/128/256/512/1024/2048, same library), and the reference's
                    forward twiddle tables tw16a/b … tw512a/b, tw1024, tw2048 (data it holds):
                    pins the oracle's forward DFT and the GPU slot_fep path.
  idft_ref.npz      inputs and outputs of the REFERENCE's own fixed-point IDFTs
                    (openair1/PHY/TOOLS/lte_dfts.c idft64/128/256/512/1024/2048, compiled unmodified
                    into oracle/_ref/libref_dfts.so by oracle/Makefile and run here): pins the
                    oracle and the GPU IDFT bit for bit.
  pipeline_C1.npz   oracle transmit vectors for config C1 (1.4 MHz, QPSK): payload bytes,
                    scrambled e bits and time-domain IQ of subframes 0, 5, 7 (regression pins
                    for the GPU path; the coding stages are pinned to the 36.212 spec model in
                    tests/spec_model.py).
  pipeline_C3.json  the same for C3 (20 MHz TM3 64-QAM, 2 CW) as SHA-256 digests of the e bits
                    and IQ plus the first samples (the full IQ is 245 KB per subframe).

Payloads come from numpy's PCG64 with fixed seeds.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

import oracle_lib as O  # noqa: E402


def aligned_i16(n):
    buf = np.zeros(n + 32, dtype=np.int16)
    off = (-buf.ctypes.data % 64) // 2
    return buf[off:off + n]


def gen_dft():
    ref = O.ref_dfts()
    if ref is None:
        raise SystemExit("oracle/_ref/libref_dfts.so missing: run make -C oracle (needs /root/reference)")
    import ctypes
    rng = np.random.default_rng(20261016)
    out = {}
    for log2n in (6, 7, 8, 9, 10, 11):
        n = 1 << log2n
        fn = getattr(ref, f"dft{n}")
        vecs = [rng.integers(-1024, 1024, 2 * n), rng.integers(-32768, 32768, 2 * n),
                rng.choice(np.array([-32768, 32767, -20000, 20000]), 2 * n),
                np.r_[np.full(2, 8000), np.zeros(2 * n - 2, dtype=np.int64)]]
        for vi, v in enumerate(vecs):
            for scale in ((0, 1) if vi == 0 else (1,)):
                x = aligned_i16(2 * n)
                x[:] = v.astype(np.int16)
                y = aligned_i16(2 * n)
                fn(O.P(x), O.P(y), scale)
                out[f"x_{n}_{vi}_{scale}"] = x.copy()
                out[f"y_{n}_{vi}_{scale}"] = y.copy()
    for name, cnt in (("tw16a", 24), ("tw16b", 24), ("tw64a", 96), ("tw64b", 96), ("tw128a", 128), ("tw128b", 128),
                      ("tw256a", 384), ("tw256b", 384), ("tw512a", 512), ("tw512b", 512), ("tw1024", 1536),
                      ("tw2048", 2048)):
        out["table_" + name] = np.ctypeslib.as_array((ctypes.c_int16 * cnt).in_dll(ref, name)).copy()
    np.savez_compressed(os.path.join(HERE, "dft_ref.npz"), **out)
    print("dft_ref.npz:", len(out), "arrays")


def gen_idft():
    ref = O.ref_dfts()
    if ref is None:
        raise SystemExit("oracle/_ref/libref_dfts.so missing: run make -C oracle (needs /root/reference)")
    rng = np.random.default_rng(20241015)
    out = {}
    for log2n in (6, 7, 8, 10, 11, 9):   # 9 appended later: earlier vectors unchanged
        n = 1 << log2n
        fn = getattr(ref, f"idft{n}")
        vecs = [rng.integers(-1024, 1024, 2 * n), rng.integers(-32768, 32768, 2 * n),
                np.r_[np.full(2, 8000), np.zeros(2 * n - 2, dtype=np.int64)]]
        for vi, v in enumerate(vecs):
            for scale in ((0, 1) if vi == 0 else (1,)):
                x = aligned_i16(2 * n)
                x[:] = v.astype(np.int16)
                y = aligned_i16(2 * n)
                fn(O.P(x), O.P(y), scale)
                out[f"x_{n}_{vi}_{scale}"] = x.copy()
                out[f"y_{n}_{vi}_{scale}"] = y.copy()
    np.savez_compressed(os.path.join(HERE, "idft_ref.npz"), **out)
    print("idft_ref.npz:", len(out) // 2, "vectors")


def G_of(p, sf, cw):
    fp = O.frame(p.N_RB_DL, p.Nid_cell, p.Ncp, p.nb_antennas_tx, p.mode1_flag, p.frame_type)
    Qm = O.orc().orc_get_Qm(p.mcs[cw])
    return O.get_G(fp.N_RB_DL, fp.Ncp, fp.mode1_flag, fp.frame_type, p.nb_rb, list(p.rb_alloc), Qm, 1,
                   p.num_pdcch_symbols, sf)


def pipeline_vectors(name, subframes, seed):
    import openair4g_amd as oai   # host-side parameter mirror only (no GPU needed)
    rng = np.random.default_rng(seed)
    res = []
    for sf in subframes:
        p = oai.make_params(name, subframe=sf)
        cfg = O.tx_cfg_from_params(p, sf)
        pays = [rng.integers(0, 256, size=p.TBS[cw] // 8, dtype=np.uint8) for cw in range(p.n_cw)]
        txd, _, es = O.tx_subframe(cfg, pays, want_e=True)
        ebits = [np.packbits(es[cw][:G_of(p, sf, cw)] & 1, bitorder="little") for cw in range(p.n_cw)]
        res.append((sf, pays, ebits, txd))
    return res


def gen_pipeline():
    out = {}
    for sf, pays, ebits, txd in pipeline_vectors("C1", (0, 5, 7), 11):
        out[f"payload0_{sf}"] = pays[0]
        out[f"ebits0_{sf}"] = ebits[0]
        out[f"iq_{sf}"] = txd
    np.savez_compressed(os.path.join(HERE, "pipeline_C1.npz"), **out)
    rows = []
    for sf, pays, ebits, txd in pipeline_vectors("C3", (7, 0), 33):
        rows.append({"subframe": sf,
                     "payload_sha256": [hashlib.sha256(pl.tobytes()).hexdigest() for pl in pays],
                     "ebits_sha256": [hashlib.sha256(e.tobytes()).hexdigest() for e in ebits],
                     "iq_sha256": hashlib.sha256(np.ascontiguousarray(txd).tobytes()).hexdigest(),
                     "iq_head": txd[:, :16].tolist()})
    json.dump({"config": "C3", "payload_rng": "numpy default_rng(33), per subframe per codeword",
               "subframes": rows}, open(os.path.join(HERE, "pipeline_C3.json"), "w"), indent=1)
    print("pipeline fixtures written")


if __name__ == "__main__":
    which = sys.argv[1:] or ["idft", "dft", "pipeline"]
    if "idft" in which:
        gen_idft()
    if "dft" in which:
        gen_dft()
    if "pipeline" in which:
        gen_pipeline()
