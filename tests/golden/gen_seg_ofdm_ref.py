"""Generates tests/golden/seg_ofdm_ref.json and seg_ofdm_ref.npz from the reference's own
lte_segmentation.c and ofdm_mod.c, compiled unmodified in this container (oracle/Makefile:
_ref/libref_seg.so, _ref/libref_ofdm.so).  The reference never travels; these outputs do.  Run
from the repo root:

    make -C oracle ref && python tests/golden/gen_seg_ofdm_ref.py

seg_ofdm_ref.npz
  seg_B       the parameter-sweep B values (tests/seg_ofdm_ref_cases.seg_B_values over the TBS
              table of dlsch_tbs_full.h:34, read here as data)
  seg_params  [len(seg_B)][7] (ret, C, Cplus, Cminus, Kplus, Kminus, F) of lte_segmentation
seg_ofdm_ref.json
  seg_data[B]            [params, digest of the C code-block buffers]
  ofdm_mod["l,n,cp"]     digest of PHY_ofdm_mod's output buffer
  npm["N_RB,Ncp,nsymb"]  digest of normal_prefix_mod's output buffer
  do_ofdm["N_RB,Ncp,nant,slot"]  digest of do_OFDM_mod's output buffers
  bench_C3[i]            per antenna, digest of subframe i of the C3 bench batch (8192 subframes,
                         subframe 7, bench.py's seed): the oracle's frequency grid of that subframe,
                         built from the batch's payload (k_fill's splitmix64 stream, restated in
                         seg_ofdm_ref_cases.bench_payload), through the reference's do_OFDM_mod for
                         slots 14 and 15 — IDFT, CP and slot layout all the reference's
"""
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle_lib as O  # noqa: E402
import seg_ofdm_ref_cases as SC  # noqa: E402

TBS_HDR = "/root/reference/openair1/PHY/LTE_TRANSPORT/dlsch_tbs_full.h"


def tbs_values():
    src = open(TBS_HDR).read()
    body = src[src.index("TBStable[TBStable_rowCnt][110]"):]
    body = body[body.index("{"):body.index("};")]
    return sorted({int(x) for r in re.findall(r"\{([^{}]*)\}", body) for x in re.findall(r"\d+", r)})


def main():
    assert O.ref_seg() is not None and O.ref_ofdm() is not None, "build oracle/_ref first (make -C oracle ref)"
    ref = SC.ref_impl(O)
    Bs = SC.seg_B_values(tbs_values())
    params = SC.run_seg_params(ref, Bs)
    out = {"seg_data": {}, "ofdm_mod": {}, "npm": {}, "do_ofdm": {}}
    for B in SC.seg_data_B(Bs):
        vals, bufs = SC.run_seg_data(ref, B)
        out["seg_data"][str(B)] = [list(vals), SC.digest(bufs)]
    for case in SC.OFDM_CASES:
        out["ofdm_mod"]["%d,%d,%d" % case] = SC.digest(SC.run_ofdm_mod(ref, case))
    for (n_rb, ncp) in SC.NPM_FRAMES:
        fp = O.frame(n_rb, Ncp=ncp)
        for nsymb in SC.NPM_NSYMB:
            out["npm"]["%d,%d,%d" % (n_rb, ncp, nsymb)] = SC.digest(SC.run_npm(ref, fp, nsymb))
    for (n_rb, ncp, na) in SC.DO_OFDM_FRAMES:
        fp = O.frame(n_rb, Ncp=ncp, nb_antennas_tx=na, mode1_flag=1 if na == 1 else 0)
        for slot in SC.DO_OFDM_SLOTS:
            out["do_ofdm"]["%d,%d,%d,%d" % (n_rb, ncp, na, slot)] = SC.digest(SC.run_do_ofdm(ref, fp, 3, slot))
    out["bench_C3"] = {str(i): SC.bench_c3_digests(ref, O, i) for i in SC.BENCH_C3_SAMPLES}
    # the chain behind the bench digests: e bits from the oracle (RM / Gold pinned to the reference),
    # then the reference's dlsch_modulation.c (when built) and do_OFDM_mod
    out["bench_C3_chain"] = ("e (oracle, RM/Gold reference-pinned) -> dlsch_modulation.c -> do_OFDM_mod (ofdm_mod.c)"
                             if "mod" in ref else "oracle grid -> do_OFDM_mod (ofdm_mod.c)")
    with open(os.path.join(HERE, "seg_ofdm_ref.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    np.savez_compressed(os.path.join(HERE, "seg_ofdm_ref.npz"), seg_B=Bs.astype(np.int32),
                        seg_params=params.astype(np.int64))


if __name__ == "__main__":
    main()
