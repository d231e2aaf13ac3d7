"""Generates tests/golden/rm_ref.json and rm_ref.npz from the reference's own rate matcher and Gold
generator, compiled unmodified in this container (oracle/Makefile: _ref/libref_rm.so =
PHY/CODING/lte_rate_matching.c, _ref/libref_gold.so = PHY/LTE_REFSIG/lte_gold.c).  The
reference never travels; these outputs do.  Run from the repo root:

    make -C oracle ref && python tests/golden/gen_rm_ref.py

rm_ref.json — digests over deterministic sweeps (tests/rm_ref_cases.py defines every case):
  sbi[K]     = (R, digest of w)           sub_block_interleaving_turbo, all 188 K
  rm[K]      = (E list, digest of e)       lte_rate_matching_turbo, 4 geometries x Kmimo x rv
  dummy_w[K] = digest of the NULL masks    generate_dummy_w, F in {0, 8, 16, 24, 40, 64}
  rm_rx[K]   = (E list, digest of w)       lte_rate_matching_turbo_rx, HARQ rounds rv 0, 2, 3, 1
  deint[K]   = digest of d                 sub_block_deinterleaving_turbo
  gold       = digest of the words         lte_gold_generic, 2701 words per c_init
rm_ref.npz — data for the bench geometries:
  map_C1 / map_C2 / map_C3: e position -> d entry (sub_block_interleaving_turbo then
    lte_rate_matching_turbo, rv 0, every block r of the configuration has this map);
  gold_sf: [10][2701] lte_gold_generic words of dlsch_scrambling's c_init for rnti 0x1234, q 0,
    Nid_cell 0, subframes 0..9 (the bench / parity configuration).
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as O  # noqa: E402
import rm_ref_cases as RC  # noqa: E402


def main():
    assert O.ref_rm() is not None and O.ref_gold() is not None, "build oracle/_ref first (make -C oracle ref)"
    ref = RC.ref_impl(O)
    out = {"sbi": {}, "rm": {}, "dummy_w": {}, "rm_rx": {}, "deint": {}}
    for K in RC.KS:
        R, w = RC.run_sbi(ref, K)
        out["sbi"][K] = [int(R), RC.digest(w)]
        Es, e = RC.run_rm_sweep(ref, K)
        out["rm"][K] = [Es, RC.digest(e)]
        out["dummy_w"][K] = RC.digest(RC.run_dummy_w(ref, K))
    for K in RC.RX_KS:
        Es, w = RC.run_rm_rx(ref, K)
        out["rm_rx"][K] = [Es, RC.digest(w)]
    for K in RC.DEINT_KS:
        out["deint"][K] = RC.digest(RC.run_deint(ref, K))
    out["gold"] = RC.digest(RC.run_gold(ref))
    with open(os.path.join(HERE, "rm_ref.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)

    arrays = {}
    for name, (K, G, C, Qm, Kmimo, Nl) in RC.MAP_GEOMS.items():
        maps = [RC.rm_map(ref, K, G, C, r, Qm, Kmimo, Nl) for r in range(C)]
        for m in maps[1:]:
            assert np.array_equal(m, maps[0]), name
        assert maps[0].min() >= 96 and len(maps[0]) == G // C
        arrays["map_" + name] = maps[0].astype(np.int16)
    arrays["gold_sf"] = np.stack([ref["gold"](RC.c_init(0x1234, 0, sf, 0), 2701) for sf in range(10)])
    np.savez_compressed(os.path.join(HERE, "rm_ref.npz"), **arrays)


if __name__ == "__main__":
    main()
