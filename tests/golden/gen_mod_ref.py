"""Generate tests/golden/mod_ref.json from the reference's dlsch_modulation.c, dlsch_scrambling.c and
pcfich.c compiled unmodified here (oracle/_ref/libref_mod.so; `make -C oracle ref`).  Inputs come from
tests/mod_ref_cases.py (splitmix64), so only the case list, return values and digests are stored.

    python tests/golden/gen_mod_ref.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import numpy as np  # noqa: E402

import oracle_lib as O  # noqa: E402
from mod_ref_cases import (cws_of, e_bits, frame_of, grid_digests, modulation_cases, pcfich_cases,  # noqa: E402
                           scrambling_cases, symbol0_digests)
from rm_ref_cases import digest  # noqa: E402


def main():
    assert O.ref_mod() is not None, "build the reference objects first: make -C oracle ref"
    out = {"source": "PHY/LTE_TRANSPORT/dlsch_modulation.c, dlsch_scrambling.c, pcfich.c (compiled unmodified, "
                     "oracle/_ref/libref_mod.so)", "modulation": [], "scrambling": [], "pcfich": []}
    for c in modulation_cases():
        fp = frame_of(O, c)
        ret, grids = O.ref_modulation(fp, c["amp"], c["subframe"], c["num_pdcch"], cws_of(c), *c["rho"])
        out["modulation"].append(dict(case=c, ret=int(ret), digests=grid_digests(grids, c, fp.ofdm_symbol_size)))
    for c in scrambling_cases():
        G = c["G"]
        e = e_bits(c["seed"])[:32 * (1 + (G >> 5))]
        s = O.ref_scrambling(e, G, c["rnti"], c["Nid_cell"], c["q"], c["Ns"])
        out["scrambling"].append(dict(case=c, digest=digest(s[:G])))
    for c in pcfich_cases():
        fp = frame_of(O, c)
        grids, reg, first = O.ref_pcfich(c["cfi"], c["amp"], fp, c["subframe"])
        out["pcfich"].append(dict(case=c, reg=reg, first=first, digests=symbol0_digests(grids, c, fp.ofdm_symbol_size)))
    path = os.path.join(HERE, "mod_ref.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path, len(out["modulation"]), "modulation cases,", len(out["scrambling"]), "scrambling cases,",
          len(out["pcfich"]), "PCFICH cases")


if __name__ == "__main__":
    main()
