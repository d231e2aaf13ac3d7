"""Generate tests/golden/llr_ref.json from the reference's dlsch_llr_computation.c compiled unmodified
here (oracle/_ref/libref_llr.so; `make -C oracle ref`).  Inputs come from tests/llr_ref_cases.py
(splitmix64), so only the case list and the digests of the LLRs the reference writes are stored.

    python tests/golden/gen_llr_ref.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import oracle_lib as O  # noqa: E402
from llr_ref_cases import digest, ia_cases, ia_written, qam_cases, qam_written  # noqa: E402
from test_ref_pin_llr_cpu import ref_ia, ref_qam  # noqa: E402


def main():
    assert O.ref_llr() is not None, "build the reference objects first: make -C oracle ref"
    out = {"source": "PHY/LTE_TRANSPORT/dlsch_llr_computation.c (compiled unmodified, oracle/_ref/libref_llr.so)",
           "qam": [], "ia": []}
    for c in qam_cases():
        n, llr = ref_qam(c)
        out["qam"].append(dict(case=c, advance=int(n), digest=digest(llr[:c["Qm"] * qam_written(c)])))
    for c in ia_cases():
        o = ref_ia(c)
        out["ia"].append(dict(case=c, digest=digest(o[:2 * ia_written(c["n"])])))
    path = os.path.join(HERE, "llr_ref.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path, len(out["qam"]), "QAM cases,", len(out["ia"]), "interference-aware cases")


if __name__ == "__main__":
    main()
