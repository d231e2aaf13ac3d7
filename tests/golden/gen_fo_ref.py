"""Generate tests/golden/fo_ref.json from the reference's lte_est_freq_offset.c compiled unmodified here
(oracle/_ref/libref_fo.so; `make -C oracle ref`): per case of tests/fo_ref_cases.py, the return value
and *freq_offset after each call of the sequence.

    python tests/golden/gen_fo_ref.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import oracle_lib as O  # noqa: E402
from fo_ref_cases import fo_cases  # noqa: E402
from test_ref_pin_fo_cpu import ref_sequence  # noqa: E402


def main():
    assert O.ref_fo() is not None, "build the reference objects first: make -C oracle ref"
    out = {"source": "PHY/LTE_ESTIMATION/lte_est_freq_offset.c (compiled unmodified, oracle/_ref/libref_fo.so)",
           "cases": [dict(case=c, calls=ref_sequence(c)) for c in fo_cases()]}
    path = os.path.join(HERE, "fo_ref.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path, len(out["cases"]), "cases")


if __name__ == "__main__":
    main()
