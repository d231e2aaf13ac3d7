"""Generates tests/golden/td_ref.json from the reference's own scalar turbo decoder, compiled
unmodified in this container (oracle/Makefile: _ref/libref_td.so = PHY/CODING/3gpplte_turbo_decoder.c,
its CRCs from _ref/libref_coding.so).  The reference never travels; these outputs do.  Run from the
repo root:

    make -C oracle ref && python tests/golden/gen_td_ref.py

td_ref.json — one row per Table 5.1.3-3 size K (tests/td_ref_cases.py defines every case):
  c        digest of the seeded CRC-terminated block (td_ref_cases.blocks)
  crc      the CRC type the decoder checks (0 = CRC24_A, 1 = CRC24_B)
  d        digest of the oracle encoder's 3K+12 entry d for it: the codeword the reference decoded
  <v>      [iterations, digest(decoded bytes)] of phy_threegpplte_turbo_decoder_scalar for variant v
           (full / nosys / z_only / zp_only / flip); the decoded digest equals c's
  neg_<v>  the same with the neighbouring K's (f1, f2): iterations = max + 1 (CRC never matched)
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as O  # noqa: E402
import td_ref_cases as TC  # noqa: E402
from ref_cases import QPP  # noqa: E402


def main():
    assert O.ref_td() is not None, "build oracle/_ref first (make -C oracle ref)"
    out = {"amp": TC.AMP, "amp_flip": TC.AMP_FLIP, "flip_frac": TC.FLIP_FRAC, "max_it": TC.MAX_IT, "blocks": {}}
    for K, crc_type, c in TC.blocks():
        d = O.turbo_encode(c, *QPP[K])
        row = TC.check_block(d, K, crc_type, c)
        row.update({"c": TC.digest(c), "crc": crc_type, "d": TC.digest(d[:3 * K + 12])})
        out["blocks"][K] = row
    with open(os.path.join(HERE, "td_ref.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)


if __name__ == "__main__":
    main()
