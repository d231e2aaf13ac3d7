#!/usr/bin/env python3
"""Generate tests/golden/ref_coding.npz from the REFERENCE's own coding translation units
(oracle/_ref/libref_coding.so, built unmodified by oracle/Makefile; run in the dev container).

For every case of tests/ref_cases.py it stores the reference's outputs plus a digest of the
input the case generator produced, so the GPU test can regenerate the inputs (seeded numpy +
the reference-pinned oracle encoder) and check that they are the same inputs:
  enc_<i>   threegpplte_turbo_encoder output bytes, packed (np.packbits), for encoder_cases()[i]
  dec_<i>   [return value, decoded bytes...] of phy_threegpplte_turbo_decoder16 for decoder_cases()[i]
  meta      JSON: per case name, K, max_it, crc_type, F and the input digest
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import oracle_lib as O  # noqa: E402
from ref_cases import decoder_cases, digest, encoder_cases  # noqa: E402


def main():
    assert O.ref_coding() is not None, "build oracle/_ref first (make -C oracle ref)"
    out, meta = {}, {"enc": [], "dec": []}
    for i, (K, c) in enumerate(encoder_cases()):
        out[f"enc_{i}"] = np.packbits(O.ref_turbo_encode(c))
        meta["enc"].append({"K": K, "in": digest(c)})
    for i, (name, K, y, max_it, crc_type, F) in enumerate(decoder_cases()):
        it, dec = O.ref_turbo_decode(y, K, max_it, crc_type, F)
        out[f"dec_{i}"] = np.concatenate([[it], dec]).astype(np.uint8)
        meta["dec"].append({"name": name, "K": K, "max_it": max_it, "crc_type": crc_type, "F": F, "in": digest(y)})
    out["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "ref_coding.npz"), **out)
    print("wrote", len(meta["enc"]), "encoder and", len(meta["dec"]), "decoder cases")


if __name__ == "__main__":
    main()
