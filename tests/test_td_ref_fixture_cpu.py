"""The oracle's turbo encoder reproduces every codeword the reference's scalar decoder was run on
(tests/golden/td_ref.json, made by tests/golden/gen_td_ref.py with PHY/CODING/3gpplte_turbo_decoder.c
compiled unmodified).  Runs everywhere (the fixture travels; the reference does not): the pin of
tests/test_ref_pin_td_cpu.py, carried to the GPU box."""
import json
import os

import numpy as np

import oracle_lib as O
import td_ref_cases as TC
from ref_cases import QPP

FIX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "td_ref.json")))


def test_fixture_covers_every_K_and_every_variant_decoded():
    assert FIX["amp"] == TC.AMP and FIX["max_it"] == TC.MAX_IT and FIX["flip_frac"] == TC.FLIP_FRAC
    assert sorted(int(k) for k in FIX["blocks"]) == list(TC.KS)
    for K, row in FIX["blocks"].items():
        for v in TC.VARIANTS:
            assert row[v][0] <= TC.MAX_IT and row[v][1] == row["c"], (K, v)
        for v in TC.NEG_VARIANTS:
            assert row["neg_" + v][0] == TC.MAX_IT + 1 and row["neg_" + v][1] != row["c"], (K, v)


def test_oracle_encoder_reproduces_the_reference_decoded_codewords():
    for K, crc_type, c in TC.blocks():
        row = FIX["blocks"][str(K)]
        assert TC.digest(c) == row["c"] and crc_type == row["crc"]
        assert TC.digest(O.turbo_encode(c, *QPP[K])[:3 * K + 12]) == row["d"], K


def test_variants_keep_their_streams():
    K = 104
    d = np.arange(3 * K + 12) % 2
    s = TC.sys_positions(K)
    assert np.all(TC.variant(d, K, "nosys")[s] == 0)
    z = TC.variant(d, K, "z_only")
    assert np.all(z[2:3 * K:3] == 0) and np.all(z[1:3 * K:3] != 0) and np.all(z[3 * K + 7::2] == 0)
    zp = TC.variant(d, K, "zp_only")
    assert np.all(zp[1:3 * K:3] == 0) and np.all(zp[2:3 * K:3] != 0) and np.all(zp[3 * K + 1:3 * K + 6:2] == 0)
    f = TC.variant(d, K, "flip")
    assert np.sum(f[0:3 * K:3] != (d[0:3 * K:3] * 2 - 1) * TC.AMP_FLIP) == int(TC.FLIP_FRAC * K)
