"""Oracle turbo encoder pinned to a reference execution: the reference's own scalar turbo decoder
(oracle/_ref/libref_td.so = PHY/CODING/3gpplte_turbo_decoder.c compiled unmodified) decodes the
oracle's codewords.  Runs only in the build container, where /root/reference exists; the fixture
tests/golden/td_ref.json (tests/golden/gen_td_ref.py) carries the result to the GPU box.

  - all 188 K of 36.212 Table 5.1.3-3: every variant of tests/td_ref_cases.py (full, nosys, z_only,
    zp_only, flip) decodes to the encoder's input with the CRC passing, the neighbouring K's QPP does
    not (negative control), and the results equal the committed fixture;
  - a whole C3 and a C2 codeword (the oracle's encoder + sub-block interleaver + rate matcher +
    scrambler, bench payload) received with the reference's Gold, lte_rate_matching_turbo_rx,
    sub_block_deinterleaving_turbo and this decoder, 3 % of the systematic bits flipped: the transport
    block and its CRC24_A come back."""
import json
import os

import numpy as np
import pytest

import oracle_lib as O
import td_ref_cases as TC
from ref_cases import QPP

pytestmark = pytest.mark.skipif(O.ref_td() is None or O.ref_rm() is None or O.ref_gold() is None,
                                reason="oracle/_ref not built (no reference tree)")
FIX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "td_ref.json")))


def test_reference_decodes_oracle_codewords_all_K():
    for K, crc_type, c in TC.blocks():
        d = O.turbo_encode(c, *QPP[K])
        row = TC.check_block(d, K, crc_type, c)
        row.update({"c": TC.digest(c), "crc": crc_type, "d": TC.digest(d[:3 * K + 12])})
        assert row == FIX["blocks"][str(K)], K


def test_tails_do_not_reach_the_reference_decisions():
    """Documents why the tails stay spec-pinned: inverting every tail LLR changes nothing the
    decoder returns (termination commented out, :583-672)."""
    for K, crc_type, c in TC.blocks()[::37]:
        d = O.turbo_encode(c, *QPP[K])
        for v in ("z_only", "zp_only"):
            y = TC.variant(d, K, v)
            y[3 * K:] = -y[3 * K:]
            it, dec = TC.decode(y, K, crc_type)
            assert it == 1 and np.array_equal(dec, c)


@pytest.mark.parametrize("name", ["C3", "C2"])
def test_reference_receives_oracle_codeword(name):
    import rm_ref_cases as RC
    import seg_ofdm_ref_cases as SC
    import openair4g_amd as oai
    p = oai.make_params(name, subframe=7)
    pay = SC.bench_payload(SC.BENCH_SEED, 2, p.n_cw, p.payload_stride)[1]
    cfg = O.tx_cfg_from_params(p, 7)
    _, _, es = O.tx_subframe(cfg, [pay[cw] for cw in range(p.n_cw)], want_e=True)
    K, G, C, Qm, Kmimo, Nl = RC.MAP_GEOMS[name]
    for cw in range(p.n_cw):
        gold = RC.gold_bits(O.ref_gold_words(RC.c_init(p.rnti, p.q[cw], 7, p.Nid_cell), G // 32 + 1), G)
        its, tb = TC.decode_codeword(es[cw], G, K, C, Qm, Kmimo, Nl, gold, p.TBS[cw])
        assert all(it <= TC.MAX_IT for it in its), its
        n = p.TBS[cw] // 8
        assert np.array_equal(tb[:n], pay[cw][:n])
        v = O.ref_crc(pay[cw][:n], 8 * n, "24a") >> 8
        assert list(tb[n:]) == [v >> 16, (v >> 8) & 255, v & 255]
