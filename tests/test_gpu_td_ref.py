"""GPU turbo encoder pinned to a reference execution: the reference's own scalar turbo decoder
(PHY/CODING/3gpplte_turbo_decoder.c, compiled unmodified into oracle/_ref/libref_td.so; the variants
and the two reference overruns that shape them are in tests/td_ref_cases.py) decodes what the GPU
encodes.

  - the drop-in oai4g_threegpplte_turbo_encoder, all 188 K: d equals the codeword the reference decoded
    in tests/golden/td_ref.json (digest), and -- where oracle/_ref travelled with the tree -- every
    variant of the GPU's own d decodes live (nosys / z_only / zp_only / flip) and the neighbouring K's
    QPP fails;
  - the fused k_encode (its debug instantiation, through the dlsch_encoding drop-in) for C3 and C2:
    every code block's d decodes live to the block's c, z_only and zp_only included;
  - the C3 bench batch (8192 subframes, the production k_encode + the bench's device payloads):
    sampled subframes' scrambled e bits received with reference functions only (lte_gold_generic,
    lte_rate_matching_turbo_rx, sub_block_deinterleaving_turbo, this decoder; 3 % of the systematic
    bits flipped) give back the payload and its CRC24_A."""
import json
import os

import numpy as np
import pytest

import oracle_lib as O
import rm_ref_cases as RC
import seg_ofdm_ref_cases as SC
import td_ref_cases as TC
from ref_cases import QPP

pytestmark = pytest.mark.gpu
FIX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "td_ref.json")))
LIVE = O.ref_td() is not None and O.ref_rm() is not None and O.ref_gold() is not None
need_live = pytest.mark.skipif(not LIVE, reason="oracle/_ref (reference decoder / RM / Gold) not in this tree")


def test_dropin_encoder_equals_reference_decoded_codewords(gpu):
    for K, crc_type, c in TC.blocks():
        d = gpu.turbo_encode(c, *QPP[K])
        row = FIX["blocks"][str(K)]
        assert TC.digest(d[:3 * K + 12]) == row["d"], K
        if LIVE:
            live = TC.check_block(d, K, crc_type, c)
            assert all(live[k] == row[k] for k in live), K


@need_live
@pytest.mark.parametrize("name", ["C3", "C2"])
def test_fused_encoder_blocks_decode_with_reference(gpu, name):
    p = gpu.make_params(name, subframe=7)
    K, G, C, Qm, Kmimo, Nl = RC.MAP_GEOMS[name]
    pay = SC.bench_payload(SC.BENCH_SEED, 3, p.n_cw, p.payload_stride)[2]
    fp = gpu.frame_parms(p.N_RB_DL, p.Nid_cell, 0, p.nb_antennas_tx, p.mode1_flag, 0)
    for cw in range(p.n_cw):
        dl = gpu.DlschHandle(Kmimo=p.Kmimo, Mdlharq=8, N_RB_DL=p.N_RB_DL)
        h = dl.h
        h.TBS, h.mcs, h.rvidx, h.round, h.mimo_mode, h.Nl = p.TBS[cw], p.mcs[cw], 0, 0, p.mimo_mode, 1
        for i in range(4):
            h.rb_alloc[i] = p.rb_alloc[i]
        h.nb_rb = p.nb_rb
        dl.d.rnti = p.rnti
        a = np.zeros(p.TBS[cw] // 8 + 16, np.uint8)
        a[:p.TBS[cw] // 8] = pay[cw][:p.TBS[cw] // 8]
        assert gpu.dlsch_encoding(a, fp, p.num_pdcch_symbols, dl, 7) == 0
        assert h.C == C and h.Kplus == K and h.F == 0
        for r in range(C):
            c = dl.view("c", K // 8, r).copy()
            d = dl.view("d", 96 + 3 * K + 12, r)[96:].copy()
            for v in ("full", "z_only", "zp_only", "flip"):
                it, dec = TC.decode(TC.variant(d, K, v), K, 1)
                assert it <= TC.MAX_IT and np.array_equal(dec, c), (name, cw, r, v, it)
        dl.close()


@need_live
def test_c3_bench_batch_received_by_reference(gpu):
    p = gpu.make_params("C3", subframe=7)
    K, G, C, Qm, Kmimo, Nl = RC.MAP_GEOMS["C3"]
    pipe = gpu.TxPipeline(p, SC.BENCH_N_SF)
    pipe.fill_payload(seed=SC.BENCH_SEED)
    pipe.run()
    pipe.sync()
    pay = pipe.download_payload()
    eb = pipe.ebits()
    assert all(pipe.G(cw, 7) == G for cw in range(p.n_cw))
    pipe.close()
    golds = [RC.gold_bits(O.ref_gold_words(RC.c_init(p.rnti, p.q[cw], 7, p.Nid_cell), G // 32 + 1), G)
             for cw in range(p.n_cw)]
    for i in (0, 4097, SC.BENCH_N_SF - 1):
        for cw in range(p.n_cw):
            its, tb = TC.decode_codeword(gpu.unpack_bits(eb[i, cw], G), G, K, C, Qm, Kmimo, Nl, golds[cw],
                                         p.TBS[cw])
            assert all(it <= TC.MAX_IT for it in its), (i, cw, its)
            n = p.TBS[cw] // 8
            assert np.array_equal(tb[:n], pay[i, cw][:n]), (i, cw)
            v = O.crc24a(pay[i, cw][:n], 8 * n) >> 8
            assert list(tb[n:]) == [v >> 16, (v >> 8) & 255, v & 255], (i, cw)
