"""GPU parity against the reference's own rate matcher and Gold generator (lte_rate_matching.c,
lte_gold.c compiled unmodified in the build container; their outputs travel as
tests/golden/rm_ref.{json,npz}, made by tests/golden/gen_rm_ref.py).

  - every drop-in (sub_block_interleaving_turbo, lte_rate_matching_turbo, generate_dummy_w,
    lte_rate_matching_turbo_rx, sub_block_deinterleaving_turbo, lte_gold_generic) reproduces the
    reference's digests over the 188-K sweeps (tests/rm_ref_cases.py);
  - the bench batch's e bits (C3 at 8192 subframes with the bench's device-generated payloads, C2 at
    1024, C1): for sampled subframes, e = the reference's composed sub-block interleaver + rate
    matcher map applied to the turbo output d of every block, XOR the reference's Gold bits of
    dlsch_scrambling's c_init.  The turbo output d comes from the library's own dlsch_encoding
    drop-in (the turbo encoder has no buildable reference TU: lte_interleaver.h is a missing blob)."""
import os

import numpy as np
import pytest

import rm_ref_cases as RC
from test_rm_ref_fixture_cpu import ARR, check_sweeps

pytestmark = pytest.mark.gpu
SEED = 0x5EED0000                           # bench.py: payload_seed(0x5EED0000, rank 0)


def test_dropins_reproduce_reference_digests(gpu):
    check_sweeps(RC.gpu_impl(gpu))


@pytest.mark.parametrize("name", sorted(RC.MAP_GEOMS))
def test_dropin_rm_map_equals_reference(gpu, name):
    K, G, C, Qm, Kmimo, Nl = RC.MAP_GEOMS[name]
    got = RC.rm_map(RC.gpu_impl(gpu), K, G, C, C - 1, Qm, Kmimo, Nl)
    assert np.array_equal(got, ARR["map_" + name].astype(np.int32))


def _expected_e(gpu, p, payload, cw, subframe, G):
    """Reference map + reference Gold over the drop-in encoder's d buffers."""
    name = {(6, 1): "C1", (100, 1): "C2", (100, 2): "C3"}[(p.N_RB_DL, p.Kmimo)]
    K, Gm, C, Qm, Kmimo, Nl = RC.MAP_GEOMS[name]
    assert G == Gm
    fp = gpu.frame_parms(p.N_RB_DL, p.Nid_cell, 0, p.nb_antennas_tx, p.mode1_flag, 0)
    dl = gpu.DlschHandle(Kmimo=p.Kmimo, Mdlharq=8, N_RB_DL=p.N_RB_DL)
    h = dl.h
    h.TBS, h.mcs, h.rvidx, h.round, h.mimo_mode, h.Nl = p.TBS[cw], p.mcs[cw], 0, 0, p.mimo_mode, 1
    for i in range(4):
        h.rb_alloc[i] = p.rb_alloc[i]
    h.nb_rb = p.nb_rb
    dl.d.rnti = p.rnti
    a = np.zeros(p.TBS[cw] // 8 + 16, np.uint8)
    a[:p.TBS[cw] // 8] = payload[:p.TBS[cw] // 8]
    assert gpu.dlsch_encoding(a, fp, p.num_pdcch_symbols, dl, subframe) == 0
    assert h.C == C and h.Kplus == K
    m = ARR["map_" + name].astype(np.int64)
    e = np.concatenate([dl.view("d", 96 + 3 * K + 12, r)[m] for r in range(C)])
    dl.close()
    gold = RC.gold_bits(ARR["gold_sf"][subframe], G)
    return (e & 1) ^ gold


@pytest.mark.parametrize("name,n_sf", [("C3", 8192), ("C2", 1024), ("C1", 64)])
def test_bench_batch_ebits_against_reference_rm_and_gold(gpu, name, n_sf):
    p = gpu.make_params(name, subframe=7)
    pipe = gpu.TxPipeline(p, n_sf)
    pipe.fill_payload(seed=SEED)
    pipe.run()
    pipe.sync()
    pay = pipe.download_payload()
    eb = pipe.ebits()
    rng = np.random.default_rng(n_sf)
    for i in sorted({0, n_sf - 1, *rng.integers(0, n_sf, 3).tolist()}):
        for cw in range(p.n_cw):
            G = pipe.G(cw, 7)
            assert np.array_equal(gpu.unpack_bits(eb[i, cw], G), _expected_e(gpu, p, pay[i, cw], cw, 7, G)), \
                (name, i, cw)
    pipe.close()
