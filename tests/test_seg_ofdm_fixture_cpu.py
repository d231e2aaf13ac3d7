"""The oracle's segmentation and OFDM modulator reproduce the reference-generated fixtures
(tests/golden/seg_ofdm_ref.{json,npz}, made by tests/golden/gen_seg_ofdm_ref.py from the reference's
lte_segmentation.c / ofdm_mod.c compiled unmodified).  Runs everywhere (the fixtures travel; the
reference does not): the pin of tests/test_ref_pin_seg_ofdm_cpu.py, carried to the GPU box."""
import json
import os

import numpy as np

import oracle_lib as O
import seg_ofdm_ref_cases as SC

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "seg_ofdm_ref.json")))
ARR = np.load(os.path.join(HERE, "golden", "seg_ofdm_ref.npz"))


def check_seg(impl, stride=1):
    """Every parameter row (every `stride`-th) and every code-block digest of the fixture."""
    Bs = ARR["seg_B"][::stride]
    got = SC.run_seg_params(impl, Bs)
    want = ARR["seg_params"][::stride]
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert len(bad) == 0, [(int(Bs[i]), got[i].tolist(), want[i].tolist()) for i in bad[:5]]
    for B, (vals, dg) in FIX["seg_data"].items():
        v, bufs = SC.run_seg_data(impl, int(B))
        assert list(v) == vals and SC.digest(bufs) == dg, ("seg_data", B)


def check_ofdm(impl, frame_parms):
    """Every OFDM digest of the fixture; frame_parms(N_RB, Ncp, n_ant) builds the frame the impl
    takes (an OrcFrame for the oracle, the same geometry is read by the GPU impl)."""
    for case in SC.OFDM_CASES:
        assert SC.digest(SC.run_ofdm_mod(impl, case)) == FIX["ofdm_mod"]["%d,%d,%d" % case], ("ofdm_mod", case)
    for (n_rb, ncp) in SC.NPM_FRAMES:
        fp = frame_parms(n_rb, ncp, 1)
        for nsymb in SC.NPM_NSYMB:
            assert SC.digest(SC.run_npm(impl, fp, nsymb)) == FIX["npm"]["%d,%d,%d" % (n_rb, ncp, nsymb)], \
                ("npm", n_rb, ncp, nsymb)
    for (n_rb, ncp, na) in SC.DO_OFDM_FRAMES:
        fp = frame_parms(n_rb, ncp, na)
        for slot in SC.DO_OFDM_SLOTS:
            assert SC.digest(SC.run_do_ofdm(impl, fp, 3, slot)) == FIX["do_ofdm"]["%d,%d,%d,%d" % (n_rb, ncp, na, slot)], \
                ("do_ofdm", n_rb, ncp, na, slot)


def oracle_frame(n_rb, ncp, na):
    return O.frame(n_rb, Ncp=ncp, nb_antennas_tx=na, mode1_flag=1 if na == 1 else 0)


def test_oracle_segmentation_reproduces_reference():
    check_seg(SC.oracle_impl(O))


def test_oracle_ofdm_reproduces_reference():
    check_ofdm(SC.oracle_impl(O), oracle_frame)


def test_fixture_coverage():
    p = ARR["seg_params"]
    assert len(ARR["seg_B"]) > 20000 and p.shape[1] == 7
    assert (p[:, 0] == -1).sum() >= 4                      # the C > 16 refusal (:69-72)
    ok = p[p[:, 0] == 0]
    assert ok[:, 1].max() == 16 and (ok[:, 6] > 0).any()   # C up to 16, filler bits F > 0
    assert ((ok[:, 1] > 1) & (ok[:, 3] > 0)).any()         # C > 1 with K- blocks
    multi = [B for B, (v, _) in FIX["seg_data"].items() if v[0] > 1]
    assert len(multi) > 50 and any(v[5] > 0 for v, _ in FIX["seg_data"].values())
    assert len(FIX["ofdm_mod"]) == len(SC.OFDM_CASES) and len(FIX["npm"]) == 9 * len(SC.NPM_NSYMB)
    assert len(FIX["do_ofdm"]) == len(SC.DO_OFDM_FRAMES) * len(SC.DO_OFDM_SLOTS)


def test_oracle_chain_bench_c3_subframes_equal_reference_ofdm():
    """The oracle's whole transmit chain (orc_tx_subframe, its own OFDM modulator) on the sampled C3
    bench subframes equals the reference's do_OFDM_mod applied to the oracle's grid."""
    p = SC.bench_c3_params()
    pay = SC.bench_payload(SC.BENCH_SEED, SC.BENCH_N_SF, p.n_cw, p.payload_stride)
    cfg = O.tx_cfg_from_params(p, 7)
    for i in SC.BENCH_C3_SAMPLES[:3]:
        txd, _, _ = O.tx_subframe(cfg, [pay[i, cw] for cw in range(p.n_cw)])
        assert [SC.digest(txd[a]) for a in range(len(txd))] == FIX["bench_C3"][str(i)], i
