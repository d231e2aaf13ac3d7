"""k_encode's two rate-matching placement paths against the oracle.

Phase 4 of k_encode places each transposed 32-bit run of w straight into the circular buffer's
output.  With no repetition (E <= Nnn for every block) it takes the `once` path, where the single
run that straddles the buffer's end (the block's wrap tile, rm_wrapt) is placed inline; any other
plan (E > Nnn, or a second straddling run, rm_wrapt = ~1, which no LTE geometry produces) takes the
general path with its repetition rounds.  OAI4G_ENC_GENERAL_RM (a host test hook, read when the
configuration is created) forces the general path for every block size.

Each case runs the batched pipeline on both paths and compares every subframe's e bits with the
oracle (lte_rate_matching_turbo restated, pinned to the reference's own TU in
test_ref_pin_rm_cpu.py): redundancy versions 0-3 (k0 = R (2 + 2 rv ceil(Ncb / 8R)) moves the wrap
tile across the block: rv 1-3 put it mid-block or on the block's last, odd tile), 1.4 / 5 / 10 /
20 MHz, QPSK to 64-QAM, 1 and 2 codewords (Kmimo 2 halves Ncb), subframes 0..9 (G changes with
the PBCH / sync exclusions), and configurations whose E exceeds Nnn (repetition: 6 PRB at a low
MCS)."""
import os

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

CASES = [("C1", {}), ("C2", {}), ("C3", {}), ("TM2", {}),
         ("C2", dict(N_RB_DL=25, rb_alloc=None, nb_rb=25, mcs=(4, 0))),
         ("C3", dict(N_RB_DL=50, rb_alloc=None, nb_rb=50, mcs=(12, 12))),
         ("C1", dict(mcs=(0, 0))),                 # 6 PRB, MCS 0: E > Nnn, the buffer repeats
         ("C1", dict(mcs=(2, 0)))]


def _run(gpu, name, over, rv, general):
    over = dict(over)
    if over.get("rb_alloc", 1) is None:
        over["rb_alloc"] = {25: gpu.FULL_ALLOC_25, 50: gpu.FULL_ALLOC_50}[over["N_RB_DL"]]
    if "mcs" in over:
        over["TBS"] = tuple(gpu.tbs_bits(m, over.get("nb_rb", 6 if name == "C1" else 100)) for m in over["mcs"])
    p = gpu.make_params(name, subframe=0, subframe_step=1, **over)
    for cw in range(p.n_cw):
        p.rvidx[cw] = rv
    if general:
        os.environ["OAI4G_ENC_GENERAL_RM"] = "1"
    try:
        pipe = gpu.TxPipeline(p, 10)
    finally:
        os.environ.pop("OAI4G_ENC_GENERAL_RM", None)
    pay = np.random.default_rng(31 * rv + len(name)).integers(0, 256, size=(10, p.n_cw, p.payload_stride),
                                                              dtype=np.uint8)
    pipe.upload_payload(pay)
    pipe.run()
    pipe.sync()
    eb = pipe.ebits()
    Gs = [[pipe.G(cw, sf) for cw in range(p.n_cw)] for sf in range(10)]
    pipe.close()
    return p, pay, eb, Gs


@pytest.mark.parametrize("name,over", CASES)
@pytest.mark.parametrize("rv", [0, 1, 2, 3])
def test_rm_placement_paths_equal_oracle(gpu, name, over, rv):
    runs = [_run(gpu, name, over, rv, general) for general in (False, True)]
    p, pay, _, Gs = runs[0]
    for sf in range(10):
        cfg = O.tx_cfg_from_params(p, sf)
        _, _, e_o = O.tx_subframe(cfg, [pay[sf, cw] for cw in range(p.n_cw)], want_e=True)
        for cw in range(p.n_cw):
            G = Gs[sf][cw]
            for k, (_, _, eb, _) in enumerate(runs):
                assert np.array_equal(gpu.unpack_bits(eb[sf, cw], G), e_o[cw][:G]), (name, over, rv, sf, cw,
                                                                                      "general" if k else "once")
