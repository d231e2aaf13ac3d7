"""generate_dci_top on the GPU (PCFICH + PDCCH kernels): bit-exact against the oracle (which
tests/test_pdcch_cpu.py pins to the 36.211/36.212 spec model) on the whole frame grid, for the
same cases: 1 / 2 antennas, 6-100 PRB, several cell ids, subframes, DCI sizes and aggregation
levels, including DCIs without a free CCE; every other RE of the grid untouched."""
import numpy as np
import pytest

import oracle_lib as O
from test_pdcch_cpu import CASES, _dcis

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}prb_{c[1]}tx_nid{c[3]}_sf{c[4]}_{len(c[5])}dci")
def test_generate_dci_top_gpu(gpu, case):
    N_RB, n_ant, mode1, nid, sf, specs = case
    rng = np.random.default_rng(N_RB * 1000 + nid)
    fpo = O.frame(N_RB, nid, 0, n_ant, mode1)
    items, npd = _dcis(rng, fpo, sf, specs)
    n_common = sum(1 for s in specs if s[2])
    order = [i for i, s in enumerate(specs) if s[2]] + [i for i, s in enumerate(specs) if not s[2]]
    items = [items[i] for i in order]
    N, nsym = fpo.ofdm_symbol_size, fpo.symbols_per_tti
    pre = [np.random.default_rng(a).integers(-999, 999, 10 * nsym * N).astype(np.int32) for a in range(n_ant)]
    ref = [p.copy() for p in pre]
    assert O.generate_dci_top(items, n_common, 512, fpo, ref, sf) == npd
    got = [p.copy() for p in pre]
    fp = gpu.frame_parms(N_RB, nid, 0, n_ant, mode1)
    assert gpu.generate_dci_top(items, n_common, 512, fp, got, sf) == npd
    for a in range(n_ant):
        assert np.array_equal(got[a], ref[a]), a


def test_dci_top_rejects_unsupported(gpu):
    fp = gpu.frame_parms(15, 0, 0, 1, 1)            # get_nquad has no 15-PRB geometry: 0 symbols
    g = [np.zeros(10 * 14 * fp.ofdm_symbol_size, np.int32)]
    assert gpu.generate_dci_top([(23, 0, 0, 0x1234, bytes(8))], 0, 512, fp, g, 0) == 0
    assert not g[0].any()
