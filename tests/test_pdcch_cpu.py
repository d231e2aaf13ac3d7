"""PDCCH / DCI oracle (orc_generate_dci_top, a restatement of dci.c:2024-2346) pinned to the
independent 36.212 5.3.3 / 36.211 6.7-6.9 spec model (tests/spec_model.py: pdcch_grid + pcfich):
the whole control region of the subframe (PCFICH + every PDCCH RE, PHICH REGs left empty) for 1
and 2 antennas (SISO / transmit diversity), 6 / 25 / 50 / 100 PRB, several cell ids, subframes,
aggregation levels, DCI sizes (the reference's 23 / 28 / 39 / 48-bit formats) and CCE positions
from get_nCCE_offset; plus the geometry helpers against the spec (nquad, PHICH REGs)."""
import numpy as np
import pytest

import oracle_lib as O
import spec_model as S


def _dcis(rng, fp, subframe, specs, mi=1):
    """specs: (length, L, common, rnti) -> items with nCCE from get_nCCE_offset (dlsim.c:1988-1999)"""
    items, table = [], np.zeros(800, np.int32)
    total = sum(1 << L for _, L, _, _ in specs)
    npd = next(n for n in (1, 2, 3) if total <= O.get_nCCE(n, fp, mi))
    nCCE = O.get_nCCE(npd, fp, mi)
    for length, L, common, rnti in specs:
        pdu = rng.integers(0, 256, 8, dtype=np.uint8)
        ncce = O.get_nCCE_offset(table, 1 << L, nCCE, common, rnti, subframe)
        items.append((length, L, ncce, rnti, pdu))
    return items, npd


CASES = [  # N_RB, n_ant, mode1, Nid, subframe, dci specs (length, L, common, rnti)
    (6, 1, 1, 0, 7, [(23, 1, 0, 0x1234)]),                       # C1: dlsim format 1, L = 2 CCEs
    (6, 2, 0, 13, 0, [(23, 0, 0, 0x1234), (28, 1, 1, 0xFFFF)]),
    (25, 1, 1, 5, 3, [(39, 1, 0, 0x1234), (28, 2, 1, 0xFFFF)]),
    (50, 2, 0, 301, 9, [(48, 1, 0, 0x1234), (39, 0, 0, 0x1235), (28, 3, 1, 0xFFFF)]),
    (100, 1, 1, 0, 7, [(39, 1, 0, 0x1234)]),                     # C2: format 1
    (100, 2, 0, 0, 7, [(48, 1, 0, 0x1234)]),                     # C3: format 2A
    (100, 2, 0, 77, 5, [(48, 2, 0, 0x2222), (39, 1, 0, 0x3333), (28, 3, 1, 0xFFFF), (28, 2, 1, 0xFFFE)]),
    (100, 1, 1, 4, 1, [(48, 3, 0, 0x1234)] * 1 + [(23, 0, 0, 0x4321 + i) for i in range(20)]),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}prb_{c[1]}tx_nid{c[3]}_sf{c[4]}_{len(c[5])}dci")
def test_generate_dci_top_matches_spec(case):
    N_RB, n_ant, mode1, nid, sf, specs = case
    rng = np.random.default_rng(N_RB * 1000 + nid)
    fp = O.frame(N_RB, nid, 0, n_ant, mode1)
    items, npd = _dcis(rng, fp, sf, specs)
    n_common = sum(1 for s in specs if s[2])
    order = [i for i, s in enumerate(specs) if s[2]] + [i for i, s in enumerate(specs) if not s[2]]
    items = [items[i] for i in order]                 # DCI_ALLOC_t: common DCIs first
    N, nsym = fp.ofdm_symbol_size, fp.symbols_per_tti
    grids = [np.zeros(10 * nsym * N, np.int32) for _ in range(n_ant)]
    got_npd = O.generate_dci_top(items, n_common, 512, fp, grids, sf)
    assert got_npd == npd
    exp = [np.zeros(nsym * N, np.uint32) for _ in range(n_ant)]
    for a, dct in enumerate(S.pcfich(N_RB, nid, sf, npd, 512, N, fp.first_carrier_offset, mode1, n_ant)):
        for k, (re, im) in dct.items():
            exp[a][k] = (re & 0xFFFF) | ((im & 0xFFFF) << 16)
    dcis = [(pdu, ln, L, ncce, rnti) for ln, L, ncce, rnti, pdu in items]
    for a, dct in enumerate(S.pdcch_grid(N_RB, nid, sf, dcis, npd, 512, N, fp.first_carrier_offset, mode1, n_ant)):
        for k, (re, im) in dct.items():
            assert exp[a][k] == 0
            exp[a][k] = (re & 0xFFFF) | ((im & 0xFFFF) << 16)
    for a in range(n_ant):
        sub = grids[a].reshape(10, nsym * N)
        assert np.array_equal(sub[sf].view(np.uint32), exp[a]), a
        assert not np.any(np.delete(sub, sf, axis=0))


@pytest.mark.parametrize("N_RB,nid", [(6, 0), (25, 7), (50, 301), (100, 0), (100, 503)])
def test_phich_regs_match_spec(N_RB, nid):
    fp = O.frame(N_RB, nid, 0, 2, 0)
    pcf, _ = O.pcfich_reg_mapping(fp)
    assert O.phich_reg_mapping(fp) == [tuple(g) for g in S.phich_regs(N_RB, nid, 6, pcf)]
    for npd in (1, 2, 3):
        assert O.get_nquad(npd, fp) == S.n_reg_pdcch(N_RB, npd) - 4 - 3 * len(S.phich_regs(N_RB, nid, 6, pcf))
