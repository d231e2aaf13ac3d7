"""Synchronisation, broadcast and HARQ-indicator channels: the CPU oracle
(oracle/oai_oracle_sync.c, a restatement of pss.c / sss.c / pbch.c / phich.c) pinned
  - to the reference's own PSS / SSS tables entry by entry (PHY/LTE_REFSIG/primary_synch.h,
    PHY/LTE_TRANSPORT/sss.h, read as data when the reference tree is present), and
  - to the independent 36.211 6.6 / 6.9 / 6.11 + 36.212 5.3.1 / 5.3.5 spec model
    (tests/spec_model.py: sync_grid, pbch_grid, phich_grid) on whole frame grids for 1 and 2
    antennas, 6 / 15 / 25 / 50 / 100 PRB, both cyclic prefixes (PSS / SSS / PBCH) and several
    cell ids, frame_mod4 values, PHICH groups, sequences and HI values.
No GPU needed."""
import os
import re

import numpy as np
import pytest

import oracle_lib as O
import spec_model as S

REF = "/root/reference/openair1/PHY"


def _ref_table(path, name, count):
    src = open(path).read()
    body = src[src.index(name + "["):]
    vals = [int(x) for x in re.findall(r"-?\d+", body[body.index("{"):body.index("}")])]
    assert len(vals) == count
    return vals


@pytest.mark.skipif(not os.path.exists(REF), reason="reference tree absent")
def test_pss_tables_equal_reference():
    path = os.path.join(REF, "LTE_REFSIG/primary_synch.h")
    for nid2 in range(3):
        ref = _ref_table(path, f"primary_synch{nid2}", 144)
        assert O.primary_synch(nid2).tolist() == ref
        spec = S.pss_seq(nid2)
        assert [v for n in range(62) for v in spec[n]] == ref[10:134]


@pytest.mark.skipif(not os.path.exists(REF), reason="reference tree absent")
def test_sss_tables_equal_reference():
    path = os.path.join(REF, "LTE_TRANSPORT/sss.h")
    d0 = _ref_table(path, "d0_sss", 504 * 62)
    d5 = _ref_table(path, "d5_sss", 504 * 62)
    for nid in range(504):
        assert O.sss_seq(nid, 0).tolist() == d0[62 * nid:62 * nid + 62], nid
        assert O.sss_seq(nid, 1).tolist() == d5[62 * nid:62 * nid + 62], nid
        if nid % 37 == 0:
            assert S.sss_seq(nid, False) == d0[62 * nid:62 * nid + 62]
            assert S.sss_seq(nid, True) == d5[62 * nid:62 * nid + 62]


def _fp(N_RB, nid, n_ant, mode1, Ncp=0):
    fp = O.frame(N_RB, Nid_cell=nid, Ncp=Ncp, nb_antennas_tx=n_ant, mode1_flag=mode1)
    return fp


def _grids(fp, n_sf=10):
    nsymb = 14 if fp.Ncp == 0 else 12
    return [np.zeros(n_sf * nsymb * fp.ofdm_symbol_size + fp.ofdm_symbol_size, np.int32)
            for _ in range(fp.nb_antennas_tx)]


def _iq(v):
    lo, hi = v & 0xFFFF, (v >> 16) & 0xFFFF
    return lo - (lo >> 15) * 65536, hi - (hi >> 15) * 65536


SYNC = [(6, 0, 1, 1, 0), (15, 7, 2, 0, 0), (25, 302, 1, 1, 1), (50, 11, 2, 0, 0), (100, 0, 2, 0, 0),
        (100, 503, 1, 1, 0), (100, 250, 2, 1, 1)]


@pytest.mark.parametrize("N_RB,nid,n_ant,mode1,Ncp", SYNC)
def test_pss_sss_match_spec(N_RB, nid, n_ant, mode1, Ncp):
    fp = _fp(N_RB, nid, n_ant, mode1, Ncp)
    g = _grids(fp)
    nsl = 7 if Ncp == 0 else 6
    for so in (0, 10):                                   # phy_procedures_lte_eNb.c:1547-1556, 1700-1711
        assert O.generate_pss(g, 512, fp, nsl - 1, so) == 0
        assert O.generate_sss(g, 512, fp, nsl - 2, so) == 0
    want = S.sync_grid(N_RB, nid, 512, fp.ofdm_symbol_size, fp.first_carrier_offset, n_ant, Ncp)
    N, nsymb = fp.ofdm_symbol_size, 2 * nsl
    for a in range(n_ant):
        nz = {int(i) for i in np.nonzero(g[a])[0]}
        for (sf, l, b), v in want.items():
            idx = (sf * nsymb + l) * N + b
            assert _iq(int(g[a][idx]) & 0xFFFFFFFF) == tuple(v), (a, sf, l, b)
            nz.discard(idx)
        assert not nz, f"stray REs {sorted(nz)[:5]}"


PBCH = [(6, 0, 1, 1, 0), (6, 5, 2, 0, 0), (25, 17, 2, 0, 1), (50, 100, 1, 1, 0), (100, 0, 2, 0, 0),
        (100, 3, 2, 0, 1), (100, 301, 1, 1, 1), (15, 8, 2, 1, 0)]


@pytest.mark.parametrize("N_RB,nid,n_ant,mode1,Ncp", PBCH)
def test_pbch_matches_spec(N_RB, nid, n_ant, mode1, Ncp):
    fp = _fp(N_RB, nid, n_ant, mode1, Ncp)
    rng = np.random.default_rng(N_RB * 1000 + nid)
    pdu = rng.integers(0, 256, 3, dtype=np.uint8)
    st = O.OrcPbch()
    N = fp.ofdm_symbol_size
    for fm4 in range(4):                                 # the encoded block persists across frame_mod4
        g = _grids(fp, 1)
        assert O.generate_pbch(st, g, 512, fp, pdu, fm4) == 0
        want = S.pbch_grid(pdu, fm4, N_RB, nid, 512, N, fp.first_carrier_offset, mode1, n_ant,
                           n_ant_enb=n_ant, Ncp=Ncp)
        for a in range(n_ant):
            nz = {int(i) for i in np.nonzero(g[a])[0]}
            assert len(want[a]) == (240 if Ncp == 0 else 216)
            for (l, b), v in want[a].items():
                assert _iq(int(g[a][l * N + b]) & 0xFFFFFFFF) == tuple(v), (fm4, a, l, b)
                nz.discard(l * N + b)
            assert not nz


PHICH = [(6, 0, 1, 1), (6, 2, 2, 0), (25, 13, 2, 0), (50, 1, 1, 1), (100, 0, 2, 0), (100, 302, 2, 0),
         (100, 7, 1, 1), (15, 26, 2, 0)]


@pytest.mark.parametrize("N_RB,nid,n_ant,mode1", PHICH)
def test_phich_matches_spec(N_RB, nid, n_ant, mode1):
    fp = _fp(N_RB, nid, n_ant, mode1)
    N = fp.ofdm_symbol_size
    regs, _ = O.pcfich_reg_mapping(fp)
    ngroups = len(O.phich_reg_mapping(fp))
    rng = np.random.default_rng(nid + 7)
    for sf in (0, 4, 9):
        g = _grids(fp)
        want = [dict() for _ in range(n_ant)]
        for _ in range(4):                               # several PHICHs accumulate (generate_phich_top)
            ngroup, nseq, hi = int(rng.integers(0, ngroups)), int(rng.integers(0, 8)), int(rng.integers(0, 2))
            assert O.generate_phich(fp, 512, nseq, ngroup, hi, sf, g) == 0
            w = S.phich_grid(N_RB, nid, sf, ngroup, nseq, hi, 512, N, fp.first_carrier_offset, mode1, n_ant,
                             regs, Ng6=fp.phich_resource)
            for a in range(n_ant):
                for b, v in w[a].items():
                    r0, i0 = want[a].get(b, (0, 0))
                    want[a][b] = (S._w16(r0 + v[0]), S._w16(i0 + v[1]))
        for a in range(n_ant):
            nz = {int(i) for i in np.nonzero(g[a])[0]}
            for b, v in want[a].items():
                idx = sf * 14 * N + b
                assert _iq(int(g[a][idx]) & 0xFFFFFFFF) == tuple(v), (sf, a, b)
                nz.discard(idx)
            assert not {i for i in nz if g[a][i] != 0}


def test_phich_rejects_extended_prefix():
    fp = _fp(25, 0, 1, 1, Ncp=1)
    g = _grids(fp)
    assert O.generate_phich(fp, 512, 0, 0, 1, 0, g) == -1
