"""GPU parity of the synchronisation, broadcast and HARQ-indicator drop-ins:
oai4g_generate_pss / _sss (pss.c:50, sss.c:47), oai4g_generate_pbch (pbch.c:161, state kept
across frame_mod4 0..3) and oai4g_generate_phich (phich.c:401) against the oracle restatement,
which tests/test_sync_cpu.py pins to the reference tables and the 36.211 / 36.212 model.
Bit-exact on whole frame grids pre-filled with random values, so the '=' (PSS / SSS) and '+='
(PBCH / PHICH, int16 wrap) semantics and the untouched REs are all checked."""
import numpy as np
import pytest

import oracle_lib as O
from test_sync_cpu import PBCH, PHICH, SYNC

pytestmark = pytest.mark.gpu


def _pair(gpu, N_RB, nid, n_ant, mode1, Ncp=0):
    fo = O.frame(N_RB, Nid_cell=nid, Ncp=Ncp, nb_antennas_tx=n_ant, mode1_flag=mode1)
    fg = gpu.frame_parms(N_RB, Nid_cell=nid, Ncp=Ncp, nb_antennas_tx=n_ant, mode1_flag=mode1)
    return fo, fg


def _rand_grids(fp, n_ant, seed, n_sf=10):
    rng = np.random.default_rng(seed)
    nsymb = 14 if fp.Ncp == 0 else 12
    base = [rng.integers(-2**31, 2**31 - 1, n_sf * nsymb * fp.ofdm_symbol_size + fp.ofdm_symbol_size,
                         dtype=np.int64).astype(np.int32) for _ in range(n_ant)]
    return [b.copy() for b in base], [b.copy() for b in base]


@pytest.mark.parametrize("N_RB,nid,n_ant,mode1,Ncp", SYNC)
def test_gpu_pss_sss(gpu, N_RB, nid, n_ant, mode1, Ncp):
    fo, fg = _pair(gpu, N_RB, nid, n_ant, mode1, Ncp)
    go, gg = _rand_grids(fo, n_ant, nid + N_RB)
    nsl = 7 if Ncp == 0 else 6
    for so in (0, 10):
        assert O.generate_pss(go, 512, fo, nsl - 1, so) == 0
        assert O.generate_sss(go, 512, fo, nsl - 2, so) == 0
        assert gpu.generate_pss(gg, 512, fg, nsl - 1, so) == 0
        assert gpu.generate_sss(gg, 512, fg, nsl - 2, so) == 0
    for a in range(n_ant):
        assert np.array_equal(gg[a], go[a]), a


@pytest.mark.parametrize("N_RB,nid,n_ant,mode1,Ncp", PBCH)
def test_gpu_pbch(gpu, N_RB, nid, n_ant, mode1, Ncp):
    fo, fg = _pair(gpu, N_RB, nid, n_ant, mode1, Ncp)
    pdu = np.random.default_rng(nid).integers(0, 256, 3, dtype=np.uint8)
    so, sg = O.OrcPbch(), gpu.Pbch()
    for fm4 in range(4):
        go, gg = _rand_grids(fo, n_ant, 100 * fm4 + nid, n_sf=1)
        assert O.generate_pbch(so, go, 512, fo, pdu, fm4) == 0
        assert gpu.generate_pbch(sg, gg, 512, fg, pdu, fm4) == 0
        E = 1920 if Ncp == 0 else 1728
        assert bytes(sg.pbch_e)[:E] == bytes(so.pbch_e)[:E]
        for a in range(n_ant):
            assert np.array_equal(gg[a], go[a]), (fm4, a)


@pytest.mark.parametrize("N_RB,nid,n_ant,mode1", PHICH)
def test_gpu_phich(gpu, N_RB, nid, n_ant, mode1):
    fo, fg = _pair(gpu, N_RB, nid, n_ant, mode1)
    ngroups = len(O.phich_reg_mapping(fo))
    rng = np.random.default_rng(nid + 3)
    for sf in (0, 5, 9):
        go, gg = _rand_grids(fo, n_ant, sf + nid)
        for _ in range(3):
            ngroup, nseq, hi = int(rng.integers(0, ngroups)), int(rng.integers(0, 8)), int(rng.integers(0, 2))
            assert O.generate_phich(fo, 512, nseq, ngroup, hi, sf, go) == 0
            assert gpu.generate_phich(fg, 512, nseq, ngroup, hi, sf, gg) == 0
        for a in range(n_ant):
            assert np.array_equal(gg[a], go[a]), (sf, a)


def test_gpu_phich_errors_and_group_seq(gpu):
    fg = gpu.frame_parms(25, Nid_cell=3)                # nushift 3: the reference reads past its arrays
    g = [np.zeros(10 * 14 * fg.ofdm_symbol_size + fg.ofdm_symbol_size, np.int32)]
    assert gpu.generate_phich(fg, 512, 0, 0, 1, 0, g) == -1
    fg = gpu.frame_parms(25, Nid_cell=1)
    assert gpu.generate_phich(fg, 512, 8, 0, 1, 0, g) == -1
    assert gpu.generate_phich(fg, 512, 0, 99, 1, 0, g) == -1
    # generate_phich_top (phich.c:1449-1465): Ngroup = ceil(6 * 25 / 48) = 4 with Ng = 1
    assert gpu.phich_group_seq(fg, 13, 2) == ((13 + 2) % 4, (13 // 4 + 2) % 8)
