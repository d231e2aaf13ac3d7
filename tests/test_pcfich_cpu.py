"""PCFICH: the oracle restatement of generate_pcfich (oracle/oai_oracle.c,
pcfich.c:48-228) against an independent 36.211 / 36.212 model (tests/spec_model.py: pcfich).  The
reference TU itself is pinned too: pcfich.c builds unmodified (oracle/_ref/libref_mod.so) and
tests/test_ref_pin_mod_cpu.py / test_mod_fixture_cpu.py / test_gpu_mod_ref.py compare against it."""
import numpy as np
import pytest

import oracle_lib as O
import spec_model as S

CASES = [(6, 0, 1, 1, 0), (25, 7, 2, 1, 3), (50, 101, 3, 0, 9), (100, 0, 1, 0, 5), (100, 503, 3, 1, 0),
         (15, 250, 2, 0, 7), (6, 5, 3, 0, 4), (50, 38, 2, 1, 8)]


@pytest.mark.parametrize("N_RB,Nid,cfi,mode1,subframe", CASES)
def test_oracle_pcfich_matches_spec_model(N_RB, Nid, cfi, mode1, subframe):
    n_ant = 1 if mode1 else 2
    fp = O.frame(N_RB, Nid_cell=Nid, nb_antennas_tx=n_ant, mode1_flag=mode1)
    N, nsymb = fp.ofdm_symbol_size, fp.symbols_per_tti
    grids = [np.full(10 * nsymb * N, 0x00070007, np.int32) for _ in range(n_ant)]
    assert O.generate_pcfich(cfi, 512, fp, grids, subframe) == 0
    exp = S.pcfich(N_RB, Nid, subframe, cfi, 512, N, fp.first_carrier_offset, mode1, n_ant)
    for a in range(n_ant):
        sym0 = grids[a][subframe * nsymb * N:(subframe * nsymb + 1) * N].view(np.int16).reshape(-1, 2)
        touched = {i for i in range(N) if tuple(sym0[i]) != (7, 7)}
        assert touched <= set(exp[a]) and len(exp[a]) == 16
        for idx, (re, im) in exp[a].items():
            assert tuple(int(v) for v in sym0[idx]) == (re, im), (a, idx)
        rest = np.delete(np.arange(len(grids[a])), [subframe * nsymb * N + i for i in exp[a]])
        assert np.all(grids[a][rest] == 0x00070007)


def test_oracle_pcfich_rejects_bad_cfi():
    fp = O.frame(25)
    g = [np.zeros(10 * 14 * fp.ofdm_symbol_size, np.int32)]
    assert O.generate_pcfich(0, 512, fp, g, 0) == -1
    assert O.generate_pcfich(4, 512, fp, g, 0) == -1
