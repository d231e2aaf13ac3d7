"""The oracle's lte_est_freq_offset (orc_fo_omega + orc_fo_update, oracle/oai_oracle_chest.c) against
the reference's own PHY/LTE_ESTIMATION/lte_est_freq_offset.c:104-193, compiled unmodified into
oracle/_ref/libref_fo.so (with PHY/TOOLS/cdot_prod.c and log2_approx.c from libref_tools.so):
*freq_offset after every call of a sequence, the static first_run and reset included, and the
refusal of a pilot row other than 0 or 4 - Ncp.  This pin found the reference's omega alias
(omega_cpx points at omega, :152-166: omega = twice the upper-half dot product), which the oracle and
the library now reproduce.  Skipped where the reference tree was not built here."""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
from fo_ref_cases import calls, fo_cases, fo_plane

pytestmark = pytest.mark.skipif(O.ref_fo() is None, reason="oracle/_ref/libref_fo.so not built (no reference tree)")


def ref_sequence(c):
    fp = O.frame(c["N_RB_DL"], Ncp=c["Ncp"])
    plane = O.aligned(fo_plane(c, fp.ofdm_symbol_size))
    f = ctypes.c_int(0)
    out = []
    for l, reset in calls(c):
        r = O.ref_fo().ref_glue_est_freq_offset(c["N_RB_DL"], c["Ncp"], fp.ofdm_symbol_size, plane.ctypes.data, l,
                                                ctypes.byref(f), reset)
        out.append((int(r), int(f.value)))
    return out


def orc_sequence(c):
    fp = O.frame(c["N_RB_DL"], Ncp=c["Ncp"])
    plane = fo_plane(c, fp.ofdm_symbol_size)
    st = O.FreqOffsetState()
    out = []
    for l, reset in calls(c):
        if l not in (0, 4 - c["Ncp"]):
            assert O.fo_omega(fp, plane, l) == -2 ** 31
            out.append((-1, int(st.f.value)))
            continue
        out.append((0, st.call(fp, plane, l, reset)))
    return out


@pytest.mark.parametrize("c", fo_cases(), ids=lambda c: f"{c['N_RB_DL']}prb-cp{c['Ncp']}-amp{c['amp']}")
def test_freq_offset_sequence_equals_reference(c):
    assert orc_sequence(c) == ref_sequence(c)
