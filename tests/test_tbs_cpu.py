"""MCS -> I_TBS -> TBS in the library (row A2): oai4g_get_I_TBS / oai4g_get_TBS_DL / oai4g_tbs_bits
(host code, no GPU needed) against the reference's own TBStable
(PHY/LTE_TRANSPORT/dlsch_tbs_full.h:34) and lte_mcs.c:45-155, entry by entry."""
import os
import re

import pytest

import openair4g_amd as oai

HDR = "/root/reference/openair1/PHY/LTE_TRANSPORT/dlsch_tbs_full.h"


def ref_table():
    src = open(HDR).read()
    body = src[src.index("TBStable[TBStable_rowCnt][110]"):]
    body = body[body.index("{"):body.index("};")]
    return [[int(x) for x in re.findall(r"\d+", r)] for r in re.findall(r"\{([^{}]*)\}", body)]


@pytest.mark.skipif(not os.path.exists(HDR), reason="reference tree absent")
def test_tbs_table_all_entries_equal_reference():
    L = oai.lib()
    t = ref_table()
    assert len(t) == 27
    for i in range(27):
        for n in range(1, 111):
            assert L.oai4g_tbs_bits(i, n) == t[i][n - 1], (i, n)
    assert L.oai4g_tbs_bits(6, 1) == 328          # the reference's entry (36.213 has 88), kept for parity
    assert L.oai4g_tbs_bits(27, 1) == 0 and L.oai4g_tbs_bits(0, 0) == 0 and L.oai4g_tbs_bits(0, 111) == 0


def test_mcs_mapping_as_lte_mcs_c():
    L = oai.lib()
    for mcs in range(32):
        i_tbs = mcs if mcs < 10 else 9 if mcs == 10 else mcs - 1 if mcs < 17 else 15 if mcs == 17 else mcs - 2
        assert L.oai4g_get_I_TBS(mcs) == i_tbs
        assert L.oai4g_get_I_TBS_UL(mcs) == (mcs if mcs <= 10 else mcs - 1 if mcs < 21 else mcs - 2)
        assert L.oai4g_get_Qm(mcs) == (2 if mcs < 10 else 4 if mcs < 17 else 6)
        assert L.oai4g_get_Qm_ul(mcs) == (2 if mcs < 11 else 4 if mcs < 21 else 6)
        for nb_rb in (0, 1, 6, 25, 100, 110):
            want = 0 if (nb_rb == 0 or mcs >= 29) else L.oai4g_tbs_bits(i_tbs, nb_rb) >> 3
            assert L.oai4g_get_TBS_DL(mcs, nb_rb) == want


def test_survey_config_tbs():
    """C1 936, C2 30576, C3 36696 per CW, C5 (UL MCS 20) 43816."""
    assert oai.tbs_bits(9, 6) == 936
    assert oai.tbs_bits(16, 100) == 30576
    assert oai.tbs_bits(19, 100) == 36696
    assert oai.lib().oai4g_get_TBS_UL(20, 100) * 8 == 43816
    for name in ("C1", "C2", "C3", "C4", "TM2", "TM2S"):
        p = oai.make_params(name)
        assert p.TBS[0] == oai.tbs_bits(p.mcs[0], p.nb_rb)
