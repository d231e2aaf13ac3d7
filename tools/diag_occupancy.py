"""Resident k_encode workgroups per CU and its dynamic LDS per workgroup for the bench configurations."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import openair4g_amd as oai  # noqa: E402

oai.init()
for name in ("C3", "C4", "C2", "C1"):
    p = oai.make_params(name, subframe=7, subframe_step=1)
    pipe = oai.TxPipeline(p, 64)
    occ, lds = ctypes.c_int(), ctypes.c_size_t()
    assert oai.lib().oai4g_diag_encode_occupancy(pipe.cfg, ctypes.byref(occ), ctypes.byref(lds)) == 0
    print(f"{name}: k_encode {occ.value} workgroups per CU, {lds.value} B LDS per workgroup")
    pipe.close()
