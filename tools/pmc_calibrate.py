"""PMC calibration dispatches: read then write a known 1 GiB at 4 B per lane (k_diag_stream)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import openair4g_amd as oai  # noqa: E402

oai.init()
L = oai.lib()
nbytes = 1 << 30
src, dst = L.oai4g_dev_alloc(nbytes), L.oai4g_dev_alloc(nbytes)
L.oai4g_memset_d(src, 1, nbytes)
for mode in (0, 1):
    assert L.oai4g_diag_stream(src, dst, nbytes, mode, None) == 0
L.oai4g_sync()
L.oai4g_dev_free(src)
L.oai4g_dev_free(dst)
print("calibration bytes", nbytes)
