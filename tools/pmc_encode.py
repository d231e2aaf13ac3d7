"""Dispatch the encoder cut after phases 2, 3, 4 and in full (diagnostic, for rocprofv3 --pmc)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import openair4g_amd as oai  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C3"
n_sf = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
p = oai.make_params(name)
pipe = oai.TxPipeline(p, n_sf)
pipe.fill_payload(1)
for ph in (0, 1, 2, 23, 3, 4, 99):
    pipe.diag_encode_phase_ms(ph, 1)
pipe.run()
pipe.sync()
print("dispatched")
