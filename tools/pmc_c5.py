"""Dispatch the C5 decoder a few times (diagnostic, for rocprofv3 --pmc)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import openair4g_amd as oai  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402

n_sf = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
oai.init()
llr = bench.c5_llrs(n_sf * bench.C5_CB, "8it", 0xC5)
dec = oai.TurboDecoderBatch(bench.C5_K, n_sf * bench.C5_CB)
dec.upload(llr)
for _ in range(2):
    dec.run(max_iterations=8, crc_type=1)
dec.results()
dec.close()
print("dispatched")
