"""Time the encoder kernel cut after each phase (diagnostic; outputs are invalid)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import openair4g_amd as oai  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C3"
n_sf = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
p = oai.make_params(name)
pipe = oai.TxPipeline(p, n_sf)
pipe.fill_payload(1)
prev = 0.0
for ph, label in [(0, "load+gold"), (1, "crc"), (2, "segment"), (23, "qpp-ilv"), (3, "turbo"), (4, "w-build"), (99, "rm+store")]:
    ms = pipe.diag_encode_phase_ms(ph, 5)
    print(f"phase<= {ph:2d} {label:10s} cumulative {ms*1e3:9.1f} us   (+{(ms-prev)*1e3:8.1f})")
    prev = ms
a, b = pipe.run_timed()
print(f"encode {a*1e3:.1f} us  modofdm {b*1e3:.1f} us  for {n_sf} subframes")
