#!/bin/bash
# Encoder A/B: GPU parity of the transmit path, then per-phase encoder times and the C3 bench for the
# in-tree library and every variants/*/libopenair4g_amd.so.
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_bench_size.py tests/test_gpu_filler.py tests/test_gpu_rm_limited.py tests/test_gpu_golden.py tests/test_gpu_control_batch.py tests/test_gpu_common_batch.py tests/test_gpu_host_c.py > gpurun_out/enc_tests.log 2>&1 || { tail -30 gpurun_out/enc_tests.log; exit 1; }
tail -2 gpurun_out/enc_tests.log
for lib in openair4g_amd/lib/libopenair4g_amd.so variants/*/libopenair4g_amd.so; do
  [ -f "$lib" ] || continue
  echo "== $lib"
  OAI4G_LIB=$PWD/$lib timeout -k 10 120 python tools/diag_phases.py C3 8192 || exit 1
  OAI4G_LIB=$PWD/$lib timeout -k 10 120 python bench.py --steps 20 --no-cpu-baseline > gpurun_out/b.log 2>&1 || exit 1
  grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}' gpurun_out/b.log
done
