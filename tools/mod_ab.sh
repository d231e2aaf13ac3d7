#!/bin/bash
# Modulator A/B: parity of the transmit path with every variants/*/libopenair4g_amd.so, then the C3
# bench (kernel times per launch) for the in-tree library and each variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in variants/*/libopenair4g_amd.so; do
  [ -f "$lib" ] || continue
  OAI4G_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu \
      tests/test_gpu_parity.py tests/test_gpu_bench_size.py tests/test_gpu_common_batch.py > gpurun_out/mod_tests.log 2>&1 \
      || { echo "FAILED tests $lib"; tail -20 gpurun_out/mod_tests.log; exit 1; }
  echo "$lib: $(tail -1 gpurun_out/mod_tests.log)"
done
for rep in 1 2; do
  for lib in openair4g_amd/lib/libopenair4g_amd.so variants/*/libopenair4g_amd.so; do
    [ -f "$lib" ] || continue
    OAI4G_LIB=$PWD/$lib timeout -k 10 120 python bench.py --steps 20 --no-cpu-baseline > gpurun_out/b.log 2>&1 || exit 1
    echo "$lib $(grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}' gpurun_out/b.log | tr '\n' ' ')"
  done
done
