#!/bin/bash
# Modulator change check: transmit-path parity of the in-tree library, then C3 / full-grid / C4 A/B
# against every variants/*/libopenair4g_amd.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    tests/test_gpu_bench_size.py tests/test_gpu_common_batch.py tests/test_gpu_control_batch.py tests/test_gpu_golden.py \
    tests/test_gpu_host_c.py tests/test_gpu_tm2.py tests/test_gpu_filler.py tests/test_gpu_dist.py > gpurun_out/mod_tests.log 2>&1 \
  || { echo "FAILED tests"; grep -E "FAILED|Error" gpurun_out/mod_tests.log | head; tail -5 gpurun_out/mod_tests.log; exit 1; }
echo "in-tree: $(tail -1 gpurun_out/mod_tests.log)"
for rep in 1 2; do
  for args in "" "--full-grid" "--config C4"; do
    for lib in openair4g_amd/lib/libopenair4g_amd.so variants/*/libopenair4g_amd.so; do
      [ -f "$lib" ] || continue
      OAI4G_LIB=$PWD/$lib timeout -k 10 120 python bench.py $args --steps 20 --no-cpu-baseline > gpurun_out/b.log 2>&1 || exit 1
      echo "[$args] $lib $(grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}' gpurun_out/b.log | tr '\n' ' ')"
    done
  done
done
