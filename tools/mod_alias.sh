#!/bin/bash
# k_modofdm residency: staged QAM addresses aliased into the IDFT exchange (19.0 KB LDS per
# workgroup) at 3 and 4 waves/SIMD against the in-tree build; parity of the TX path per variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in variants/*/libopenair4g_amd.so; do
  OAI4G_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_tm2.py tests/test_gpu_tm3.py tests/test_gpu_golden.py tests/test_gpu_bench_size.py tests/test_gpu_control_batch.py > gpurun_out/alias_pytest.log 2>&1 || { echo "$lib FAILED"; tail -30 gpurun_out/alias_pytest.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/alias_pytest.log)"
done
for rep in 1 2; do
  for lib in openair4g_amd/lib/libopenair4g_amd.so variants/*/libopenair4g_amd.so; do
    OAI4G_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/alias.log 2>&1 || exit 1
    echo "$lib $(grep -o '"value": [0-9.]*\|"modulate_idft_cp": [0-9.]*' gpurun_out/alias.log | tr '\n' ' ')"
  done
done
for lib in openair4g_amd/lib/libopenair4g_amd.so variants/*/libopenair4g_amd.so; do
  OAI4G_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --full-grid --steps 20 --no-cpu-baseline > gpurun_out/alias.log 2>&1 || exit 1
  echo "full_grid $lib $(grep -o '"value": [0-9.]*\|"modulate_idft_cp": [0-9.]*' gpurun_out/alias.log | tr '\n' ' ')"
done
