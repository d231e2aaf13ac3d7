#!/bin/bash
# decoder tuning sweep: parity of every variant library first, then the C5 bench per library (x2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
for lib in variants/*/libopenair4g_amd.so; do
  OAI4G_LIB=$PWD/$lib timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_decoder.py tests/test_gpu_decoder_cases.py > gpurun_out/sweep/p.log 2>&1 || { echo "$lib parity FAIL"; tail -5 gpurun_out/sweep/p.log; exit 1; }
done
for rep in 1 2; do
  for lib in openair4g_amd/lib/libopenair4g_amd.so variants/*/libopenair4g_amd.so; do
    OAI4G_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --config C5 --no-cpu-baseline > gpurun_out/sweep/b.log 2>&1 || exit 1
    echo "$lib $(grep -o '"value": [0-9.]*' gpurun_out/sweep/b.log)"
  done
done
