#!/bin/bash
# 8-bit decoder: parity of every library, then the C5 8-bit bench per library (x2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep8
for lib in openair4g_amd/lib/libopenair4g_amd.so variants/*/libopenair4g_amd.so; do
  OAI4G_LIB=$PWD/$lib timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_decoder8.py > gpurun_out/sweep8/p.log 2>&1 || { echo "$lib parity FAIL"; tail -5 gpurun_out/sweep8/p.log; exit 1; }
done
echo parity ok
for rep in 1 2; do
  for lib in openair4g_amd/lib/libopenair4g_amd.so variants/*/libopenair4g_amd.so; do
    OAI4G_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --config C5 --c5-bits 8 --no-cpu-baseline > gpurun_out/sweep8/b.log 2>&1 || { tail -3 gpurun_out/sweep8/b.log; exit 1; }
    echo "$lib $(grep -o '"value": [0-9.]*' gpurun_out/sweep8/b.log)"
  done
done
