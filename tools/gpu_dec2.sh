#!/bin/bash
# decoder parity (unit + cases + UL chain + bench size), then C5 bench for the in-tree library and variants/*
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_decoder.py tests/test_gpu_decoder_cases.py tests/test_gpu_ul_chain.py tests/test_gpu_bench_size.py > gpurun_out/pytest_dec.log 2>&1 || { tail -20 gpurun_out/pytest_dec.log; exit 1; }
tail -2 gpurun_out/pytest_dec.log
for rep in 1 2; do
  for lib in openair4g_amd/lib/libopenair4g_amd.so variants/*/libopenair4g_amd.so; do
    [ -f "$lib" ] || continue
    OAI4G_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --config C5 --no-cpu-baseline > gpurun_out/bench_C5.log 2>&1 || exit 1
    echo "$lib $(grep -o '"value": [0-9.]*' gpurun_out/bench_C5.log)"
  done
done
