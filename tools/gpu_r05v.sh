#!/bin/bash
# round 5: C5 batch sweep, in-tree (2 waves per SIMD) vs variants/w3 (TD16_WAVES=3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in ${C5_BATCHES:-2048 4096 8192 16384}; do
  for lib in openair4g_amd/lib/libopenair4g_amd.so variants/w3/libopenair4g_amd.so; do
    OAI4G_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --config C5 --batch $b --steps 5 --no-cpu-baseline > gpurun_out/c5b.log 2>&1 || { tail -5 gpurun_out/c5b.log; exit 1; }
    echo "batch=$b $lib $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/c5b.log | tr '\n' ' ')"
  done
done
