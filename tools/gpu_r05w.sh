#!/bin/bash
# round 5: C5 at large batches with variants/w3 (TD16_WAVES=3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in 32768 49152; do
  OAI4G_LIB=$PWD/variants/w3/libopenair4g_amd.so timeout -k 10 300 python3 bench.py --config C5 --batch $b --steps 5 --no-cpu-baseline > gpurun_out/c5b.log 2>&1 || { tail -5 gpurun_out/c5b.log; exit 1; }
  echo "batch=$b w3 $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/c5b.log | tr '\n' ' ')"
done
