#!/bin/bash
# A/B of the 8-bit decoder (C5 workload, --c5-bits 8): the in-tree library and every variants/*/ build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in openair4g_amd/lib/libopenair4g_amd.so variants/*/libopenair4g_amd.so; do
  [ -f "$lib" ] || continue
  for mode in 8it snr; do
    OAI4G_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --config C5 --c5-bits 8 --c5-mode $mode --steps 5 --warmup 1 \
        --no-cpu-baseline > gpurun_out/ab_td8.log 2>&1 || { echo "FAILED $lib"; tail -5 gpurun_out/ab_td8.log; exit 1; }
    echo "$lib $mode $(grep -o '"value": [0-9.]*' gpurun_out/ab_td8.log)"
  done
done
