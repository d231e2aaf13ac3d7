#!/bin/bash
# A/B of the C5 decoder: the in-tree library and every variants/*/libopenair4g_amd.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in openair4g_amd/lib/libopenair4g_amd.so variants/*/libopenair4g_amd.so; do
  [ -f "$lib" ] || continue
  OAI4G_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --config C5 --batch ${C5_BATCH:-4096} --steps 3 --warmup 1 \
      --no-cpu-baseline > gpurun_out/ab_c5.log 2>&1 || { echo "FAILED $lib"; tail -5 gpurun_out/ab_c5.log; exit 1; }
  echo "$lib $(grep -o '"value": [0-9.]*' gpurun_out/ab_c5.log)"
done
