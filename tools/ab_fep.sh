#!/bin/bash
# A/B of the FEP kernel: the in-tree library and every variants/*/libopenair4g_amd.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in openair4g_amd/lib/libopenair4g_amd.so variants/*/libopenair4g_amd.so; do
  [ -f "$lib" ] || continue
  OAI4G_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --config FEP --steps 20 --warmup 3 \
      --no-cpu-baseline > gpurun_out/ab_fep.log 2>&1 || { echo "FAILED $lib"; tail -5 gpurun_out/ab_fep.log; exit 1; }
  echo "$lib $(grep -o '"value": [0-9.]*' gpurun_out/ab_fep.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/ab_fep.log)"
done
