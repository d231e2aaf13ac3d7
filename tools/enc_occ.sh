#!/bin/bash
# k_encode residency sensitivity (diagnostic builds with unused LDS: 6 -> 5 -> 4 workgroups per CU at C3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in openair4g_amd/lib/libopenair4g_amd.so variants/*/libopenair4g_amd.so; do
    OAI4G_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/occ.log 2>&1 || exit 1
    echo "$lib $(grep -o '"encode_rm_scramble": [0-9.]*' gpurun_out/occ.log)"
  done
done
