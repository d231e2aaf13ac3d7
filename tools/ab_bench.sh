#!/bin/bash
# A/B: bench the in-tree library and every variants/*/libopenair4g_amd.so (kernel experiments).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in openair4g_amd/lib/libopenair4g_amd.so variants/*/libopenair4g_amd.so; do
  [ -f "$lib" ] || continue
  echo "== $lib"
  OAI4G_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --steps ${BENCH_STEPS:-20} --warmup 3 --no-cpu-baseline \
      > gpurun_out/ab.log 2>&1 || { echo "FAILED rc=$?"; tail -5 gpurun_out/ab.log; exit 1; }
  grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}' gpurun_out/ab.log | tr '\n' ' '; echo
done
