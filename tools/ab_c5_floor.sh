#!/bin/bash
# C5 decoder floor: the in-tree library against abvar/l2ring*/ (TD_DIAG_L2: the waves share
# scratch regions, so the scratch working set stays in L2 / MALL; results are wrong by design,
# the time is the kernel's no-HBM floor).  16- and 8-bit decoders, 8 iterations, bench batch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for bits in 16; do
  for lib in openair4g_amd/lib/libopenair4g_amd.so abvar/l2ring*/libopenair4g_amd.so; do
    [ -f "$lib" ] || continue
    OAI4G_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --config C5 --c5-bits $bits --steps 3 --warmup 1 \
        --no-cpu-baseline > gpurun_out/ab_c5f.log 2>&1 || { echo "FAILED $lib"; tail -5 gpurun_out/ab_c5f.log; exit 1; }
    echo "bits $bits $lib $(grep -o '"value": [0-9.]*' gpurun_out/ab_c5f.log) $(grep -o '"kernel_ms": [^}]*' gpurun_out/ab_c5f.log)"
  done
done
