#!/bin/bash
# round 5 modulator diagnostics (timing only; the diagnostic builds' outputs are wrong by design):
# in-tree vs no IDFT barriers (OAI4G_DIAG_NOSYNC), no IQ stores (OAI4G_DIAG_MODOFDM=1), 3 waves
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in openair4g_amd/lib/libopenair4g_amd.so abvar/nosync/libopenair4g_amd.so abvar/nostore/libopenair4g_amd.so abvar/w3/libopenair4g_amd.so; do
    OAI4G_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/ab05.log 2>&1 || { tail -5 gpurun_out/ab05.log; exit 1; }
    echo "C3 $lib $(grep -o '"kernel_ms": {[^}]*}' gpurun_out/ab05.log | tr '\n' ' ')"
  done
done
echo ALL_OK
