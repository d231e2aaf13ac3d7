#!/bin/bash
# round 5: whole GPU suite on the in-tree build, C3 A/B against abvar/base (HEAD's modulator), VALU pass
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_all.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_all.log
for rep in 1 2 3; do
  for lib in openair4g_amd/lib/libopenair4g_amd.so abvar/base/libopenair4g_amd.so; do
    OAI4G_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/ab05.log 2>&1 || { tail -5 gpurun_out/ab05.log; exit 1; }
    echo "C3 $lib $(grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}' gpurun_out/ab05.log | tr '\n' ' ')"
  done
done
TAG=r05b CONFIG=C3 NAME=C3 BATCH=8192 bash tools/gpu_pmc_valu.sh > gpurun_out/valu_r05b.log 2>&1 || { tail -20 gpurun_out/valu_r05b.log; exit 1; }
grep "k_encode\|k_modofdm" gpurun_out/pmc/valu_C3.md
echo ALL_OK
