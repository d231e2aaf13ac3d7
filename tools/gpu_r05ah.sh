#!/bin/bash
# round 5 closing measurement (after the encoder barrier-latency cuts): whole GPU suite, smoke, C3 rocprofv3 trace + calibrated PMC + VALU pass, the C3 bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r05ah}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_${T}_gpu_all.log 2>&1 || { tail -30 gpurun_out/pytest_${T}_gpu_all.log; exit 1; }
tail -1 gpurun_out/pytest_${T}_gpu_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_${T}.log 2>&1 || { tail -20 gpurun_out/smoke_${T}.log; exit 1; }
tail -1 gpurun_out/smoke_${T}.log
TAG=$T CONFIG=C3 bash tools/gpu_profile.sh > gpurun_out/prof_$T.log 2>&1 || { tail -20 gpurun_out/prof_$T.log; exit 1; }
rm -rf gpurun_out/prof_C3 && cp -r gpurun_out/prof gpurun_out/prof_C3 && rm -rf gpurun_out/prof
tail -6 gpurun_out/prof_$T.log
TAG=$T CONFIG=C3 NAME=C3 BATCH=8192 bash tools/gpu_pmc_valu.sh > gpurun_out/valu_$T.log 2>&1 || { tail -20 gpurun_out/valu_$T.log; exit 1; }
grep "k_encode\|k_modofdm" gpurun_out/pmc/valu_C3.md
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${T}_C3.json.log 2>&1 || { tail -5 gpurun_out/bench_${T}_C3.json.log; exit 1; }
tail -1 gpurun_out/bench_${T}_C3.json.log | cut -c1-300
echo ALL_OK
