#!/bin/bash
# round 4 closing pass: C5 rocprof trace + calibrated traffic + VALU pass at the final decoder, the
# whole GPU suite, smoke(), and the bench lines (C3 default, C5, C5 8-bit)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r04d CONFIG=C5 bash tools/gpu_profile.sh || exit 1
TAG=r04d CONFIG=C5 NAME=C5 BATCH=2048 bash tools/gpu_pmc_valu.sh || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_all.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python3 bench.py > gpurun_out/bench_r04d_C3.json.log 2>&1 || { tail -5 gpurun_out/bench_r04d_C3.json.log; exit 1; }
timeout -k 10 300 python3 bench.py --config C5 > gpurun_out/bench_r04d_C5.json.log 2>&1 || { tail -5 gpurun_out/bench_r04d_C5.json.log; exit 1; }
for f in C3 C5; do tail -1 gpurun_out/bench_r04d_$f.json.log | cut -c1-250; done
echo ALL_OK
