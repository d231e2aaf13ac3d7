#!/bin/bash
# round 4, after the decoder / encoder changes: rocprofv3 trace + calibrated traffic and a VALU pass
# for C5 and C3, then the bench lines (C3 default with cpu_baseline, C4, C5, C5 8-bit)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r04c CONFIG=C5 bash tools/gpu_profile.sh || exit 1
TAG=r04c CONFIG=C5 NAME=C5 BATCH=2048 bash tools/gpu_pmc_valu.sh || exit 1
TAG=r04c CONFIG=C3 bash tools/gpu_profile.sh || exit 1
TAG=r04c CONFIG=C3 NAME=C3 BATCH=8192 bash tools/gpu_pmc_valu.sh || exit 1
timeout -k 10 400 python3 bench.py > gpurun_out/bench_r04c_C3.json.log 2>&1 || { tail -5 gpurun_out/bench_r04c_C3.json.log; exit 1; }
timeout -k 10 300 python3 bench.py --config C4 > gpurun_out/bench_r04c_C4.json.log 2>&1 || { tail -5 gpurun_out/bench_r04c_C4.json.log; exit 1; }
timeout -k 10 300 python3 bench.py --config C5 > gpurun_out/bench_r04c_C5.json.log 2>&1 || { tail -5 gpurun_out/bench_r04c_C5.json.log; exit 1; }
timeout -k 10 300 python3 bench.py --config C5 --c5-bits 8 > gpurun_out/bench_r04c_C5_8bit.json.log 2>&1 || { tail -5 gpurun_out/bench_r04c_C5_8bit.json.log; exit 1; }
for f in C3 C4 C5 C5_8bit; do tail -1 gpurun_out/bench_r04c_$f.json.log | cut -c1-300; done
echo ALL_OK
