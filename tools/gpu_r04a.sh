#!/bin/bash
# round 4, first GPU pass: VALU-rate microbenchmark at 1/2/4/8 waves per SIMD with encoding-size
# controls, the default C3 bench line, rocprofv3 trace + PMC traffic for C3 and C4, VALU pass for C4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 tools/ubench/valu_rate > gpurun_out/valu_rate_r04.txt 2>&1 || { echo "ubench failed"; exit 1; }
echo "ubench ok"
timeout -k 10 300 python3 bench.py > gpurun_out/bench_r04_C3.json.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_r04_C3.json.log; exit 1; }
tail -1 gpurun_out/bench_r04_C3.json.log | cut -c1-400
TAG=r04 CONFIG=C3 bash tools/gpu_profile.sh || exit 1
TAG=r04 CONFIG=C4 bash tools/gpu_profile.sh || exit 1
TAG=r04 CONFIG=C4 NAME=C4 BATCH=1024 bash tools/gpu_pmc_valu.sh || exit 1
echo ALL_OK
