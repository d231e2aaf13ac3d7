#!/bin/bash
# round 5 final measurement pass, part 2: C5 rocprofv3 trace + calibrated PMC and VALU pass at the bench batch,
# then the bench lines C3 (default command), C4, C2, full grid, C5 (8it / snr / chain)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r05z}
TAG=$T CONFIG=C5 bash tools/gpu_profile.sh > gpurun_out/prof_${T}_C5.log 2>&1 || { tail -20 gpurun_out/prof_${T}_C5.log; exit 1; }
rm -rf gpurun_out/prof_C5 && cp -r gpurun_out/prof gpurun_out/prof_C5 && rm -rf gpurun_out/prof
tail -6 gpurun_out/prof_${T}_C5.log
TAG=$T CONFIG=C5 NAME=C5 BATCH=49152 bash tools/gpu_pmc_valu.sh > gpurun_out/valu_${T}_C5.log 2>&1 || { tail -20 gpurun_out/valu_${T}_C5.log; exit 1; }
grep "k_td16" gpurun_out/pmc/valu_C5.md
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${T}_C3.json.log 2>&1 || { tail -5 gpurun_out/bench_${T}_C3.json.log; exit 1; }
timeout -k 10 300 python3 bench.py --config C4 > gpurun_out/bench_${T}_C4.json.log 2>&1 || { tail -5 gpurun_out/bench_${T}_C4.json.log; exit 1; }
timeout -k 10 300 python3 bench.py --config C2 > gpurun_out/bench_${T}_C2.json.log 2>&1 || { tail -5 gpurun_out/bench_${T}_C2.json.log; exit 1; }
timeout -k 10 300 python3 bench.py --full-grid > gpurun_out/bench_${T}_full_grid.json.log 2>&1 || { tail -5 gpurun_out/bench_${T}_full_grid.json.log; exit 1; }
timeout -k 10 400 python3 bench.py --config C5 > gpurun_out/bench_${T}_C5.json.log 2>&1 || { tail -5 gpurun_out/bench_${T}_C5.json.log; exit 1; }
timeout -k 10 400 python3 bench.py --config C5 --c5-mode snr --no-cpu-baseline > gpurun_out/bench_${T}_C5_snr.json.log 2>&1 || { tail -5 gpurun_out/bench_${T}_C5_snr.json.log; exit 1; }
timeout -k 10 400 python3 bench.py --config C5 --c5-mode chain --no-cpu-baseline > gpurun_out/bench_${T}_C5_chain.json.log 2>&1 || { tail -5 gpurun_out/bench_${T}_C5_chain.json.log; exit 1; }
for f in C3 C4 C2 full_grid C5 C5_snr C5_chain; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/bench_${T}_$f.json.log | head -1)"; done
echo ALL_OK
