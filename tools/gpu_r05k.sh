#!/bin/bash
# round 5 measurement pass (after the modulator wait fixes): whole GPU suite, smoke, C3 rocprof trace + calibrated PMC + VALU pass,
# bench lines C3 (default command) / C4 / C2 / C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r05k}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_all.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
TAG=$T CONFIG=C3 bash tools/gpu_profile.sh > gpurun_out/prof_$T.log 2>&1 || { tail -20 gpurun_out/prof_$T.log; exit 1; }
cp -r gpurun_out/prof gpurun_out/prof_C3 && rm -rf gpurun_out/prof
tail -8 gpurun_out/prof_$T.log
TAG=$T CONFIG=C4 bash tools/gpu_profile.sh > gpurun_out/prof_${T}_C4.log 2>&1 || { tail -20 gpurun_out/prof_${T}_C4.log; exit 1; }
cp -r gpurun_out/prof gpurun_out/prof_C4 && rm -rf gpurun_out/prof
tail -8 gpurun_out/prof_${T}_C4.log
TAG=$T CONFIG=C3 NAME=C3 BATCH=8192 bash tools/gpu_pmc_valu.sh > gpurun_out/valu_$T.log 2>&1 || { tail -20 gpurun_out/valu_$T.log; exit 1; }
grep "k_encode\|k_modofdm" gpurun_out/pmc/valu_C3.md
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${T}_C3.json.log 2>&1 || { tail -5 gpurun_out/bench_${T}_C3.json.log; exit 1; }
timeout -k 10 300 python3 bench.py --config C4 > gpurun_out/bench_${T}_C4.json.log 2>&1 || { tail -5 gpurun_out/bench_${T}_C4.json.log; exit 1; }
timeout -k 10 300 python3 bench.py --config C2 > gpurun_out/bench_${T}_C2.json.log 2>&1 || { tail -5 gpurun_out/bench_${T}_C2.json.log; exit 1; }
timeout -k 10 400 python3 bench.py --config C5 > gpurun_out/bench_${T}_C5.json.log 2>&1 || { tail -5 gpurun_out/bench_${T}_C5.json.log; exit 1; }
for f in C3 C4 C2 C5; do tail -1 gpurun_out/bench_${T}_$f.json.log | cut -c1-300; done
echo ALL_OK
