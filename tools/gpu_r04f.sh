#!/bin/bash
# round-4 close: occupancy, the whole GPU suite, smoke, C3 rocprof + VALU pass,
# bench lines C3 / C4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/diag_occupancy.py > gpurun_out/encode_occupancy_r04.txt 2>&1 || { cat gpurun_out/encode_occupancy_r04.txt; exit 1; }
cat gpurun_out/encode_occupancy_r04.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_all.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
TAG=r04f CONFIG=C3 bash tools/gpu_profile.sh > gpurun_out/prof_r04f.log 2>&1 || { tail -20 gpurun_out/prof_r04f.log; exit 1; }
TAG=r04f CONFIG=C3 NAME=C3 BATCH=8192 bash tools/gpu_pmc_valu.sh > gpurun_out/valu_r04f.log 2>&1 || { tail -20 gpurun_out/valu_r04f.log; exit 1; }
grep "k_encode\|k_modofdm" gpurun_out/pmc/valu_C3.md
timeout -k 10 400 python3 bench.py > gpurun_out/bench_r04f_C3.json.log 2>&1 || { tail -5 gpurun_out/bench_r04f_C3.json.log; exit 1; }
timeout -k 10 300 python3 bench.py --config C4 > gpurun_out/bench_r04f_C4.json.log 2>&1 || { tail -5 gpurun_out/bench_r04f_C4.json.log; exit 1; }
for f in C3 C4; do tail -1 gpurun_out/bench_r04f_$f.json.log | cut -c1-200; done
echo ALL_OK
