#!/bin/bash
# round 5 verification after the dlsch_modulation / dlsch_scrambling reference pins: whole GPU suite, smoke, C3 bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r05r}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_${T}_gpu_all.log 2>&1 || { tail -30 gpurun_out/pytest_${T}_gpu_all.log; exit 1; }
tail -1 gpurun_out/pytest_${T}_gpu_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_${T}.log 2>&1 || { tail -20 gpurun_out/smoke_${T}.log; exit 1; }
tail -1 gpurun_out/smoke_${T}.log
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${T}_C3.json.log 2>&1 || { tail -5 gpurun_out/bench_${T}_C3.json.log; exit 1; }
tail -1 gpurun_out/bench_${T}_C3.json.log | cut -c1-400
echo ALL_OK
