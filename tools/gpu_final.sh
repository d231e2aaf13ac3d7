#!/bin/bash
# round-end check: the whole GPU suite, smoke(), and the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_all.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python3 bench.py > gpurun_out/bench_final.json.log 2>&1 || { tail -5 gpurun_out/bench_final.json.log; exit 1; }
tail -1 gpurun_out/bench_final.json.log | cut -c1-400
timeout -k 10 300 python3 bench.py --config C5 --c5-bits 8 --no-cpu-baseline > gpurun_out/bench_final_C5_8bit.json.log 2>&1 || { tail -5 gpurun_out/bench_final_C5_8bit.json.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/bench_final_C5_8bit.json.log
