#!/bin/bash
# encoder parity (TX chain + fillers + RM fixtures + bench-size), phase timings and the C3 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_filler.py tests/test_gpu_rm_ref.py tests/test_gpu_rm_limited.py tests/test_gpu_golden.py tests/test_gpu_bench_size.py > gpurun_out/pytest_enc.log 2>&1 || { tail -30 gpurun_out/pytest_enc.log; exit 1; }
tail -2 gpurun_out/pytest_enc.log
timeout -k 10 200 python3 tools/diag_phases.py C3 8192 > gpurun_out/phases_C3.txt 2>&1 || exit 1
cat gpurun_out/phases_C3.txt
for rep in 1 2; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/bench_C3.log 2>&1 || exit 1
  grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}' gpurun_out/bench_C3.log | tr '\n' ' '; echo
done
