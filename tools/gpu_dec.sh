#!/bin/bash
# decoder parity (unit + cases + UL chain) then two C5 bench runs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_decoder.py tests/test_gpu_decoder_cases.py tests/test_gpu_ul_chain.py > gpurun_out/pytest_dec.log 2>&1 || { tail -20 gpurun_out/pytest_dec.log; exit 1; }
tail -2 gpurun_out/pytest_dec.log
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --config C5 --no-cpu-baseline > gpurun_out/bench_C5.log 2>&1 || exit 1
  grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/bench_C5.log | tr '\n' ' '; echo
done
