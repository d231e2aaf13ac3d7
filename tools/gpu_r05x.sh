#!/bin/bash
# round 5: decoder at 3 waves per SIMD (TD16_WAVES=3) -- decoder / UL-chain / dlsim GPU tests, then the C5 line at its new default batch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bench_size.py tests/test_gpu_decoder.py tests/test_gpu_ul_chain.py tests/test_gpu_dlsim.py > gpurun_out/r05x_pytest.log 2>&1 || { tail -30 gpurun_out/r05x_pytest.log; exit 1; }
tail -1 gpurun_out/r05x_pytest.log
timeout -k 10 400 python3 bench.py --config C5 > gpurun_out/bench_r05x_C5.json.log 2>&1 || { tail -5 gpurun_out/bench_r05x_C5.json.log; exit 1; }
tail -1 gpurun_out/bench_r05x_C5.json.log | cut -c1-600
