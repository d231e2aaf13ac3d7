#!/bin/bash
# round 5: the misaligned-IQ test, full-grid and C4 bench lines after the modulator wait fixes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_parity.py -k misaligned > gpurun_out/r05o_pytest.log 2>&1 || { tail -30 gpurun_out/r05o_pytest.log; exit 1; }
tail -1 gpurun_out/r05o_pytest.log
timeout -k 10 300 python3 bench.py --full-grid --no-cpu-baseline > gpurun_out/bench_r05o_full_grid.json.log 2>&1 || { tail -5 gpurun_out/bench_r05o_full_grid.json.log; exit 1; }
tail -1 gpurun_out/bench_r05o_full_grid.json.log | cut -c1-400
echo ALL_OK
