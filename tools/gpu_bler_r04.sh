#!/bin/bash
# round 4 BLER evidence: the GPU dlsim loop (16-bit, all 28 MCS; 8-bit at the four pin MCS) against the
# reference's Perf_Curves_Abs set, then the GPU pin tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u tools/bler_sweep.py --mcs $(seq 0 27) --trials 32768 --curves perf_curves_abs --out gpurun_out/bler_r04_perf16_all28.json > gpurun_out/bler_r04_perf16_all28.log 2>&1 || { tail -5 gpurun_out/bler_r04_perf16_all28.log; exit 1; }
grep "rows within" gpurun_out/bler_r04_perf16_all28.log
timeout -k 10 300 python3 -u tools/bler_sweep.py --mcs 0 9 16 27 --trials 32768 --llr8 --curves perf_curves_abs --out gpurun_out/bler_r04_perf8.json > gpurun_out/bler_r04_perf8.log 2>&1 || { tail -5 gpurun_out/bler_r04_perf8.log; exit 1; }
grep "rows within\|best shift" gpurun_out/bler_r04_perf8.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_dlsim.py > gpurun_out/pytest_dlsim.log 2>&1 || { tail -20 gpurun_out/pytest_dlsim.log; exit 1; }
tail -3 gpurun_out/pytest_dlsim.log
