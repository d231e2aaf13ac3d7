#!/bin/bash
# round 6: the new reference pins on the GPU (turbo encoder through the reference decoder, the compiled shim)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_td_ref.py tests/test_gpu_shim_ref.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r06a_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED" gpurun_out/r06a_tests.log | tail -30
tail -3 gpurun_out/r06a_tests.log
exit $rc
