#!/bin/bash
# Selected -m gpu tests on one GPU, one pytest process, a hang ends at the per-test timeout.
# usage: TAG=name bash tools/gpu_tests.sh tests/test_a.py tests/test_b.py ...   (no files: the whole suite)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-sel}
timeout -k 10 ${LIMIT:-900} python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread ${@:-tests} \
  > gpurun_out/tests_${TAG}.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/tests_${TAG}.log | head -20
tail -1 gpurun_out/tests_${TAG}.log
exit $rc
