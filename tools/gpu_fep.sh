#!/bin/bash
# GPU session for the receive front end: parity tests, FEP bench, rocprofv3 kernel trace of the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
TAG=${TAG:-r01}
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name"; date +%T
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 6 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step pytest_fep 300 python -u -m pytest tests/test_gpu_fep.py tests/test_gpu_golden.py -v --timeout 120 --timeout-method thread
step bench_FEP 300 python bench.py --steps 20 --warmup 3 --config FEP --cpu-seconds 5
step prof_FEP 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/fep_$TAG -o run -- python3 bench.py --steps 10 --warmup 2 --config FEP --no-cpu-baseline
