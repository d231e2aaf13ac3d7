#!/bin/bash
# Full GPU session: parity tests -> smoke -> C3 bench -> C4 bench -> C5 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name" ; date +%T
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 6 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_C3 600 python bench.py --steps 20 --warmup 3
step bench_C4 600 python bench.py --steps 10 --warmup 2 --config C4 --cpu-seconds 5
step bench_C5 600 python bench.py --steps 5 --warmup 1 --config C5 --cpu-seconds 5
step bench_FEP 600 python bench.py --steps 20 --warmup 3 --config FEP --cpu-seconds 5
