#!/bin/bash
# GPU-box session: parity tests -> smoke -> short bench.  Every GPU step has its own time
# limit; after a crash/abort/timeout (exit status other than 0/1) nothing else is started.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name" ; date +%T
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
if [ -n "$PYTEST_K" ]; then KARG=(-k "$PYTEST_K"); else KARG=(); fi
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread "${KARG[@]}"
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps ${BENCH_STEPS:-10} --warmup 2 --cpu-seconds ${CPU_SECONDS:-8}
