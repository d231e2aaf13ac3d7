#!/bin/bash
# rocprofv3 passes over the bench: kernel trace + stats, then one PMC pass per counter
# (FETCH_SIZE and WRITE_SIZE need separate passes on gfx950's TCC slots), each also over the
# 4 B/lane calibration stream (tools/pmc_calibrate.py).  Summarise with tools/summarize_prof.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
TAG=${TAG:-r01}
CMD="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --kernel-reps 2 --config ${CONFIG:-C3}"
# counter passes serialise every dispatch: no clock-settle runs there (durations come from the trace pass)
CMDP="$CMD --settle-ms 0"
run() {
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/prof/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -n 3 "gpurun_out/prof/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP"; exit $rc; fi
}
run trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace_$TAG -o run -- $CMD
run pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch_$TAG -o run -- $CMDP
run pmc_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write_$TAG -o run -- $CMDP
run cal_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/calfetch_$TAG -o run -- python3 tools/pmc_calibrate.py
run cal_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/calwrite_$TAG -o run -- python3 tools/pmc_calibrate.py
python3 tools/summarize_prof.py gpurun_out/prof $TAG ${CONFIG:-C3} gpurun_out/prof/summary > gpurun_out/prof/summary.log 2>&1
echo "summary rc=$?"; cat gpurun_out/prof/summary.log | tail -20
