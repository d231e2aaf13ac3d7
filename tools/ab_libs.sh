#!/bin/bash
# A/B of library builds on one bench config: tools/ab_libs.sh CONFIG REPS lib1 lib2 ...
# (timing only; each variant's parity is checked separately before it is adopted)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
cfg=$1; reps=$2; shift 2
for rep in $(seq $reps); do
  for lib in "$@"; do
    OAI4G_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --config $cfg --steps 20 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    echo "$cfg $lib $(grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}' gpurun_out/ab.log | tr '\n' ' ')"
  done
done
echo ALL_OK
