#!/bin/bash
# round 5: the other transmit bench lines after the encoder SALU cuts (C4, C2, full grid)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r05af}
timeout -k 10 300 python3 bench.py --config C4 > gpurun_out/bench_${T}_C4.json.log 2>&1 || { tail -5 gpurun_out/bench_${T}_C4.json.log; exit 1; }
timeout -k 10 300 python3 bench.py --config C2 > gpurun_out/bench_${T}_C2.json.log 2>&1 || { tail -5 gpurun_out/bench_${T}_C2.json.log; exit 1; }
timeout -k 10 300 python3 bench.py --full-grid > gpurun_out/bench_${T}_full_grid.json.log 2>&1 || { tail -5 gpurun_out/bench_${T}_full_grid.json.log; exit 1; }
for f in C4 C2 full_grid; do echo "$f $(grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}' gpurun_out/bench_${T}_$f.json.log | head -2 | tr '\n' ' ')"; done
