#!/bin/bash
# round 5: C3 throughput against the batch (subframes per step)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in ${C3_BATCHES:-8192 16384 32768}; do
  timeout -k 10 300 python3 bench.py --config C3 --batch $b --steps 10 --no-cpu-baseline > gpurun_out/c3b.log 2>&1 || { tail -5 gpurun_out/c3b.log; exit 1; }
  echo "batch=$b $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"kernel_ms": {[^}]*}' gpurun_out/c3b.log | head -3 | tr '\n' ' ')"
done
