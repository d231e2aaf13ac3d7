#!/bin/bash
# round 5: wall step vs HIP-event kernel sum: warmup length vs step count (C3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "3 20" "100 20" "300 20" "3 20" "3 200" "100 5"; do
  set -- $cfg
  timeout -k 10 120 python3 bench.py --warmup $1 --steps $2 --no-cpu-baseline > gpurun_out/st.log 2>&1 || { tail -5 gpurun_out/st.log; exit 1; }
  echo "warmup=$1 steps=$2 $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": {[^}]*}' gpurun_out/st.log | tr '\n' ' ')"
done
echo ALL_OK
