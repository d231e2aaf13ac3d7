#!/bin/bash
# round 5: the UE-side bench lines (FEP, UE, UE3) and the 8-bit decoder line at the current build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r05ad}
for cfg in FEP UE UE3; do
  timeout -k 10 300 python3 bench.py --config $cfg > gpurun_out/bench_${T}_$cfg.json.log 2>&1 || { tail -5 gpurun_out/bench_${T}_$cfg.json.log; exit 1; }
  echo "$cfg $(grep -o '"value": [0-9.]*' gpurun_out/bench_${T}_$cfg.json.log | head -1)"
done
timeout -k 10 400 python3 bench.py --config C5 --c5-bits 8 --no-cpu-baseline > gpurun_out/bench_${T}_C5_8bit.json.log 2>&1 || { tail -5 gpurun_out/bench_${T}_C5_8bit.json.log; exit 1; }
echo "C5_8bit $(grep -o '"value": [0-9.]*' gpurun_out/bench_${T}_C5_8bit.json.log | head -1)"
