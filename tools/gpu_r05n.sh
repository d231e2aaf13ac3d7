#!/bin/bash
# round 5: encoder || modulator chunk pipeline (OAI4G_PIPE_CHUNK) with the modulator grid capped
# (OAI4G_MODOFDM_OCC) so encoder workgroups share the CUs; C3 bench values
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "0 0" "2048 0" "2048 6" "4096 6" "1024 7" "2048 7"; do
    set -- $cfg
    env $( [ $1 -gt 0 ] && echo OAI4G_PIPE_CHUNK=$1 ) $( [ $2 -gt 0 ] && echo OAI4G_MODOFDM_OCC=$2 ) \
      timeout -k 10 120 python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/pp.log 2>&1 || { tail -5 gpurun_out/pp.log; exit 1; }
    echo "chunk=$1 occ=$2 $(grep -o '"value": [0-9.]*' gpurun_out/pp.log)"
  done
done
echo ALL_OK
