#!/bin/bash
# C3: serial pair vs the two-stream chunk pipeline with the modulator grid capped per CU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_pipe.log 2>&1 \
    || { echo "FAILED $*"; tail -5 gpurun_out/ab_pipe.log; exit 1; }
  echo "$* $(grep -o '"value": [0-9.]*' gpurun_out/ab_pipe.log)"
}
run X=serial
run OAI4G_MODOFDM_OCC=5 X=occ5_serial
run OAI4G_PIPE_CHUNK=4096
run OAI4G_PIPE_CHUNK=2048
run OAI4G_PIPE_CHUNK=4096 OAI4G_MODOFDM_OCC=5
run OAI4G_PIPE_CHUNK=2048 OAI4G_MODOFDM_OCC=5
run OAI4G_PIPE_CHUNK=2048 OAI4G_MODOFDM_OCC=4
run OAI4G_PIPE_CHUNK=1024 OAI4G_MODOFDM_OCC=4
run OAI4G_PIPE_CHUNK=4096 OAI4G_MODOFDM_OCC=4
run X=serial_again
