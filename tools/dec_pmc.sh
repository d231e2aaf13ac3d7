#!/bin/bash
# decoder stall evidence: one SQ/SQC PMC pass per library (in-tree + variants/*) over a short C5 run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/dpmc
CTRS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_IFETCH SQC_ICACHE_MISSES SQC_ICACHE_REQ GRBM_GUI_ACTIVE"
i=0
for lib in openair4g_amd/lib/libopenair4g_amd.so variants/*/libopenair4g_amd.so; do
  i=$((i+1))
  OAI4G_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/dpmc/p$i -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --config C5 > gpurun_out/dpmc/p$i.log 2>&1 || exit 1
  echo "== $i $lib"
  python3 tools/pmc_dump.py gpurun_out/dpmc/p$i k_td16
done
