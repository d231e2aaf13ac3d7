#!/bin/bash
# VALU-issue evidence for the bench kernels: one rocprofv3 --pmc pass (8 SQ counters + GRBM_GUI_ACTIVE)
# over a short bench run; summarised per kernel by tools/valu_table.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02}; CONFIG=${CONFIG:-C3}; NAME=${NAME:-$CONFIG}
mkdir -p gpurun_out/pmc
CTRS="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/pmc/valu_${NAME} -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --kernel-reps 1 --settle-ms 0 --config $CONFIG ${EXTRA:-} > gpurun_out/pmc/valu_${NAME}.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -2 gpurun_out/pmc/valu_${NAME}.log
[ $rc -eq 0 ] || exit $rc
python3 tools/valu_table.py gpurun_out/pmc/valu_${NAME} $NAME ${BATCH:-8192} > gpurun_out/pmc/valu_${NAME}.md
cat gpurun_out/pmc/valu_${NAME}.md
