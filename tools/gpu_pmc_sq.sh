#!/bin/bash
# SQ counter pass over a diagnostic script (default: encoder phase cuts).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
SCRIPT=${SCRIPT:-tools/pmc_encode.py}
CTRS=${CTRS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU"}
timeout -k 10 400 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/pmc/sq -o run -- python3 $SCRIPT > gpurun_out/pmc/sq.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -3 gpurun_out/pmc/sq.log
find gpurun_out/pmc -name '*.csv'
