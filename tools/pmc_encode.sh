#!/bin/bash
# Per-phase encoder counters: tools/pmc_encode.py dispatches k_encode cut after each phase, then in
# full; one rocprofv3 --pmc pass (SQ counters) over it.  Table: tools/pmc_table.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc/enc -o run -- python3 tools/pmc_encode.py C3 ${BATCH:-8192} > gpurun_out/pmc/enc.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 gpurun_out/pmc/enc.log; exit $rc
