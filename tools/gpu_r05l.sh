#!/bin/bash
# round 5: encoder phase timings (cut builds) + per-phase SQ counters
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/diag_phases.py C3 8192 > gpurun_out/enc_phases.log 2>&1 || { tail -5 gpurun_out/enc_phases.log; exit 1; }
cat gpurun_out/enc_phases.log
bash tools/pmc_encode.sh && python3 tools/pmc_table.py gpurun_out/pmc/enc > gpurun_out/enc_pmc.txt 2>&1; cat gpurun_out/enc_pmc.txt | cut -c1-200
