#!/bin/bash
# round 5: encoder phase cut timings + per-phase SQ counters (current build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/diag_phases.py C3 8192 > gpurun_out/phases_C3.txt 2>&1 || { cat gpurun_out/phases_C3.txt; exit 1; }
cat gpurun_out/phases_C3.txt
bash tools/pmc_encode.sh || exit 1
f=$(ls gpurun_out/pmc/enc/*counter_collection.csv 2>/dev/null | head -1)
[ -z "$f" ] && f=$(find gpurun_out/pmc/enc -name "*counter_collection.csv" | head -1)
python3 tools/pmc_table.py "$f" > gpurun_out/enc_phase_counters.txt && cat gpurun_out/enc_phase_counters.txt
