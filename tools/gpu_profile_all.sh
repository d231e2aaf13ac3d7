#!/bin/bash
# rocprofv3 sessions for C3 and FEP (trace+stats, FETCH_SIZE and WRITE_SIZE passes, calibration):
# tools/gpu_profile.sh once per config, summaries under gpurun_out/prof/summary_<config>.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in ${CONFIGS:-C3 FEP}; do
  CONFIG=$c TAG=r01 bash tools/gpu_profile.sh || exit $?
  mkdir -p gpurun_out/prof/summary_$c && cp -r gpurun_out/prof/summary/* gpurun_out/prof/summary_$c/ 2>/dev/null
  rm -rf gpurun_out/prof/summary gpurun_out/prof/trace_r01 gpurun_out/prof/fetch_r01 gpurun_out/prof/write_r01
done
