#!/bin/bash
# round 5: C5 decoder residency variants (variants/*: 3 waves per SIMD with shorter operand prefetch)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do C5_BATCH=16384 bash tools/ab_c5.sh || exit 1; done
