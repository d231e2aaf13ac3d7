#!/bin/bash
# A/B of kernel variants (variants/*/libopenair4g_amd.so) against the in-tree library on one GPU:
# the transmit-path parity tests on every variant, then REPS interleaved bench lines per variant.
# usage: bash tools/gpu_ab.sh [bench args...]     env: REPS (3), TESTS (default transmit set), TAG,
#        NOTESTS=1 (timing-only diagnostic variants whose output is wrong by design)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
REPS=${REPS:-3}
TAG=${TAG:-ab}
TESTS=${TESTS:-"tests/test_gpu_parity.py tests/test_gpu_bench_size.py tests/test_gpu_golden.py tests/test_gpu_seg_ofdm_ref.py tests/test_gpu_tm2.py"}
for lib in variants/*/libopenair4g_amd.so; do
  [ -f "$lib" ] && [ -z "$NOTESTS" ] || continue
  OAI4G_LIB=$PWD/$lib timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu $TESTS \
      > gpurun_out/${TAG}_tests_$(basename $(dirname $lib)).log 2>&1 \
    || { echo "FAILED tests with $lib"; grep -E "FAILED|Error" gpurun_out/${TAG}_tests_*.log | head; exit 1; }
  echo "$lib: $(tail -1 gpurun_out/${TAG}_tests_$(basename $(dirname $lib)).log)"
done
for rep in $(seq $REPS); do
  for lib in openair4g_amd/lib/libopenair4g_amd.so variants/*/libopenair4g_amd.so; do
    [ -f "$lib" ] || continue
    OAI4G_LIB=$PWD/$lib timeout -k 10 120 python bench.py "$@" --steps 20 --no-cpu-baseline > gpurun_out/${TAG}_b.log 2>&1 \
      || { tail -5 gpurun_out/${TAG}_b.log; exit 1; }
    echo "[$*] $lib $(grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}' gpurun_out/${TAG}_b.log | tr '\n' ' ')"
  done
done
