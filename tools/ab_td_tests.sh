#!/bin/bash
# Decoder parity (bit-exact drop-in cases) for the in-tree library and every variants/*/ build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in openair4g_amd/lib/libopenair4g_amd.so variants/*/libopenair4g_amd.so; do
  [ -f "$lib" ] || continue
  OAI4G_LIB=$PWD/$lib timeout -k 10 120 python3 -m pytest -x -q --timeout 60 --timeout-method thread \
      "tests/test_gpu_decoder.py::test_drop_in_decoder_bit_exact" > gpurun_out/ab_td_tests.log 2>&1
  rc=$?
  echo "$lib rc=$rc $(tail -1 gpurun_out/ab_td_tests.log)"
  [ $rc -le 1 ] || exit $rc
done
