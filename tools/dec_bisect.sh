#!/bin/bash
# decoder parity per library (in-tree + variants/*), first failure only
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bis
for lib in openair4g_amd/lib/libopenair4g_amd.so variants/*/libopenair4g_amd.so; do
  OAI4G_LIB=$PWD/$lib timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_decoder.py > gpurun_out/bis/p.log 2>&1
  rc=$?
  echo "$lib rc=$rc $(tail -1 gpurun_out/bis/p.log)"
  [ $rc -le 1 ] || exit $rc
done
