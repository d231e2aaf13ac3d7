#!/bin/bash
# Round 5 k_modofdm A/B: the in-tree build (SGPR twiddle operands, affine LDS addressing, twiddle
# companions rebuilt at use, pass C h-outer; 3 waves/SIMD) against abvar/new4 (the same code, 4
# waves/SIMD with the staged QAM addresses aliased into the IDFT exchange) and abvar/base (HEAD's
# kernel).  Parity first for every library, then interleaved 20-step benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIBS="openair4g_amd/lib/libopenair4g_amd.so abvar/new4/libopenair4g_amd.so abvar/base/libopenair4g_amd.so abvar/w5/libopenair4g_amd.so"
for lib in $LIBS; do
  OAI4G_LIB=$PWD/$lib timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_tm2.py tests/test_gpu_tm3.py tests/test_gpu_golden.py \
    tests/test_gpu_bench_size.py tests/test_gpu_control_batch.py tests/test_gpu_fep.py tests/test_gpu_seg_ofdm_ref.py \
    > gpurun_out/ab05_pytest.log 2>&1 || { echo "$lib FAILED"; tail -30 gpurun_out/ab05_pytest.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/ab05_pytest.log)"
done
for rep in 1 2; do
  for lib in $LIBS; do
    OAI4G_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/ab05.log 2>&1 || { tail -5 gpurun_out/ab05.log; exit 1; }
    echo "C3 $lib $(grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}' gpurun_out/ab05.log | tr '\n' ' ')"
  done
done
for lib in $LIBS; do
  OAI4G_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --config C2 --steps 20 --no-cpu-baseline > gpurun_out/ab05.log 2>&1 || exit 1
  echo "C2 $lib $(grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}' gpurun_out/ab05.log | tr '\n' ' ')"
  OAI4G_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --config C4 --steps 20 --no-cpu-baseline > gpurun_out/ab05.log 2>&1 || exit 1
  echo "C4 $lib $(grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}' gpurun_out/ab05.log | tr '\n' ' ')"
  OAI4G_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --full-grid --steps 20 --no-cpu-baseline > gpurun_out/ab05.log 2>&1 || exit 1
  echo "full $lib $(grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}' gpurun_out/ab05.log | tr '\n' ' ')"
done
