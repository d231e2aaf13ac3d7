#!/bin/bash
# round 5: idft2048 pair stores / modulator memory-wait fixes — modulator parity subset + C3 A/B (in-tree vs abvar/base = previous commit)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_tm2.py tests/test_gpu_tm3.py tests/test_gpu_golden.py tests/test_gpu_bench_size.py tests/test_gpu_control_batch.py tests/test_gpu_common_batch.py tests/test_gpu_seg_ofdm_ref.py tests/test_gpu_fep.py tests/test_gpu_host_c.py > gpurun_out/r05i_pytest.log 2>&1 || { tail -30 gpurun_out/r05i_pytest.log; exit 1; }
tail -1 gpurun_out/r05i_pytest.log
for rep in 1 2 3; do
  for lib in openair4g_amd/lib/libopenair4g_amd.so abvar/base/libopenair4g_amd.so; do
    OAI4G_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/ab05.log 2>&1 || { tail -5 gpurun_out/ab05.log; exit 1; }
    echo "C3 $lib $(grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}' gpurun_out/ab05.log | tr '\n' ' ')"
  done
done
echo ALL_OK
