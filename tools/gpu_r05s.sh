#!/bin/bash
# round 5: LDS-only barriers + first QPP gather entries loaded ahead of the plane build — encoder parity subset + C3 A/B vs abvar/base (previous commit)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bench_size.py tests/test_gpu_rm_ref.py tests/test_gpu_filler.py tests/test_gpu_rm_limited.py tests/test_gpu_seg_ofdm_ref.py tests/test_gpu_golden.py > gpurun_out/r05s_pytest.log 2>&1 || { tail -30 gpurun_out/r05s_pytest.log; exit 1; }
tail -1 gpurun_out/r05s_pytest.log
bash tools/ab_libs.sh C3 3 openair4g_amd/lib/libopenair4g_amd.so abvar/base/libopenair4g_amd.so > gpurun_out/ab_r05s.txt 2>&1; rc=$?; cat gpurun_out/ab_r05s.txt; exit $rc
