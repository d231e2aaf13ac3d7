#!/bin/bash
# round 5: decoder vmcnt fixes — decoder parity subset + C5 A/B (in-tree vs abvar/base = previous commit)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_decoder.py tests/test_gpu_decoder_cases.py tests/test_gpu_ul_chain.py > gpurun_out/r05j_pytest.log 2>&1 || { tail -30 gpurun_out/r05j_pytest.log; exit 1; }
tail -1 gpurun_out/r05j_pytest.log
bash tools/ab_libs.sh C5 3 openair4g_amd/lib/libopenair4g_amd.so abvar/base/libopenair4g_amd.so
