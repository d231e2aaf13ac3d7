#!/bin/bash
# round 5: modulation / scrambling reference pins on the GPU (drop-ins vs reference fixtures, the C3
# bench batch vs the reference chain) + the C3 line with the new CPU baseline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mod_ref.py tests/test_gpu_seg_ofdm_ref.py tests/test_mod_fixture_cpu.py tests/test_seg_ofdm_fixture_cpu.py > gpurun_out/r05q_pytest.log 2>&1 || { tail -30 gpurun_out/r05q_pytest.log; exit 1; }
tail -1 gpurun_out/r05q_pytest.log
timeout -k 10 400 python3 bench.py > gpurun_out/bench_r05q_C3.json.log 2>&1 || { tail -5 gpurun_out/bench_r05q_C3.json.log; exit 1; }
tail -1 gpurun_out/bench_r05q_C3.json.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['cpu_baseline'])[:900])"
echo ALL_OK
