cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_decoder.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dec.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_dec.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --config C5 --no-cpu-baseline > gpurun_out/bench_C5.log 2>&1; rc=$?; tail -1 gpurun_out/bench_C5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --config C5 --c5-mode snr --no-cpu-baseline > gpurun_out/bench_C5snr.log 2>&1; rc=$?; tail -1 gpurun_out/bench_C5snr.log; exit $rc
