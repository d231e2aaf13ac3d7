cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_decoder.py tests/test_gpu_decoder8.py > gpurun_out/p_dec.log 2>&1 || { tail -5 gpurun_out/p_dec.log; exit 1; }
tail -1 gpurun_out/p_dec.log
timeout -k 10 300 python3 bench.py --config C5 --c5-mode chain > gpurun_out/bench_r04_C5_chain.json.log 2>&1 || { tail -5 gpurun_out/bench_r04_C5_chain.json.log; exit 1; }
timeout -k 10 300 python3 bench.py --config C5 --c5-mode snr --no-cpu-baseline > gpurun_out/bench_r04_C5_snr.json.log 2>&1 || { tail -5 gpurun_out/bench_r04_C5_snr.json.log; exit 1; }
for f in chain snr; do grep -o '"value": [0-9.]*\|"mean_iterations": [0-9.]*' gpurun_out/bench_r04_C5_$f.json.log | tr '\n' ' '; echo; done
