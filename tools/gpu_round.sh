#!/bin/bash
# Round check on one GPU: the whole -m gpu suite, smoke, then one bench line per configuration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/round_tests.log 2>&1 \
  || { echo "TESTS FAILED"; grep -E "FAILED|Error" gpurun_out/round_tests.log | head -20; tail -5 gpurun_out/round_tests.log; exit 1; }
tail -1 gpurun_out/round_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/round_smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -5 gpurun_out/round_smoke.log; exit 1; }
echo "smoke ok"
for args in "" "--full-grid" "--config C4" "--config C5" "--config C5 --c5-bits 8" "--config FEP" "--config UE" "--config UE3"; do
  name=$(echo "bench $args" | tr ' -' '__')
  timeout -k 10 300 python bench.py $args > gpurun_out/$name.log 2>&1 || { echo "BENCH FAILED: $args"; tail -5 gpurun_out/$name.log; exit 1; }
  echo "$args: $(grep -o '"value": [0-9.]*' gpurun_out/$name.log | head -1)"
done
