#!/bin/bash
# One-GPU session driver.  Folds the one-off drivers of rounds 1-5 (tools/gpu_r04*.sh, gpu_r05*.sh,
# the ab_* / mod_* / dec_* / enc_* sweeps; they stay in git history) into steps run in order:
#
#   bash tools/gpu_round.sh STEP [STEP ...]
#
#   tests[:FILES]     -m gpu tests (default the whole suite; FILES comma-separated)   tools/gpu_tests.sh
#   smoke             __graft_entry__.smoke()
#   bench[:ARGS]      one bench.py line, ARGS comma-separated (bench:--config,C5)  -> gpurun_out/bench_TAG_*.log
#   lines             the bench line of every configuration (C3, full grid, C2, C4, C5 x3, FEP, UE, UE3)
#   profile[:CONFIG]  rocprofv3 kernel trace + stats, calibrated FETCH / WRITE passes   tools/gpu_profile.sh
#   valu[:CONFIG]     one rocprofv3 --pmc VALU / LDS / wait pass                        tools/gpu_pmc_valu.sh
#   ab[:ARGS]         variants/*/libopenair4g_amd.so against the in-tree library      tools/gpu_ab.sh
#   encphases         k_encode cut after each phase (tools/diag_phases.py) + its SQ counters (tools/pmc_encode.sh)
#
# env TAG (outputs), BATCH (C3 8192, C5 49152 for profile / valu).  Every GPU step has its own time limit;
# the first failing step ends the session (no retries).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-round}
fail() { echo "STEP FAILED: $1"; exit 1; }
bench_line() {   # $1 = name, rest = bench.py args
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/bench_${TAG}_${name}.json.log 2>&1 \
    || { tail -5 gpurun_out/bench_${TAG}_${name}.json.log; fail "bench $*"; }
  echo "bench [$*]: $(grep -o '"value": [0-9.]*' gpurun_out/bench_${TAG}_${name}.json.log | head -1)"
}
for step in "$@"; do
  name=${step%%:*}; arg=""; [ "$name" != "$step" ] && arg=${step#*:}
  case $name in
    tests) TAG=$TAG bash tools/gpu_tests.sh ${arg//,/ } || fail tests ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 \
             || { tail -5 gpurun_out/smoke_${TAG}.log; fail smoke; }
           tail -1 gpurun_out/smoke_${TAG}.log ;;
    bench) a=${arg//,/ }; bench_line "$(echo "C3 $a" | tr -cd 'A-Za-z0-9 ' | tr ' ' '_')" $a ;;
    lines) bench_line C3; bench_line full_grid --full-grid; bench_line C2 --config C2; bench_line C4 --config C4
           bench_line C5 --config C5; bench_line C5_snr --config C5 --c5-mode snr; bench_line C5_chain --config C5 --c5-mode chain
           bench_line C5_8bit --config C5 --c5-bits 8; bench_line FEP --config FEP; bench_line UE --config UE
           bench_line UE3 --config UE3 ;;
    profile) c=${arg:-C3}; TAG=$TAG CONFIG=$c bash tools/gpu_profile.sh > gpurun_out/prof_${TAG}_$c.log 2>&1 \
               || { tail -20 gpurun_out/prof_${TAG}_$c.log; fail "profile $c"; }
             rm -rf gpurun_out/prof_$c && mv gpurun_out/prof gpurun_out/prof_$c
             tail -8 gpurun_out/prof_${TAG}_$c.log ;;
    valu) c=${arg:-C3}; b=${BATCH:-$(case $c in C5) echo 49152 ;; C2) echo 2048 ;; C4) echo 1024 ;; *) echo 8192 ;; esac)}
          TAG=$TAG CONFIG=$c NAME=$c BATCH=$b bash tools/gpu_pmc_valu.sh > gpurun_out/valu_${TAG}_$c.log 2>&1 \
            || { tail -20 gpurun_out/valu_${TAG}_$c.log; fail "valu $c"; }
          tail -6 gpurun_out/valu_${TAG}_$c.log ;;
    ab) TAG=$TAG bash tools/gpu_ab.sh ${arg//,/ } || fail ab ;;
    encphases) timeout -k 10 300 python tools/diag_phases.py C3 8192 > gpurun_out/encphases_${TAG}.txt 2>&1 \
                 || { tail -5 gpurun_out/encphases_${TAG}.txt; fail encphases; }
               cat gpurun_out/encphases_${TAG}.txt
               bash tools/pmc_encode.sh || fail "pmc_encode" ;;
    *) fail "unknown step $step" ;;
  esac
done
echo ALL_OK
