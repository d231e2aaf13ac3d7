#!/bin/bash
# Modulator timing diagnostics (variants with wrong output: no parity run): C3 bench kernel times
# per variant, then one SQ PMC pass each for the LDS instruction / bank-conflict counts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/diag
for rep in 1 2; do
  for lib in openair4g_amd/lib/libopenair4g_amd.so variants/*/libopenair4g_amd.so; do
    [ -f "$lib" ] || continue
    OAI4G_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/diag/b.log 2>&1 || exit 1
    echo "$lib $(grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}' gpurun_out/diag/b.log | tr '\n' ' ')"
  done
done
CTRS="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
i=0
for lib in openair4g_amd/lib/libopenair4g_amd.so variants/*/libopenair4g_amd.so; do
  [ -f "$lib" ] || continue
  i=$((i+1))
  OAI4G_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/diag/pmc_$i -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --kernel-reps 1 > gpurun_out/diag/pmc_$i.log 2>&1 || exit 1
  echo "pmc $i = $lib"
  python3 tools/valu_table.py gpurun_out/diag/pmc_$i C3 8192 | grep modofdm
done
