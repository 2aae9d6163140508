#!/bin/bash
# PMC passes over the fold prototype (microbench/fold_bench.py), one counter group per pass.
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/fold_pmc"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "fold" --output-format csv \
    -d "$OUT/$name" -o run -- python3 "$R/microbench/fold_bench.py" ${FOLD_N:-262144} > "$OUT/$name.log" 2>&1 || { echo "pass $name failed"; tail -20 "$OUT/$name.log"; exit 1; }
}
pass a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
pass b SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA
find "$OUT" -name "*counter_collection.csv"
