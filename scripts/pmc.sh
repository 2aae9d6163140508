#!/bin/bash
# rocprofv3 PMC passes over bench.py (counters only, one group per pass, no
# tracing domains besides the kernel trace the counters attach to).
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/pmc"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH=(python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --headline-only ${BENCH_ARGS:-})
pass() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex "k_rsa|k_grant_prep|k_tally" --output-format csv \
    -d "$OUT/$name" -o run -- "${BENCH[@]}" > "$OUT/$name.log" 2>&1 || { echo "pass $name failed"; tail -20 "$OUT/$name.log"; exit 1; }
}
pass sq1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU
pass sq2 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_IFETCH SQ_WAVES GRBM_GUI_ACTIVE
pass sq3 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE
pass write WRITE_SIZE
echo "pmc passes done"
