#!/bin/bash
# k_rsa_pow variants A/B on one box (scripts/gpu_ab.sh) after a quick parity check
# of every variant on the C2-sized GPU parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
for v in ${AB_LIBS}; do
  MOCHI_HIP_LIB=$PWD/$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "golden or branch or synthetic or c2 or bucketing or edge" --timeout 120 --timeout-method thread > $OUT/par_$(basename $v .so).log 2>&1 || { tail -20 $OUT/par_$(basename $v .so).log; exit 1; }
  tail -1 $OUT/par_$(basename $v .so).log
done
bash scripts/gpu_ab.sh
