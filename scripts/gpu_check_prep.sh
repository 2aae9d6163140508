#!/bin/bash
# Parity of the grant-prep / signer paths (SHA-256 message loading) and the
# prep serial-vs-beside A/B on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sign.py tests/test_write2_wire_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/prep_tests.log 2>&1 || { tail -30 $OUT/prep_tests.log; exit 1; }
tail -1 $OUT/prep_tests.log
bash scripts/gpu_prep_ab.sh
