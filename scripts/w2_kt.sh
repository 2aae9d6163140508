#!/bin/bash
# Wire-path tests + per-kernel times of the device decoder (rocprofv3 kernel trace).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_write2_wire_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/w2_tests.log 2>&1 || { tail -30 $OUT/w2_tests.log; exit 1; }
tail -2 $OUT/w2_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/w2_kt" -o run -- python3 "$R/scripts/w2_prof.py" > "$R/$OUT/w2_kt.log" 2>&1 || { tail -20 "$R/$OUT/w2_kt.log"; exit 1; }
grep -E "k_w2|k_rsa|k_grant|k_tally|k_bucket|Scan" "$R/$OUT/w2_kt/run_kernel_stats.csv" | cut -d, -f1-4 | sed 's/(.*)"/"/'
