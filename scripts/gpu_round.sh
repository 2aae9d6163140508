#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel trace.  Every GPU step
# has its own time limit and the chain stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_kt" -o run -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --headline-only > "$R/$OUT/prof_kt.log" 2>&1 || { tail -20 "$R/$OUT/prof_kt.log"; exit 1; }
find "$R/$OUT/prof_kt" -name "*stats*" | head
timeout -k 10 120 rocprofv3 -L > "$R/$OUT/counters.txt" 2>&1 || true
