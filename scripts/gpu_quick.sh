#!/bin/bash
# Quick GPU check: parity tests + one bench line (no CPU baseline, no profiler).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench_quick.json 2> $OUT/bench_quick.err || { tail -20 $OUT/bench_quick.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_quick.json'));print(round(d['value']/1e6,2),'M grants/s', d['stage_ms'], d['roofline']['frac'])"
