#!/bin/bash
# Headline bench only (no tests, no side legs): quick A/B of a kernel change.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --headline-only ${BENCH_ARGS:-} > $OUT/bench_only.json 2> $OUT/bench_only.err || { tail -20 $OUT/bench_only.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_only.json'));print(round(d['value']/1e6,2),'M grants/s', d['stage_ms'])"
