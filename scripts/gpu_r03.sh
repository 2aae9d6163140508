#!/bin/bash
# Round-3 session: the default bench (C4 headline + every leg), then the
# rocprofv3 kernel trace + stats of the headline and the PMC passes.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; OUT=gpurun_out; mkdir -p $OUT
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-900} python -u bench.py --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench.json'));print(round(d['value']/1e6,2),'M grants/s', d['stage_ms'], d['roofline']['frac'])"
fi
[ -n "$NO_PROF" ] && exit 0
bash scripts/prof_r02.sh
