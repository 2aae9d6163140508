#!/bin/bash
# Round-2 GPU check: parity tests, then the default bench (C4 headline + legs).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
TESTS=${TESTS:-tests/}
timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(round(d['value']/1e6,2),'M grants/s', d['stage_ms'], d['roofline']['frac'])"
