#!/bin/bash
# Round-3 session check: parity tests, smoke, then the default bench.  Every GPU
# step has its own time limit and the chain stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(round(d['value']/1e6,2),'M grants/s', d.get('stage_ms'), d['roofline'])"
