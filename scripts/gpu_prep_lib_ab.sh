#!/bin/bash
# Grant prep serialised on the launch stream (MOCHI_PREP_SERIAL=1, so its
# stage time is its standalone time): the in-tree build vs $AB_LIBS, alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
for i in 1 2; do for L in "" ${AB_LIBS}; do
  [ -n "$L" ] && L="$PWD/$L"
  MOCHI_HIP_LIB=$L MOCHI_PREP_SERIAL=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --headline-only > $OUT/pser.json 2> $OUT/pser.err || { tail -20 $OUT/pser.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/pser.json'));print('serial lib=${L##*/}', round(d['value']/1e6,2), d['stage_ms'], 'ok=', d.get('correct_vs_ground_truth'))"
done; done
