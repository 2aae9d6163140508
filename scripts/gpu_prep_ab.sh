#!/bin/bash
# Grant prep beside k_rsa_pow (aux stream) vs serialised on the launch stream
# (MOCHI_PREP_SERIAL=1): headline bench alternated on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
for i in 1 2; do
  for ser in 0 1; do
    MOCHI_PREP_SERIAL=$ser timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --headline-only > $OUT/prep_ab_$ser$i.json 2> $OUT/prep_ab_$ser$i.err || { tail -20 $OUT/prep_ab_$ser$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/prep_ab_$ser$i.json'));print('serial=$ser', round(d['value']/1e6,2),'M grants/s', d['ms_per_step'], d['stage_ms'])"
  done
done
