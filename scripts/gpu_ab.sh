#!/bin/bash
# A/B of two builds of the library on one box: headline bench only, alternated
# A B A B so clock drift hits both.  B = $AB_LIB (default libmochi_hip_ab.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
B=${AB_LIB:-mochi-db_amd/libmochi_hip_ab.so}
for i in 1 2; do
  for v in A B; do
    if [ $v = A ]; then L=""; else L="$PWD/$B"; fi
    MOCHI_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --headline-only ${BENCH_ARGS:-} > $OUT/ab_$v$i.json 2> $OUT/ab_$v$i.err || { tail -20 $OUT/ab_$v$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/ab_$v$i.json'));print('$v$i', round(d['value']/1e6,2),'M grants/s', d['stage_ms'])"
  done
done
