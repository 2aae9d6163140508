#!/bin/bash
# A/B(/C...) of builds of the library on one box: headline bench only,
# alternated A B C A B C so clock drift hits all.  A = the in-tree build;
# the others = $AB_LIBS (default: mochi-db_amd/libmochi_hip_ab.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
LIBS=(A ${AB_LIBS:-mochi-db_amd/libmochi_hip_ab.so})
for i in 1 2; do
  for k in "${!LIBS[@]}"; do
    v=${LIBS[$k]}; tag=$(basename $v .so)
    if [ $v = A ]; then L=""; else L="$PWD/$v"; fi
    MOCHI_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --headline-only ${BENCH_ARGS:-} > $OUT/ab_$tag$i.json 2> $OUT/ab_$tag$i.err || { tail -20 $OUT/ab_$tag$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/ab_$tag$i.json'));print('$tag$i', round(d['value']/1e6,2),'M grants/s', d['stage_ms'], 'ok=',d.get('correct_vs_ground_truth'))"
  done
done
