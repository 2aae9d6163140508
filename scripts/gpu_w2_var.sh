#!/bin/bash
# Wire-path A/B over library variants (scripts/w2_prof.py: 250k messages, ms/step).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
for i in 1 2; do
  for v in $W2_VARIANTS; do
    MOCHI_HIP_LIB=$PWD/mochi-db_amd/libmochi_hip_$v.so timeout -k 10 200 python scripts/w2_prof.py > $OUT/w2var_$v$i.log 2>&1 || { tail -20 $OUT/w2var_$v$i.log; exit 1; }
    echo "$v$i $(grep 'wire path' $OUT/w2var_$v$i.log)"
  done
done
