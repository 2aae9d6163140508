#!/bin/bash
# Wire path (scripts/w2_prof.py: 250k messages decode + verify, device-resident)
# with the in-tree library and each of $AB_LIBS, alternated, one box; then the
# kernel trace of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
LIBS=(A ${AB_LIBS})
for i in 1 2; do
  for v in "${LIBS[@]}"; do
    if [ $v = A ]; then L=""; else L="$PWD/$v"; fi
    echo -n "$(basename $v) "; MOCHI_HIP_LIB=$L timeout -k 10 300 python scripts/w2_prof.py 2>/dev/null | tail -1 || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for v in "${LIBS[@]}"; do
  if [ $v = A ]; then L=""; else L="$GRAFT_REPO_ROOT/$v"; fi
  t=$(basename $v .so)
  MOCHI_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/w2l_$t" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/w2_prof.py" > /dev/null 2>&1 || exit 1
  echo "== $t"; python3 "$GRAFT_REPO_ROOT/scripts/kstats.py" "$GRAFT_REPO_ROOT/$OUT/w2l_$t/run_kernel_stats.csv" | grep k_w2
done
