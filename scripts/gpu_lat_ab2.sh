# A/B of k_rsa_pow_lat variants (in-tree lib, and each of $LIBS) on single small
# mochi_verify_write2 calls, alternated, then a kernel trace of each.
LIBS="${LIBS:-mochi-db_amd/libmochi_hip_seq.so mochi-db_amd/libmochi_hip_raw.so}"
for i in 1 2; do
  for v in A $LIBS; do
    if [ $v = A ]; then L=""; t=A; else L="$PWD/$v"; t=$(basename $v .so); fi
    echo -n "$t$i "; MOCHI_HIP_LIB=$L REPS=200 timeout -k 10 200 python scripts/small_batch_prof.py || exit 1
  done
done
for v in A $LIBS; do
  if [ $v = A ]; then L=""; t=A; else L="$PWD/$v"; t=$(basename $v .so); fi
  (cd /tmp && export TMPDIR=/tmp && MOCHI_HIP_LIB=$L REPS=100 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/lat_$t -o run -- python3 $GRAFT_REPO_ROOT/scripts/small_batch_prof.py > $GRAFT_REPO_ROOT/gpurun_out/lat_$t.log 2>&1) || exit 1
  echo "$t $(grep -h k_rsa_pow_lat gpurun_out/lat_$t/run_kernel_stats.csv | cut -d, -f2-6)"
done
