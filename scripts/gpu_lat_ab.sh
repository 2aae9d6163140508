# A/B of the small-batch pow kernel: single small mochi_verify_write2 calls with
# k_rsa_pow_lat and with k_rsa_pow (MOCHI_NO_LAT=1), alternated, each under a kernel trace.
for i in 1 2; do
  for v in lat big; do
    if [ $v = big ]; then export MOCHI_NO_LAT=1; else unset MOCHI_NO_LAT; fi
    echo -n "$v$i "; REPS=200 timeout -k 10 200 python scripts/small_batch_prof.py || exit 1
  done
done
unset MOCHI_NO_LAT
(cd /tmp && export TMPDIR=/tmp && REPS=100 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/lat_kt -o run -- python3 $GRAFT_REPO_ROOT/scripts/small_batch_prof.py > $GRAFT_REPO_ROOT/gpurun_out/lat_kt.log 2>&1) || exit 1
(cd /tmp && export TMPDIR=/tmp && MOCHI_NO_LAT=1 REPS=100 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/big_kt -o run -- python3 $GRAFT_REPO_ROOT/scripts/small_batch_prof.py > $GRAFT_REPO_ROOT/gpurun_out/big_kt.log 2>&1) || exit 1
grep -h "k_rsa_pow" gpurun_out/lat_kt/run_kernel_stats.csv gpurun_out/big_kt/run_kernel_stats.csv | cut -c1-200
