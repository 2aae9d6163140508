# Small-batch latency A/B (one GPU call): single small mochi_verify_write2 calls
# (scripts/small_batch_prof.py) with the default env and with each ';'-separated
# setting of $AB_ENVS, alternated twice, then a kernel trace of each.
#   AB_ENVS="MOCHI_NO_FINAL_LAT=1" bash scripts/gpu_small_ab.sh
IFS=';' read -ra ENVS <<< "${AB_ENVS}"
for i in 1 2; do
  for j in $(seq 0 ${#ENVS[@]}); do
    if [ $j = 0 ]; then E=""; t=A; else E="${ENVS[$((j-1))]}"; t="E$j"; fi
    echo -n "$t$i [$E] "; env $E REPS=200 timeout -k 10 200 python scripts/small_batch_prof.py || exit 1
  done
done
for j in $(seq 0 ${#ENVS[@]}); do
  if [ $j = 0 ]; then E=""; t=A; else E="${ENVS[$((j-1))]}"; t="E$j"; fi
  rm -rf gpurun_out/small_$t
  (cd /tmp && export TMPDIR=/tmp && env $E REPS=100 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/small_$t -o run -- python3 $GRAFT_REPO_ROOT/scripts/small_batch_prof.py > $GRAFT_REPO_ROOT/gpurun_out/small_$t.log 2>&1) || exit 1
  echo "$t $(grep -h 'k_rsa_final\|k_rsa_pow_lat' gpurun_out/small_$t/run_kernel_stats.csv | cut -d, -f1-6 | tr '\n' ' ')"
done
