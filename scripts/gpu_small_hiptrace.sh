# HIP API + kernel trace of single small mochi_verify_write2 calls (no counters):
# where a call's host time goes.
rm -rf gpurun_out/sb_hip
(cd /tmp && export TMPDIR=/tmp && REPS=60 timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/sb_hip -o run -- python3 $GRAFT_REPO_ROOT/scripts/small_batch_prof.py > $GRAFT_REPO_ROOT/gpurun_out/sb_hip.log 2>&1) || { tail -20 gpurun_out/sb_hip.log; exit 1; }
ls gpurun_out/sb_hip
