# Batcher / small-batch latency probe (one GPU call): batcher GPU tests, single
# small mochi_verify_write2 calls (wall time, then a kernel trace of them), and the
# bench's native batcher leg on a 2M-grant stream.  Run: bash scripts/gpu_batcher_probe.sh
timeout -k 10 300 python -u -m pytest tests/test_write2_wire_gpu.py -x -q -m gpu -k "batcher or context_closed" --timeout 120 --timeout-method thread > gpurun_out/bt.log 2>&1; tail -2 gpurun_out/bt.log
timeout -k 10 200 python scripts/small_batch_prof.py || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/sb_kt -o run -- python3 $GRAFT_REPO_ROOT/scripts/small_batch_prof.py > $GRAFT_REPO_ROOT/gpurun_out/sb_kt.log 2>&1) || exit 1
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --grants-total 2000000 --no-c3 --no-cluster --no-shard-sizes --no-separate --no-cpu-baseline > gpurun_out/bench_small.json 2> gpurun_out/bench_small.err || exit 1
python -c "
import json;d=json.load(open('gpurun_out/bench_small.json'))
for r in d['write2_wire_path']['batcher_native']['rows']: print(r['mode'],r['threads'],r['contexts'],r['requests_per_s'],r['latency_us'],r['mean_batch_msgs'])"
