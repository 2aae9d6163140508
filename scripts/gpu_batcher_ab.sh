# The bench's native batcher leg (2M-grant stream) with the default env and with
# each ';'-separated setting of $AB_ENVS, alternated twice.
IFS=';' read -ra ENVS <<< "${AB_ENVS}"
for i in 1 2; do
  for j in $(seq 0 ${#ENVS[@]}); do
    if [ $j = 0 ]; then E=""; t=A; else E="${ENVS[$((j-1))]}"; t="E$j"; fi
    env $E timeout -k 10 600 python bench.py --steps 3 --warmup 1 --grants-total 2000000 --no-c3 --no-cluster --no-shard-sizes --no-separate --no-cpu-baseline > gpurun_out/bab_$t$i.json 2> gpurun_out/bab_$t$i.err || { tail -20 gpurun_out/bab_$t$i.err; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/bab_$t$i.json'))
print('$t$i [$E]', ' | '.join(f\"{r['mode']} {r['threads']}/{r['contexts']} {r['requests_per_s']:.0f} p50 {r['latency_us']['p50']}\" for r in d['write2_wire_path']['batcher_native']['rows'][:2]+d['write2_wire_path']['batcher_native']['rows'][4:5]))"
  done
done
