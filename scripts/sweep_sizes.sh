#!/bin/bash
# Per-grant k_rsa_pow time vs batch size (wave-quantisation / tail study).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/sweep
for g in ${SIZES:-786432 900000 983040 1000000 1100000 1179648 1572864}; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --grants-per-gpu $g > gpurun_out/sweep/$g.json 2> gpurun_out/sweep/$g.err || { tail -5 gpurun_out/sweep/$g.err; exit 1; }
  python -c "import json,sys;d=json.load(open('gpurun_out/sweep/$g.json'));s=d['stage_ms'];n=d['config']['grants_per_gpu'];print(n, round(d['value']/1e6,1), s, 'pow ns/grant', round(s['rsa_pow']*1e6/n,3))"
done
