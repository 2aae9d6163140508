#!/bin/bash
# rocprofv3 kernel trace + stats of one bench run (no CPU baseline).
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${PROF_NAME:-prof_kt}"; rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 "$R/bench.py" --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT.log" 2>&1 || { tail -20 "$OUT.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f'{float(r["AverageNs"])/1e3:10.1f} us  x{r["Calls"]:>4}  {r["Name"][:90]}')
PY
