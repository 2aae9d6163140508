#!/bin/bash
# Round-2 profile session: rocprofv3 kernel trace + stats of the C4 headline,
# then the PMC passes (scripts/pmc.sh).  Every step has its own time limit.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; OUT=gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
rm -rf "$R/$OUT/prof_kt"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_kt" -o run -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --headline-only > "$R/$OUT/prof_kt.log" 2>&1 || { tail -20 "$R/$OUT/prof_kt.log"; exit 1; }
tail -1 "$R/$OUT/prof_kt.log"
python3 - "$R/$OUT/prof_kt" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f'{float(r["AverageNs"])/1e3:10.1f} us  x{r["Calls"]:>4}  {r["Name"][:90]}')
PY
bash "$R/scripts/pmc.sh"
