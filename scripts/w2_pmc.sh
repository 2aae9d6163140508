#!/bin/bash
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/w2pmc"; rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P=(python3 "$R/scripts/w2_prof.py" 250000)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- "${P[@]}" > "$OUT/kt.log" 2>&1 || { tail -20 "$OUT/kt.log"; exit 1; }
tail -2 "$OUT/kt.log"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES --kernel-include-regex "k_w2" --output-format csv -d "$OUT/p1" -o run -- "${P[@]}" > "$OUT/p1.log" 2>&1 || { tail -20 "$OUT/p1.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
f = glob.glob(d + "/kt/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f'{float(r["AverageNs"])/1e3:10.1f} us  x{r["Calls"]:>4}  {r["Name"][:70]}')
f = glob.glob(d + "/p1/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    m = {c: sum(x) / len(x) for c, x in v.items()}
    w = m.get("SQ_WAVES", 1)
    print(k, {c: round(val / w, 1) for c, val in m.items()}, "(per wave)")
PY
