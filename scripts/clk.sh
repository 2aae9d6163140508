#!/bin/bash
# Effective GPU clock per kernel: GRBM_GUI_ACTIVE cycles over the kernel-trace
# duration, for the in-tree library and each of $AB_LIBS (headline bench, 2 steps).
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/clk"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in A ${AB_LIBS}; do
  if [ $v = A ]; then L=""; t=A; else L="$R/$v"; t=$(basename $v .so); fi
  MOCHI_HIP_LIB=$L timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES --kernel-trace \
    --kernel-include-regex "k_rsa_pow|k_rsa_final|k_grant_prep" --output-format csv -d "$OUT/$t" -o run -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --headline-only ${BENCH_ARGS:-} > "$OUT/$t.log" 2>&1 \
    || { echo "clk $t failed"; tail -20 "$OUT/$t.log"; exit 1; }
  python3 - "$OUT/$t" "$t" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
cc = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
kt = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)
vals = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for r in csv.DictReader(open(cc)):
    vals[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    names[r["Dispatch_Id"]] = r["Kernel_Name"][:40]
dur = {}
if kt:
    for r in csv.DictReader(open(kt[0])):
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for k, v in vals.items():
    us = dur.get(k)
    ghz = v["GRBM_GUI_ACTIVE"] / (us * 1e3) if us else float("nan")
    print(sys.argv[2], names[k], f"{us} us", {c: int(x) for c, x in v.items()}, f"clk {ghz:.3f} GHz")
PY
done
