#!/bin/bash
# One GPU session driver (replaces the one-off gpu_*.sh scripts).  Steps run in
# the order given, each under its own time limit; the chain stops at the first
# failure (no retries).  Usage on the box:
#   bash scripts/gpu.sh STEP [STEP ...]
# Steps:
#   tests        every -m gpu test (TESTS= to narrow, e.g. TESTS=tests/test_gpu_parity.py)
#   parity       the quick parity subset for the in-tree lib and each of $AB_LIBS
#   smoke        __graft_entry__.smoke()
#   bench        the default bench (C4 headline + every leg) -> gpurun_out/bench.json
#   ab           headline-only bench, in-tree lib vs each of $AB_LIBS, alternated twice
#                (AB_ENV="A=... B=..." per-variant env overrides are not supported: use libs)
#   abenv        headline-only bench, default env vs each ';'-separated env setting of
#                $AB_ENVS (e.g. AB_ENVS="MOCHI_NO_DEDUP=1;MOCHI_PREP_SERIAL=1"), alternated twice
#   kt           rocprofv3 kernel trace + stats of the headline (-> gpurun_out/prof_kt)
#   pmc          the PMC passes (scripts/pmc.sh)
#   w2           wire-path tests + kernel trace of the device decoder (w2_prof.py)
#   w2ab         wire path (w2_prof.py), in-tree lib vs each of $AB_LIBS, alternated
# Environment: BENCH_ARGS (extra bench.py flags), STEPS, AB_LIBS.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; OUT=gpurun_out; mkdir -p $OUT
fail() { echo "step $1 failed"; tail -40 "$2"; exit 1; }
kstats() {
  python3 - "$1" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f'{float(r["AverageNs"])/1e3:10.1f} us  x{r["Calls"]:>4}  {r["Name"][:90]}')
PY
}
for step in "$@"; do
  case $step in
  tests)
    timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests/} -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || fail tests $OUT/pytest_gpu.log
    tail -3 $OUT/pytest_gpu.log ;;
  parity)
    for v in A ${AB_LIBS}; do
      if [ $v = A ]; then L=""; t=A; else L="$PWD/$v"; t=$(basename $v .so); fi
      MOCHI_HIP_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "golden or branch or synthetic or c2 or bucketing or edge" --timeout 120 --timeout-method thread > $OUT/par_$t.log 2>&1 || fail parity $OUT/par_$t.log
      echo "$t: $(tail -1 $OUT/par_$t.log)"
    done ;;
  smoke)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || fail smoke $OUT/smoke.log
    tail -1 $OUT/smoke.log ;;
  bench)
    timeout -k 10 ${BENCH_TIMEOUT:-900} python -u bench.py --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || fail bench $OUT/bench.err
    python -c "import json;d=json.load(open('$OUT/bench.json'));print(round(d['value']/1e6,2),'M grants/s', d.get('stage_ms'), d['roofline']['frac'])" ;;
  ab)
    for i in 1 2; do
      for v in A ${AB_LIBS}; do
        if [ $v = A ]; then L=""; t=A; else L="$PWD/$v"; t=$(basename $v .so); fi
        MOCHI_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --headline-only ${BENCH_ARGS:-} > $OUT/ab_$t$i.json 2> $OUT/ab_$t$i.err || fail ab $OUT/ab_$t$i.err
        python -c "import json;d=json.load(open('$OUT/ab_$t$i.json'));print('$t$i', round(d['value']/1e6,2),'M grants/s', d['ms_per_step'], d['stage_ms'], 'ok=',d.get('correct_vs_ground_truth'))"
      done
    done ;;
  abenv)
    IFS=';' read -ra ENVS <<< "${AB_ENVS}"
    for i in 1 2; do
      for j in $(seq 0 ${#ENVS[@]}); do
        if [ $j = 0 ]; then E=""; t=A; else E="${ENVS[$((j-1))]}"; t="E$j"; fi
        env $E timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --headline-only ${BENCH_ARGS:-} > $OUT/abenv_$t$i.json 2> $OUT/abenv_$t$i.err || fail abenv $OUT/abenv_$t$i.err
        python -c "import json;d=json.load(open('$OUT/abenv_$t$i.json'));print('$t$i [$E]', round(d['value']/1e6,2),'M grants/s', d['ms_per_step'], d['stage_ms'], 'ok=',d.get('correct_vs_ground_truth'))"
      done
    done ;;
  kt)
    rm -rf "$R/$OUT/prof_kt"
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_kt" -o run -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --headline-only ${BENCH_ARGS:-} > "$R/$OUT/prof_kt.log" 2>&1) || fail kt $OUT/prof_kt.log
    tail -1 $OUT/prof_kt.log; kstats "$R/$OUT/prof_kt" ;;
  pmc)
    bash scripts/pmc.sh || exit 1 ;;
  w2)
    timeout -k 10 300 python -u -m pytest tests/test_write2_wire_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/w2_tests.log 2>&1 || fail w2 $OUT/w2_tests.log
    tail -2 $OUT/w2_tests.log
    rm -rf "$R/$OUT/w2_kt"
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/w2_kt" -o run -- python3 "$R/scripts/w2_prof.py" > "$R/$OUT/w2_kt.log" 2>&1) || fail w2kt $OUT/w2_kt.log
    kstats "$R/$OUT/w2_kt" | grep -E "k_w2|Scan|k_rsa|k_grant|k_tally|k_bucket" ;;
  w2ab)
    for i in 1 2; do
      for v in A ${AB_LIBS}; do
        if [ $v = A ]; then L=""; t=A; else L="$PWD/$v"; t=$(basename $v .so); fi
        echo -n "$t$i "; MOCHI_HIP_LIB=$L timeout -k 10 300 python scripts/w2_prof.py 2>/dev/null | tail -1 || exit 1
      done
    done ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
