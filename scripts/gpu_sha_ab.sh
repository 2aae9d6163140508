set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sign.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/par_x3.log 2>&1 || { tail -30 $OUT/par_x3.log; exit 1; }
tail -1 $OUT/par_x3.log
AB_LIBS=mochi-db_amd/libmochi_hip_prev.so bash scripts/gpu_ab.sh || exit 1
for i in 1 2; do for L in "" "$PWD/mochi-db_amd/libmochi_hip_prev.so"; do
  MOCHI_HIP_LIB=$L MOCHI_PREP_SERIAL=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --headline-only > $OUT/pser.json 2> $OUT/pser.err || { tail -20 $OUT/pser.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/pser.json'));print('serial lib=${L##*/}', round(d['value']/1e6,2), d['stage_ms'])"
done; done
