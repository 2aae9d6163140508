set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_write2_wire_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t13.log 2>&1 || { tail -40 gpurun_out/t13.log; exit 1; }
tail -1 gpurun_out/t13.log
MOCHI_HIP_LIB=mochi-db_amd/libmochi_hip_w2st.so timeout -k 10 200 python scripts/w2_stamps.py > gpurun_out/w2st13.json 2>gpurun_out/w2st13.err || { tail gpurun_out/w2st13.err; exit 1; }
cat gpurun_out/w2st13.json
AB_LIBS="mochi-db_amd/libmochi_hip_m0.so" bash scripts/gpu.sh w2ab
