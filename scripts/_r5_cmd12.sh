set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "c2 or c3 or golden or synthetic or edge or repeatable or bucketing" --timeout 300 --timeout-method thread > gpurun_out/t12.log 2>&1 || { tail -30 gpurun_out/t12.log; exit 1; }
tail -1 gpurun_out/t12.log
AB_LIBS="mochi-db_amd/libmochi_hip_fstat.so mochi-db_amd/libmochi_hip_pw4.so" bash scripts/gpu.sh parity || exit 1
AB_LIBS="mochi-db_amd/libmochi_hip_fstat.so mochi-db_amd/libmochi_hip_pw4.so" bash scripts/gpu.sh ab
