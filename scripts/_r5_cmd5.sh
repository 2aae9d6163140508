set -o pipefail
mkdir -p gpurun_out
AB_LIBS="mochi-db_amd/libmochi_hip_pipe.so" bash scripts/gpu.sh parity || exit 1
MOCHI_HIP_LIB=$PWD/mochi-db_amd/libmochi_hip_pipe.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "c3 or bucketing or repeatable or device_resident or chunking" --timeout 300 --timeout-method thread > gpurun_out/t5.log 2>&1 || { tail -30 gpurun_out/t5.log; exit 1; }
tail -1 gpurun_out/t5.log
AB_LIBS="mochi-db_amd/libmochi_hip_pipe.so" BENCH_ARGS="--shard-sizes" bash scripts/gpu.sh ab
