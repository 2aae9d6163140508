set -o pipefail
mkdir -p gpurun_out
AB_LIBS="mochi-db_amd/libmochi_hip_nah0.so" bash scripts/gpu.sh parity || exit 1
AB_LIBS="mochi-db_amd/libmochi_hip_nah0.so" BENCH_ARGS="--shard-sizes" bash scripts/gpu.sh ab
