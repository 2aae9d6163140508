set -o pipefail
mkdir -p gpurun_out
AB_LIBS="mochi-db_amd/libmochi_hip_t128.so" bash scripts/gpu.sh ab || exit 1
TEST_TIMEOUT=1500 bash scripts/gpu.sh tests
