set -o pipefail
mkdir -p gpurun_out
AB_LIBS="mochi-db_amd/libmochi_hip_fph.so" bash scripts/gpu.sh parity || exit 1
AB_LIBS="mochi-db_amd/libmochi_hip_fph.so" bash scripts/gpu.sh ab
