set -o pipefail
mkdir -p gpurun_out
STEPS=20 BENCH_TIMEOUT=1000 bash scripts/gpu.sh bench || exit 1
bash scripts/gpu.sh kt pmc
