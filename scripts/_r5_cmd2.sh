set -o pipefail
mkdir -p gpurun_out
MOCHI_PREP_SERIAL=1 bash scripts/gpu.sh kt || exit 1
bash scripts/gpu.sh w2
