set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "c2 or golden or synthetic or edge or dedup" --timeout 300 --timeout-method thread > gpurun_out/t18.log 2>&1 || { tail -30 gpurun_out/t18.log; exit 1; }
tail -1 gpurun_out/t18.log
MOCHI_PREP_FIRST=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "c2 or golden or synthetic or edge or dedup" --timeout 300 --timeout-method thread > gpurun_out/t18b.log 2>&1 || { tail -30 gpurun_out/t18b.log; exit 1; }
tail -1 gpurun_out/t18b.log
AB_ENVS="MOCHI_PREP_FIRST=1" bash scripts/gpu.sh abenv
