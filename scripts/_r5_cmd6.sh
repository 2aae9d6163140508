set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_write2_wire_gpu.py -x -q -m gpu -k "shapes or dedup or golden or branch or synthetic or c2 or edge or long or group_depth or ten_byte or callback or fallback or fuzz or wire" --timeout 300 --timeout-method thread > gpurun_out/t6.log 2>&1 || { tail -30 gpurun_out/t6.log; exit 1; }
tail -2 gpurun_out/t6.log
AB_ENVS="MOCHI_PREP_SERIAL=1;MOCHI_NO_DEDUP=1 MOCHI_PREP_SERIAL=1" bash scripts/gpu.sh abenv || exit 1
MOCHI_PREP_SERIAL=1 bash scripts/gpu.sh kt || exit 1
bash scripts/gpu.sh w2
