set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_write2_wire_gpu.py -x -q -m gpu -k "shapes or dedup or golden or branch or synthetic or c2 or edge or long or ten_byte or fuzz or wire" --timeout 300 --timeout-method thread > gpurun_out/t10.log 2>&1 || { tail -30 gpurun_out/t10.log; exit 1; }
tail -1 gpurun_out/t10.log
AB_LIBS="mochi-db_amd/libmochi_hip_pdirect.so" bash scripts/gpu.sh parity || exit 1
MOCHI_PREP_SERIAL=1 AB_LIBS="mochi-db_amd/libmochi_hip_pdirect.so" bash scripts/gpu.sh ab || exit 1
AB_LIBS="mochi-db_amd/libmochi_hip_pdirect.so" bash scripts/gpu.sh ab
