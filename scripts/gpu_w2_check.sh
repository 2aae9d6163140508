set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_write2_wire_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/w2_tests.log 2>&1 || { tail -30 gpurun_out/w2_tests.log; exit 1; }
tail -2 gpurun_out/w2_tests.log
W2_VARIANTS="${W2_VARIANTS:-new v1}" bash scripts/gpu_w2_var.sh
