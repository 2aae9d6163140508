# Round-6 GPU call for the small-batch latency kernel: every -m gpu test (small
# batches take k_rsa_pow_lat), then the batcher / small-batch probe.
TEST_TIMEOUT=700 bash scripts/gpu.sh tests || exit 1
bash scripts/gpu_batcher_probe.sh || exit 1
