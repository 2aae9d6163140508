# Round-6 records of one tree (one GPU call): the batcher / small-batch probe, the
# default bench (every leg), the headline kernel trace and the PMC passes.
bash scripts/gpu_batcher_probe.sh || exit 1
bash scripts/gpu.sh bench kt pmc || exit 1
