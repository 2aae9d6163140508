set -o pipefail
mkdir -p gpurun_out
echo "== C3"; BENCH_ARGS="--config c3" bash scripts/clk.sh 2>&1 | grep k_rsa_pow | tail -2 || exit 1
echo "== C4 stream at 4M"; BENCH_ARGS="--grants-total 4000000" bash scripts/clk.sh 2>&1 | grep k_rsa_pow | tail -2 || exit 1
echo "== C4 stream at 4M, R=7 keys"; BENCH_ARGS="--grants-total 4000000 --replication 7" bash scripts/clk.sh 2>&1 | grep k_rsa_pow | tail -2
