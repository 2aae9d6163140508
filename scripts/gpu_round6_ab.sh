# Round-6 GPU call: every -m gpu test, then the A/B of the two-level Karatsuba
# k_rsa_pow variants (parity subset, alternated headline steps, GRBM clock of each).
TEST_TIMEOUT=700 bash scripts/gpu.sh tests || exit 1
AB_LIBS="mochi-db_amd/libmochi_hip_k2l.so mochi-db_amd/libmochi_hip_k2lh.so" bash scripts/gpu.sh parity ab || exit 1
AB_LIBS="mochi-db_amd/libmochi_hip_k2l.so mochi-db_amd/libmochi_hip_k2lh.so" bash scripts/clk.sh 2>&1 | grep -E "k_rsa_pow" || exit 1
