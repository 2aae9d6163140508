# A/B of round-6 k_rsa_pow variants (two-level Karatsuba): parity subset, alternated headline
# steps, and the clock of each (GRBM_GUI_ACTIVE over the kernel trace).
AB_LIBS="mochi-db_amd/libmochi_hip_k2l.so mochi-db_amd/libmochi_hip_k2lh.so" bash scripts/gpu.sh parity ab || exit 1
AB_LIBS="mochi-db_amd/libmochi_hip_k2l.so mochi-db_amd/libmochi_hip_k2lh.so" bash scripts/clk.sh 2>&1 | grep -E "k_rsa_pow" || exit 1
