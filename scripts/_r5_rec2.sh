set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu.sh kt pmc w2
MOCHI_HIP_LIB=$PWD/mochi-db_amd/libmochi_hip_w2st.so timeout -k 10 300 python scripts/w2_stamps.py > gpurun_out/w2_stamps.json 2> gpurun_out/w2_stamps.err && cat gpurun_out/w2_stamps.json
