set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu.sh tests smoke w2 || exit 1
MOCHI_HIP_LIB=mochi-db_amd/libmochi_hip_w2st.so timeout -k 10 200 python scripts/w2_stamps.py > gpurun_out/w2st_rec3.json 2>gpurun_out/w2st_rec3.err || { tail gpurun_out/w2st_rec3.err; exit 1; }
cat gpurun_out/w2st_rec3.json
