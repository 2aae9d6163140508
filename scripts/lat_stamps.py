"""Phase times of k_rsa_pow_lat from a MOCHI_LAT_STAMPS build (MOCHI_HIP_LIB points
at it): small mochi_verify_write2 calls (2 messages, R = 4), then per wave the
s_memtime cycles per squaring in each phase -- squares, barrier 1, combine +
barrier 2, fold (+ barrier 3), barrier 4, carry chain, barrier 5, and the whole
squaring -- averaged over the blocks that ran.  One JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mochi-db_amd"), ROOT]

import numpy as np  # noqa: E402

import mochi_hip as mh  # noqa: E402
import workload as W  # noqa: E402

R = 4
pool = W.build_pool(R=R, k=1, P=256, P_f=32, cache_dir=os.environ.get("MOCHI_CACHE", "/tmp/mochi_bench_cache"))
ver = mh.Verifier(pool.moduli, device=0)
ver.set_server_ids(W.SERVER_IDS[:R])
s = W.make_batch(pool, 2, first_cert=100, faults=False)
wb = W.encode_wire_batch(s)
lib = ctypes.CDLL(os.environ["MOCHI_HIP_LIB"])
names = ["squares", "bar1", "combine_bar2", "fold_bar3", "bar4", "carry", "bar5", "loop"]
acc = []
for _ in range(20):
    ver.verify_write2(wb, R, True)
    buf = (ctypes.c_ulonglong * (256 * 4 * 8))()
    assert lib.mochi_debug_lat_stamps(buf, 256) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(256, 4, 8).astype(np.float64)
    ran = a[:, 0, 7] > 0
    acc.append(a[ran].mean(axis=0) / 16.0)
    ctypes.memset(buf, 0, ctypes.sizeof(buf))
m = np.mean(acc[5:], axis=0)  # [wave][phase] cycles per squaring
res = {"blocks_ran": int(ran.sum()), "cycles_per_squaring": {f"wave{w}": {n: round(float(m[w][i])) for i, n in enumerate(names)} for w in range(4)}}
ver.close()
print(json.dumps(res))
