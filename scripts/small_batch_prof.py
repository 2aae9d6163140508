"""Latency of one small Write2ToServer batch through mochi_verify_write2 (the
host path the batcher's flusher calls): wall time per call for batches of 1, 2
and 8 messages, best and median over many calls.  Run under rocprofv3
--kernel-trace (and --runtime-trace) to see where one call's time goes."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mochi-db_amd"), ROOT]

import numpy as np  # noqa: E402

import mochi_hip as mh  # noqa: E402
import workload as W  # noqa: E402

R = 4
reps = int(os.environ.get("REPS", "300"))
pool = W.build_pool(R=R, k=1, P=256, P_f=32, cache_dir=os.environ.get("MOCHI_CACHE", "/tmp/mochi_bench_cache"))
ver = mh.Verifier(pool.moduli, device=0)
ver.set_server_ids(W.SERVER_IDS[:R])
res = {}
for m in (1, 2, 8):
    s = W.make_batch(pool, m, first_cert=100)
    wb = W.encode_wire_batch(s)
    for _ in range(20):
        ver.verify_write2(wb, R, True)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ver.verify_write2(wb, R, True)
        ts.append(time.perf_counter() - t0)
    ts = np.sort(np.asarray(ts)) * 1e6
    res[f"msgs_{m}"] = {"best_us": round(float(ts[0]), 1), "p50_us": round(float(np.percentile(ts, 50)), 1),
                        "p90_us": round(float(np.percentile(ts, 90)), 1)}
ver.close()
print(json.dumps(res))
