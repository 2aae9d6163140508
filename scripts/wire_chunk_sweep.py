"""Host wire path (mochi_verify_write2 on pinned Write2ToServer bodies) at
several pipeline chunk sizes: where PCIe, fill/drain and per-chunk overheads
balance.  One JSON line per chunk size."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mochi-db_amd"), ROOT]

import numpy as np  # noqa: E402

import bench  # noqa: E402
import mochi_hip as mh  # noqa: E402
import workload as W  # noqa: E402

R = 4
certs = int(os.environ.get("CERTS", "250000"))
synth = W.make_batch_unique(R, certs, 1, first_cert=0, device=0)
wb = W.encode_wire_batch(synth)
moduli = [mh.pem_modulus(p) for p in W.load_keys(R)]
ver = mh.Verifier(moduli, device=0)
ver.set_server_ids(W.SERVER_IDS[:R])
pwb, keep = bench.pinned_wire(wb)
ref = None
for cg in [int(x) for x in os.environ.get("CHUNKS", "16384,32768,65536,131072,262144").split(",")]:
    ver.set_chunk_grants(cg)
    best, best_wall = float("inf"), float("inf")
    for _ in range(4):
        t0 = time.perf_counter()
        hv, _ = ver.verify_write2(pwb, R, True)
        best_wall = min(best_wall, time.perf_counter() - t0)
        best = min(best, hv.timing_ms["total"] / 1e3)
    if ref is None:
        ref = hv.cert_reason.copy()
    same = bool(np.array_equal(ref, hv.cert_reason))
    print(json.dumps({"chunk_grants": cg, "chunk_wire_mb": round(cg * 256 / 1e6, 1),
                      "grants_per_s": round(synth.batch.n_grants / best, 1),
                      "wire_gb_per_s": round(wb.wire.nbytes / best / 1e9, 2),
                      "wall_wire_gb_per_s": round(wb.wire.nbytes / best_wall / 1e9, 2), "same": same}), flush=True)
