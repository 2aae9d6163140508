#!/usr/bin/env python3
"""Wire-path profiling driver: 250k Write2ToServer messages (R=4) decoded +
verified on the device a few times (run under rocprofv3)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mochi-db_amd"))

import torch  # noqa: E402

import mochi_hip as mh  # noqa: E402
import workload as W  # noqa: E402

n_certs = int(sys.argv[1]) if len(sys.argv) > 1 else 250000
pool = W.build_pool(R=4, k=1, P=256, P_f=64)
s = W.make_batch(pool, n_certs)
t0 = time.time()
wb = W.encode_wire_batch(s)
print(f"encoded {wb.n_msgs} msgs, {wb.wire.nbytes / 1e6:.0f} MB in {time.time() - t0:.1f}s", flush=True)
ver = mh.Verifier(pool.moduli, 0)
ver.set_server_ids(W.SERVER_IDS[:4])
dwb = mh.DeviceWireBatch(wb, 0)
out = mh.DeviceVerdicts(0, wb.n_msgs, 0, full=True)
out.grant_flags = out.grant_ts = None
st = torch.cuda.current_stream()
for _ in range(3):
    ver.verify_write2_device(dwb, out, 4, True, stream=st.cuda_stream)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(st)
for _ in range(3):
    ver.verify_write2_device(dwb, out, 4, True, stream=st.cuda_stream)
e1.record(st)
torch.cuda.synchronize()
print(f"wire path {e0.elapsed_time(e1) / 3:.3f} ms/step, {s.batch.n_grants / (e0.elapsed_time(e1) / 3e3) / 1e6:.1f} M grants/s")
