"""Phase times of k_w2_mg from a MOCHI_W2_STAMPS build (MOCHI_HIP_LIB points at
it): s_memtime ticks per wave in each phase of the level-2 walk, summed over the
grid-stride loop.  One JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mochi-db_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mochi_hip as mh  # noqa: E402
import workload as W  # noqa: E402

pool = W.build_pool(R=4, k=1, P=256, P_f=64)
s = W.make_batch(pool, int(os.environ.get("CERTS", "250000")))
wb = W.encode_wire_batch(s)
ver = mh.Verifier(pool.moduli, 0)
ver.set_server_ids(W.SERVER_IDS[:4])
dwb = mh.DeviceWireBatch(wb, 0)
out = mh.DeviceVerdicts(0, wb.n_msgs, 0, full=True)
out.grant_flags = out.grant_ts = None
st = torch.cuda.current_stream()
for _ in range(2):
    ver.verify_write2_device(dwb, out, 4, True, stream=st.cuda_stream)
torch.cuda.synchronize()
lib = ctypes.CDLL(os.environ["MOCHI_HIP_LIB"])
buf = (ctypes.c_ulonglong * (16384 * 8))()
assert lib.mochi_debug_w2_stamps(buf, 16384) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(16384, 8).astype(np.float64)
a = a[a[:, 7] > 0]
names = ["dedup", "scan", "canonical", "signer", "key_slot", "records"]
tot = a[:, 1:7].sum(axis=1).mean()
print(json.dumps({"waves": int(a.shape[0]), "ticks_per_wave": round(float(tot)),
                  "share": {n: round(float(a[:, i + 1].mean() / tot), 3) for i, n in enumerate(names)}}))
