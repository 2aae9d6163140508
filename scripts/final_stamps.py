"""Phase times of k_rsa_final from a MOCHI_FINAL_STAMPS build (MOCHI_HIP_LIB
points at it): per wave, s_memtime cycles per 64-grant item in the operand
loads (meaningful with MOCHI_FINAL_STAMPS=2, which waits for them explicitly),
the z*s product, the digest load + fold, and the final Montgomery step + flag
store, and the kernel's cycles per item overall.  One JSON line."""
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
certs = int(os.environ.get("CERTS", "1000000"))
waves_rec = int(os.environ.get("WAVES", "1024"))  # stamp rows read back (4 per block, <= 4096)
synth = W.make_batch_unique(R, certs, 1, first_cert=0, device=0)
moduli = [mh.pem_modulus(p) for p in W.load_keys(R)]
ver = mh.Verifier(moduli, device=0)
dev = mh.DeviceBatch(synth.batch, 0)
out = mh.DeviceVerdicts(dev.n_grants, dev.n_certs, 0, full=True, n_ops=dev.n_ops)
import torch  # noqa: E402

for _ in range(3):
    ver.verify_device(dev, out, R, True)
torch.cuda.synchronize()
ok = bool(np.array_equal(out.to_host().grant_flags, synth.expected_flags))
ver.set_profiling(True)
for _ in range(3):
    ver.verify_device(dev, out, R, True)
torch.cuda.synchronize()
ver.set_profiling(False)
prof = ver.read_profile()
lib = ctypes.CDLL(os.environ["MOCHI_HIP_LIB"])
buf = (ctypes.c_ulonglong * (4096 * 6))()
assert lib.mochi_debug_final_stamps(buf, waves_rec) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 6)[:waves_rec].astype(np.float64)
keep = a[:, 4] > 0
b = a[keep]
n = b[:, 4]
res = {"lib": os.path.basename(os.environ["MOCHI_HIP_LIB"]), "grants": synth.batch.n_grants, "flags_ok": ok,
       "final_ms": round(prof["rsa_final"], 4), "waves": int(b.shape[0]), "items_per_wave": float(n.mean())}
for i, name in enumerate(("load", "product", "fold", "check")):
    res[f"{name}_cyc_per_item"] = round(float((b[:, i] / n).mean()), 1)
res["kernel_cyc_per_item"] = round(float((b[:, 5] / n).mean()), 1)
res["sum_phases"] = round(sum(res[f"{k}_cyc_per_item"] for k in ("load", "product", "fold", "check")), 1)
print(json.dumps(res))
