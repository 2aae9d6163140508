"""Phase times of k_rsa_pow from a MOCHI_POW_STAMPS build (MOCHI_HIP_LIB points
at it): per wave, s_memtime cycles per squaring in x^2 and in the fold (each
between its phase barriers), and the kernel's cycles per squaring overall
(stamp column 4 is unused since grant prep left the kernel); split by the leading
(waves 0-3) and lagging (waves 4-7) halves.  One JSON line."""
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
waves_rec = int(os.environ.get("WAVES", "2048"))  # stamp rows read back (8 per block, <= 4096)
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
lib = ctypes.CDLL(os.environ["MOCHI_HIP_LIB"])
buf = (ctypes.c_ulonglong * (4096 * 5))()
assert lib.mochi_debug_pow_stamps(buf, waves_rec) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 5)[:waves_rec].astype(np.float64)
wave = np.arange(a.shape[0]) % 8
keep = a[:, 3] > 0
res = {"lib": os.path.basename(os.environ["MOCHI_HIP_LIB"]), "grants": synth.batch.n_grants, "flags_ok": ok}
for name, sel in (("all", keep), ("lead", keep & (wave < 4)), ("lag", keep & (wave >= 4))):
    b = a[sel]
    n = b[:, 3]
    res[name] = {"waves": int(b.shape[0]), "squarings_per_wave": float(n.mean()),
                 "x2_cyc_per_sq": round(float((b[:, 0] / n).mean()), 1),
                 "fold_cyc_per_sq": round(float((b[:, 1] / n).mean()), 1),
                 "kernel_cyc_per_sq": round(float((b[:, 2] / n).mean()), 1),
                 "kernel_cyc_p0_p100": [round(float(np.percentile(b[:, 2], q)), 1) for q in (0, 50, 100)],
                 "groups_min_max": [int(n.min() / 16), int(n.max() / 16)],
                 "x2_p10_p90": [round(float(np.percentile(b[:, 0] / n, q)), 1) for q in (10, 90)],
                 "fold_p10_p90": [round(float(np.percentile(b[:, 1] / n, q)), 1) for q in (10, 90)]}
print(json.dumps(res))
