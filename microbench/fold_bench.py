"""GPU check + timing of the MFMA fold squaring prototype (fold_pow.hip).

python microbench/fold_bench.py [N] : N signatures, 16 squarings each; checks a
sample against Python pow and prints ms per launch and ns per signature."""
import ctypes
import os
import random
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import fold_model as FR  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    lib = ctypes.CDLL(os.path.join(HERE, os.environ.get("FOLD_LIB", "libfold_pow.so")))
    lib.fold_pow.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
    rnd = random.Random(7)
    n = rnd.getrandbits(2048) | (1 << 2047) | 1
    t0 = time.time()
    img, cadd, _ = FR.make_weights(n)
    print(f"weights {time.time() - t0:.1f}s", flush=True)
    # inputs: random s < n, 64-bit chunks via numpy for speed
    rng = np.random.default_rng(1)
    limbs = rng.integers(0, 1 << 28, size=(FR.L, N), dtype=np.uint32)
    limbs[73:, :] = 0  # < 2^2044 < n
    limbs[72, :] &= (1 << 27) - 1
    dev = torch.device("cuda", 0)
    x = torch.from_numpy(limbs.view(np.int32)).to(dev)
    w = torch.from_numpy(img.reshape(-1).view(np.uint8)).to(dev)
    c = torch.from_numpy(cadd.view(np.int32)).to(dev)
    z = torch.empty_like(x)
    st = torch.cuda.current_stream(dev).cuda_stream
    rc = lib.fold_pow(x.data_ptr(), w.data_ptr(), c.data_ptr(), z.data_ptr(), N, 16, st)
    assert rc == 0
    torch.cuda.synchronize()
    zh = z.cpu().numpy().view(np.uint32)
    bad = 0
    for i in list(range(0, N, max(1, N // 500))) + [N - 1]:
        s = FR.from_limbs(limbs[:, i])
        zi = FR.from_limbs(zh[:, i])
        if zi >= 1 << 2064 or zi % n != pow(s, 1 << 16, n):
            bad += 1
    print(f"checked sample: bad={bad}", flush=True)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    times = []
    for _ in range(5):
        ev[0].record()
        lib.fold_pow(x.data_ptr(), w.data_ptr(), c.data_ptr(), z.data_ptr(), N, 16, st)
        ev[1].record()
        torch.cuda.synchronize()
        times.append(ev[0].elapsed_time(ev[1]))
    ms = sorted(times)[2]
    if os.environ.get("FOLD_STAMPS"):
        lib.fold_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
        torch.cuda.synchronize()
        lib.fold_stamps(None, 1)
        ev[0].record()
        lib.fold_pow(x.data_ptr(), w.data_ptr(), c.data_ptr(), z.data_ptr(), N, 16, st)
        ev[1].record()
        torch.cuda.synchronize()
        kms = ev[0].elapsed_time(ev[1])
        out = np.zeros(6, np.uint64)
        lib.fold_stamps(out.ctypes.data, 0)
        waves = int(out[3])
        per = [int(v) / waves / 16 for v in out[:3]]
        life = int(out[4]) / waves
        # 2 waves per SIMD, 1,024 SIMDs: sum of wave lifetimes / 2,048 ~ kernel ticks
        rate = int(out[4]) / 2048 / (kms / 1e3) / 1e9
        print(f"stamps per wave-squaring (s_memtime ticks): sqr {per[0]:.0f}  bops {per[1]:.0f}  fold {per[2]:.0f}  "
              f"waves={waves}  wave lifetime {life:.0f} (loop {16 * sum(per):.0f})  kernel {kms:.3f} ms -> "
              f"{rate:.3f} G ticks/s if SIMDs always hold 2 waves")
    print(f"N={N} 16 squarings: {ms:.3f} ms/launch  {ms * 1e6 / N:.3f} ns/sig  "
          f"(k_rsa_pow r02: 4.19 ns/sig)  times={['%.3f' % t for t in times]}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
