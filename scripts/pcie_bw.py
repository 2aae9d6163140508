"""H2D / D2H copy bandwidth of pinned host memory on this box (the ceiling the
host wire path is measured against).  Prints one JSON line."""
import json
import time

import torch

n = 1 << 30
h = torch.empty(n, dtype=torch.uint8).pin_memory()
d = torch.empty(n, dtype=torch.uint8, device="cuda")
res = {}
for name, fn in (("h2d", lambda: d.copy_(h, non_blocking=True)), ("d2h", lambda: h.copy_(d, non_blocking=True))):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    res[name + "_GB_per_s"] = round(5 * n / (time.perf_counter() - t) / 1e9, 2)
print(json.dumps(res))
