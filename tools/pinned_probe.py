"""CPU read/write speed of torch pinned host memory vs ordinary memory (ingest design)."""
import time
import numpy as np
import torch

n = 256 << 20
a = torch.empty(n, dtype=torch.uint8).pin_memory()
b = np.empty(n, np.uint8)
src = np.random.default_rng(0).integers(0, 256, n, dtype=np.uint8)
for name, arr in (("pinned", a.numpy()), ("pageable", b)):
    t0 = time.perf_counter(); arr[:] = src; tw = time.perf_counter() - t0
    t0 = time.perf_counter(); c = arr.tobytes(); tr = time.perf_counter() - t0
    print("%-9s write %.2f GB/s  read %.2f GB/s" % (name, n / tw / 1e9, n / tr / 1e9))
d = torch.empty(n, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
for name, h in (("pinned", a), ("pageable", torch.from_numpy(b))):
    t0 = time.perf_counter(); d.copy_(h); torch.cuda.synchronize(); t1 = time.perf_counter()
    h.copy_(d); torch.cuda.synchronize(); t2 = time.perf_counter()
    print("%-9s H2D %.2f GB/s  D2H %.2f GB/s" % (name, n / (t1 - t0) / 1e9, n / (t2 - t1) / 1e9))
