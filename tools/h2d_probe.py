"""Host<->device copy rates the host-buffer API sees (pageable numpy vs pinned)."""
import time
import numpy as np
import torch

n = 4032 * 3008 * 3 // 2
a = np.random.randint(0, 255, n, dtype=np.uint8)
d = torch.empty(n, dtype=torch.uint8, device="cuda")
p = torch.empty(n, dtype=torch.uint8).pin_memory()
def t(f, k=10):
    f(); torch.cuda.synchronize()
    ts = []
    for _ in range(k):
        t0 = time.perf_counter(); f(); torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
    return sorted(ts)[k // 2]
ta = torch.from_numpy(a)
print("H2D pageable %.2f GB/s" % (n / t(lambda: d.copy_(ta)) / 1e9))
print("H2D pinned   %.2f GB/s" % (n / t(lambda: d.copy_(p, non_blocking=True)) / 1e9))
print("D2H pageable %.2f GB/s" % (n / t(lambda: ta.copy_(d)) / 1e9))
print("D2H pinned   %.2f GB/s" % (n / t(lambda: p.copy_(d, non_blocking=True)) / 1e9))
print("host memcpy  %.2f GB/s" % (n / t(lambda: p.numpy().__setitem__(slice(None), a)) / 1e9))
