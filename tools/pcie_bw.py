"""Raw host<->device copy bandwidth on this box (torch, pinned and pageable), for DESIGN.md."""
import time

import torch

n = 512 << 20
d = torch.empty(n, dtype=torch.uint8, device="cuda")
for pinned in (True, False):
    h = torch.empty(n, dtype=torch.uint8, pin_memory=pinned)
    h.fill_(1)
    for name, fn in (("h2d", lambda: d.copy_(h, non_blocking=True)), ("d2h", lambda: h.copy_(d, non_blocking=True))):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 5
        print(f"pinned={pinned} {name}: {n / dt / 1e9:.1f} GB/s", flush=True)
