"""H2D copy rate of a C2-sized packed batch (~1.9 MB) from pinned host memory: one copy on one
stream against the same bytes split over 2 / 4 streams (copy engines), and larger sizes."""
import time

import torch

def rate(nbytes, parts, reps=200):
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(parts)]
    chunk = (nbytes + parts - 1) // parts
    def once():
        for i, s in enumerate(streams):
            with torch.cuda.stream(s):
                d[i * chunk:(i + 1) * chunk].copy_(h[i * chunk:(i + 1) * chunk], non_blocking=True)
    for _ in range(10):
        once()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        once()
        for s in streams:
            s.synchronize()
    el = (time.perf_counter() - t) / reps
    return el * 1e6, nbytes / el / 1e9

for nb in (1_900_000, 8_000_000, 64_000_000):
    for parts in (1, 2, 4):
        us, gbs = rate(nb, parts)
        print(f"{nb/1e6:6.1f} MB parts {parts}: {us:8.1f} us/copy  {gbs:6.1f} GB/s", flush=True)
