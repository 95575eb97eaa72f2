"""H2D / D2H bandwidth from pinned host memory with 1, 2 and 4 streams (diagnostic)."""
import torch, time
dev = torch.device("cuda")
n = 4000 << 20
h = torch.empty(n, dtype=torch.uint8).pin_memory()
d = torch.empty(n, dtype=torch.uint8, device=dev)
o = torch.empty(n, dtype=torch.uint8).pin_memory()
d2 = torch.empty(n, dtype=torch.uint8, device=dev)
for ns in (1, 2, 4):
    ss = [torch.cuda.Stream(dev) for _ in range(ns)]
    for rep in range(3):
        torch.cuda.synchronize(); t = time.perf_counter()
        part = n // ns
        for k, s in enumerate(ss):
            with torch.cuda.stream(s):
                d[k * part:(k + 1) * part].copy_(h[k * part:(k + 1) * part], non_blocking=True)
        torch.cuda.synchronize(); dt = time.perf_counter() - t
    print(f"H2D {ns} streams: {n / dt / 1e9:.1f} GB/s", flush=True)
# H2D and D2H at once
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
for rep in range(3):
    torch.cuda.synchronize(); t = time.perf_counter()
    with torch.cuda.stream(s1): d.copy_(h, non_blocking=True)
    with torch.cuda.stream(s2): o.copy_(d2, non_blocking=True)
    torch.cuda.synchronize(); dt = time.perf_counter() - t
print(f"H2D + D2H concurrently: {2 * n / dt / 1e9:.1f} GB/s total", flush=True)
