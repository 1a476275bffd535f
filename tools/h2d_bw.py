import torch, time
n = 32 << 20
h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
h.fill_(7)
d = torch.empty(n, dtype=torch.uint8, device="cuda")
for _ in range(5): d.copy_(h, non_blocking=True)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(50): d.copy_(h, non_blocking=True)
torch.cuda.synchronize()
el = (time.perf_counter() - t) / 50
print(f"H2D pinned 32MB: {el*1e3:.3f} ms  {n/el/1e9:.1f} GB/s")
s2 = torch.cuda.Stream()
h2 = torch.empty(n, dtype=torch.uint8, pin_memory=True); d2 = torch.empty_like(d)
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(25):
    d.copy_(h, non_blocking=True)
    with torch.cuda.stream(s2): d2.copy_(h2, non_blocking=True)
torch.cuda.synchronize(); el = (time.perf_counter() - t) / 50
print(f"two streams: {el*1e3:.3f} ms per 32MB {n/el/1e9:.1f} GB/s")
hp = torch.empty(n, dtype=torch.uint8); hp.fill_(3)
t = time.perf_counter()
for _ in range(10): d.copy_(hp)
torch.cuda.synchronize(); el = (time.perf_counter() - t) / 10
print(f"H2D pageable 32MB: {el*1e3:.3f} ms  {n/el/1e9:.1f} GB/s")

# does an H2D copy overlap a long kernel on another stream?
a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
def mm(k=20):
    for _ in range(k): torch.mm(a, a)
mm(3); torch.cuda.synchronize()
t = time.perf_counter(); mm(); torch.cuda.synchronize(); t_mm = time.perf_counter() - t
t = time.perf_counter()
for _ in range(20): d.copy_(h, non_blocking=True)
torch.cuda.synchronize(); t_cp = time.perf_counter() - t
s3 = torch.cuda.Stream()
torch.cuda.synchronize(); t = time.perf_counter()
with torch.cuda.stream(s3):
    for _ in range(20): d.copy_(h, non_blocking=True)
mm(); torch.cuda.synchronize(); t_both = time.perf_counter() - t
print(f"matmuls {t_mm*1e3:.2f} ms, 20 copies {t_cp*1e3:.2f} ms, both on two streams {t_both*1e3:.2f} ms")
