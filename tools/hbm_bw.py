import torch, time
for mb in (64, 256, 1024):
    n = mb * 2**20
    x = torch.empty(n, dtype=torch.uint8, device='cuda'); y = torch.empty_like(x)
    for _ in range(3): y.copy_(x)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): y.copy_(x)
    e1.record(); torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 20 * 1e-3
    print(f"copy {mb} MB: {2*n/t/1e12:.2f} TB/s (read+write) {t*1e6:.1f} us")
    xf = x.view(torch.float32)
    for _ in range(3): s = xf.sum()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(20): s = xf.sum()
    e1.record(); torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 20 * 1e-3
    print(f"sum {mb} MB: {n/t/1e12:.2f} TB/s read {t*1e6:.1f} us")
    for _ in range(3): y.fill_(1)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(20): y.fill_(1)
    e1.record(); torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 20 * 1e-3
    print(f"fill {mb} MB: {n/t/1e12:.2f} TB/s write {t*1e6:.1f} us")
