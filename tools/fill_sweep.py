import torch
torch.cuda.set_device(0)
for mb in (95.2, 760, 2400, 6000, 12000, 24400):
    x = torch.empty(int(mb * 1e6 / 4), device="cuda")
    x.fill_(0.0)
    reps = max(3, int(3000 / mb))
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for r in range(reps):
        x.fill_(float(r & 1))
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    print(f"fill {mb:.1f} MB: {x.numel() * 4 / ms / 1e6:.0f} GB/s", flush=True)
    del x
    torch.cuda.empty_cache()
