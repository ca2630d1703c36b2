"""Write-bandwidth ceilings on this GPU: torch fill_ of an observation-sized buffer
(95 MB, re-written in place: MALL-resident) and of a rollout-sized one (2.4 GB,
fresh HBM lines), HIP-event timed."""
import torch

torch.cuda.set_device(0)
for mb, reps in ((95.2, 300), (2380.0, 20)):
    x = torch.empty(int(mb * 1e6 / 4), device="cuda")
    x.fill_(0.0)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for r in range(reps):
        x.fill_(float(r & 1))
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    print(f"fill {mb:.1f} MB: {ms * 1e3:.1f} us  {x.numel() * 4 / ms / 1e9:.0f} GB/s", flush=True)
    del x
