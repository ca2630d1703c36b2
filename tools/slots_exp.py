"""Experiment: the c2 rollout into [S]-slot buffers vs in place.  S slots are written by
launches of T = S steps (launch length barely matters: DESIGN.md §6); 'obs only' passes no
step-output buffers (the partial-line small outputs are then not written at all)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "primal-ppo_amd")]

import torch  # noqa: E402

from mapf_amd.config import make_config  # noqa: E402
from mapf_amd.env import BatchedMapfGym  # noqa: E402
from mapf_amd.maps import generate_warehouse  # noqa: E402

B, N, H, F, C = 4096, 8, 20, 11, 6
K = int(os.environ.get("K", "1024"))
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
env = BatchedMapfGym(make_config(B, H, H, num_agents=N, fov=F, num_channel=C, human_mode="random",
                                 goal_mode="random", fix_choice=1, seed=1234), device=dev)
env.reset_seeded(generate_warehouse(H, H))


def timed(fn, steps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 0
    a.record()
    while n < K:
        fn()
        n += steps
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


us = timed(lambda: env.rollout_random(256), 256)
print(f"in place T=256: {us:.2f} us/step", flush=True)
for S in [int(x) for x in os.environ.get("SLOTS", "2,8,32,256").split(",")]:
    for outs in (True, False):
        bufs = dict(actions=torch.zeros(S, B, N, dtype=torch.int32, device=dev),
                    obs=torch.zeros(S, B, N, C, F, F, device=dev), vec=torch.zeros(S, B, N, 4, device=dev),
                    out={k: torch.zeros((S,) + tuple(v.shape), dtype=v.dtype, device=dev)
                         for k, v in env.out.items()} if outs else {})
        us = timed(lambda: env.rollout_random(S, slots=True, **bufs), S)
        print(f"slots S={S} ({S * 95.2 / 1e3:.2f} GB obs) {'all outputs' if outs else 'obs only'}: {us:.2f} us/step",
              flush=True)
        del bufs
        torch.cuda.empty_cache()
for mb, reps in ((95.2, 300), (24400.0, 4)):
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
    print(f"fill {mb:.1f} MB: {x.numel() * 4 / ms / 1e9:.0f} GB/s -> 95.2 MB in {95.2e6 / (x.numel() * 4 / ms) / 1e3 * 1e3:.2f} us", flush=True)
    del x
