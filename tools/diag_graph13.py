"""The captured-update replay hazard (diag_graph12: even with no twin, m1's replays go NaN once small
tensors are allocated and freed between them; diag_graph6: big NaN-filled blocks do not).
  churn_small   between m1's updates allocate ~2,000 small tensors (4 B .. 512 KiB: the caching
                allocator's small pool), fill them with NaN, free them
  churn_large   the same with 2 MiB .. 64 MiB blocks
  none          nothing
Then the forensic pass: capture m1 with the graph's debug mode on, dump the hipGraph (DOT), and
list every kernel-argument word that points into device memory NOT owned by the graph's private
pool or by any tensor alive after the capture -- with the allocator history's Python stack of the
allocation that last held that address."""
import os
import re
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, "primal-ppo_amd")
from test_gpu_update_graph import _batch  # noqa: E402
from mapf_amd.model import Model  # noqa: E402

torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False


def fresh(graph=True):
    torch.manual_seed(0)
    m = Model(0, "cuda", global_model=True, numChannel=6, num_agents=8, fov=9)
    m.graph_update = graph
    m.network.eval()
    m.net_scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 8)
    return m


def train(m, b):
    obs, vec, ret, cret, v, cv, act, ps, tv = b
    return m.train(obs, vec, ret, cret, v, cv, act, ps, None, tv, 1.0)


def finite(s):
    return all(torch.isfinite(torch.tensor(float(x))) for x in s[:9])


def churn(sizes):
    ts = [torch.full((n,), float("nan"), device="cuda") for n in sizes]
    torch.cuda.synchronize()
    del ts


SMALL = [1 << (k % 17) for k in range(2000)]            # 4 B .. 512 KiB of float32
LARGE = [(1 << 19) << (k % 5) for k in range(40)]        # 2 MiB .. 32 MiB


def run_churn(kind):
    g = torch.Generator(device="cuda").manual_seed(1)
    batches = [_batch(g) for _ in range(12)]
    m = fresh()
    res = []
    for k, b in enumerate(batches):
        if k >= 3 and kind != "none":
            churn(SMALL if kind == "churn_small" else LARGE)
        res.append(finite(train(m, b)))
    print(f"{kind:12s} replay finite per update {res}", flush=True)


def forensic():
    g = torch.Generator(device="cuda").manual_seed(1)
    batches = [_batch(g) for _ in range(4)]
    m = fresh()
    torch.cuda.memory._record_memory_history(max_entries=400000)
    orig = torch.cuda.CUDAGraph

    class Dbg(orig):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            self.enable_debug_mode()
    torch.cuda.CUDAGraph = Dbg
    try:
        for b in batches[:3]:
            train(m, b)
    finally:
        torch.cuda.CUDAGraph = orig
    torch.cuda.synchronize()
    upd = next(iter(m._updates.values()))
    path = os.path.abspath("gpurun_out/r5f_graph.dot")
    upd.graph.debug_dump(path)
    snap = torch.cuda.memory._snapshot()
    torch.cuda.memory._record_memory_history(enabled=None)
    segs = [(s["address"], s["address"] + s["total_size"], tuple(s.get("segment_pool_id", (0, 0)))) for s in snap["segments"]]
    live = []
    for s in snap["segments"]:
        for blk in s["blocks"]:
            if blk["state"] == "active_allocated":
                live.append((blk["address"] if "address" in blk else 0, blk["size"]))
    # blocks: compute addresses from segment layout
    live = []
    for s in snap["segments"]:
        a = s["address"]
        for blk in s["blocks"]:
            if blk["state"] == "active_allocated":
                live.append((a, a + blk["size"], tuple(s.get("segment_pool_id", (0, 0)))))
            a += blk["size"]
    text = open(path).read()
    words = set(int(x, 16) for x in re.findall(r"0x([0-9a-fA-F]{8,16})", text))
    words |= set(int(x) for x in re.findall(r"\b(1[0-9]{13,15})\b", text))
    dev_words = [w for w in words if any(a <= w < e for a, e, _ in segs)]
    dangling = []
    for w in sorted(dev_words):
        owner = [(a, e, p) for a, e, p in live if a <= w < e]
        if not owner:
            dangling.append(w)
        elif all(p == (0, 0) for *_, p in owner):
            pass
    print(f"graph DOT: {len(text)} bytes, {len(words)} numeric words, {len(dev_words)} inside allocator segments, "
          f"{len(dangling)} pointing at memory no live block holds", flush=True)
    trace = snap["device_traces"][0]
    for w in dangling[:20]:
        last = None
        for ev in trace:
            if ev["action"] == "alloc" and ev["addr"] <= w < ev["addr"] + ev["size"]:
                last = ev
        frames = [f"{f['filename'].split('/')[-1]}:{f['line']}:{f['name']}" for f in (last or {}).get("frames", [])
                  if f["filename"].endswith(".py")][:8] if last else []
        print(f"  0x{w:x}: last allocation there size {last['size'] if last else None} {frames}", flush=True)


if __name__ == "__main__":
    import warnings
    from mapf_amd.model import _DeviceUpdate
    for same in (False, True):
        _DeviceUpdate.SAME_STREAM = same
        print(f"warm-ups and capture on {'one side stream' if same else 'a new stream each'}:", flush=True)
        with warnings.catch_warnings(record=True) as wl:
            warnings.simplefilter("always")
            run_churn("churn_small")
        acc = [str(w.message)[:160] for w in wl if "AccumulateGrad" in str(w.message)]
        print(f"   AccumulateGrad stream warnings: {len(acc)} {acc[:1]}", flush=True)
