"""The captured-update replay hazard, forensics: the captured backward's bias gradients go non-finite
after small-pool churn once the eager warm-ups' tensors are freed (diag_graph14).  So the graph reads
(or writes) a block a warm-up tensor held.  Record the allocator history through warm-ups, capture
and one churn; then list the warm-up-phase allocations (freed before the capture began) whose blocks
the churn re-used, with their Python stacks -- the stale-pointer candidates."""
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, "tools")
sys.path.insert(0, "primal-ppo_amd")
import diag_graph14 as D  # noqa: E402
from test_gpu_update_graph import _batch  # noqa: E402
from mapf_amd.model import Model, _DeviceUpdate  # noqa: E402
from mapf_amd.config import TrainingParameters as T  # noqa: E402


def mark():
    return len(torch.cuda.memory._snapshot()["device_traces"][0])


def main():
    g = torch.Generator(device="cuda").manual_seed(1)
    batches = [_batch(g) for _ in range(5)]
    torch.manual_seed(0)
    torch.cuda.memory._record_memory_history(max_entries=1000000)
    m = Model(0, "cuda", global_model=True, numChannel=6, num_agents=8, fov=9)
    m.network.eval()
    m.net_scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 8)
    m.net_scaler._lazy_init_scale_growth_tracker(m.device)
    obs, vec, ret, cret, v, cv, act, ps, tv = batches[0]
    u = _DeviceUpdate(m, obs, vec, ret, ps, tv, act.unsqueeze(-1))
    coef = (T.CLIP_RANGE, T.ENTROPY_COEF, T.VALUE_COEF, T.VALID_COEF, T.COST_VALUE_COEF, T.COST_COEF)
    out = {}
    m_warm0 = mark()
    for k in range(2):
        u.load(*batches[k][:6], batches[k][6].unsqueeze(-1), batches[k][7], batches[k][8], coef=coef, lam=0.0)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            D.body(m, u, "bwd", out)
        torch.cuda.current_stream().wait_stream(s)
        out.clear()
    torch.cuda.synchronize()
    m_cap0 = mark()
    graph = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            D.body(m, u, "bwd", out)
    torch.cuda.current_stream().wait_stream(s)
    m_cap1 = mark()
    graph.replay()
    torch.cuda.synchronize()
    print("first replay non-finite grads:", D.bad(out["bwd"]), flush=True)
    m_churn0 = mark()
    D.churn()
    m_churn1 = mark()
    graph.replay()
    torch.cuda.synchronize()
    bad = [n for n, t in zip(out["bwd_names"], out["bwd"]) if not torch.isfinite(t.float()).all()]
    print("after churn non-finite grads:", bad, flush=True)
    snap = torch.cuda.memory._snapshot()
    torch.cuda.memory._record_memory_history(enabled=None)
    tr = snap["device_traces"][0]
    # warm-up-phase allocations freed before the capture began
    warm = {}
    for i in range(m_warm0, m_cap0):
        ev = tr[i]
        if ev["action"] == "alloc":
            warm[ev["addr"]] = ev
        elif ev["action"] in ("free_requested", "free_completed"):
            pass
    freed_before_cap = {}
    live = {}
    for i in range(0, m_cap0):
        ev = tr[i]
        if ev["action"] == "alloc":
            live[ev["addr"]] = (i, ev)
        elif ev["action"] == "free_requested" and ev["addr"] in live:
            j, a = live.pop(ev["addr"])
            if j >= m_warm0:
                freed_before_cap[ev["addr"]] = a
    churned = [tr[i] for i in range(m_churn0, m_churn1) if tr[i]["action"] == "alloc"]
    # allocations during capture that were NOT in the private pool
    cap_allocs = [tr[i] for i in range(m_cap0, m_cap1) if tr[i]["action"] == "alloc"]
    print(f"warm-up allocations freed before capture: {len(freed_before_cap)}; churn allocations: {len(churned)}; "
          f"allocations during capture: {len(cap_allocs)} (streams {sorted(set(e['stream'] for e in cap_allocs))})",
          flush=True)
    hits = []
    for c in churned:
        c0, c1 = c["addr"], c["addr"] + c["size"]
        for a0, a in freed_before_cap.items():
            if a0 < c1 and c0 < a0 + a["size"]:
                hits.append(a)
    seen = set()
    print(f"{len(hits)} warm-up blocks re-used by the churn; their allocations:")
    for a in hits:
        key = (a["size"], tuple((f["filename"], f["line"]) for f in a.get("frames", []) if f["filename"].endswith(".py")))
        if key in seen:
            continue
        seen.add(key)
        frames = [f"{f['filename'].split('/')[-1]}:{f['line']}:{f['name']}" for f in a.get("frames", [])
                  if f["filename"].endswith(".py")][:7]
        print(f"  size {a['size']} stream {a['stream']}: {frames}", flush=True)


if __name__ == "__main__":
    main()
