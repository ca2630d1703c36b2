"""Tuned GEMM solutions for SCRIMPNet's shapes (PyTorch TunableOp results, shipped with the package).

torch's hipBLASLt heuristic picks slow solutions for the network's tall GEMMs -- e.g. the acting
forward's QKV projection (557,056 x 512 -> 1,536) in 1.22 ms where the best solution hipBLASLt has
takes 0.86 ms, the KV projection 0.74 -> 0.51 ms (tools/bench_gemm_backends.py,
profiles/r05_gemm_backends.jsonl).  tools/tune_gemms.sh benchmarks every candidate solution for every
GEMM shape the c3 rollout and the c3 / c4 PPO updates run (TunableOp tuning on), and the resulting
CSV ships as tunableop_gfx950.csv.  use_tuned_gemms() loads it with tuning OFF: shapes in the file use
their measured-best solution, any other shape torch's default -- no benchmarking at run time, so a
captured hipGraph never sees a tuning step.  The file's validators (PyTorch, HIP, hipBLASLt versions,
gfx950) must match the running stack; if they do not, read_file fails and TunableOp is switched off
again (torch's defaults).  A process that configures TunableOp itself (PYTORCH_TUNABLEOP_ENABLED in
the environment) is left alone."""
import os

TUNED = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tunableop_gfx950.csv")
_state = {"done": False, "active": False}


def use_tuned_gemms():
    """Load the shipped TunableOp results (idempotent).  Returns whether they are in use."""
    if _state["done"]:
        return _state["active"]
    _state["done"] = True
    if "PYTORCH_TUNABLEOP_ENABLED" in os.environ or not os.path.exists(TUNED):
        return False
    import torch
    if not torch.cuda.is_available():
        return False
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(False)
    ok = False
    try:
        ok = bool(tun.read_file(TUNED))
    except RuntimeError:
        ok = False
    if not ok:
        tun.enable(False)
    _state["active"] = ok
    return ok
