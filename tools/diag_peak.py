"""Peak device memory of Model.train (256 x 8 rows, graphed: 2 eager warm-ups + capture + replays)
with round 5's training-path features toggled one at a time (tests/test_gpu_rollout.py bounds the
driver block's peak at 2 GiB)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "primal-ppo_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402


def run(feat):
    from mapf_amd import net as N
    from mapf_amd.model import Model
    from test_gpu_update_graph import _batch
    N.SCRIMPNet.cast_params = "cast" in feat
    N._PreNorm.hip_layernorm = "ln" in feat
    N._SplitKLinear.SPLIT = 4 if "split" in feat else 10 ** 9
    torch.manual_seed(0)
    m = Model(0, "cuda", global_model=True, numChannel=6, num_agents=8, fov=9)
    g = torch.Generator(device="cuda").manual_seed(1)
    b = _batch(g, rows=256)
    torch.cuda.synchronize()
    before = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    for _ in range(5):
        m.train(*b[:8], None, b[8], 1.0)
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated() - before
    print(json.dumps({"features": feat, "peak_mb": round(peak / 2 ** 20, 1),
                      "tuned": torch.cuda.tunable.is_enabled()}), flush=True)


if __name__ == "__main__":
    run(sys.argv[1] if len(sys.argv) > 1 else "")
