"""Graph capture vs the per-step API's deferred searches (mapf_api.cpp: join_deferred).

Wide maps (N > 8, the split path) defer the humans' next-path search onto a second stream and
join it two steps later.  A search deferred BEFORE a stream capture began cannot be joined
inside the capture (the graph would depend on work outside itself): the call fails loudly
with MAPF_ESTATE instead, and after mapf_flush on an uncaptured stream the same capture
works.  (Runs last: it exercises a failing capture.)"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_capture_after_deferred_search_needs_flush():
    from mapf_amd.config import make_config
    from mapf_amd.env import BatchedMapfGym
    from mapf_amd.maps import generate_warehouse
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    env = BatchedMapfGym(make_config(8, 40, 40, num_agents=16, fov=9, num_channel=6, human_mode="random",
                                     goal_mode="random", fix_choice=1, seed=3))
    env.reset_seeded(generate_warehouse(40, 40))
    assert not env.fused
    for _ in range(4):                       # leaves a deferred search pending on the aux stream
        env.step_observe(random_policy=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with pytest.raises(RuntimeError, match="mapf_flush"):
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                env.step_observe(random_policy=True)
    torch.cuda.synchronize()
    env.flush()                              # joins the deferred search on the current stream
    torch.cuda.synchronize()
    st = env.get_state()
    assert (st["pos"] >= 0).all()
