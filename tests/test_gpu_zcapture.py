"""Graph capture vs the per-step API's deferred searches (mapf_api.cpp: join_deferred), and
captured persistent rollouts vs the argument ring (mapf_kernels.h: ArgRing).

Wide maps (N > 8, the split path) defer the humans' next-path search onto a second stream and
join it two steps later.  A search deferred BEFORE a stream capture began cannot be joined
inside the capture (the graph would depend on work outside itself): the call fails loudly
with MAPF_ESTATE instead, and after mapf_flush on an uncaptured stream the same capture
works.  (Runs last: it exercises a failing capture.)"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def c4_env(B=8, seed=3):
    from mapf_amd.config import make_config
    from mapf_amd.env import BatchedMapfGym
    from mapf_amd.maps import generate_warehouse
    env = BatchedMapfGym(make_config(B, 40, 40, num_agents=16, fov=9, num_channel=6, human_mode="random",
                                     goal_mode="random", fix_choice=1, seed=seed))
    env.reset_seeded(generate_warehouse(40, 40))
    return env


def assert_same_env(a, b, what):
    sa, sb = a.get_state(), b.get_state()
    for k in sb:
        np.testing.assert_array_equal(sa[k], sb[k], err_msg=f"{what}: state {k}")
    assert torch.equal(a.bfs(), b.bfs()), what


def test_captured_rollouts_between_direct_rollouts():
    """A captured mapf_rollout_random of the three-wave c4 form (arguments through a device
    block) keeps its own argument slot: replayed between direct launches that cycle the
    16-slot ring several times, the env ends exactly where a twin that ran every rollout
    directly does; capture slots are per handle and finite (MAPF_ESTATE past them)."""
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    env, twin = c4_env(), c4_env()
    assert env.rollout_plan().startswith("rollout_wide3_kernel<u64,1,false>"), env.rollout_plan()
    env.rollout_random(5)
    twin.rollout_random(5)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            env.rollout_random(4)            # recorded, not run
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
        twin.rollout_random(4)
        for _ in range(20):                  # > 16 ring slots between replays
            env.rollout_random(1)
            twin.rollout_random(1)
    torch.cuda.synchronize()
    assert torch.equal(env.obs, twin.obs) and torch.equal(env.vec, twin.vec)
    for k in twin.out:
        assert torch.equal(env.out[k], twin.out[k]), k
    assert_same_env(env, twin, "after replays")
    assert not env.counters()[:8].any()


def test_capture_after_deferred_search_needs_flush():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    env, twin = c4_env(), c4_env()
    assert not env.fused
    for _ in range(4):                       # leaves a deferred search pending on the aux stream
        env.step_observe(random_policy=True)
        twin.step_observe(random_policy=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with pytest.raises(RuntimeError, match="mapf_flush"):
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                env.step_observe(random_policy=True)
    torch.cuda.synchronize()
    env.flush()                              # joins the deferred search on the current stream
    twin.flush()
    torch.cuda.synchronize()
    assert_same_env(env, twin, "after the refused capture")   # the refused call changed nothing
    # ... and the same capture now works: three steps recorded, replayed twice == six direct steps
    s2 = torch.cuda.Stream()
    s2.wait_stream(torch.cuda.current_stream())
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s2):
        with torch.cuda.graph(g2, stream=s2):
            for _ in range(3):
                env.step_observe(random_policy=True)
    torch.cuda.synchronize()
    for _ in range(2):
        g2.replay()
        for _ in range(3):
            twin.step_observe(random_policy=True)
    torch.cuda.synchronize()
    assert torch.equal(env.obs, twin.obs) and torch.equal(env.vec, twin.vec)
    assert torch.equal(env.actions, twin.actions)
    assert_same_env(env, twin, "after the replays")


def test_capture_slots_run_out_loudly_and_can_be_released():
    """16 captured persistent launches per handle (ArgRing): the 17th capture fails with
    MAPF_ESTATE and records nothing (the env is unchanged, no other kernel form is launched in
    its place); after the graphs are destroyed, mapf_release_captures hands the slots back."""
    import gc
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    env, twin = c4_env(), c4_env()
    env.rollout_random(2)
    twin.rollout_random(2)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())

    def capture():
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                env.rollout_random(1)
        torch.cuda.synchronize()
        return g

    graphs = [capture() for _ in range(16)]
    with pytest.raises(RuntimeError, match="argument slot"):
        capture()
    torch.cuda.synchronize()
    assert_same_env(env, twin, "after the refused capture")     # nothing ran
    graphs[3].replay()                                          # a held slot still replays
    twin.rollout_random(1)
    torch.cuda.synchronize()
    assert_same_env(env, twin, "after a replay")
    del graphs
    gc.collect()
    env.release_captures()
    g = capture()
    for _ in range(2):
        g.replay()
        twin.rollout_random(1)
    torch.cuda.synchronize()
    assert torch.equal(env.obs, twin.obs)
    assert_same_env(env, twin, "after the released slots were captured again")
