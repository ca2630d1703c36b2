"""GPU tests of the rollout side and the drop-in adapters.

* DeviceRunner (runner.py:26-151 on device): buffer contract, GAE bit-exact
  against the oracle on the rollout's own buffers.
* Model.train on device (normalisation kernel + PPO update).
* Env sharding: ranks own disjoint env ranges via env_offset and draw exactly
  what one device running all envs draws (weak-scaling correctness).
* mapf_gym adapter (FixedMapfGym) driven with the reference's call sequence
  reproduces a golden episode.
"""
import numpy as np
import pytest
import torch

from golden_io import load, unpack_obs
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")


def make_env(B, N=8, H=20, W=20, F=9, offset=0, seed=99):
    from mapf_amd.config import make_config
    from mapf_amd.env import BatchedMapfGym
    from mapf_amd.maps import generate_warehouse
    env = BatchedMapfGym(make_config(B, H, W, num_agents=N, fov=F, num_channel=6, human_mode="random",
                                     goal_mode="random", fix_choice=1, seed=seed, env_offset=offset))
    env.reset_seeded(generate_warehouse(H, W))
    return env


def test_device_runner_contract_and_gae():
    from mapf_amd.model import Model
    from mapf_amd.runner import DeviceRunner
    B, N, T = 16, 8, 12
    env = make_env(B, N)
    model = Model(0, "cuda", global_model=True, numChannel=6, num_agents=N, fov=9)
    runner = DeviceRunner(env, model, n_steps=T, seed=5)
    mb, perf = runner.run()
    torch.cuda.synchronize()
    assert mb["observations"].shape == (T * B, N, 6, 9, 9)
    assert mb["vectors"].shape == (T * B, N, 4)
    assert mb["ps"].shape == (T * B, N, 5) and mb["trainValid"].shape == (T * B, N, 5)
    assert mb["actions"].dtype == torch.int64 and mb["hiddenState"].shape == (T * B, 2, N, 512)
    for k in ("rewards", "values", "returns", "costRewards", "costValues", "costReturns"):
        assert mb[k].shape == (T * B, N), k
    assert torch.isfinite(mb["returns"].materialize()).all()
    # env-major rows: row b*T + t is env b's step t
    np.testing.assert_array_equal(mb.observations[np.arange(T)].cpu().numpy(), runner.obs[:T, 0].cpu().numpy())
    np.testing.assert_array_equal(mb.rewards[T * 3 + 5].cpu().numpy(), runner.rewards[5, 3].cpu().numpy())
    # sampled actions have support under ps
    p_taken = mb["ps"].materialize().gather(-1, mb["actions"].materialize().unsqueeze(-1))
    assert (p_taken > 0).all()
    # GAE == oracle GAE on the same buffers, bit-exact
    r = runner.rewards.reshape(T, -1).cpu().numpy()
    v = runner.values.reshape(T, -1).cpu().numpy()
    # (the net keeps dropout active during rollouts, net.py:50-51 / model.py:26 -- use the runner's own bootstrap)
    lv, lcv = runner.last_v, runner.last_cv
    adv, ret = O.gae(r, v, lv.reshape(-1).cpu().numpy())
    np.testing.assert_array_equal(runner.returns.reshape(T, -1).cpu().numpy(), ret)
    cr = runner.cost_rewards.reshape(T, -1).cpu().numpy()
    cv = runner.cost_values.reshape(T, -1).cpu().numpy()
    _, cret = O.gae(cr, cv, lcv.reshape(-1).cpu().numpy())
    np.testing.assert_array_equal(runner.cost_returns.reshape(T, -1).cpu().numpy(), cret)
    assert perf.staticCollide + perf.humanCollide + perf.agentCollide >= 0
    # one PPO update on device from the rollout
    rows = slice(0, 64)
    stats = model.train(mb["observations"][rows], mb["vectors"][rows], mb["returns"][rows], mb["costReturns"][rows],
                        mb["values"][rows], mb["costValues"][rows], mb["actions"][rows], mb["ps"][rows], None,
                        mb["trainValid"][rows], float(perf.episodeCostReward))
    # losses finite (grad_norm, stats[8], may be inf on the first AMP steps: GradScaler then skips the step)
    assert all(np.isfinite(float(np.asarray(s))) for k, s in enumerate(stats) if k != 8)


def test_env_shards_draw_like_one_device():
    full = make_env(32, offset=0)
    parts = [make_env(16, offset=0), make_env(16, offset=16)]
    for _ in range(40):
        full.step_random()
        full.observe()
        for p in parts:
            p.step_random()
            p.observe()
    torch.cuda.synchronize()
    sf = full.get_state()
    s0, s1 = parts[0].get_state(), parts[1].get_state()
    for k in ("pos", "goal", "human", "clock"):
        np.testing.assert_array_equal(sf[k][:16], s0[k])
        np.testing.assert_array_equal(sf[k][16:], s1[k])
    np.testing.assert_array_equal(full.obs[16:].cpu().numpy(), parts[1].obs.cpu().numpy())


def test_fixed_mapf_gym_adapter_reproduces_golden_episode():
    from mapf_amd.config import EnvParameters
    from mapf_amd.mapf_gym import FixedMapfGym
    z = load("g1_c1")
    n, fov, nch = int(z["n"]), int(z["fov"]), int(z["nch"])
    seqs = [list(map(tuple, z["seq"][i, :z["seq_len"][i]])) for i in range(n)]
    EnvParameters.FOV_SIZE = fov
    env = FixedMapfGym(z["map"], seqs, tuple(z["hstart"]), tuple(z["hgoal"]), numChannel=nch)
    obs, vec = env.getAllObservations()
    np.testing.assert_array_equal(obs[0], unpack_obs(z["obs0"], (n, nch, fov, fov)))
    for t in range(60):
        a = z["actions"][t].astype(np.float64)
        st = env.getActionStatus(a)
        rw, sh = env.calculateActionReward(a, st)
        cost = env.calculateCostReward(a)
        tv = env.getTrainValid(a)
        goals, constr = env.jointStep(a, st)
        np.testing.assert_array_equal(st, z["status"][t].astype(np.float64))
        np.testing.assert_array_equal(rw[0], z["reward"][t])
        assert sh == int(z["shadow"][t])
        np.testing.assert_array_equal(cost[0], z["cost"][t])
        np.testing.assert_array_equal(tv, z["valid"][t])
        np.testing.assert_array_equal(goals, z["goals"][t].astype(np.float64))
        np.testing.assert_array_equal(constr, z["constr"][t].astype(np.float64))
        obs, vec = env.getAllObservations()
        np.testing.assert_array_equal(obs[0], unpack_obs(z["obs"][t], (n, nch, fov, fov)))
        np.testing.assert_array_equal(vec[0], z["vec"][t])


def test_policy_forward_on_device_matches_reference():
    """SCRIMPNet as the rollout runs it on the GPU (autocast fp16, NHWC convolutions,
    fused scaled_dot_product_attention) against the reference's fp32 outputs
    (tests/golden/g5_net.npz, net.py:101-155), dropout off: fp16 tolerance."""
    from golden_io import load
    from mapf_amd.model import Model
    from test_net import det_weights
    z = load("g5_net")
    m = Model(0, "cuda", global_model=False, numChannel=6, num_agents=2, fov=9)
    m.network.load_state_dict(det_weights(m.network.state_dict()))
    m.network.eval()
    with torch.no_grad():
        outs = m.network(torch.from_numpy(z["obs"]).cuda(), torch.from_numpy(z["vec"]).cuda())
    for name, o in zip(["policy", "value", "blocking", "policy_sig", "x", "logits", "cost_value"], outs):
        want = z[f"out_{name}"]
        got = o.float().cpu().numpy()
        tol = 2e-2 * max(1.0, float(np.abs(want).max()))
        np.testing.assert_allclose(got, want, rtol=0, atol=tol, err_msg=name)


def test_device_runner_fresh_reference_envs_each_rollout():
    """DeviceRunner(new_maps=reference_maps(env)): every run() starts from a fresh
    MapfGym() per env (runner.py:30) -- its own random-size warehouse in the padded
    stack, new agents and human -- and every agent stays on its env's real map."""
    from mapf_amd.config import make_config
    from mapf_amd.env import BatchedMapfGym
    from mapf_amd.model import Model
    from mapf_amd.runner import DeviceRunner, reference_maps
    B, N, T = 32, 8, 6
    env = BatchedMapfGym(make_config(B, 40, 60, num_agents=N, fov=9, num_channel=6, human_mode="random",
                                     goal_mode="random", fix_choice=1, seed=5, shared_map=False))
    model = Model(0, "cuda", global_model=False, numChannel=6, num_agents=N, fov=9)
    draw = reference_maps(env, seed=3)
    runner = DeviceRunner(env, model, n_steps=T, seed=1, new_maps=draw)
    starts = []
    for r in range(2):
        mb, perf = runner.run()
        assert mb["observations"].shape == (T * B, N, 6, 9, 9)
        maps = draw(r)
        st = env.get_state()
        for b in range(B):
            cells = maps[b][st["pos"][b][:, 0], st["pos"][b][:, 1]]
            assert (cells == 0).all(), f"rollout {r} env {b}: agent off its warehouse"
        starts.append(mb["observations"][::T].cpu().numpy())     # every env's first observation
    assert not np.array_equal(starts[0], starts[1])      # a new env each rollout
    c = env.counters()
    assert not c[:8].any(), c[:8]


class _GuardedModel:
    """Model.train behind driver.py:131-134: every minibatch argument must arrive as a device
    tensor; the model's own one stats copy is the only host copy allowed (HostGuard)."""

    def __init__(self, model, guard):
        self.model, self.guard, self.obs, self.returns = model, guard, [], []

    def train(self, *args):
        for k, a in enumerate(args[:10]):
            assert isinstance(a, torch.Tensor) and a.is_cuda, f"train argument {k} is not a device tensor"
        self.obs.append(args[0])
        self.returns.append(args[2])
        with self.guard.allow():
            return self.model.train(*args)


@pytest.mark.parametrize("n_runners", [1, 2])
def test_driver_block_verbatim_over_device_runners_c3(n_runners):
    """driver.py:97-134 run unchanged (tests/driver_block.py: the attribute appends :101-107, the
    np.nanmean of :110-117, np.concatenate(..., axis=0) of :119-121, the minibatch loop of
    :123-134) over one and two DeviceRunner results at the c3 shape (4096 envs x 8 agents,
    20x20, FOV 9) with the reference's rollout length T = N_STEPS = 256.  No buffer leaves the
    device (HostGuard + peak-memory bound: one runner's observations alone are 16.3 GB), the
    concatenation is lazy, and `inds = np.arange(N_STEPS)` trains on env 0's rollout of the
    first runner -- as the reference trains on its first runner's rollout."""
    from driver_block import HostGuard, ReferenceBatchValues, ReferenceOneEpPerformance, expected_minibatches, \
        run_driver_block
    from mapf_amd.config import TrainingParameters as TP
    from mapf_amd.model import Model
    from mapf_amd.runner import BATCH_FIELDS, PERF_FIELDS, DeviceRunner
    B, N, T = 4096, 8, TP.N_STEPS
    model = Model(0, "cuda", global_model=True, numChannel=6, num_agents=N, fov=9)
    runners = [DeviceRunner(make_env(B, N, F=9, offset=k * B, seed=99), model, n_steps=T, seed=11 + k)
               for k in range(n_runners)]
    job_results = [r.run() for r in runners]
    torch.cuda.synchronize()
    # GAE on runner 0's whole rollout (B*N columns) == the oracle's numpy-f32 loop, bit-exact
    r0 = runners[0]
    for rew, val, last, ret in ((r0.rewards, r0.values, r0.last_v, r0.returns),
                                (r0.cost_rewards, r0.cost_values, r0.last_cv, r0.cost_returns)):
        _, want = O.gae(rew.reshape(T, -1).cpu().numpy(), val.reshape(T, -1).cpu().numpy(),
                        last.reshape(-1).cpu().numpy())
        np.testing.assert_array_equal(ret.reshape(T, -1).cpu().numpy(), want)
    want_perf = {f: getattr(job_results[-1][1], f) for f in PERF_FIELDS}
    before = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    np.random.seed(2024)
    with HostGuard() as guard:
        proxy = _GuardedModel(model, guard)
        mb, performance, losses, steps, episodes = run_driver_block(
            job_results, proxy, ReferenceBatchValues, ReferenceOneEpPerformance, TP)
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated() - before
    # (3 GiB: the update's own working set is ~1.8 GB, plus ~0.5 GB of hipBLASLt workspace for the
    # tuned GEMM solutions, mapf_amd/gemm_tuning.py -- a materialised rollout would be 16 GB)
    assert not guard.hits and peak < 3 << 30, (guard.hits, peak)
    assert steps == n_runners * T and episodes == n_runners
    for k in BATCH_FIELDS:
        v = getattr(mb, k)
        assert not isinstance(v, np.ndarray) and len(v) == n_runners * T * B and v.device.type == "cuda", k
    for f in PERF_FIELDS:                    # the last result's per-env means, through two nanmeans
        assert getattr(performance, f) == want_perf[f], f
    per_env = runners[-1].performance_per_env()
    assert performance.episodeCostReward == np.mean(per_env["episodeCostReward"])
    # the minibatches: env 0's rollout of runner 0, in the shuffled order of the global numpy RNG
    mbs = expected_minibatches(2024, TP)
    assert len(losses) == len(mbs) == TP.N_EPOCHS * (T // TP.MINIBATCH_SIZE)
    for obs, ret, inds in zip(proxy.obs, proxy.returns, mbs):
        assert torch.equal(obs, r0.obs[torch.as_tensor(inds, device="cuda"), 0])
        assert torch.equal(ret, r0.returns[torch.as_tensor(inds, device="cuda"), 0])
    if n_runners == 2:                       # runner 1's rows follow runner 0's
        r1 = runners[1]
        rows = np.array([T * B, T * B + 7, 2 * T * B - 1])
        got = mb.observations[rows]
        assert torch.equal(got[0], r1.obs[0, 0]) and torch.equal(got[1], r1.obs[7, 0])
        assert torch.equal(got[2], r1.obs[T - 1, B - 1])
    assert all(np.isfinite(float(np.asarray(s))) for k, s in enumerate(losses[-1]) if k != 8)


class _ScriptedModel:
    """Model.step / Model.value stand-in that plays a g1 episode's scripted actions (the
    reference's recorded actions) into DeviceRunner's buffers: the runner's counter loop then
    sees exactly the reference episode."""

    def __init__(self, actions, B):
        self.actions = torch.from_numpy(np.ascontiguousarray(actions)).cuda()    # [T, N]
        self.B = B

    def step(self, obs, vec, hidden, seed=0, step=0, actions_out=None, actions32_out=None):
        t = step % self.actions.shape[0]
        a = self.actions[t].unsqueeze(0).expand(self.B, -1)
        actions_out.copy_(a)
        actions32_out.copy_(a)
        z = torch.zeros(self.B, a.shape[1], 1, device="cuda")
        return actions_out, torch.full((self.B, a.shape[1], 5), 0.2, device="cuda"), z, None, None, z

    def value(self, obs, vec, hidden):
        z = torch.zeros(self.B, self.actions.shape[1], 1, device="cuda")
        return z, z


@pytest.mark.parametrize("name", ["g1_c1", "g1_c2", "g1_dahp", "g1_dense", "g1_fixedpath"])
def test_device_runner_performance_matches_reference(name):
    """OneEpPerformance (runner.py:66-99) of DeviceRunner over a reference episode (g1, replayed
    with its scripted actions on B replicas) == the reference's own counter loop over the same
    episode (g1_perf, util.OneEpPerformance), every env, every counter bit for bit -- the float32
    episodeReward / episodeCostReward accumulation included (episodeCostReward feeds the
    Lagrangian, model.py:180)."""
    from mapf_amd.config import make_config
    from mapf_amd.env import BatchedMapfGym
    from mapf_amd.runner import PERF_FIELDS, DeviceRunner
    z = load(name)
    perf = load("g1_perf")
    n, fov, nch = int(z["n"]), int(z["fov"]), int(z["nch"])
    world = z["map"]
    H, W = world.shape
    hmode = int(z["human_mode"])
    B, T = 5, int(z["steps"])
    env = BatchedMapfGym(make_config(B, H, W, num_agents=n, fov=fov, num_channel=nch, use_da=int(z["use_da"]),
                                     use_hp=int(z["use_hp"]), human_mode=hmode, goal_mode="sequence", fix_choice=0,
                                     max_seq=z["seq"].shape[1], max_human_seq=max(2, len(z["hseq"]))))
    seqs = [z["seq"][i, :z["seq_len"][i]] for i in range(n)]
    if hmode == 2:
        env.reset_fixed(world, [seqs] * B, human_seq=[z["hseq"]] * B)
    else:
        env.reset_fixed(world, [seqs] * B, [z["hstart"]] * B, [z["hgoal"]] * B)
    runner = DeviceRunner(env, _ScriptedModel(z["actions"], B), n_steps=T)
    _, p = runner.run()
    per_env = runner.performance_per_env()
    np.testing.assert_array_equal(runner.status.cpu().numpy()[:, 0], z["status"])   # the reference episode
    for k in PERF_FIELDS:
        want = perf[f"{name}__{k}"][T - 1]
        np.testing.assert_array_equal(per_env[k], np.full(B, want), err_msg=k)
        assert getattr(p, k) == want, k
    assert per_env["episodeReward"].dtype == np.float64


def test_episode_sum_matches_oracle():
    from mapf_amd.env import episode_sum
    g = np.random.default_rng(9)
    vals = np.array([-0.3, -0.5, -1.0, 0.0, 1.5, -0.25, 1.2, -0.02], np.float32)
    for N in (1, 4, 7, 8, 9, 16, 17, 64):
        x = np.where(g.random((256, 33, N)) < 0.5, g.choice(vals, (256, 33, N)),
                     g.normal(size=(256, 33, N))).astype(np.float32)
        got = episode_sum(torch.from_numpy(x).cuda()).cpu().numpy()
        np.testing.assert_array_equal(got, O.episode_sum(x), err_msg=f"N={N}")


def _norm_worker(rank, world, port, x, y, lam, q):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path[:0] = [root, os.path.join(root, "primal-ppo_amd")]
        from mapf_amd.env import normalize_advantages_distributed
        torch.cuda.set_device(0)
        sl = slice(rank * len(x) // world, (rank + 1) * len(x) // world)
        xt, yt = torch.from_numpy(x[sl]).cuda(), torch.from_numpy(y[sl]).cuda()
        zero = torch.zeros_like(xt)
        adv, cadv = normalize_advantages_distributed(xt, zero, yt, zero, lagrange=lam, mix=True)
        q.put((rank, adv.cpu().numpy(), cadv.cpu().numpy()))
    finally:
        dist.destroy_process_group()


def test_normalize_distributed_two_ranks_equal_one_process():
    """two ranks (gloo, both on this GPU) each holding half of a minibatch,
    normalised by the HIP path with all-reduced two-pass moments (mapf_advantage_moments,
    mapf_normalize_advantages_stats), give the one-process HIP normalisation of the whole
    minibatch within 1e-5 -- the product path Model.train takes when distributed."""
    import socket
    import torch.multiprocessing as mp
    from mapf_amd.env import normalize_advantages
    z = load("g4_gae")
    x, y = z["norm_x"].reshape(-1), z["norm_y"].reshape(-1)
    lam = float(z["norm_lam"])
    xt, yt = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    zero = torch.zeros_like(xt)
    adv1, cadv1 = normalize_advantages(xt, zero, yt, zero, lagrange=lam, mix=True)
    np.testing.assert_allclose(adv1.cpu().numpy(), z["norm_mixed"].reshape(-1), rtol=1e-5, atol=1e-5)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_norm_worker, args=(r, 2, port, x, y, lam, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    adv2 = np.concatenate([r[1] for r in res])
    cadv2 = np.concatenate([r[2] for r in res])
    np.testing.assert_allclose(adv2, adv1.cpu().numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(cadv2, cadv1.cpu().numpy(), rtol=1e-5, atol=1e-6)
