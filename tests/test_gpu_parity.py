"""GPU parity: the HIP path (through the C ABI) against the reference's golden
vectors and the CPU oracle.  Bit-exact for every integer output, every
observation bit and every float the reference computes (rewards, costs,
vectors are exact restatements); GAE bit-exact; advantage normalisation
within 1e-5 of torch fp32 (model.py:106-113 computes it in torch).
"""
import collections

import numpy as np
import pytest
import torch

from golden_io import G1_NAMES, Fuzz, load, unpack_obs
from kernel_registry import record_rollout_kernel
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")


def mk_env(tuning=None, **kw):
    from mapf_amd.config import make_config
    from mapf_amd.env import BatchedMapfGym
    B = kw.pop("B")
    H, W = kw.pop("H"), kw.pop("W")
    return BatchedMapfGym(make_config(B, H, W, **kw), tuning=tuning)


def host(out):
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items()}


def assert_no_errors(env, allow=()):
    c = env.counters()
    for k in range(8):
        if k not in allow:
            assert c[k] == 0, f"device counter {k} = {c[k]}"


# --------------------------------------------------------------------------- g1
@pytest.mark.parametrize("name", G1_NAMES)
def test_g1_episode_on_device(name):
    run_g1(name, pad=None)


@pytest.mark.parametrize("name", G1_NAMES[:3])
def test_g1_episode_on_padded_map(name):
    """The same reference episode on the map padded with obstacle rows/columns at the
    bottom/right (how a batch of the reference's random-size warehouses shares one
    H x W, maps.random_warehouse_batch): off-map and padding read alike, so every
    output and observation is unchanged."""
    run_g1(name, pad=(6, 5))


def run_g1(name, pad):
    z = load(name)
    n, fov, nch = int(z["n"]), int(z["fov"]), int(z["nch"])
    world = z["map"]
    H0, W0 = world.shape
    if pad is not None:
        world = np.pad(world, ((0, pad[0]), (0, pad[1])), constant_values=-1)
    H, W = world.shape
    hmode = int(z["human_mode"])
    B = 37   # replicas: partial last workgroup, several envs per wave
    env = mk_env(B=B, H=H, W=W, num_agents=n, fov=fov, num_channel=nch, use_da=int(z["use_da"]),
                 use_hp=int(z["use_hp"]), human_mode=hmode, goal_mode="sequence", fix_choice=0,
                 max_seq=z["seq"].shape[1], max_human_seq=max(2, len(z["hseq"])))
    seqs = [z["seq"][i, :z["seq_len"][i]] for i in range(n)]
    if hmode == 2:
        env.reset_fixed(world, [seqs] * B, human_seq=[z["hseq"]] * B)
    else:
        env.reset_fixed(world, [seqs] * B, [z["hstart"]] * B, [z["hgoal"]] * B)
    st = env.get_state()
    for b in (0, B - 1):
        np.testing.assert_array_equal(st["pos"][b], z["pos0"])
        L = st["human"][b, 7]
        np.testing.assert_array_equal(st["human_path"][b, :L], z["hpath0"])
    bfs = env.bfs().cpu().numpy()
    np.testing.assert_array_equal(bfs[:, :, :H0, :W0], np.broadcast_to(z["bfs0"], (B,) + z["bfs0"].shape))
    if pad is not None:
        assert (bfs[:, :, H0:, :] == -1).all() and (bfs[:, :, :, W0:] == -1).all()
    obs, vec = env.observe()
    ref = unpack_obs(z["obs0"], (n, nch, fov, fov))
    o = obs.cpu().numpy()
    for b in range(B):
        np.testing.assert_array_equal(o[b], ref, err_msg=f"obs0 env {b}")
        np.testing.assert_array_equal(vec.cpu().numpy()[b], z["vec0"][0])
    acts = torch.zeros(B, n, dtype=torch.int32, device="cuda")
    for t in range(int(z["steps"])):
        acts.copy_(torch.from_numpy(np.tile(z["actions"][t].astype(np.int32), (B, 1))))
        out = host(env.step(acts))
        for k, key in [("status", "status"), ("reward", "reward"), ("cost", "cost"), ("train_valid", "valid"),
                       ("actions_fixed", "fixed"), ("goals_reached", "goals"), ("constraints", "constr")]:
            ref = np.broadcast_to(z[key][t].astype(out[k].dtype), out[k].shape)
            np.testing.assert_array_equal(out[k], ref, err_msg=f"{name} t={t} {k}")
        assert (out["shadow_goals"] == int(z["shadow"][t])).all()
        rt = z["reward"][t] + np.where(z["goals"][t] == 1, np.float32(1.5), np.float32(0)).astype(np.float32)
        np.testing.assert_array_equal(out["reward_total"][0], rt.astype(np.float32))
        obs, vec = env.observe()
        o = obs.cpu().numpy()
        ref = unpack_obs(z["obs"][t], (n, nch, fov, fov))
        for b in (0, B // 2, B - 1):
            np.testing.assert_array_equal(o[b], ref, err_msg=f"{name} t={t} obs env {b}")
            np.testing.assert_array_equal(vec.cpu().numpy()[b], z["vec"][t])
        if t % 25 == 0 or t == int(z["steps"]) - 1:
            st = env.get_state()
            np.testing.assert_array_equal(st["pos"][B - 1], z["pos"][t])
            np.testing.assert_array_equal(st["goal"][B - 1], z["goal"][t])
            np.testing.assert_array_equal(st["human"][0, 0:2], z["hpos"][t])
            np.testing.assert_array_equal(st["human"][0, 2:4], z["hnext"][t])
    np.testing.assert_array_equal(env.bfs().cpu().numpy()[B - 1][:, :H0, :W0], z["bfs_final"])
    assert_no_errors(env)


# --------------------------------------------------------------------------- g2
@pytest.mark.parametrize("fixture", ["g2_fuzz", "g2_evict"])
def test_g2_fuzz_on_device(fixture):
    """g2_fuzz: one-step scenarios; g2_evict: scenarios whose fixActions evicts two
    agents with one pick, appended in the reference's set order (mapf_pyset.h)."""
    fz = Fuzz(fixture)
    groups = collections.defaultdict(list)
    for k in range(fz.count):
        c = fz.case(k)
        groups[(int(c["H"]), int(c["W"]), int(c["n"]), int(c["fov"]), int(c["use_da"]), int(c["use_hp"]))].append(c)
    bad = []
    for (H, W, n, fov, da, hp), cases in groups.items():
        B = len(cases)
        env = mk_env(B=B, H=H, W=W, num_agents=n, fov=fov, num_channel=6, use_da=da, use_hp=hp,
                     human_mode="looping", goal_mode="sequence", fix_choice=0, max_seq=3, shared_map=False)
        maps = np.stack([c["map"].reshape(H, W) for c in cases])
        hps = [c["hpath"] for c in cases]
        env.reset_fixed(maps, [list(c["seq"]) for c in cases], [p[0] for p in hps], [p[len(p) // 2] for p in hps])
        st = env.get_state()
        human = st["human"].copy()
        for b, c in enumerate(cases):
            hs = int(c["hstep0"])
            human[b, 6] = hs
            human[b, 0:2] = hps[b][hs]
        prev = np.stack([c["prev"] if c["prev"].size == n else np.full(n, -1) for c in cases]).astype(np.int32)
        env.set_state(human=human, last_action=prev)
        obs0, vec0 = [x.cpu().numpy().copy() for x in env.observe()]
        acts = torch.from_numpy(np.stack([c["actions"] for c in cases]).astype(np.int32)).cuda()
        out = host(env.step(acts))
        obs1, vec1 = [x.cpu().numpy().copy() for x in env.observe()]
        st = env.get_state()
        for b, c in enumerate(cases):
            if not np.array_equal(obs0[b], unpack_obs(c["obs0"], (n, 6, fov, fov))) or not np.array_equal(vec0[b], c["vec0"]):
                bad.append(("obs0", H, W, n, b))
            for k, key in [("status", "status"), ("reward", "reward"), ("cost", "cost"), ("train_valid", "valid"),
                           ("actions_fixed", "fixed"), ("goals_reached", "goals"), ("constraints", "constr")]:
                if not np.array_equal(out[k][b], c[key].astype(out[k].dtype)):
                    bad.append((k, H, W, n, b))
            if out["shadow_goals"][b] != int(c["shadow"]):
                bad.append(("shadow", H, W, n, b))
            if not np.array_equal(st["pos"][b], c["pos1"]) or not np.array_equal(st["goal"][b], c["goal1"]):
                bad.append(("pos1", H, W, n, b))
            if not np.array_equal(obs1[b], unpack_obs(c["obs1"], (n, 6, fov, fov))) or not np.array_equal(vec1[b], c["vec1"]):
                bad.append(("obs1", H, W, n, b))
        env.close()
    assert not bad, f"{len(bad)} mismatches: {bad[:20]}"


# --------------------------------------------------------------------------- g3
def test_g3_astar_paths_and_bfs_on_device():
    z = load("g3_search")
    offs = np.concatenate([[0], np.cumsum(z["path_len"])])
    boffs = [0]
    for k in range(len(z["mi"])):
        boffs.append(boffs[-1] + z[f"map{int(z['mi'][k])}"].size)
    for mi in range(int(z["nmaps"])):
        world = z[f"map{mi}"]
        H, W = world.shape
        ks = [k for k in range(len(z["mi"])) if int(z["mi"][k]) == mi and not np.array_equal(z["s"][k], z["g"][k])]
        if not ks:
            continue
        free = np.argwhere(world == 0)
        B = len(ks)
        env = mk_env(B=B, H=H, W=W, num_agents=1, fov=3, num_channel=5, human_mode="looping", goal_mode="sequence",
                     fix_choice=0, max_seq=2)
        seqs = [[[free[0], z["g"][k]]] for k in ks]
        env.reset_fixed(world, seqs, [z["s"][k] for k in ks], [z["g"][k] for k in ks])
        st = env.get_state()
        bfs = env.bfs().cpu().numpy()
        unreachable = 0
        for b, k in enumerate(ks):
            ref_bfs = z["bfs"][boffs[k]:boffs[k + 1]].reshape(H, W)
            np.testing.assert_array_equal(bfs[b, 0], ref_bfs, err_msg=f"bfs map {mi} case {k}")
            if not z["ok"][k]:
                unreachable += 1
                assert st["human"][b, 7] == 3      # stays put three steps
                continue
            path = z["path"][offs[k]:offs[k + 1]]            # goal -> start (construct_path_from_dict)
            want = np.concatenate([path[::-1], path[1:]])     # Human.getAstarPath (mapf_gym.py:33-37)
            L = st["human"][b, 7]
            np.testing.assert_array_equal(st["human_path"][b, :L], want, err_msg=f"astar map {mi} case {k}")
        assert env.counters()[4] == unreachable


# ------------------------------------------------------------ random mode vs oracle
RANDOM_CASES = {
    "c2_20x20_n8_f11": dict(B=64, H=20, W=20, n=8, fov=11, nch=6, steps=300, map="wh"),
    "c1_10x10_n4_f11": dict(B=33, H=10, W=10, n=4, fov=11, nch=6, steps=300, map="wh"),
    "dense_12x12_n16_f9_dahp": dict(B=16, H=12, W=12, n=16, fov=9, nch=6, steps=200, map="wh", da=1, hp=1),
    "c4_40x40_n16_f9_looping": dict(B=16, H=40, W=40, n=16, fov=9, nch=6, steps=100, map="wh", human="looping"),
    "c5_80x80_n64_f11_bfsch": dict(B=3, H=80, W=80, n=64, fov=11, nch=7, steps=40, map="rand"),
    # one shared random 12x12 map (seed 6) on which fixActions deadlocks (the reference loops
    # forever, mapf_gym.py:563) and empty viable sets (it raises, :588) occur: counters 1 and 2
    # equal the oracle's, every step bit-exact through them
    "r_n8_12x12_f11_deadlock": dict(B=64, H=12, W=12, n=8, fov=11, nch=6, steps=200, map="rand_shared",
                                    map_seed=6, allow=(1, 2), min_deadlocks=1),
}


def build_maps(case, B, rng):
    from mapf_amd.maps import generate_warehouse, keep_largest_component, random_map
    if case["map"] == "wh":
        return generate_warehouse(case["H"], case["W"]), True
    if case["map"] == "rand_shared":
        m = random_map(np.random.default_rng(case["map_seed"]), case["H"], case["W"], 0.3)
        return keep_largest_component(m), True
    return np.stack([keep_largest_component(random_map(rng, case["H"], case["W"], 0.3)) for _ in range(B)]), False


FUSED_CASES = {
    "c2_20x20_n8_f11": RANDOM_CASES["c2_20x20_n8_f11"],
    "c1_10x10_n4_f11": RANDOM_CASES["c1_10x10_n4_f11"],
    "n2_16x16_f9_dahp": dict(B=40, H=16, W=16, n=2, fov=9, nch=6, steps=150, map="wh", da=1, hp=1),
    "n1_12x12_f7_looping": dict(B=300, H=12, W=12, n=1, fov=7, nch=6, steps=100, map="wh", human="looping"),
    # random 30% maps: an agent boxed in by obstacles + human has no viable action
    # (the reference's random.choice([]) raises); counter 2 counts it on both sides
    "n7_24x24_f11_rand_dahp": dict(B=37, H=24, W=24, n=7, fov=11, nch=6, steps=150, map="rand", da=1, hp=1,
                                   allow=(2,)),
    "n8_40x40_f9_wide": dict(B=16, H=40, W=40, n=8, fov=9, nch=6, steps=100, map="wh"),
}


@pytest.mark.parametrize("name", list(RANDOM_CASES))
def test_random_mode_matches_oracle(name):
    """(idx % 2) == 1: mapf_step_random (actions drawn in the step kernel), else mapf_step."""
    run_random_case(name, RANDOM_CASES[name], "random" if list(RANDOM_CASES).index(name) % 2 == 1 else "plain")


@pytest.mark.parametrize("name", list(FUSED_CASES) + ["r_n8_12x12_f11_deadlock"])
def test_fused_step_observe_matches_oracle(name):
    """mapf_step_observe_random: step + observations in one launch, search one launch behind."""
    run_random_case(name, FUSED_CASES.get(name) or RANDOM_CASES[name], "fused")


# configurations the one-launch rollout kernel covers (N in 5..8 with whole float4s
# per env, a shared map whose padded bitmap fits 64 words -- W + 2*(F//2) <= 32 --,
# Human / LoopingHuman, random goals): ragged B
# (not a multiple of the 4 envs per workgroup), FOV 7/9/11, DA + HP channels, dense maps
ROLLOUT_CASES = {
    "r_n6_16x16_f9_dahp": dict(B=37, H=16, W=16, n=6, fov=9, nch=6, steps=120, map="wh", da=1, hp=1),
    "r_n8_22x22_f11_looping": dict(B=18, H=22, W=22, n=8, fov=11, nch=6, steps=120, map="wh", human="looping"),
    "r_n6_12x12_f7_dense": dict(B=41, H=12, W=12, n=6, fov=7, nch=6, steps=150, map="wh", allow=(2,)),
    "r_n8_24x24_f9": dict(B=9, H=24, W=24, n=8, fov=9, nch=6, steps=100, map="wh"),   # padded row = 32 bits
    "r_n8_12x12_f11_deadlock": RANDOM_CASES["r_n8_12x12_f11_deadlock"],
}


@pytest.mark.parametrize("name", list(FUSED_CASES) + list(ROLLOUT_CASES) +
                         ["c5_80x80_n64_f11_bfsch", "c4_40x40_n16_f9_looping", "dense_12x12_n16_f9_dahp"])
def test_rollout_random_matches_oracle(name):
    """mapf_rollout_random into [T]-slot rollout buffers, 23 steps per call, one launch
    each (each wave loops step -> observe -> its own search): the pair-lane kernel for
    the ROLLOUT_CASES and the c2 shape, the one-wave-per-env kernel for the rest (up to
    64 agents, per-env maps, the BFS channel) -- every slot bit-exact vs the oracle."""
    case = FUSED_CASES.get(name) or ROLLOUT_CASES.get(name) or RANDOM_CASES[name]
    kind = 1 if name in ROLLOUT_CASES or name.startswith("c2") else (2 if case["n"] > 8 else (1, 2))
    run_random_case(name, case, "rollout", expect_rollout_kernel=kind)


GROUP_CASES = {
    "g_n8_20x20_f11": dict(B=64, H=20, W=20, n=8, fov=11, nch=6, steps=60, map="wh"),
    "g_n8_20x20_f11_ragged61": dict(B=61, H=20, W=20, n=8, fov=11, nch=6, steps=60, map="wh"),
    "g_n6_16x16_f9_dahp_ragged": dict(B=45, H=16, W=16, n=6, fov=9, nch=6, steps=60, map="wh", da=1, hp=1),
}


@pytest.mark.parametrize("name,slack", [("g_n8_20x20_f11", 1), ("g_n8_20x20_f11", 0), ("g_n8_20x20_f11", -1),
                                        ("g_n6_16x16_f9_dahp_ragged", 1), ("g_n6_16x16_f9_dahp_ragged", 3),
                                        ("g_n8_20x20_f11_ragged61", 1)])
def test_rollout_random_cu_groups_match_oracle(name, slack):
    """The pair-lane rollout with all 16 waves of a CU in one workgroup (four 4-env quarters
    at their own LDS offsets, the waves paced within `slack` steps of the group's slowest;
    ragged B -- 45: a short last quarter, 61: the last group's last quarter holds one env --
    the envs past B never count) -- every slot bit-exact vs the oracle."""
    run_random_case(name, GROUP_CASES[name], "rollout", expect_rollout_kernel=1,
                    tuning=dict(roll_occ=4, roll_group=1, roll_slack=slack), expect_name="rollout_random_kernel<true,4>")


@pytest.mark.parametrize("name,fair,path", [("g_n8_20x20_f11", 4, "rollout"), ("g_n6_16x16_f9_dahp_ragged", 1, "rollout"),
                                            ("g_n8_20x20_f11", 4, "inplace1"), ("g_n8_20x20_f11", 4, "inplace"),
                                            ("g_n8_20x20_f11_ragged61", 4, "inplace")])
def test_rollout_random_fair_priority_matches_oracle(name, fair, path):
    """The pair-lane rollout with all 16 waves of a CU in one workgroup and issue priority by
    progress (a wave more than `fair` steps ahead of the group's slowest env drops to priority
    0; ragged B: the envs past B never count) -- slot buffers, and the in-place [B] buffers
    (the form and plain stores c2's in-place rollout uses: rollout_random_kernel<false,4>) in
    one-step launches and in 23-step launches -- bit-exact vs the oracle."""
    run_random_case(name, GROUP_CASES[name], path, expect_rollout_kernel=1, tuning=dict(roll_occ=4, roll_fair=fair),
                    expect_name="rollout_random_kernel<%s,4>" % ("true" if path == "rollout" else "false"))


# the one-wave-per-env kernel's other search row layouts (u32 rows on two lane slots, u64 on
# two, 128-bit rows on one) and the BFS channel on a non-square map
WIDE_SHAPES = {
    "w_n12_70x30_f9": dict(B=11, H=70, W=30, n=12, fov=9, nch=6, steps=60, map="rand"),
    "w_n20_48x90_f11_bfsch": dict(B=5, H=48, W=90, n=20, fov=11, nch=7, steps=50, map="rand"),
    "w_n10_96x60_f7_looping": dict(B=7, H=96, W=60, n=10, fov=7, nch=6, steps=50, map="rand", human="looping"),
}


@pytest.mark.parametrize("name", list(WIDE_SHAPES))
def test_rollout_wide_row_layouts_match_oracle(name):
    run_random_case(name, WIDE_SHAPES[name], "rollout", expect_rollout_kernel=2)


@pytest.mark.parametrize("name", G1_NAMES)
def test_rollout_on_fixed_episodes_equals_step_observe(name):
    """The reference's fixed episodes (agent goal sequences, LoopingHuman or FixedPathHuman)
    under the random policy: one mapf_rollout_random launch of T steps == T launches of
    mapf_step_observe_random, on two envs reset alike (every slot's actions, outputs and
    observation; state and BFS maps after) -- the rollout kernels' goal_mode 0 and human
    modes 0 / 2, which the seeded cases do not reach."""
    z = load(name)
    n, fov, nch = int(z["n"]), int(z["fov"]), int(z["nch"])
    world = z["map"]
    H, W = world.shape
    hmode = int(z["human_mode"])
    B = 9
    envs = []
    for _ in range(2):
        e = mk_env(B=B, H=H, W=W, num_agents=n, fov=fov, num_channel=nch, use_da=int(z["use_da"]),
                   use_hp=int(z["use_hp"]), human_mode=hmode, goal_mode="sequence", fix_choice=1,
                   max_seq=z["seq"].shape[1], max_human_seq=max(2, len(z["hseq"])), seed=77)
        seqs = [z["seq"][i, :z["seq_len"][i]] for i in range(n)]
        if hmode == 2:
            e.reset_fixed(world, [seqs] * B, human_seq=[z["hseq"]] * B)
        else:
            e.reset_fixed(world, [seqs] * B, [z["hstart"]] * B, [z["hgoal"]] * B)
        envs.append(e)
    ro, so = envs
    assert ro.rollout_fused, name
    T = 40
    dev = ro.device
    acts = torch.zeros(T, B, n, dtype=torch.int32, device=dev)
    obs = torch.full((T, B, n, nch, fov, fov), float("nan"), device=dev)
    vec = torch.full((T, B, n, 4), float("nan"), device=dev)
    out = {key: torch.full((T,) + tuple(v.shape), -7, dtype=v.dtype, device=dev) for key, v in ro.out.items()}
    ro.rollout_random(T, slots=True, actions=acts, obs=obs, vec=vec, out=out)
    out = host(out)
    for t in range(T):
        o_s, obs_s, vec_s = so.step_observe(random_policy=True)
        o_s = host(o_s)
        np.testing.assert_array_equal(acts[t].cpu().numpy(), so.actions.cpu().numpy(), err_msg=f"{name} t={t}")
        for key in o_s:
            np.testing.assert_array_equal(out[key][t], o_s[key], err_msg=f"{name} t={t} {key}")
        assert torch.equal(obs[t], obs_s) and torch.equal(vec[t], vec_s), f"{name} t={t} obs"
    sr, ss = ro.get_state(), so.get_state()
    for key in ss:
        np.testing.assert_array_equal(sr[key], ss[key], err_msg=f"{name} state {key}")
    assert torch.equal(ro.bfs(), so.bfs())
    assert (ro.counters()[:8] == so.counters()[:8]).all()


@pytest.mark.parametrize("name,grid", [("c4_40x40_n16_f9_looping", 1), ("dense_12x12_n16_f9_dahp", 1),
                                       ("n7_24x24_f11_rand_dahp", 1), ("dense_12x12_n16_f9_dahp", 0)])
def test_rollout_wide_one_wave_form_matches_oracle(name, grid):
    """The one-wave-per-env kernel in its unpipelined form (one wave steps and observes;
    the form c5 runs in) -- small configs otherwise run the two-wave pipelined form --
    with the step's neighbour grid over the scratch, and without it (the agent loop)."""
    case = FUSED_CASES.get(name) or RANDOM_CASES[name]
    run_random_case(name, case, "rollout", expect_rollout_kernel=(1, 2), tuning=dict(wide_pipe=0, wide_grid=grid))


@pytest.mark.parametrize("name,pipe,epw,pair,slack", [
    ("c4_40x40_n16_f9_looping", 1, 4, 0, 4), ("c4_40x40_n16_f9_looping", 1, 4, 1, 0),
    ("dense_12x12_n16_f9_dahp", 1, 2, 0, -1), ("dense_12x12_n16_f9_dahp", 0, 8, 0, 4),
    ("c5_80x80_n64_f11_bfsch", 0, 3, 0, 1), ("dense_12x12_n16_f9_dahp", 0, 4, 0, -3)])
def test_rollout_wide_env_groups_match_oracle(name, pipe, epw, pair, slack):
    """Several envs per workgroup (all the envs of a CU at full size), each at its own LDS
    offset, their pacing waves kept within `slack` steps of the group's slowest env: the
    same trajectories and observations as the oracle, in both wave-to-env orders."""
    tuning = dict(wide_pipe=pipe, wide_epw=epw, wide_pair=pair, wide_slack=max(slack, -1))
    if slack < -1:      # issue priority by progress instead of waits (wide_fair = -slack - 1)
        tuning["wide_fair"] = -slack - 1
    case = FUSED_CASES.get(name) or RANDOM_CASES[name]
    run_random_case(name, case, "rollout", expect_rollout_kernel=(1, 2), tuning=tuning)


@pytest.mark.parametrize("name,nobs,bfsobs", [("c4_40x40_n16_f9_looping", 1, 1), ("dense_12x12_n16_f9_dahp", 1, 1),
                                              ("w_n12_70x30_f9", 1, 1), ("w_n10_96x60_f7_looping", 2, 1),
                                              ("dense_12x12_n16_f9_dahp", 2, 0), ("c4_40x40_n16_f9_looping", 2, 0)])
def test_rollout_wide_observer_count_matches_oracle(name, nobs, bfsobs):
    """The overlapped two-wave form (wide_obs 1: one stepping, one observing wave) and the
    three-wave form (2: two observers taking alternate steps, the default where it fits), with
    the BFS maps searched by the observers (the default) or by the stepper -- every slot and
    the BFS maps bit-exact vs the oracle."""
    case = FUSED_CASES.get(name) or RANDOM_CASES.get(name) or WIDE_SHAPES[name]
    run_random_case(name, case, "rollout", expect_rollout_kernel=(1, 2), tuning=dict(wide_obs=nobs, wide_bfsobs=bfsobs))


# In place: every step of a launch re-writes the same [B]-leading buffers (mapf_rollout_random
# slots = 0) with plain stores where the buffer stays cache-resident -- the kernels the in-place
# rollouts of c1 / c2 / c4 run (rollout_wide3_kernel<u32/u64,1,false>, rollout_random_kernel<false,*>),
# which the slot-buffer cases above never launch (slot buffers force nontemporal stores).
# "inplace1": one-step launches, every step compared; "inplace": 23-step launches, each launch's
# last step compared (its buffers hold only that step), the oracle stepping through the others.
@pytest.mark.parametrize("name,path", [("c4_40x40_n16_f9_looping", "inplace1"), ("c4_40x40_n16_f9_looping", "inplace"),
                                       ("dense_12x12_n16_f9_dahp", "inplace1"), ("dense_12x12_n16_f9_dahp", "inplace"),
                                       ("c1_10x10_n4_f11", "inplace1"), ("c1_10x10_n4_f11", "inplace"),
                                       ("c5_80x80_n64_f11_bfsch", "inplace1"), ("w_n12_70x30_f9", "inplace"),
                                       ("c2_20x20_n8_f11", "inplace1"), ("r_n6_16x16_f9_dahp", "inplace")])
def test_rollout_in_place_matches_oracle(name, path):
    case = FUSED_CASES.get(name) or ROLLOUT_CASES.get(name) or RANDOM_CASES.get(name) or WIDE_SHAPES[name]
    run_random_case(name, case, path, expect_rollout_kernel=(1, 2))


def run_random_case(name, case, path, expect_rollout_kernel=None, tuning=None, expect_name=None):
    B, H, W, n, fov, nch = case["B"], case["H"], case["W"], case["n"], case["fov"], case["nch"]
    rng = np.random.default_rng(5)
    maps, shared = build_maps(case, B, rng)
    human = case.get("human", "random")
    seed = 0x5EED0000 + len(name)
    env = mk_env(B=B, H=H, W=W, num_agents=n, fov=fov, num_channel=nch, use_da=case.get("da", 0),
                 use_hp=case.get("hp", 0), human_mode=human, goal_mode="random", fix_choice=1, shared_map=shared,
                 seed=seed, env_offset=7, tuning=tuning)
    env.reset_seeded(maps)
    if expect_rollout_kernel is not None:
        assert env.rollout_kernel in np.atleast_1d(expect_rollout_kernel), name
    rolling = path in ("rollout", "inplace", "inplace1")
    if rolling:
        kname = env.rollout_kernel_name(slots=path == "rollout")
        if expect_name is not None:
            assert kname == expect_name, (name, env.rollout_plan(slots=path == "rollout"))
    hm = {"random": 1, "looping": 0}[human]
    cfg = O.make_config(H, W, n, fov, nch, use_da=case.get("da", 0), use_hp=case.get("hp", 0), human_mode=hm,
                        goal_mode=1, fix_choice=1, seed=seed, env_offset=7)
    oracles = []
    for b in range(B):
        oe = O.OracleEnv(cfg, env_id=7 + b)
        oe.reset_random(maps if shared else maps[b])
        oracles.append(oe)
    st = env.get_state()
    for b in range(B):
        p, g = oracles[b].agents()
        np.testing.assert_array_equal(st["pos"][b], p)
        np.testing.assert_array_equal(st["goal"][b], g)
        hp = oracles[b].human_path()
        np.testing.assert_array_equal(st["human_path"][b, :len(hp)], hp)
    checked_obs = 0
    RT = 1 if path == "inplace1" else 23      # rollout paths: steps per mapf_rollout_random call
    roll = None
    T = 0
    for t in range(case["steps"]):
        compare = True
        if rolling:
            if t % RT == 0:
                T = min(RT, case["steps"] - t)
                k = T if path == "rollout" else 1          # in place: one [B]-leading set of buffers
                roll = dict(actions=torch.full((k, B, n), -9, dtype=torch.int32, device=env.device),
                            obs=torch.full((k, B, n, nch, fov, fov), float("nan"), device=env.device),
                            vec=torch.full((k, B, n, 4), float("nan"), device=env.device),
                            out={key: torch.full((k,) + tuple(v.shape), -7, dtype=v.dtype, device=env.device)
                                 for key, v in env.out.items()})
                env.rollout_random(T, slots=path == "rollout", **roll)
                roll = dict(actions=roll["actions"].cpu().numpy(), obs=roll["obs"], vec=roll["vec"],
                            out=host(roll["out"]))
            k = t % RT if path == "rollout" else 0
            compare = path == "rollout" or t % RT == T - 1
            a_host = roll["actions"][k]
            out = {key: v[k] for key, v in roll["out"].items()}
            obs, vec = roll["obs"][k], roll["vec"][k]
        elif path == "fused":
            acts = env.actions
            env.obs.fill_(float("nan"))     # every float of the observation must be written by the launch
            env.vec.fill_(float("nan"))
            out, obs, vec = env.step_observe(acts, random_policy=True)
            out = host(out)
            a_host = acts.cpu().numpy()
        elif path == "random":   # mapf_step_random: actions drawn inside the step kernel
            acts = env.actions
            out = host(env.step_random(acts))
            a_host = acts.cpu().numpy()
            obs, vec = env.observe()
        else:
            acts = env.random_actions()
            a_host = acts.cpu().numpy()
            out = host(env.step(acts))
            obs, vec = env.observe()
        if not compare:                           # in place, inside a launch: the oracle steps on its own
            for oe in oracles:
                oe.step(oe.random_actions())
            continue
        obs, vec = obs.cpu().numpy(), vec.cpu().numpy()
        for b in range(B):
            oe = oracles[b]
            np.testing.assert_array_equal(a_host[b], oe.random_actions(), err_msg=f"{name} actions t={t} b={b}")
            o = oe.step(a_host[b])
            for k, key in [("status", "status"), ("reward", "reward"), ("cost", "cost"), ("train_valid", "valid"),
                           ("actions_fixed", "fixed"), ("goals_reached", "goals"), ("constraints", "constr")]:
                np.testing.assert_array_equal(out[k][b], o[key].astype(out[k].dtype), err_msg=f"{name} t={t} b={b} {k}")
            assert out["shadow_goals"][b] == o["shadow"]
            if b % 4 == t % 4 or path in ("inplace", "inplace1"):
                oo, ov = oe.observe()
                np.testing.assert_array_equal(obs[b], oo, err_msg=f"{name} t={t} b={b} obs")
                np.testing.assert_array_equal(vec[b], ov, err_msg=f"{name} t={t} b={b} vec")
                checked_obs += 1
        # device state after the step (rollout paths: only at the end of a call's T steps)
        if (t % 20 == 19) if not rolling else (t % RT == T - 1):
            st = env.get_state()
            bfs = env.bfs().cpu().numpy()
            for b in range(B):
                p, g = oracles[b].agents()
                np.testing.assert_array_equal(st["pos"][b], p)
                np.testing.assert_array_equal(st["goal"][b], g)
                h = oracles[b].human()
                np.testing.assert_array_equal(st["human"][b, 0:2], h["pos"])
                np.testing.assert_array_equal(st["human"][b, 4:6], h["goal"])
                np.testing.assert_array_equal(bfs[b], oracles[b].bfs())
    assert checked_obs > 0
    allow = case.get("allow", ())
    assert_no_errors(env, allow=allow)
    if rolling:       # this instantiation is now oracle-compared (tests/test_gpu_ycoverage.py)
        record_rollout_kernel(kname, f"{name} {path} vs oracle")
    if allow:   # the oracle counts the same events
        assert int(env.counters()[:8].sum()) == sum(oe.errors() for oe in oracles)
        fix = np.sum([oe.fix_counts() for oe in oracles], axis=0)
        assert (int(env.counters()[2]), int(env.counters()[1])) == tuple(int(x) for x in fix)
        assert fix[1] >= case.get("min_deadlocks", 0)
    else:
        for oe in oracles:
            assert oe.errors() == 0


# ---------------------------------------------------------------- full-size c5
def c5_maps(count, seed=1234):
    """c5's maps: 80x80, p = 0.3 (random_generator's rule), largest 4-connected component."""
    from mapf_amd.maps import keep_largest_component, random_map
    rng = np.random.default_rng(seed)
    return np.stack([keep_largest_component(random_map(rng, 80, 80, 0.3)) for _ in range(count)])


def test_c5_full_size_invariants_and_sampled_oracle():
    """BASELINE config c5 per GPU (2048 envs x 64 agents, 80x80 random maps, FOV 11,
    BFS channel): agents on free cells and pairwise distinct in every env after
    every step, legal statuses, sampled envs bit-exact vs the oracle (step outputs,
    observations incl. the BFS channel), and the fixActions counters equal to the
    oracle's on those envs."""
    B, n, H, W, fov, C = 2048, 64, 80, 80, 11, 7
    maps = c5_maps(B)
    env = mk_env(B=B, H=H, W=W, num_agents=n, fov=fov, num_channel=C, human_mode="random", goal_mode="random",
                 fix_choice=1, shared_map=False, seed=1234)
    env.reset_seeded(maps)
    cfg = O.make_config(H, W, n, fov, C, human_mode=1, goal_mode=1, fix_choice=1, seed=1234)
    sample = [0, 1, 777, 2047]
    oracles = {b: O.OracleEnv(cfg, env_id=b) for b in sample}
    for b, oe in oracles.items():
        oe.reset_random(maps[b])
    free = maps == 0
    bidx = np.arange(B)[:, None]
    for t in range(30):
        acts = env.random_actions()
        a_host = acts.cpu().numpy()
        out = host(env.step(acts))
        obs, vec = env.observe()
        pos = env.get_state()["pos"]
        assert free[bidx, pos[..., 0], pos[..., 1]].all(), f"t={t}: agent off the free cells"
        srt = np.sort(pos[..., 0] * W + pos[..., 1], axis=1)
        assert (np.diff(srt, axis=1) > 0).all(), f"t={t}: two agents share a cell"
        assert np.isin(out["status"], [1, -1, -2, -3, -4]).all()
        for b, oe in oracles.items():
            r = oe.step(a_host[b])
            np.testing.assert_array_equal(out["status"][b], r["status"], err_msg=f"t={t} b={b}")
            np.testing.assert_array_equal(out["actions_fixed"][b], r["fixed"], err_msg=f"t={t} b={b}")
            np.testing.assert_array_equal(out["train_valid"][b], r["valid"], err_msg=f"t={t} b={b}")
            if b == sample[t % len(sample)]:
                oo, ov = oe.observe()
                np.testing.assert_array_equal(obs[b].cpu().numpy(), oo, err_msg=f"t={t} b={b} obs")
                np.testing.assert_array_equal(vec[b].cpu().numpy(), ov, err_msg=f"t={t} b={b} vec")
    assert_no_errors(env, allow=(1, 2))
    for oe in oracles.values():
        assert oe.errors() == sum(oe.fix_counts())


# fixActions deadlocks found by the oracle on c5's maps (c5_maps, seed 1234): env id ->
# steps to run past it.  An agent pushed by the human into a dead end held by another
# agent: each one's only viable actions evict the other, and the reference's while
# loop (mapf_gym.py:563) never ends.
DEADLOCK_ENVS = {512: 470, 763: 920, 1081: 800, 1862: 380}


def test_fix_deadlocks_match_oracle():
    """Through the deadlocks: the device declares them where the oracle does (after
    fix_draws(N) draws), resolves them to the same conflict-free moves (unplaced agents
    stay, blocked movers revert), and agents stay on distinct free cells."""
    maps = c5_maps(max(DEADLOCK_ENVS) + 1)
    H = W = 80
    n = 64
    for b, T in DEADLOCK_ENVS.items():
        env = mk_env(B=1, H=H, W=W, num_agents=n, fov=11, num_channel=6, human_mode="random", goal_mode="random",
                     fix_choice=1, shared_map=False, keep_bfs=False, seed=1234, env_offset=b)
        env.reset_seeded(maps[b:b + 1])
        oe = O.OracleEnv(O.make_config(H, W, n, 11, 6, human_mode=1, goal_mode=1, fix_choice=1, keep_bfs=0,
                                       seed=1234), env_id=b)
        oe.reset_random(maps[b])
        free = maps[b] == 0
        for t in range(T):
            acts = env.random_actions()
            a_host = acts.cpu().numpy()[0]
            out = host(env.step(acts))
            r = oe.step(a_host)
            np.testing.assert_array_equal(out["status"][0], r["status"], err_msg=f"env {b} t={t}")
            np.testing.assert_array_equal(out["actions_fixed"][0], r["fixed"], err_msg=f"env {b} t={t}")
            pos = env.get_state()["pos"][0]
            assert free[pos[:, 0], pos[:, 1]].all()
            assert len(np.unique(pos[:, 0] * W + pos[:, 1])) == n, f"env {b} t={t}: shared cell"
        p, _ = oe.agents()
        np.testing.assert_array_equal(env.get_state()["pos"][0], p)
        empty, deadlocks = oe.fix_counts()
        assert deadlocks >= 1, f"env {b}: the oracle saw no deadlock"
        c = env.counters()
        assert (int(c[1]), int(c[2])) == (deadlocks, empty), f"env {b}: counters {c[:3]}"
        env.close()


# ---------------------------------------------------------------- full-size c2
def test_c2_full_size_invariants_and_sampled_oracle():
    """BASELINE config c2 (4096 envs x 8 agents, 20x20, FOV 11): size-independent
    invariants on every env + bit-exact oracle replays of sampled envs."""
    from mapf_amd.maps import generate_warehouse
    B, n, H, W, fov = 4096, 8, 20, 20, 11
    world = generate_warehouse(H, W)
    env = mk_env(B=B, H=H, W=W, num_agents=n, fov=fov, num_channel=6, human_mode="random", goal_mode="random",
                 fix_choice=1, seed=1234)
    env.reset_seeded(world)
    cfg = O.make_config(H, W, n, fov, 6, human_mode=1, goal_mode=1, fix_choice=1, seed=1234)
    sample = [0, 1, 63, 64, 2047, 4095]
    oracles = {b: O.OracleEnv(cfg, env_id=b) for b in sample}
    for b, oe in oracles.items():
        oe.reset_random(world)
    free = world == 0
    for t in range(60):
        acts = env.random_actions()
        a_host = acts.cpu().numpy()
        out = host(env.step(acts))
        obs, vec = env.observe()
        st = env.get_state()
        pos = st["pos"]
        # invariants: agents on free cells, pairwise distinct, statuses legal, fixed moves legal
        assert free[pos[..., 0], pos[..., 1]].all()
        flat = pos[..., 0] * W + pos[..., 1]
        srt = np.sort(flat, axis=1)
        assert (np.diff(srt, axis=1) > 0).all()
        assert np.isin(out["status"], [1, -1, -2, -3, -4]).all()
        if t % 10 == 0:
            o = obs.cpu().numpy()
            c = fov // 2
            assert (o[:, :, 0, c, c] == 1).all()                  # self marked in ch0
            assert ((o == 0) | (o == 1)).all()
        for b, oe in oracles.items():
            r = oe.step(a_host[b])
            np.testing.assert_array_equal(out["status"][b], r["status"])
            np.testing.assert_array_equal(out["actions_fixed"][b], r["fixed"])
            np.testing.assert_array_equal(out["train_valid"][b], r["valid"])
            oo, ov = oe.observe()
            np.testing.assert_array_equal(obs[b].cpu().numpy(), oo)
            np.testing.assert_array_equal(vec[b].cpu().numpy(), ov)
    assert_no_errors(env)


def test_c2_full_size_fused_equals_two_launches():
    """c2 at full size: mapf_step_observe (one launch) and mapf_step + mapf_observe on
    two envs with the same seed give identical outputs, observations and state."""
    from mapf_amd.maps import generate_warehouse
    B, n, H, W, fov = 4096, 8, 20, 20, 11
    world = generate_warehouse(H, W)
    envs = []
    for _ in range(2):
        e = mk_env(B=B, H=H, W=W, num_agents=n, fov=fov, num_channel=6, human_mode="random", goal_mode="random",
                   fix_choice=1, seed=99)
        e.reset_seeded(world)
        envs.append(e)
    fz, pl = envs
    for t in range(90):
        fz.obs.fill_(float("nan"))          # the fused launch (incl. its zero-band workgroups) writes every float
        out_f, obs_f, vec_f = fz.step_observe(fz.actions, random_policy=True)
        out_f = host(out_f)
        out_p = host(pl.step_random(pl.actions))
        obs_p, vec_p = pl.observe()
        np.testing.assert_array_equal(fz.actions.cpu().numpy(), pl.actions.cpu().numpy())
        for k in out_p:
            np.testing.assert_array_equal(out_f[k], out_p[k], err_msg=f"t={t} {k}")
        assert torch.equal(obs_f, obs_p) and torch.equal(vec_f, vec_p), f"t={t} obs"
        if t % 30 == 29:
            sf, sp = fz.get_state(), pl.get_state()
            for k in sp:
                np.testing.assert_array_equal(sf[k], sp[k], err_msg=f"t={t} state {k}")
            assert torch.equal(fz.bfs(), pl.bfs())
    assert_no_errors(fz)
    assert_no_errors(pl)


# BASELINE configs at full per-GPU size: (B, N, H=W, FOV, C, shared warehouse?, rollout kernel, T per call)
FULL_ROLLOUT = {"c2": (4096, 8, 20, 11, 6, True, 1, (1, 31, 45)),
                "c4": (1024, 16, 40, 9, 6, True, 2, (1, 31, 45)),
                "c5": (2048, 64, 80, 11, 7, False, 2, (1, 9, 23))}


@pytest.mark.parametrize("cfg,slots", [("c2", True), ("c2", False), ("c4", True), ("c4", False), ("c5", True),
                                       ("c5", False)])
def test_full_size_rollout_equals_step_observe(cfg, slots):
    """c2 / c4 / c5 at full size: mapf_rollout_random (one launch of T steps) and T
    launches of mapf_step_observe_random on two envs with the same seed give identical
    actions, outputs, observations, state and BFS maps (slots: every step's; else the
    last).  c2 runs the pair-lane kernel, c4 and c5 (16 / 64 agents, c5 with per-env
    80x80 maps and the BFS channel) the one-wave-per-env kernel."""
    from mapf_amd.maps import generate_warehouse
    B, n, H, fov, C, shared, kind, Ts = FULL_ROLLOUT[cfg]
    W = H
    world = generate_warehouse(H, W) if shared else c5_maps(B)
    envs = []
    for _ in range(2):
        e = mk_env(B=B, H=H, W=W, num_agents=n, fov=fov, num_channel=C, human_mode="random", goal_mode="random",
                   fix_choice=1, seed=4321, shared_map=shared)
        e.reset_seeded(world)
        envs.append(e)
    ro, so = envs
    assert ro.rollout_kernel == kind
    for _ in range(3):                       # a step_observe first: pending search work is flushed
        ro.step_observe(random_policy=True)
        so.step_observe(random_policy=True)
    for T in Ts:
        k = T if slots else 1
        dev = ro.device
        acts = torch.zeros(k, B, n, dtype=torch.int32, device=dev)
        obs = torch.full((k, B, n, C, fov, fov), float("nan"), device=dev)
        vec = torch.full((k, B, n, 4), float("nan"), device=dev)
        out = {key: torch.full((k,) + tuple(v.shape), -7, dtype=v.dtype, device=dev) for key, v in ro.out.items()}
        ro.rollout_random(T, slots=slots, actions=acts, obs=obs, vec=vec, out=out)
        out = host(out)
        for t in range(T):
            o_s, obs_s, vec_s = so.step_observe(random_policy=True)
            if slots or t == T - 1:
                j = t if slots else 0
                np.testing.assert_array_equal(acts[j].cpu().numpy(), so.actions.cpu().numpy(), err_msg=f"T={T} t={t}")
                o_s = host(o_s)
                for key in o_s:
                    np.testing.assert_array_equal(out[key][j], o_s[key], err_msg=f"T={T} t={t} {key}")
                assert torch.equal(obs[j], obs_s) and torch.equal(vec[j], vec_s), f"T={T} t={t} obs"
        sr, ss = ro.get_state(), so.get_state()
        for key in ss:
            np.testing.assert_array_equal(sr[key], ss[key], err_msg=f"T={T} state {key}")
        assert torch.equal(ro.bfs(), so.bfs()), f"T={T} bfs"
    allow = (1, 2) if cfg == "c5" else ()     # c5: the states the reference does not survive
    assert_no_errors(ro, allow=allow)
    assert_no_errors(so, allow=allow)
    assert (ro.counters()[:8] == so.counters()[:8]).all()
    # equal to the per-step launches, which the oracle-compared cases pin
    record_rollout_kernel(ro.rollout_kernel_name(slots), f"full-size {cfg} slots={slots} == step_observe")


# --------------------------------------------------------------- GAE / normalise
def test_gae_bit_exact_vs_golden():
    from mapf_amd.env import gae
    z = load("g4_gae")
    for r, v, lv, want in [("rewards", "values", "last_v", "returns"),
                           ("cost_rewards", "cost_values", "last_cv", "cost_returns")]:
        adv, ret = gae(torch.from_numpy(z[r]).cuda(), torch.from_numpy(z[v]).cuda(), torch.from_numpy(z[lv]).cuda(),
                       float(z["gamma"]), float(z["lam"]))
        np.testing.assert_array_equal(ret.cpu().numpy(), z[want])


def test_gae_large_matches_oracle():
    from mapf_amd.env import gae
    g = np.random.default_rng(1)
    T, M = 256, 4096 * 8
    r = g.normal(size=(T, M)).astype(np.float32)
    v = g.normal(size=(T, M)).astype(np.float32)
    lv = g.normal(size=M).astype(np.float32)
    adv, ret = gae(torch.from_numpy(r).cuda(), torch.from_numpy(v).cuda(), torch.from_numpy(lv).cuda())
    cols = g.choice(M, 64, replace=False)
    oa, orr = O.gae(r[:, cols], v[:, cols], lv[cols])
    np.testing.assert_array_equal(adv.cpu().numpy()[:, cols], oa)
    np.testing.assert_array_equal(ret.cpu().numpy()[:, cols], orr)


def test_normalize_advantages_vs_torch():
    from mapf_amd.env import normalize_advantages
    z = load("g4_gae")
    x = torch.from_numpy(z["norm_x"]).cuda()
    y = torch.from_numpy(z["norm_y"]).cuda()
    zero = torch.zeros_like(x)
    adv, cadv = normalize_advantages(x, zero, y, zero, lagrange=float(z["norm_lam"]), mix=True)
    np.testing.assert_allclose(cadv.cpu().numpy(), z["norm_cadv"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(adv.cpu().numpy(), z["norm_mixed"], rtol=0, atol=1e-5)
    adv, _ = normalize_advantages(x, zero, y, zero, mix=False)
    np.testing.assert_allclose(adv.cpu().numpy(), z["norm_adv"], rtol=0, atol=1e-5)


def test_sample_actions_distribution():
    from mapf_amd.env import sample_actions
    M = 200000
    p = torch.tensor([0.1, 0.2, 0.3, 0.15, 0.25]).cuda().expand(M, 5).contiguous()
    a = torch.zeros(M, dtype=torch.int32, device="cuda")
    sample_actions(p, 99, 3, out32=a)
    freq = np.bincount(a.cpu().numpy(), minlength=5) / M
    np.testing.assert_allclose(freq, [0.1, 0.2, 0.3, 0.15, 0.25], atol=5e-3)
    b = torch.zeros(M, dtype=torch.int64, device="cuda")
    sample_actions(p, 99, 3, out64=b)
    assert torch.equal(a.long(), b)


def test_vector_every_offset_on_80x80():
    """observe's vector [dx/d, dy/d, d, 0], d = (dx^2 + dy^2) ** .5 in float64
    (mapf_gym.py:316-323), for EVERY goal offset (dx, dy) in [0, 79]^2 of an
    80x80 grid: the device's fp64 sqrt + divides must equal Python's pow / divide
    bit for bit (the kernel has no distance table)."""
    B, N, H = 100, 64, 80
    env = mk_env(B=B, H=H, W=H, num_agents=N, fov=11, num_channel=6, human_mode="looping", goal_mode="random",
                 fix_choice=1, shared_map=True, seed=3, keep_bfs=False)
    env.reset_seeded(np.zeros((H, H), np.int8))
    idx = np.arange(B * N)
    dx, dy = idx // H, idx % H
    pos = np.zeros((B, N, 2), np.int32)
    goal = np.stack([dx, dy], -1).reshape(B, N, 2).astype(np.int32)
    env.set_state(pos=pos, goal=goal)
    _, vec = env.observe()
    got = vec.cpu().numpy().reshape(-1, 4)
    want = np.zeros_like(got)
    for k in range(B * N):
        d2 = int(dx[k]) ** 2 + int(dy[k]) ** 2
        if d2:
            d = d2 ** .5
            want[k] = [np.float32(dx[k] / d), np.float32(dy[k] / d), np.float32(d), 0.0]
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("name,B,H,n,fov,nch,steps", [("c4_split_40x40_n16", 48, 40, 16, 9, 6, 80),
                                                      ("c5_split_80x80_n64_bfsch", 4, 80, 64, 11, 7, 40)])
def test_split_path_back_to_back_steps_match_oracle(name, B, H, n, fov, nch, steps):
    """The per-step split path (step launch, then observe with the step's search forked onto
    aux streams; the humans' next paths joined only two steps later, mapf_api.cpp
    join_deferred) driven back to back with NO host synchronisation, get_state or bfs in
    between -- every step's outputs and observation into [T]-slot device buffers -- so each
    deferred search really runs beside the next step.  Compared with the oracle at the end."""
    rng = np.random.default_rng(11)
    from mapf_amd.maps import keep_largest_component, random_map
    maps = np.stack([keep_largest_component(random_map(rng, H, H, 0.3)) for _ in range(B)])
    seed = 0xD0F + B
    env = mk_env(B=B, H=H, W=H, num_agents=n, fov=fov, num_channel=nch, human_mode="random", goal_mode="random",
                 fix_choice=1, shared_map=False, seed=seed, env_offset=3)
    env.reset_seeded(maps)
    assert not env.fused, "expected the split (step + observe) path"
    dev = env.device
    acts = torch.zeros(steps, B, n, dtype=torch.int32, device=dev)
    obs = torch.full((steps, B, n, nch, fov, fov), float("nan"), device=dev)
    vec = torch.full((steps, B, n, 4), float("nan"), device=dev)
    outs = {k: torch.zeros((steps,) + tuple(v.shape), dtype=v.dtype, device=dev) for k, v in env.out.items()}
    for t in range(steps):
        env.step_observe(acts[t], obs[t], vec[t], random_policy=True, out={k: v[t] for k, v in outs.items()})
    torch.cuda.synchronize()
    acts, obs, vec, outs = acts.cpu().numpy(), obs.cpu().numpy(), vec.cpu().numpy(), host(outs)
    cfg = O.make_config(H, H, n, fov, nch, human_mode=1, goal_mode=1, fix_choice=1, seed=seed, env_offset=3)
    for b in range(B):
        oe = O.OracleEnv(cfg, env_id=3 + b)
        oe.reset_random(maps[b])
        for t in range(steps):
            np.testing.assert_array_equal(acts[t, b], oe.random_actions(), err_msg=f"{name} actions t={t} b={b}")
            o = oe.step(acts[t, b])
            for k, key in [("status", "status"), ("reward", "reward"), ("cost", "cost"), ("train_valid", "valid"),
                           ("actions_fixed", "fixed"), ("goals_reached", "goals"), ("constraints", "constr")]:
                np.testing.assert_array_equal(outs[k][t, b], o[key].astype(outs[k].dtype),
                                              err_msg=f"{name} t={t} b={b} {k}")
            oo, ov = oe.observe()
            np.testing.assert_array_equal(obs[t, b], oo, err_msg=f"{name} t={t} b={b} obs")
            np.testing.assert_array_equal(vec[t, b], ov, err_msg=f"{name} t={t} b={b} vec")
    assert_no_errors(env, allow=(1, 2))
