"""Generate the golden fixtures under tests/golden/ from the reference itself.

Run in the build container (the only place /root/reference exists):

    python tests/golden/make_golden.py

The reference (Nielsencu/primal-ppo, /root/reference) is imported with its
off-path modules stubbed: skimage, cv2, imageio, wandb,
setproctitle and ray.  Nothing from the reference is copied: this script
drives the reference's own classes and records inputs and outputs as .npz
data.  The committed fixtures are data only.

Fixtures
  g1_*.npz   scripted FixedMapfGym episodes (LoopingHuman / FixedPathHuman),
             recorded per step in runner.py:64-100 order.  random.choice in
             fixActions is patched to a rotating deterministic pick (see
             rotating_choice); the oracle's fix_choice=0 rule.
  g2_fuzz.npz  thousands of one-step scenarios on small dense maps (conflict
             resolution, -3 overwrites, fixActions eviction, FOV edges).
  g3_search.npz  astar_4 paths and makeBfsMap outputs.
  g4_gae.npz  Runner.run GAE (runner.py:117-149) on a short rollout.
  g8_render.npz  renderWorld's colours and shape vertices (util.py:88-187).
"""
import copy
import json
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def import_reference():
    for name in ["skimage", "skimage.measure", "skimage.morphology", "cv2", "imageio",
                 "wandb", "setproctitle"]:
        sys.modules.setdefault(name, types.ModuleType(name))
    ray = types.ModuleType("ray")
    ray.remote = lambda *a, **k: (lambda c: c)
    sys.modules["ray"] = ray
    sys.path.insert(0, REF)
    import alg_parameters, astar_4, map_generator, mapf_gym, util  # noqa: E401
    return alg_parameters, astar_4, map_generator, mapf_gym, util


alg, astar_mod, mapgen, mg, util = import_reference()
CHOICE_HITS = [0]
ROUND = [0]
EVICT_LOG = []   # per random.choice in fixActions: the agents its pick evicts, in the reference's order


def rotating_choice(seq):
    """Deterministic stand-in for random.choice in fixActions (mapf_gym.py:588):
    the k-th draw inside one fixActions call takes seq[k % len(seq)] (the
    oracle's fix_choice=0 rule).  A literal seq[0] can cycle forever."""
    CHOICE_HITS[0] += 1
    k = ROUND[0]
    ROUND[0] += 1
    if k > 1000:
        raise RuntimeError("fixActions did not terminate")
    choice = seq[k % len(seq)]
    # record what the pick will evict: the same set expression fixActions
    # evaluates next (mapf_gym.py:590-591), read from its frame
    f = sys._getframe(1).f_locals
    agent, pairs = f.get("agent"), f.get("agentActionPairs")
    if agent is not None and pairs is not None and choice in agent.restrictedAction:
        conf = [x for x in set(tuple(x) for x in pairs) & set(tuple(x) for x in np.array(agent.restrictedAction[choice]))]
        EVICT_LOG.append([int(x[0]) for x in conf])
    return choice


mg.random.choice = rotating_choice


def set_params(n_agents, fov):
    alg.EnvParameters.N_AGENTS = n_agents
    alg.EnvParameters.FOV_SIZE = fov


def warehouse(h, w):
    """generateWarehouse (map_generator.py:127-138) with breadth = w."""
    # drive the reference generator itself with length=h; then re-derive the
    # breadth-w variant used by the benchmark configs.
    world = mapgen.generateWarehouse(num_block=[-1, -1], length=h, lbRatio=h / (w + 1e-9))
    assert world.shape == (h, w), world.shape
    return world


def free_cells(world):
    return [tuple(x) for x in np.argwhere(world == 0).tolist()]


def make_sequences(rng, world, n, n_goals, human_start):
    temp = world.copy()
    temp[human_start] = 1
    seqs = []
    free = free_cells(temp)
    starts = []
    for i in range(n):
        cand = [c for c in free if temp[c] == 0]
        s = cand[rng.integers(len(cand))]
        temp[s] = 2
        starts.append(s)
        seqs.append([s])
    allfree = free_cells(world)
    for i in range(n):
        for k in range(n_goals):
            while True:
                g = allfree[rng.integers(len(allfree))]
                if g != seqs[i][-1]:
                    break
            seqs[i].append(g)
    return seqs


def greedy_actions(rng, env, n, p_greedy):
    acts = np.zeros(n)
    for i, ag in enumerate(env.agentList):
        if rng.random() < p_greedy and len(ag.bfsMap) > 0:
            pos = ag.getPos()
            best, bestd = [], None
            for a in range(5):
                d = mg.Agent.dirDict[a]
                r, c = pos[0] + d[0], pos[1] + d[1]
                if 0 <= r < ag.bfsMap.shape[0] and 0 <= c < ag.bfsMap.shape[1] and ag.bfsMap[r, c] >= 0:
                    if bestd is None or ag.bfsMap[r, c] < bestd:
                        best, bestd = [a], ag.bfsMap[r, c]
                    elif ag.bfsMap[r, c] == bestd:
                        best.append(a)
            acts[i] = best[rng.integers(len(best))] if best else rng.integers(5)
        else:
            acts[i] = rng.integers(5)
    return acts


PERF = {}        # g1 episode -> the reference's OneEpPerformance counters after every step (g1_perf.npz)
PERF_FIELDS = ["staticCollide", "humanCollide", "agentCollide", "shadowGoals", "episodeReward", "episodeCostReward",
               "totalGoals", "constraintViolations"]


def run_episode(name, world, n, fov, nch, steps, seed, use_da=False, use_hp=False,
                human_seq=None, n_goals=60, p_greedy=0.6, save=True):
    set_params(n, fov)
    rng = np.random.default_rng(seed)
    free = free_cells(world)
    edge = [c for c in free if c[0] == 0 or c[1] == 0]
    hs = edge[rng.integers(len(edge))]
    while True:
        hg = free[rng.integers(len(free))]
        if hg != hs:
            break
    seqs = make_sequences(rng, world, n, n_goals, hs)
    agentsSequence = [util.Sequence(itemsIn=[tuple(map(int, c)) for c in s]) for s in seqs]
    hseq_in = None
    if human_seq is not None:
        hseq_in = [hs] + [free[rng.integers(len(free))] for _ in range(human_seq)]
        # consecutive poses must differ (astar of start==goal returns [])
        for k in range(1, len(hseq_in)):
            while hseq_in[k] == hseq_in[k - 1]:
                hseq_in[k] = free[rng.integers(len(free))]
    env = mg.FixedMapfGym(world, agentsSequence, tuple(map(int, hs)), tuple(map(int, hg)), numChannel=nch,
                          useDA=use_da, useHP=use_hp, humanSequence=hseq_in)
    fixed_log = []
    orig_fix = env.fixActions

    def fix_wrap(actions, st):
        ROUND[0] = 0
        out = orig_fix(actions, st)
        fixed_log.append(np.array(out, dtype=np.int64))
        return out

    env.fixActions = fix_wrap
    rec = {k: [] for k in ["actions", "status", "reward", "shadow", "cost", "valid", "fixed",
                           "goals", "constr", "pos", "goal", "hpos", "hnext", "obs", "vec"]}
    obs0, vec0 = env.getAllObservations()
    init = dict(
        pos0=np.array([a.getPos() for a in env.agentList]), goal0=np.array([a.getGoal() for a in env.agentList]),
        hpath0=np.array(env.human.path), obs0=np.packbits(obs0.astype(np.uint8)), vec0=vec0,
        bfs0=np.array([a.bfsMap for a in env.agentList]).astype(np.int16))
    choice0 = CHOICE_HITS[0]
    # runner.py:66-99's counter loop, statement for statement, with the reference's own class
    # (util.OneEpPerformance) over this episode's steps; a copy of the rewards takes the
    # GOAL_REWARD additions (rec keeps calculateActionReward's values)
    oneEpisodePerformance = util.OneEpPerformance()
    perf_log = {k: [] for k in PERF_FIELDS}
    perf_types = {}
    for t in range(steps):
        actions = greedy_actions(rng, env, n, p_greedy)
        pos_before = np.array([a.getPos() for a in env.agentList])
        st = env.getActionStatus(actions)
        rw, sh = env.calculateActionReward(actions, st)
        cost = env.calculateCostReward(actions)
        tv = env.getTrainValid(actions)
        nfix = len(fixed_log)
        goals, constr = env.jointStep(actions, st)
        fixed = fixed_log[-1] if len(fixed_log) > nfix else actions.astype(np.int64)
        pos_after = np.array([a.getPos() for a in env.agentList])
        # sanity: fixed actions explain the motion
        for i in range(n):
            d = mg.Agent.dirDict[int(fixed[i])]
            assert tuple(pos_before[i] + np.array(d)) == tuple(pos_after[i])
        actionStatus, rewards, shadowGoals, costRewards = st, rw.copy(), sh, cost
        goalsReached, constraintsViolated = goals, constr
        for value in actionStatus:
            if value == -1:
                oneEpisodePerformance.staticCollide += 1
            elif value == -2:
                oneEpisodePerformance.humanCollide += 1
            elif value == -3:
                oneEpisodePerformance.agentCollide += 1
        oneEpisodePerformance.shadowGoals += shadowGoals
        for i, value in enumerate(goalsReached):
            if (value == 1):
                rewards[0, i] += alg.EnvParameters.GOAL_REWARD
        oneEpisodePerformance.episodeReward += np.sum(rewards)
        oneEpisodePerformance.episodeCostReward += np.sum(costRewards)
        oneEpisodePerformance.totalGoals += np.sum(goalsReached)
        oneEpisodePerformance.constraintViolations += np.sum(constraintsViolated)
        for k in PERF_FIELDS:
            v = getattr(oneEpisodePerformance, k)
            perf_log[k].append(float(v))
            perf_types[k] = type(v).__name__
        obs, vec = env.getAllObservations()
        rec["actions"].append(actions.astype(np.int64)); rec["status"].append(st.astype(np.int8))
        rec["reward"].append(rw[0]); rec["shadow"].append(sh); rec["cost"].append(cost[0])
        rec["valid"].append(tv); rec["fixed"].append(fixed); rec["goals"].append(goals.astype(np.float32))
        rec["constr"].append(constraints_f32(constr)); rec["pos"].append(pos_after)
        rec["goal"].append(np.array([a.getGoal() for a in env.agentList]))
        rec["hpos"].append(np.array(env.human.getPos())); rec["hnext"].append(np.array(env.human.getNextPos()))
        rec["obs"].append(np.packbits(obs.astype(np.uint8))); rec["vec"].append(vec[0])
    final_bfs = np.array([a.bfsMap for a in env.agentList]).astype(np.int16)
    S = max(len(s) for s in seqs)
    seq_arr = np.zeros((n, S, 2), np.int32)
    seq_len = np.array([len(s) for s in seqs], np.int32)
    for i, s in enumerate(seqs):
        seq_arr[i, :len(s)] = np.array(s)
    out = {k: np.array(v) for k, v in rec.items()}
    out.update(init)
    out.update(dict(map=world.astype(np.int8), seq=seq_arr, seq_len=seq_len, hstart=np.array(hs),
                    hgoal=np.array(hg), n=n, fov=fov, nch=nch, use_da=int(use_da), use_hp=int(use_hp),
                    human_mode=0 if human_seq is None else 2, bfs_final=final_bfs,
                    hseq=np.array(hseq_in if hseq_in is not None else [hs]), steps=steps,
                    choice_hits=CHOICE_HITS[0] - choice0))
    PERF[name] = {k: np.array(v, np.float64) for k, v in perf_log.items()}
    PERF[name]["types"] = np.array([perf_types[k] for k in PERF_FIELDS])
    if not save:    # g1perf: the episode must be the committed one
        old = np.load(os.path.join(OUT, f"{name}.npz"))
        for k in ("actions", "status", "reward", "shadow", "cost", "goals", "constr", "pos"):
            assert np.array_equal(old[k], out[k]), (name, k)
        return
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **out)
    nfix_total = sum(1 for s in out["status"] if np.any((s < 0) & (s > -4)))
    print(f"{name}: steps={steps} goals={out['goals'].sum():.0f} fixsteps={nfix_total} "
          f"choice_hits={CHOICE_HITS[0] - choice0} statuses={np.unique(out['status'], return_counts=True)}")


def constraints_f32(c):
    return np.asarray(c, dtype=np.float32)


def g2_fuzz(count, seed, name="g2_fuzz", size=(4, 9), density=(0.0, 0.3), agents=(2, 9), keep=None):
    """One-step scenarios on small dense maps.  keep(evictions) selects scenarios by
    the eviction lists their fixActions call produced (None: keep all)."""
    rng = np.random.default_rng(seed)
    recs = []
    skipped = 0
    for sc in range(count):
        H = int(rng.integers(*size)); W = int(rng.integers(*size))
        world = -(rng.random((H, W)) < rng.uniform(*density)).astype(np.int64)
        free = free_cells(world)
        n = int(rng.integers(*agents))
        if len(free) < n + 2:
            skipped += 1
            continue
        fov = int(rng.choice([3, 5, 9, 11]))
        set_params(n, fov)
        perm = rng.permutation(len(free))
        starts = [free[k] for k in perm[:n]]
        goals = [free[k] for k in rng.integers(0, len(free), n)]
        hs = free[perm[n]]
        hg = free[perm[n + 1]]
        if astar_mod.astar_4(world, hs, hg).__class__ is ValueError:
            skipped += 1
            continue
        seqs = [util.Sequence(itemsIn=[s, g, free[int(rng.integers(len(free)))]]) for s, g in zip(starts, goals)]
        use_da = bool(rng.integers(2)); use_hp = bool(rng.integers(2))
        try:
            env = mg.FixedMapfGym(world, seqs, hs, hg, numChannel=6, useDA=use_da, useHP=use_hp)
            # advance the human a random number of steps (exercise step / path end)
            for _ in range(int(rng.integers(0, 6))):
                env.human.nextStep()
            env.getUnconditionallyGoodActions()
            # optional previous action (repeat masks)
            prev = None
            if rng.random() < 0.5:
                prev = rng.integers(0, 5, n)
                for i, ag in enumerate(env.agentList):
                    ag.setInvalidActions(2, [mg.Agent.oppositeAction[int(prev[i])]])
                env.getUnconditionallyGoodActions()
            pos0 = np.array([a.getPos() for a in env.agentList])
            goal0 = np.array([a.getGoal() for a in env.agentList])
            hstep0 = env.human.step
            actions = rng.integers(0, 5, n).astype(np.float64)
            obs0, vec0 = env.getAllObservations()
            fixed_log = []
            orig_fix = env.fixActions

            def fix_wrap(a, s):
                ROUND[0] = 0
                out = orig_fix(a, s)
                fixed_log.append(np.array(out, dtype=np.int64))
                return out
            env.fixActions = fix_wrap
            c0 = CHOICE_HITS[0]
            e0 = len(EVICT_LOG)
            st = env.getActionStatus(actions)
            rw, sh = env.calculateActionReward(actions, st)
            cost = env.calculateCostReward(actions)
            tv = env.getTrainValid(actions)
            gr, cv = env.jointStep(actions, st)
            fixed = fixed_log[-1] if fixed_log else actions.astype(np.int64)
            obs1, vec1 = env.getAllObservations()
        except Exception:
            skipped += 1
            continue
        if keep is not None and not keep(EVICT_LOG[e0:]):
            continue
        recs.append(dict(H=H, W=W, n=n, fov=fov, map=world.astype(np.int8).ravel(), pos0=pos0, goal0=goal0,
                         seq=np.array([s.items for s in seqs]), hpath=np.array(env.human.path), hstep0=hstep0,
                         prev=(-1 if prev is None else prev), actions=actions.astype(np.int64),
                         use_da=int(use_da), use_hp=int(use_hp),
                         obs0=np.packbits(obs0.astype(np.uint8)), vec0=vec0[0], status=st.astype(np.int8),
                         reward=rw[0], shadow=sh, cost=cost[0], valid=tv, fixed=fixed,
                         goals=np.asarray(gr, np.float32), constr=np.asarray(cv, np.float32),
                         pos1=np.array([a.getPos() for a in env.agentList]),
                         goal1=np.array([a.getGoal() for a in env.agentList]),
                         obs1=np.packbits(obs1.astype(np.uint8)), vec1=vec1[0],
                         choice=CHOICE_HITS[0] - c0))
    # ragged -> object-free flat storage: one json index + concatenated arrays
    flat = {}
    keys = [k for k in recs[0].keys()]
    for k in keys:
        arrs = [np.asarray(r[k]) for r in recs]
        flat[k + "__len"] = np.array([a.size for a in arrs])
        flat[k + "__shape"] = json.dumps([list(a.shape) for a in arrs])
        flat[k] = np.concatenate([a.ravel() for a in arrs]) if arrs else np.zeros(0)
    flat["count"] = len(recs)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **flat)
    allst = np.concatenate([r["status"] for r in recs])
    print(f"{name}: {len(recs)} scenarios ({skipped} skipped), statuses {np.unique(allst, return_counts=True)}, "
          f"choice hits {sum(r['choice'] for r in recs)}")


def g3_search(seed):
    rng = np.random.default_rng(seed)
    cases = []
    maps = []
    for h, w in [(10, 10), (20, 20), (12, 18), (40, 40)]:
        maps.append(warehouse(h, w))
    for _ in range(6):
        H = int(rng.integers(6, 30)); W = int(rng.integers(6, 30))
        maps.append(-(rng.random((H, W)) < 0.3).astype(np.int64))
    for _ in range(3):
        H = int(rng.integers(5, 16)); W = int(rng.integers(5, 16))
        maps.append(np.zeros((H, W), np.int64))       # tie-heavy open grids
    for mi, world in enumerate(maps):
        free = free_cells(world)
        for _ in range(25 if world.size <= 900 else 10):
            s = free[rng.integers(len(free))]; g = free[rng.integers(len(free))]
            res = astar_mod.astar_4(world, s, g)
            if isinstance(res, ValueError):
                path = np.zeros((0, 2), np.int64); ok = 0
            else:
                path = np.array(res[0], dtype=np.int64).reshape(-1, 2); ok = 1
            # makeBfsMap from g: drive the reference method on a stub agent
            ag = mg.Agent(); ag.setGoal(g)
            env = mg.MapfGym.__new__(mg.MapfGym); env.obstacleMap = world
            env.makeBfsMap(ag)
            cases.append(dict(mi=mi, s=np.array(s), g=np.array(g), ok=ok, path=path,
                              bfs=ag.bfsMap.astype(np.int16)))
    flat = {"nmaps": len(maps)}
    for i, m in enumerate(maps):
        flat[f"map{i}"] = m.astype(np.int8)
    for k in ["mi", "s", "g", "ok"]:
        flat[k] = np.array([c[k] for c in cases])
    flat["path_len"] = np.array([len(c["path"]) for c in cases])
    flat["path"] = np.concatenate([c["path"] for c in cases]).astype(np.int32)
    flat["bfs"] = np.concatenate([c["bfs"].ravel() for c in cases])
    np.savez_compressed(os.path.join(OUT, "g3_search.npz"), **flat)
    print(f"g3_search: {len(cases)} cases on {len(maps)} maps, {sum(1 for c in cases if not c['ok'])} unreachable")


def g4_gae():
    set_params(2, 9)          # before importing model.py: Model.step binds N_AGENTS as a default
    import torch
    import runner as runner_mod
    import model as model_mod
    alg.TrainingParameters.N_STEPS = 256
    np.random.seed(7); torch.manual_seed(7)
    captured = {}
    orig_value = model_mod.Model.value

    def value_wrap(self, obs, vector, input_state):
        v, cv = orig_value(self, obs, vector, input_state)
        captured["v"], captured["cv"] = v.copy(), cv.copy()
        return v, cv
    model_mod.Model.value = value_wrap
    r = runner_mod.Runner(0)
    weights = r.local_model.network.state_dict()
    mb, perf = r.run(weights)
    model_mod.Model.value = orig_value
    out = dict(rewards=mb.rewards, values=mb.values, cost_rewards=mb.costRewards, cost_values=mb.costValues,
               last_v=np.squeeze(captured["v"]), last_cv=np.squeeze(captured["cv"]), returns=mb.returns,
               cost_returns=mb.costReturns, gamma=alg.TrainingParameters.GAMMA, lam=alg.TrainingParameters.LAM,
               obs_shape=np.array(mb.observations.shape), hidden_shape=np.array(mb.hiddenState.shape),
               valid_shape=np.array(mb.trainValid.shape), ps_shape=np.array(mb.ps.shape),
               actions_dtype=str(mb.actions.dtype))
    # random long GAE stress case through the same runner code path is not
    # reachable without the net; the normalisation vectors use torch ops as
    # written at model.py:106-113.
    g = np.random.default_rng(3)
    x = g.normal(size=(256, 8)).astype(np.float32) * 3 + 1
    y = g.normal(size=(256, 8)).astype(np.float32)
    xt, yt = torch.from_numpy(x), torch.from_numpy(y)
    norm = lambda t: (t - t.mean()) / (t.std() + 1e-6)  # model.py:106
    adv, cadv = norm(xt), norm(yt)
    lam_ = torch.nn.functional.softplus(torch.tensor(1.0)).item()
    mixed = (adv - lam_ * cadv) / (lam_ + 1)
    out.update(norm_x=x, norm_y=y, norm_adv=adv.numpy(), norm_cadv=cadv.numpy(), norm_lam=lam_,
               norm_mixed=mixed.numpy())
    np.savez_compressed(os.path.join(OUT, "g4_gae.npz"), **out)
    print("g4_gae:", {k: np.asarray(v).shape for k, v in out.items() if hasattr(v, 'shape')})


def det_weights(state_dict):
    """Deterministic parameter values from the key names (shared with tests/test_net.py)."""
    import zlib
    out = {}
    for k, v in state_dict.items():
        n = v.numel()
        phase = (zlib.crc32(k.encode()) % 1000) / 1000.0
        x = np.sin(np.arange(n, dtype=np.float64) * 0.37 + phase * 6.283) * 0.05
        out[k] = x.reshape(tuple(v.shape)).astype(np.float32)
    return out


def g5_net():
    """SCRIMPNet forward (net.py:101-155) and Model.train (model.py:78-199) on CPU,
    deterministic weights, dropout disabled (eval mode)."""
    set_params(2, 9)
    import torch
    import net as net_mod
    import model as model_mod
    torch.manual_seed(0)
    ref = net_mod.SCRIMPNet(numChannel=6)
    sd = ref.state_dict()
    keys = sorted(sd.keys())
    w = det_weights(sd)
    ref.load_state_dict({k: torch.from_numpy(w[k]) for k in sd})
    ref.eval()
    g = np.random.default_rng(9)
    obs = (g.random((3, 2, 6, 9, 9)) < 0.2).astype(np.float32)
    vec = g.normal(size=(3, 2, 4)).astype(np.float32)
    with torch.no_grad():
        outs = ref(torch.from_numpy(obs), torch.from_numpy(vec), None)
    names = ["policy", "value", "blocking", "policy_sig", "x", "logits", "cost_value"]
    out = {f"out_{n}": o.numpy() for n, o in zip(names, outs)}
    out.update(obs=obs, vec=vec, keys=np.array(keys), shapes=np.array(json.dumps([list(sd[k].shape) for k in keys])))
    # one PPO-Lagrangian update on a fixed minibatch
    m = model_mod.Model(0, torch.device("cpu"), global_model=True, numChannel=6)
    m.network.load_state_dict({k: torch.from_numpy(w[k]) for k in sd})
    m.network.eval()
    mb = 16
    tr = dict(observation=(g.random((mb, 2, 6, 9, 9)) < 0.2).astype(np.float32),
              vector=g.normal(size=(mb, 2, 4)).astype(np.float32),
              returns=g.normal(size=(mb, 2)).astype(np.float32), cost_returns=g.random((mb, 2)).astype(np.float32),
              old_v=g.normal(size=(mb, 2)).astype(np.float32), old_cv=g.random((mb, 2)).astype(np.float32),
              action=g.integers(0, 5, (mb, 2)).astype(np.int64),
              train_valid=(g.random((mb, 2, 5)) < 0.7).astype(np.float32))
    ps = g.random((mb, 2, 5)).astype(np.float32)
    tr["old_ps"] = ps / ps.sum(-1, keepdims=True)
    hidden = np.zeros((mb, 2, 2, 512), np.float32)
    stats = m.train(tr["observation"], tr["vector"], tr["returns"], tr["cost_returns"], tr["old_v"], tr["old_cv"],
                    tr["action"], tr["old_ps"], hidden, tr["train_valid"], 3.0)
    after = m.network.state_dict()
    probe = ["conv1.weight", "fully_connected_2.bias", "transformer.layers.1.0.fn.fn.to_qkv.weight", "policy_layer.weight"]
    out.update({f"train_{k}": v for k, v in tr.items()})
    out["train_stats"] = np.array([float(np.asarray(x)) for x in stats])
    for k in probe:
        out["after_" + k.replace(".", "_")] = after[k].numpy().reshape(-1)[:2048]
    np.savez_compressed(os.path.join(OUT, "g5_net.npz"), **out)
    print("g5_net: stats", out["train_stats"])


def g6_episodes():
    """The reference's own fixed-episode files (evaluate.py:50-123, generated and
    written by its generateFixedEpisodeInfos / saveFixedEpisodeInfos) plus the
    OneEpPerformance sums of its evaluate() loop (evaluate.py:210-256) on them,
    with recorded uniform actions in place of the policy: LoopingHuman episodes
    without DA/HP, and FixedPathHuman episodes with DA+HP."""
    import evaluate as ev
    folder = os.path.join(OUT, "g6_episodes")
    alg.EvalParameters.EPISODES = 4
    alg.EvalParameters.N_AGENTS = 2
    alg.EvalParameters.MAX_STEPS = 30
    alg.EvalParameters.FIXED_EPISODE_INFOS_PATH = folder
    alg.EnvParameters.WORLD_SIZE = (10, 14)
    set_params(2, 9)
    np.random.seed(61)
    ev.saveFixedEpisodeInfos(ev.generateFixedEpisodeInfos())
    rng = np.random.default_rng(62)
    steps = 80
    out = {}
    for mtype, da, hp in [(0, False, False), (1, True, True)]:
        infos = ev.loadFixedEpisodeInfos()
        acts = np.zeros((4, steps, 2), np.int64)
        metrics = np.zeros((4, 8), np.float64)
        for e in range(4):
            hseq = infos["humanSequence"][e] if mtype == 1 else None
            env = mg.FixedMapfGym(infos["obstacleMap"][e], infos["agentsSequence"][e], infos["humanStart"][e],
                                  infos["humanGoal"][e], numChannel=6, useDA=da, useHP=hp, humanSequence=hseq)
            orig_fix = env.fixActions

            def fix_wrap(actions, st, orig_fix=orig_fix):
                ROUND[0] = 0
                return orig_fix(actions, st)
            env.fixActions = fix_wrap
            perf = util.OneEpPerformance()
            env.getAllObservations()
            for t in range(steps):
                actions = greedy_actions(rng, env, 2, 0.7).astype(np.float64)
                acts[e, t] = actions
                st = env.getActionStatus(actions)
                perf.staticCollide += int(np.sum(st == -1))
                perf.humanCollide += int(np.sum(st == -2))
                perf.agentCollide += int(np.sum(st == -3))
                rewards, shadow = env.calculateActionReward(actions, st)
                cost = env.calculateCostReward(actions)
                perf.shadowGoals += shadow
                goals, constr = env.jointStep(actions, st)
                for i, v in enumerate(goals):
                    if v == 1:
                        rewards[0, i] += alg.EnvParameters.GOAL_REWARD
                perf.episodeReward += np.sum(rewards)
                perf.totalGoals += np.sum(goals)
                perf.episodeCostReward += np.sum(cost)
                perf.constraintViolations += np.sum(constr)
                env.getAllObservations()
            metrics[e] = [perf.episodeReward, perf.episodeCostReward, perf.humanCollide, perf.staticCollide,
                          perf.agentCollide, perf.totalGoals, perf.shadowGoals, perf.constraintViolations]
        out[f"actions_type{mtype}"] = acts.astype(np.int32)
        out[f"metrics_type{mtype}"] = metrics
        print(f"g6 type {mtype}: metrics\n{metrics}")
    np.savez_compressed(os.path.join(folder, "expected.npz"), **out)


def g7_warehouses():
    """generateWarehouse(length=L) (map_generator.py:127-138) for every L of WORLD_SIZE
    (10..40), the map MapfGym() builds once L is drawn (mapf_gym.py:166)."""
    maps = {}
    for L in range(10, 41):
        w = mapgen.generateWarehouse(num_block=[-1, -1], length=L)
        maps[f"L{L}"] = w.astype(np.int8)
    np.savez_compressed(os.path.join(OUT, "g7_warehouses.npz"), **maps)
    print("g7_warehouses:", {k: v.shape for k, v in maps.items()})


def g2_evict():
    """One-step scenarios whose fixActions evicts two agents with one pick
    (mapf_gym.py:588-596): the eviction order is the iteration order of a
    Python set of (agent, action) tuples.  Dense maps, 3..16 agents."""
    g2_fuzz(60000, 22, name="g2_evict", size=(4, 8), density=(0.1, 0.4), agents=(3, 17),
            keep=lambda ev: any(len(x) >= 2 for x in ev))


def g8_render():
    """renderWorld's geometry and colours (util.py:88-187), from the reference functions:
    init_colors for several EnvParameters.N_AGENTS (the float colours and the uint8 they
    become, scene * 255 -> astype('uint8'), :229-230); getArrowPoints in the four directions
    with renderWorld's tailWidth / headWidth (:214); drawStar (diameter = scale, 5 points,
    :211); getRectPoints, getCenter, getTriPoints -- over a grid of cells and scales (renderWorld
    itself forces scale = 20, :199).  cv2's fill is not exercised (absent here)."""
    out = {}
    n_keep = alg.EnvParameters.N_AGENTS
    try:
        for n in (1, 2, 3, 4, 6, 7, 8, 16, 64):
            alg.EnvParameters.N_AGENTS = n
            util.EnvParameters.N_AGENTS = n
            c = util.init_colors()
            keys = [0, -1, -2] + [a + 1 for a in range(n)]
            f = np.array([np.asarray(c[k], dtype=np.float64) for k in keys])
            out[f"colors_f_{n}"] = f
            out[f"colors_u8_{n}"] = (f * 255).astype(np.uint8)
    finally:
        alg.EnvParameters.N_AGENTS = n_keep
        util.EnvParameters.N_AGENTS = n_keep
    coords = np.array([(r, c) for r in (0, 1, 3, 7, 19, 39) for c in (0, 2, 5, 13, 39, 59)], dtype=np.int64)
    scales = np.array([20, 10, 16, 7, 24, 11], dtype=np.int64)
    dirs = np.array([(0, 1), (1, 0), (0, -1), (-1, 0)], dtype=np.int64)
    arrows = np.zeros((len(scales), len(dirs), len(coords), 7, 2), np.int64)
    stars = np.zeros((len(scales), len(coords), 15, 2), np.int64)
    rects = np.zeros((len(scales), len(coords), 4, 2), np.int64)
    tris = np.zeros((len(scales), len(coords), 3, 2), np.int64)
    centers = np.zeros((len(scales), len(coords), 2), np.int64)
    for si, sc in enumerate(scales):
        sc = int(sc)
        for ci, (r, cc) in enumerate(coords):
            coord = (int(r), int(cc))
            for di, d in enumerate(dirs):
                arrows[si, di, ci] = util.getArrowPoints(direction=d, coord=coord, scale=sc, tailWidth=sc / 10,
                                                         headWidth=sc / 2 - 2)
            stars[si, ci] = util.drawStar(coord=coord, scale=sc, diameter=sc, numPoints=5)
            rects[si, ci] = util.getRectPoints(coord=coord, scale=sc)
            tris[si, ci] = util.getTriPoints(coord=coord, scale=sc)
            centers[si, ci] = util.getCenter(coord=coord, scale=sc)
    out.update(coords=coords, scales=scales, dirs=dirs, arrows=arrows, stars=stars, rects=rects, tris=tris,
               centers=centers)
    np.savez_compressed(os.path.join(OUT, "g8_render.npz"), **out)
    print("g8_render:", {k: v.shape for k, v in out.items() if not k.startswith("colors")})


def g1_episodes(save=True):
    run_episode("g1_c1", warehouse(10, 10), 4, 11, 6, 200, 11, save=save)
    run_episode("g1_c2", warehouse(20, 20), 8, 11, 6, 200, 12, save=save)
    run_episode("g1_f9", warehouse(20, 20), 8, 9, 6, 200, 13, save=save)
    run_episode("g1_dahp", warehouse(20, 20), 8, 9, 6, 150, 14, use_da=True, use_hp=True, save=save)
    np.random.seed(5)
    run_episode("g1_randwh", mapgen.generateWarehouse(num_block=[10, 16]), 6, 9, 5, 150, 15, save=save)
    run_episode("g1_dense", warehouse(10, 10), 16, 9, 6, 200, 16, p_greedy=0.3, save=save)
    run_episode("g1_fixedpath", warehouse(12, 12), 6, 9, 6, 150, 17, human_seq=12, use_da=True, use_hp=True,
                save=save)
    out = {f"{name}__{k}": v for name, d in PERF.items() for k, v in d.items()}
    out["fields"] = np.array(PERF_FIELDS)
    np.savez_compressed(os.path.join(OUT, "g1_perf.npz"), **out)
    print("g1_perf:", {name: {k: d[k][-1] for k in PERF_FIELDS} for name, d in PERF.items()})


if __name__ == "__main__":
    if sys.argv[1:] == ["g1perf"]:     # the reference's counter loop over the committed g1 episodes only
        g1_episodes(save=False)
        sys.exit(0)
    if sys.argv[1:] == ["g8"]:
        g8_render()
        sys.exit(0)
    if sys.argv[1:] == ["g7"]:
        g7_warehouses()
        sys.exit(0)
    if sys.argv[1:] == ["g2_evict"]:
        g2_evict()
        sys.exit(0)
    if sys.argv[1:] == ["g6"]:
        g6_episodes()
        sys.exit(0)
    if sys.argv[1:] == ["g4"]:
        g4_gae()
        sys.exit(0)
    if sys.argv[1:] == ["g5"]:
        g5_net()
        sys.exit(0)
    g1_episodes()
    g2_fuzz(3000, 21)
    g2_evict()
    g7_warehouses()
    g3_search(31)
    g4_gae()
    g6_episodes()
    g8_render()
