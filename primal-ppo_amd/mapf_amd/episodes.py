"""Fixed evaluation episodes: the reference's on-disk format and a batched
evaluation loop on the device env.

On-disk format (evaluate.py:32-135): a folder holding
  infos.json          {"obstacleMap": ["obstacleMap0.npy", ...],
                       "agentsSequence": [[[[r, c], ...] per agent] per episode],
                       "humanSequence": [[[r, c], ...] per episode],
                       "humanStart": [[r, c], ...], "humanGoal": [[r, c], ...],
                       "numEpisodes": E}        (json.dump indent=4, sort_keys)
  obstacleMap{i}.npy  int64 [H, W], 0 free / -1 obstacle (np.save)
Files are read with json and np.load(allow_pickle=False) only.

generate_fixed_episode_infos restates generateFixedEpisodeInfos
(evaluate.py:50-103) with a numpy Generator in place of the global
np.random stream (the reference's MT19937 draws are not reproducible on the
device; the episodes themselves are the parity anchor once written).

evaluate_fixed_episodes runs evaluate() (evaluate.py:169-269) for every
episode at once: one BatchedMapfGym per map shape (FixedMapfGym semantics:
agentsSequence goals, LoopingHuman or FixedPathHuman, useDA / useHP), the
policy forward batched over episodes, and the OneEpPerformance sums
(evaluate.py:226-256) accumulated on the device.
"""
import json
import os

import numpy as np
import torch

from .config import make_config
from .maps import generate_warehouse


def create_fixed_episode_info():
    return {"obstacleMap": [], "agentsSequence": [], "humanSequence": [], "humanStart": [], "humanGoal": [],
            "numEpisodes": 0}


def _manhattan(a, b):
    return abs(a[0] - b[0]) + abs(a[1] - b[1])


def _free_cell(rng, world):
    """util.getFreeCell (util.py:67-76): rejection-sample a cell whose value is 0."""
    H, W = world.shape
    while True:
        i, j = int(rng.integers(0, H)), int(rng.integers(0, W))
        if world[i, j] == 0:
            return (i, j)


def _entrance(rng, world):
    """Human.getEntrance (mapf_gym.py:17-22): a free cell on row 0 or column 0."""
    while True:
        e = _free_cell(rng, world)
        if e[0] == 0 or e[1] == 0:
            return e


def generate_fixed_episode_infos(episodes, n_agents, max_steps, world_size=(10, 40), rng=None):
    """evaluate.py:50-103 (generateFixedEpisodeInfos), same marking protocol on tempMap."""
    rng = np.random.default_rng(0) if rng is None else rng
    infos = create_fixed_episode_info()
    for _ in range(episodes):
        length = int(rng.integers(world_size[0], world_size[1] + 1))
        obstacle_map = generate_warehouse(length).astype(np.int64)
        temp = obstacle_map.copy()
        human_start = _entrance(rng, temp)
        human_seq = [human_start]
        temp[human_start] = 1
        path_len = 0
        human_goal = human_start
        while path_len <= max_steps:
            prev = human_seq[-1]
            human_goal = _free_cell(rng, temp)
            path_len += _manhattan(prev, human_goal)
            temp[human_goal] = 1
            temp[human_start] = 0
            human_seq.append(human_goal)
        temp[human_seq[-1]] = 0
        temp[human_start] = 1
        seqs = [[] for _ in range(n_agents)]
        for a in range(n_agents):
            s = _free_cell(rng, temp)
            temp[s] = 2
            seqs[a].append(s)
        lens = [0] * n_agents
        done = [False] * n_agents
        while not all(done):
            for a in range(n_agents):
                if done[a]:
                    continue
                start = seqs[a][-1]
                goal = _free_cell(rng, temp)
                temp[goal] = 3
                seqs[a].append(goal)
                lens[a] += _manhattan(start, goal)
                if lens[a] > max_steps:
                    done[a] = True
            for s in seqs:       # free the cell before the last one
                temp[s[-2]] = 0
        infos["obstacleMap"].append(obstacle_map)
        infos["agentsSequence"].append(seqs)
        infos["humanSequence"].append(human_seq)
        infos["humanStart"].append(human_start)
        infos["humanGoal"].append(human_goal)
        infos["numEpisodes"] += 1
    return infos


def save_fixed_episode_infos(infos, folder):
    """saveFixedEpisodeInfos (evaluate.py:105-123)."""
    os.makedirs(folder, exist_ok=True)
    out = dict(infos)
    names = []
    for i in range(infos["numEpisodes"]):
        name = f"obstacleMap{i}.npy"
        np.save(os.path.join(folder, name), np.asarray(infos["obstacleMap"][i], dtype=np.int64))
        names.append(name)
    out["obstacleMap"] = names
    out["agentsSequence"] = [[[list(map(int, c)) for c in seq] for seq in ep] for ep in infos["agentsSequence"]]
    out["humanSequence"] = [[list(map(int, c)) for c in ep] for ep in infos["humanSequence"]]
    out["humanStart"] = [list(map(int, c)) for c in infos["humanStart"]]
    out["humanGoal"] = [list(map(int, c)) for c in infos["humanGoal"]]
    with open(os.path.join(folder, "infos.json"), "w", encoding="utf-8") as f:
        json.dump(out, f, ensure_ascii=False, indent=4, sort_keys=True)


def load_fixed_episode_infos(folder):
    """loadFixedEpisodeInfos (evaluate.py:125-137): cells as tuples, maps via np.load (no pickle)."""
    with open(os.path.join(folder, "infos.json")) as f:
        js = json.load(f)
    infos = create_fixed_episode_info()
    for i in range(js["numEpisodes"]):
        infos["obstacleMap"].append(np.load(os.path.join(folder, js["obstacleMap"][i]), allow_pickle=False))
        infos["agentsSequence"].append([[tuple(c) for c in seq] for seq in js["agentsSequence"][i]])
        infos["humanSequence"].append([tuple(c) for c in js["humanSequence"][i]])
    infos["humanStart"] = [tuple(c) for c in js["humanStart"]]
    infos["humanGoal"] = [tuple(c) for c in js["humanGoal"]]
    infos["numEpisodes"] = js["numEpisodes"]
    return infos


def _groups_by_shape(infos):
    groups = {}
    for i in range(infos["numEpisodes"]):
        groups.setdefault(tuple(np.shape(infos["obstacleMap"][i])), []).append(i)
    return groups


METRIC_KEYS = ("episodeReward", "episodeCostReward", "humanCollide", "staticCollide", "agentCollide", "totalGoals",
               "shadowGoals", "constraintViolations")


def evaluate_fixed_episodes(infos, policy, device=None, num_channel=6, fov=9, use_da=False, use_hp=False,
                            human_movement_type=0, max_steps=256, k_predict=5, fix_choice=1):
    """evaluate() (evaluate.py:169-269) for every episode at once.

    policy(obs [B,N,C,F,F], vec [B,N,4], env, t) -> int32 [B,N] device actions
    (e.g. make_network_policy(network) below, or a random policy); env.episodes
    lists the episode indices of env's rows (one env per map shape).
    fix_choice: fixActions' random.choice -- 1 Philox, 0 the rotating rule.
    human_movement_type 0: LoopingHuman(humanStart, humanGoal); 1: FixedPathHuman(humanSequence).
    Returns {metric: float64 numpy [E]} in episode order (OneEpPerformance fields)."""
    from .env import BatchedMapfGym
    device = torch.device("cuda") if device is None else torch.device(device)
    E = infos["numEpisodes"]
    res = {k: np.zeros(E, np.float64) for k in METRIC_KEYS}
    for (H, W), idx in sorted(_groups_by_shape(infos).items()):
        n = len(infos["agentsSequence"][idx[0]])
        S = max(len(s) for i in idx for s in infos["agentsSequence"][i])
        HS = max(len(infos["humanSequence"][i]) for i in idx) if human_movement_type == 1 else 2
        cfg = make_config(len(idx), H, W, num_agents=n, fov=fov, num_channel=num_channel, use_da=int(use_da),
                          use_hp=int(use_hp), human_mode="fixed_path" if human_movement_type == 1 else "looping",
                          goal_mode="sequence", fix_choice=fix_choice, shared_map=False, keep_bfs=False, max_seq=S,
                          max_human_seq=HS)
        cfg.k_predict = k_predict
        env = BatchedMapfGym(cfg, device=device)
        env.episodes = idx
        maps = np.stack([np.asarray(infos["obstacleMap"][i]) for i in idx]).astype(np.int8)
        seqs = [infos["agentsSequence"][i] for i in idx]
        if human_movement_type == 1:
            env.reset_fixed(maps, seqs, human_seq=[infos["humanSequence"][i] for i in idx])
        else:
            env.reset_fixed(maps, seqs, human_start=[infos["humanStart"][i] for i in idx],
                            human_goal=[infos["humanGoal"][i] for i in idx])
        acc = torch.zeros((len(idx), len(METRIC_KEYS)), dtype=torch.float64, device=device)
        obs, vec = env.observe()
        for t in range(max_steps):
            acts = policy(obs, vec, env, t)
            out, obs, vec = env.step_observe(acts)
            st = out["status"]
            acc[:, 0] += out["reward_total"].double().sum(1)
            acc[:, 1] += out["cost"].double().sum(1)
            acc[:, 2] += (st == -2).sum(1)
            acc[:, 3] += (st == -1).sum(1)
            acc[:, 4] += (st == -3).sum(1)
            acc[:, 5] += out["goals_reached"].double().sum(1)
            acc[:, 6] += out["shadow_goals"].double()
            acc[:, 7] += out["constraints"].double().sum(1)
        a = acc.cpu().numpy()
        for k, key in enumerate(METRIC_KEYS):
            res[key][idx] = a[:, k]
        env.close()
    return res


def make_network_policy(network, greedy=False, seed=0):
    """Model.evaluate (model.py:43-60): softmax policy, argmax when greedy, else a
    per-agent categorical draw (Philox inverse CDF in place of np.random.choice)."""
    from .env import sample_actions

    @torch.no_grad()
    def policy(obs, vec, env, t):
        network.num_agents = env.N
        ps = network(obs, vec)[0].float().reshape(env.B, env.N, -1).contiguous()
        if greedy:
            return ps.argmax(-1).to(torch.int32).contiguous()
        return sample_actions(ps, seed, t, out32=env.actions)
    return policy


def summarize(res):
    """The per-metric mean / std over episodes that evaluate() writes to METRICS_JSON_PATH."""
    key = {"hc": "humanCollide", "ecr": "episodeCostReward", "cv": "constraintViolations", "goals": "totalGoals"}
    return {k: {"mean": float(np.mean(res[v])), "std": float(np.std(res[v]))} for k, v in key.items()}
