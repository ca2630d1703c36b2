"""ctypes front-end of the CPU oracle (oracle/mapf_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg.  The product (primal-ppo_amd) never imports it.

The oracle is a literal single-environment restatement of the reference
env (mapf_gym.py), A* (astar_4.py), BFS (mapf_gym.py:211-244) and GAE
(runner.py:117-149); see mapf_oracle.c for per-function citations.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")


class OracleConfig(ctypes.Structure):
    """Layout-identical to include/mapf.h mapf_config."""
    _fields_ = [(n, ctypes.c_int32) for n in (
        "num_envs", "num_agents", "height", "width", "fov", "num_channel",
        "use_da", "use_hp", "lifelong", "human_mode", "goal_mode", "fix_choice",
        "shared_map", "keep_bfs", "max_seq", "max_human_seq", "k_predict", "penalty_radius")] + \
        [(n, ctypes.c_float) for n in ("action_cost", "collision_cost", "human_collision_cost",
                                       "repeat_cost", "goal_reward")] + \
        [("env_offset", ctypes.c_int32), ("reserved", ctypes.c_uint32), ("seed", ctypes.c_uint64)]


def make_config(H, W, N, F=11, C=6, *, use_da=0, use_hp=0, lifelong=1, human_mode=0, goal_mode=0,
                fix_choice=0, keep_bfs=1, max_seq=1, max_human_seq=1, seed=1234, num_envs=1,
                env_offset=0, shared_map=1):
    """Defaults follow alg_parameters.py (EnvParameters :27-48, TrainingParameters :76-78)."""
    c = OracleConfig()
    c.num_envs, c.num_agents, c.height, c.width, c.fov, c.num_channel = num_envs, N, H, W, F, C
    c.use_da, c.use_hp, c.lifelong, c.human_mode, c.goal_mode, c.fix_choice = use_da, use_hp, lifelong, human_mode, goal_mode, fix_choice
    c.shared_map, c.keep_bfs, c.max_seq, c.max_human_seq = shared_map, keep_bfs, max_seq, max_human_seq
    c.k_predict, c.penalty_radius = 5, 5
    c.action_cost, c.collision_cost, c.human_collision_cost, c.repeat_cost, c.goal_reward = -0.3, -2.0, -2.0, -0.35, 1.5
    c.env_offset, c.seed = env_offset, seed
    return c


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.oc_create.restype = P
        L.oc_create.argtypes = [ctypes.POINTER(OracleConfig), ctypes.c_uint32]
        L.oc_destroy.argtypes = [P]
        L.oc_reset_fixed.argtypes = [P, P, P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, ctypes.c_int]
        L.oc_reset_random.argtypes = [P, P]
        L.oc_step.argtypes = [P] + [P] * 9
        L.oc_observe.argtypes = [P, P, P]
        L.oc_get_agents.argtypes = [P, P, P]
        L.oc_get_masks.argtypes = [P, P, P, P, P]
        L.oc_get_human.argtypes = [P, P]
        L.oc_get_human_path.argtypes = [P, P, ctypes.c_int]
        L.oc_get_bfs.argtypes = [P, P]
        L.oc_get_errors.argtypes = [P]; L.oc_get_errors.restype = ctypes.c_uint32
        L.oc_get_clock.argtypes = [P]; L.oc_get_clock.restype = ctypes.c_uint32
        L.oc_get_fix_counts.argtypes = [P, P]
        L.oc_evict_order.argtypes = [P, ctypes.c_int, P, P, ctypes.c_int, P]
        L.oc_evict_order.restype = ctypes.c_int
        L.oc_gen_map.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_uint32,
                                 ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_int, P]
        L.oc_gen_map.restype = ctypes.c_int
        L.oc_py_hash_pair.argtypes = [ctypes.c_int64, ctypes.c_int64]
        L.oc_py_hash_pair.restype = ctypes.c_uint64
        L.oc_random_actions.argtypes = [P, P]
        L.oc_debug_set.argtypes = [P, ctypes.c_int, P]
        L.oc_astar.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, ctypes.c_int]
        L.oc_bfs_map.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
        L.oc_gae.argtypes = [P, P, P, P, P, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double]
        L.oc_episode_sum.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
        L.oc_philox_word.argtypes = [ctypes.c_uint32] * 4 + [ctypes.c_uint64, ctypes.c_int]
        L.oc_philox_word.restype = ctypes.c_uint32
        L.oc_batch_create.restype = P
        L.oc_batch_create.argtypes = [ctypes.POINTER(OracleConfig), P, ctypes.c_int]
        L.oc_batch_destroy.argtypes = [P]
        L.oc_batch_run.argtypes = [P, ctypes.c_int, P, P]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleEnv:
    """One environment.  Method names follow the reference (mapf_gym.py)."""

    def __init__(self, cfg, env_id=0):
        self.cfg = cfg
        self.N, self.H, self.W, self.F, self.C = cfg.num_agents, cfg.height, cfg.width, cfg.fov, cfg.num_channel
        self.h = lib().oc_create(ctypes.byref(cfg), env_id)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oc_destroy(self.h)
            self.h = None

    def reset_fixed(self, world, seqs, hstart, hgoal, hseq=None):
        """FixedMapfGym(world, agentsSequence, humanStart, humanGoal, humanSequence=hseq)."""
        S = self.cfg.max_seq
        seq = np.zeros((self.N, S, 2), np.int32)
        ln = np.zeros(self.N, np.int32)
        for i, s in enumerate(seqs):
            s = np.asarray(s, np.int32).reshape(-1, 2)
            assert len(s) <= S
            seq[i, :len(s)] = s
            ln[i] = len(s)
        m = np.ascontiguousarray(world, np.int8)
        hs = np.zeros((max(1, self.cfg.max_human_seq), 2), np.int32)
        nh = 0
        if hseq is not None:
            hq = np.asarray(hseq, np.int32).reshape(-1, 2)
            hs[:len(hq)] = hq
            nh = len(hq)
        return lib().oc_reset_fixed(self.h, _p(m), _p(seq), _p(ln), int(hstart[0]), int(hstart[1]),
                                    int(hgoal[0]), int(hgoal[1]), _p(hs), nh)

    def reset_random(self, world):
        m = np.ascontiguousarray(world, np.int8)
        return lib().oc_reset_random(self.h, _p(m))

    def step(self, actions):
        N = self.N
        a = np.ascontiguousarray(actions, np.int32)
        out = dict(status=np.zeros(N, np.int8), reward=np.zeros(N, np.float32), shadow=np.zeros(1, np.int32),
                   cost=np.zeros(N, np.float32), valid=np.zeros((N, 5), np.float32), fixed=np.zeros(N, np.int32),
                   goals=np.zeros(N, np.float32), constr=np.zeros(N, np.float32))
        lib().oc_step(self.h, _p(a), _p(out["status"]), _p(out["reward"]), _p(out["shadow"]), _p(out["cost"]),
                      _p(out["valid"]), _p(out["fixed"]), _p(out["goals"]), _p(out["constr"]))
        out["shadow"] = int(out["shadow"][0])
        return out

    def observe(self):
        obs = np.zeros((self.N, self.C, self.F, self.F), np.float32)
        vec = np.zeros((self.N, 4), np.float32)
        lib().oc_observe(self.h, _p(obs), _p(vec))
        return obs, vec

    def agents(self):
        p = np.zeros((self.N, 2), np.int32); g = np.zeros((self.N, 2), np.int32)
        lib().oc_get_agents(self.h, _p(p), _p(g))
        return p, g

    def masks(self):
        m = [np.zeros(self.N, np.int32) for _ in range(4)]
        lib().oc_get_masks(self.h, *[_p(x) for x in m])
        return dict(static=m[0], human=m[1], repeat=m[2], good=m[3])

    def human(self):
        o = np.zeros(9, np.int32)
        lib().oc_get_human(self.h, _p(o))
        return dict(pos=o[0:2].copy(), next=o[2:4].copy(), goal=o[4:6].copy(), step=int(o[6]), len=int(o[7]),
                    replans=int(o[8]))

    def human_path(self):
        cap = 2 * self.H * self.W + 4
        rc = np.zeros((cap, 2), np.int32)
        n = lib().oc_get_human_path(self.h, _p(rc), cap)
        return rc[:n].copy()

    def bfs(self):
        b = np.zeros((self.N, self.H, self.W), np.int16)
        lib().oc_get_bfs(self.h, _p(b))
        return b

    def debug_set(self, hstep, prev):
        p = np.ascontiguousarray(prev, np.int32)
        lib().oc_debug_set(self.h, int(hstep), _p(p))

    def errors(self):
        return int(lib().oc_get_errors(self.h))

    def fix_counts(self):
        """(empty viable sets, fixActions deadlocks) since reset: the states the
        reference raises on (mapf_gym.py:588) or never leaves (:563)."""
        o = np.zeros(2, np.uint32)
        lib().oc_get_fix_counts(self.h, _p(o))
        return int(o[0]), int(o[1])

    def random_actions(self):
        a = np.zeros(self.N, np.int32)
        lib().oc_random_actions(self.h, _p(a))
        return a


def astar(world, start, goal):
    """astar_4 (astar_4.py:21-109): returns the goal->start list, [] for start==goal, None if unreachable."""
    w = np.ascontiguousarray(world, np.int8)
    H, W = w.shape
    cap = H * W + 4
    rc = np.zeros((cap, 2), np.int32)
    n = lib().oc_astar(_p(w), H, W, int(start[0]), int(start[1]), int(goal[0]), int(goal[1]), _p(rc), cap)
    if n < 0:
        return None
    return rc[:n].copy()


def bfs_map(world, goal):
    w = np.ascontiguousarray(world, np.int8)
    H, W = w.shape
    out = np.zeros((H, W), np.int16)
    lib().oc_bfs_map(_p(w), H, W, int(goal[0]), int(goal[1]), _p(out))
    return out


def gae(rewards, values, last_values, gamma=0.95, lam=0.95):
    r = np.ascontiguousarray(rewards, np.float32); v = np.ascontiguousarray(values, np.float32)
    T = r.shape[0]
    M = int(np.prod(r.shape[1:]))
    lv = np.ascontiguousarray(last_values, np.float32).reshape(M)
    adv = np.zeros_like(r); ret = np.zeros_like(r)
    lib().oc_gae(_p(r), _p(v), _p(lv), _p(adv), _p(ret), T, M, gamma, lam)
    return adv, ret


def episode_sum(x):
    """runner.py:95-96's per-env episodeReward: x [T, B, N] float32 -> [B] float32 (oc_episode_sum)."""
    x = np.ascontiguousarray(x, np.float32)
    T, B, N = x.shape
    out = np.zeros(B, np.float32)
    lib().oc_episode_sum(_p(x), T, B, N, _p(out))
    return out


def evict_order(pairs, restricted):
    """Agents evicted by fixActions' random branch (mapf_gym.py:590-596), in the
    iteration order of CPython's set(pairs) & set(restricted).  pairs[j] = agent
    j's assigned action or -1; restricted = [(j, b), ...] in list order."""
    pr = np.ascontiguousarray(pairs, np.int32)
    rs = np.asarray(restricted, np.int32).reshape(-1, 2)
    rj = np.ascontiguousarray(rs[:, 0]); rb = np.ascontiguousarray(rs[:, 1])
    out = np.zeros(8, np.int32)
    n = lib().oc_evict_order(_p(pr), len(pr), _p(rj), _p(rb), len(rs), _p(out))
    return out[:n].tolist()


def gen_map(kind, H, W, env_id, epoch=0, seed=1234, lo=10, hi=40, density=0.3):
    """The device map generators (mapf_reset_generated) restated: kind 0 warehouse of a Philox
    length in [lo, hi] padded into H x W (returns (map, L)); kind 1 random -(rand < p) (map, 0)."""
    out = np.zeros((H, W), np.int8)
    L = lib().oc_gen_map(kind, lo, hi, density, epoch, seed, env_id, H, W, _p(out))
    return out, L


def py_hash_pair(a, b):
    return int(lib().oc_py_hash_pair(a, b))


def philox_word(c0, c1, c2, c3, seed, w):
    return int(lib().oc_philox_word(c0, c1, c2, c3, seed, w))


class OracleBatch:
    """B independent envs stepped with the random policy (CPU baseline)."""

    def __init__(self, cfg, world, B):
        self.cfg = cfg
        m = np.ascontiguousarray(world, np.int8)
        self.h = lib().oc_batch_create(ctypes.byref(cfg), _p(m), B)
        self.obs = np.zeros((cfg.num_agents, cfg.num_channel, cfg.fov, cfg.fov), np.float32)
        self.vec = np.zeros((cfg.num_agents, 4), np.float32)

    def run(self, steps):
        return lib().oc_batch_run(self.h, steps, _p(self.obs), _p(self.vec))

    def __del__(self):
        if getattr(self, "h", None):
            lib().oc_batch_destroy(self.h)
            self.h = None
