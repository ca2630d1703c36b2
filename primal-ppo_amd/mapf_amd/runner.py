"""On-device rollout worker: Runner.run (runner.py:26-151) for B envs at once.

The reference runs one env per Ray actor on a CPU and pickles ~3 MB per
rollout back to the driver.  Here B environments live in HBM; every buffer of
the rollout is a device tensor written in place:

  obs[0], vec[0] <- mapf_observe
  for t in range(T):                       (runner.py:43-100)
      actions, ps, values, cost values <- policy forward + mapf_sample_actions
      mapf_step_observe: status/reward/cost/trainValid/goals/constraints written
      straight into the slices [t] of the buffers, obs[t+1]/vec[t+1] likewise
  last values <- policy value head on obs[T]   (:117-118)
  advantages / returns <- mapf_gae for reward and cost (:121-149)

Buffers are laid out [T, B, N, ...] (t-major: each step writes one contiguous
slice).  `batch()` exposes them as util.BatchValues (util.py:41-54: attribute
names, read by driver.py with getattr) whose rows are ENV-MAJOR [B*T, N, ...]
views: env 0's T steps, then env 1's -- the order driver.py:101-121 produces by
concatenating one runner's result after another, so driver.py:125-131's
`inds = np.arange(N_STEPS)` selects env 0's rollout as it selects runner 0's.
Indexing a view gathers only the minibatch rows.  hiddenState is all zeros in
the reference (runner.py:47-48, never read by the net): expanded zero views.
OneEpPerformance (util.py:56-65) is per env (the mean over the B envs; every
env's counters via performance_per_env()).
"""
import numpy as np
import torch

from .config import EnvParameters, NetParameters, TrainingParameters
from .env import BatchedMapfGym, gae


class DeviceMaps:
    """new_maps for DeviceRunner that never leaves the GPU: every rollout re-generates every
    env's map on the device (env.reset_generated, epoch = rollout index) -- by default
    MapfGym()'s random-length warehouse (mapf_gym.py:166, map_generator.py:127-138) --
    then the seeded reset.  No host maps, no upload."""

    def __init__(self, kind="warehouse", lo=None, hi=None, density=0.3, largest=False):
        self.kind, self.lo, self.hi, self.density, self.largest = kind, lo, hi, density, largest

    def reset(self, env, rollout, seed):
        env.reset_generated(self.kind, self.lo, self.hi, self.density, self.largest, epoch=rollout, seed=seed)


def reference_maps(env: BatchedMapfGym, world_size=None, seed=0):
    """new_maps for DeviceRunner: per rollout, every env gets its own MapfGym() warehouse
    (random length in EnvParameters.WORLD_SIZE) in the padded [B, Lmax, Wmax] stack the
    env was created with (maps.random_warehouse_batch; create the env with
    height, width = that stack's shape and shared_map=False)."""
    import numpy as np
    from .maps import random_warehouse_batch
    ws = EnvParameters.WORLD_SIZE if world_size is None else world_size

    def draw(rollout):
        return random_warehouse_batch(np.random.default_rng((seed, rollout)), env.B, ws)
    return draw


class OneEpPerformance:
    """util.py:56-65: the counters of ONE env's rollout (runner.py:66-99 sums them over one
    env's steps).  DeviceRunner.run() returns the mean over its B envs: driver.py:108-117
    passes one runner's object on (its loop overwrites `performance` with each result in
    turn), and Model.train feeds performance.episodeCostReward to the Lagrangian
    (model.py:180, lagrange.py) -- a per-env quantity.  performance_per_env() has all B."""

    FIELDS = ("totalGoals", "shadowGoals", "episodeReward", "staticCollide", "humanCollide", "agentCollide",
              "episodeCostReward", "constraintViolations")

    def __init__(self):
        for f in self.FIELDS:
            setattr(self, f, 0)


class EnvMajorRows:
    """The [B*T, ...] rows of a t-major [T, B, ...] rollout buffer in ENV-MAJOR order:
    row r = env r // T, step r % T -- the order driver.py:101-121 builds by concatenating
    the runners' results (runner k's T rows, then runner k+1's).  Rows [0, T) are env 0's
    rollout, i.e. what `inds = np.arange(N_STEPS)` (driver.py:125) trains on, like the
    reference's first runner.  Zero-copy: indexing gathers just the rows asked for (a
    minibatch) from the buffer; materialize() copies all of them."""

    def __init__(self, buf, T, B):
        self.buf, self.T, self.B = buf, T, B
        self.shape = torch.Size((B * T,) + tuple(buf.shape[2:]))
        self.dtype, self.device = buf.dtype, buf.device

    def __len__(self):
        return self.shape[0]

    def __getitem__(self, idx):
        n = self.shape[0]
        if isinstance(idx, int):
            if not -n <= idx < n:
                raise IndexError(idx)
            idx %= n
            return self.buf[idx % self.T, idx // self.T]
        if isinstance(idx, slice):
            idx = torch.arange(*idx.indices(n), device=self.device)
        else:
            idx = torch.as_tensor(np.asarray(idx) if not isinstance(idx, torch.Tensor) else idx,
                                  device=self.device).long()
            if idx.numel() and (int(idx.min()) < -n or int(idx.max()) >= n):
                raise IndexError("row index out of range")
            idx = idx % n
        return self.buf[idx % self.T, idx // self.T]

    def materialize(self):
        return self.buf.transpose(0, 1).reshape(self.shape)


class ZeroRows:
    """hiddenState rows: all zeros in the reference (runner.py:47-48, never read by the
    net), handed out as expanded zero views, never materialised."""

    def __init__(self, n, row_shape, device):
        self.shape = torch.Size((n,) + tuple(row_shape))
        self.dtype, self.device = torch.float32, device

    def __len__(self):
        return self.shape[0]

    def __getitem__(self, idx):
        k = len(range(*idx.indices(self.shape[0]))) if isinstance(idx, slice) else len(np.atleast_1d(
            idx.cpu().numpy() if isinstance(idx, torch.Tensor) else np.asarray(idx)))
        return torch.zeros((), device=self.device).expand((k,) + tuple(self.shape[1:]))


class BatchValues:
    """util.py:41-54: the rollout's arrays by the reference's attribute names (driver.py reads
    them with getattr), each an EnvMajorRows view over the device buffers; mb["name"] works too."""

    FIELDS = ("observations", "vectors", "rewards", "values", "ps", "actions", "hiddenState", "returns",
              "trainValid", "costRewards", "costValues", "costReturns")

    def __init__(self, **fields):
        for k in self.FIELDS:
            setattr(self, k, fields[k])

    def __getitem__(self, name):
        return getattr(self, name)

    def keys(self):
        return self.FIELDS


class DeviceRunner:
    """new_maps: DeviceMaps() (maps generated on the GPU) or a callable(rollout index) ->
    host maps for env.reset_seeded, at the start of every run(), i.e. Runner.run's
    `env = MapfGym()` (runner.py:30: a NEW random-size warehouse and new agents/human
    every rollout) -- e.g. reference_maps(env).  None: the envs continue from where the
    previous rollout left them (lifelong)."""

    def __init__(self, env: BatchedMapfGym, model, n_steps=None, seed=0, new_maps=None):
        self.env = env
        self.model = model
        self.T = TrainingParameters.N_STEPS if n_steps is None else n_steps
        self.seed = seed
        self.new_maps = new_maps
        self.rollouts = 0
        B, N, C, F = env.B, env.N, env.C, env.F
        dev = env.device
        T = self.T
        z = lambda *s, dt=torch.float32: torch.zeros(*s, dtype=dt, device=dev)
        self.obs = z(T + 1, B, N, C, F, F)          # obs[T] = bootstrap observation
        self.vec = z(T + 1, B, N, NetParameters.VECTOR_LEN)
        self.rewards = z(T, B, N)
        self.values = z(T, B, N)
        self.cost_rewards = z(T, B, N)
        self.cost_values = z(T, B, N)
        self.ps = z(T, B, N, EnvParameters.N_ACTIONS)
        self.actions = z(T, B, N, dt=torch.int64)
        self.actions32 = z(B, N, dt=torch.int32)
        self.train_valid = z(T, B, N, EnvParameters.N_ACTIONS)
        self.status = z(T, B, N, dt=torch.int8)
        self.goals = z(T, B, N)
        self.constraints = z(T, B, N)
        self.shadow = z(T, B, dt=torch.int32)
        self.adv = self.returns = self.cost_adv = self.cost_returns = None

    @torch.no_grad()
    def run(self, weights=None):
        """Runner.run: returns (BatchValues, OneEpPerformance) -- env-major rows over the device
        buffers, and the per-env mean of the episode counters."""
        if weights is not None:
            self.model.set_weights(weights)
        env, T = self.env, self.T
        if isinstance(self.new_maps, DeviceMaps):   # runner.py:30 -- a fresh MapfGym() per rollout
            self.new_maps.reset(env, self.rollouts, (self.seed << 20) + self.rollouts + 1)
        elif self.new_maps is not None:
            env.reset_seeded(self.new_maps(self.rollouts), seed=(self.seed << 20) + self.rollouts + 1)
        env.observe(self.obs[0], self.vec[0])
        for t in range(T):
            a, ps, v, _, _, cv = self.model.step(self.obs[t], self.vec[t], None, seed=self.seed,
                                                 step=self.rollouts * T + t, actions_out=self.actions[t],
                                                 actions32_out=self.actions32)
            self.ps[t].copy_(ps.reshape(self.ps[t].shape))
            self.values[t].copy_(v.reshape(self.values[t].shape))
            self.cost_values[t].copy_(cv.reshape(self.cost_values[t].shape))
            env.step_observe(self.actions32, self.obs[t + 1], self.vec[t + 1], out={
                "reward_total": self.rewards[t],            # reward + GOAL_REWARD (runner.py:89-91)
                "cost": self.cost_rewards[t], "train_valid": self.train_valid[t], "status": self.status[t],
                "goals_reached": self.goals[t], "constraints": self.constraints[t], "shadow_goals": self.shadow[t]})
        last_v, last_cv = self.model.value(self.obs[T], self.vec[T], None)
        self.last_v = last_v.reshape(self.values[0].shape).contiguous()
        self.last_cv = last_cv.reshape(self.values[0].shape).contiguous()
        self.adv, self.returns = gae(self.rewards, self.values, self.last_v,
                                     TrainingParameters.GAMMA, TrainingParameters.LAM)
        self.cost_adv, self.cost_returns = gae(self.cost_rewards, self.cost_values, self.last_cv,
                                               TrainingParameters.GAMMA, TrainingParameters.LAM)
        self.rollouts += 1
        return self.batch(), self.performance()

    def batch(self):
        """BatchValues over this rollout's buffers, rows env-major (EnvMajorRows)."""
        T, B, N = self.T, self.env.B, self.env.N
        rows = lambda x: EnvMajorRows(x, T, B)   # noqa: E731
        return BatchValues(
            observations=rows(self.obs[:T]), vectors=rows(self.vec[:T]), rewards=rows(self.rewards),
            values=rows(self.values), ps=rows(self.ps), actions=rows(self.actions),
            hiddenState=ZeroRows(T * B, (2, N, NetParameters.NET_SIZE), self.env.device),
            returns=rows(self.returns), trainValid=rows(self.train_valid), costRewards=rows(self.cost_rewards),
            costValues=rows(self.cost_values), costReturns=rows(self.cost_returns))

    def performance_per_env(self):
        """OneEpPerformance's counters of every env (runner.py:66-99), float64 numpy [B] each."""
        st = self.status
        per = {
            "staticCollide": (st == -1).sum(dim=(0, 2)), "humanCollide": (st == -2).sum(dim=(0, 2)),
            "agentCollide": (st == -3).sum(dim=(0, 2)), "shadowGoals": self.shadow.sum(dim=0),
            # np.sum over float32 rewards per step, accumulated in a python float (runner.py:95-98)
            "episodeReward": self.rewards.sum(dim=2).double().sum(dim=0),
            "episodeCostReward": self.cost_rewards.sum(dim=2).double().sum(dim=0),
            "totalGoals": self.goals.sum(dim=(0, 2)), "constraintViolations": self.constraints.sum(dim=(0, 2))}
        return {k: v.double().cpu().numpy() for k, v in per.items()}

    def performance(self):
        """The mean over envs of performance_per_env() (see OneEpPerformance)."""
        p = OneEpPerformance()
        for k, v in self.performance_per_env().items():
            setattr(p, k, float(np.mean(v)))
        return p
