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
slice); `batch()` exposes them with the BatchValues field names (util.py:41-54)
reshaped to [T*B, N, ...] rows, the contract driver.py:101-121 concatenates on
axis 0.  hiddenState is all zeros in the reference (runner.py:47-48, never read
by the net) and is returned as an expanded zero view, not materialised.
OneEpPerformance counters (util.py:56-65) are reduced on the device.
"""
import torch

from .config import EnvParameters, NetParameters, TrainingParameters
from .env import BatchedMapfGym, gae


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
    """util.py:56-65 (sums over all B envs of the rollout)."""

    def __init__(self):
        self.totalGoals = 0
        self.shadowGoals = 0
        self.episodeReward = 0
        self.staticCollide = 0
        self.humanCollide = 0
        self.agentCollide = 0
        self.episodeCostReward = 0
        self.constraintViolations = 0


class BatchValues:
    """util.py:41-54 field names; tensors on the device."""

    FIELDS = ("observations", "vectors", "rewards", "values", "ps", "actions", "hiddenState", "returns",
              "trainValid", "costRewards", "costValues", "costReturns")


class DeviceRunner:
    """new_maps: callable(rollout index) -> maps for env.reset_seeded at the start of every
    run(), i.e. Runner.run's `env = MapfGym()` (runner.py:30: a NEW random-size warehouse
    and new agents/human every rollout) -- e.g. reference_maps(env) below.  None: the
    envs continue from where the previous rollout left them (lifelong)."""

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
        """Runner.run: returns (BatchValues-like dict of device tensors, OneEpPerformance)."""
        if weights is not None:
            self.model.set_weights(weights)
        env, T = self.env, self.T
        if self.new_maps is not None:        # runner.py:30 -- a fresh MapfGym() per rollout
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
        T, B, N = self.T, self.env.B, self.env.N
        rows = lambda x: x.reshape(T * B, N, *x.shape[3:])
        return {
            "observations": rows(self.obs[:T]), "vectors": rows(self.vec[:T]), "rewards": rows(self.rewards),
            "values": rows(self.values), "ps": rows(self.ps), "actions": rows(self.actions),
            "hiddenState": torch.zeros((), device=self.env.device).expand(T * B, 2, N, NetParameters.NET_SIZE),
            "returns": rows(self.returns), "trainValid": rows(self.train_valid), "costRewards": rows(self.cost_rewards),
            "costValues": rows(self.cost_values), "costReturns": rows(self.cost_returns)}

    def performance(self):
        p = OneEpPerformance()
        st = self.status
        p.staticCollide = int((st == -1).sum())
        p.humanCollide = int((st == -2).sum())
        p.agentCollide = int((st == -3).sum())
        p.shadowGoals = int(self.shadow.sum())
        p.episodeReward = float(self.rewards.sum())
        p.episodeCostReward = float(self.cost_rewards.sum())
        p.totalGoals = float(self.goals.sum())
        p.constraintViolations = float(self.constraints.sum())
        return p
