"""Single-environment adapter with the reference's method names.

`FixedMapfGym` / `MapfGym` here expose exactly the seven calls runner.py:30-100
and evaluate.py:218-269 make on the reference env (mapf_gym.py), backed by a
B=1 BatchedMapfGym on the GPU.  Return types follow the reference:
  getAllObservations() -> (float32 [1,N,C,F,F], float32 [1,N,4])
  getActionStatus(a)   -> float64 [N] in {1,-1,-2,-3,-4}
  calculateActionReward(a, st) -> (float32 [1,N], int shadowGoals)
  calculateCostReward(a) -> float32 [1,N]
  getTrainValid(a)     -> float32 [N,5]
  jointStep(a, st)     -> (float64 [N] goalsReached, float64 [N] constraintsViolated)
getActionStatus / calculate* / getTrainValid run the device step WITHOUT
committing (no state change), jointStep commits -- the same observable
semantics as the reference's methods.
"""
import numpy as np
import torch

from .config import EnvParameters, NetParameters, make_config
from .env import BatchedMapfGym
from .maps import random_warehouse


class _SingleEnv:
    def _init_batched(self, cfg):
        self._env = BatchedMapfGym(cfg)
        self._pending = None

    def _run(self, actions, commit):
        a = torch.as_tensor(np.asarray(actions, dtype=np.float64).astype(np.int32)).reshape(1, -1)
        self._env.actions.copy_(a.to(self._env.device))
        out = self._env.step(self._env.actions, commit=commit)
        host = {k: v.cpu().numpy().copy() for k, v in out.items()}
        return host

    def _outputs(self, actions):
        key = tuple(np.asarray(actions, dtype=np.float64).astype(np.int64).tolist())
        if self._pending is None or self._pending[0] != key:
            self._pending = (key, self._run(actions, commit=False))
        return self._pending[1]

    def getAllObservations(self):
        obs, vec = self._env.observe()
        return obs.cpu().numpy().copy(), vec.cpu().numpy().copy()

    def getActionStatus(self, actions):
        return self._outputs(actions)["status"][0].astype(np.float64)

    def calculateActionReward(self, actions, actionStatus):
        o = self._outputs(actions)
        return o["reward"].astype(np.float32), int(o["shadow_goals"][0])

    def calculateCostReward(self, actions):
        return self._outputs(actions)["cost"].astype(np.float32)

    def getTrainValid(self, actions):
        return self._outputs(actions)["train_valid"][0].astype(np.float32)

    def jointStep(self, actions, actionStatus):
        o = self._run(actions, commit=True)
        self._pending = None
        return o["goals_reached"][0].astype(np.float64), o["constraints"][0].astype(np.float64)

    def _render(self, scale=20):
        """MapfGym._render (mapf_gym.py:639-646): renderWorld of this env, uint8 [H*20, W*20, 3],
        drawn on the device (mapf_render)."""
        return self._env.render([0], scale=scale)[0].cpu().numpy()

    # state views used by tests / rendering
    def agent_positions(self):
        return self._env.get_state()["pos"][0]

    def agent_goals(self):
        return self._env.get_state()["goal"][0]

    def human_state(self):
        return self._env.get_state()["human"][0]


class FixedMapfGym(_SingleEnv):
    """mapf_gym.FixedMapfGym(obstaclesMap, agentsSequence, humanStart, humanGoal, numChannel, useDA, useHP,
    humanSequence) -- sequences are lists of (row, col) (util.Sequence items)."""

    def __init__(self, obstaclesMap, agentsSequence, humanStart, humanGoal, numChannel=None, useDA=False,
                 useHP=False, humanSequence=None, fov=None, num_agents=None):
        world = np.asarray(obstaclesMap)
        seqs = [list(getattr(s, "items", s)) for s in agentsSequence]
        n = len(seqs) if num_agents is None else num_agents
        cfg = make_config(1, world.shape[0], world.shape[1], num_agents=n,
                          fov=EnvParameters.FOV_SIZE if fov is None else fov,
                          num_channel=NetParameters.NUM_CHANNEL if numChannel is None else numChannel,
                          use_da=useDA, use_hp=useHP,
                          human_mode="looping" if humanSequence is None else "fixed_path",
                          goal_mode="sequence", fix_choice=0, max_seq=max(len(s) for s in seqs),
                          max_human_seq=max(2, len(humanSequence) if humanSequence is not None else 2))
        self._init_batched(cfg)
        self.num_channel = cfg.num_channel
        self.use_da, self.use_hp = useDA, useHP
        if humanSequence is None:
            self._env.reset_fixed(world, [seqs], [humanStart], [humanGoal])
        else:
            self._env.reset_fixed(world, [seqs], human_seq=[humanSequence])


class MapfGym(_SingleEnv):
    """mapf_gym.MapfGym(num_agents, size): random warehouse, Human with random goals."""

    def __init__(self, num_agents=None, size=None, seed=None, fov=None):
        rng = np.random.default_rng(seed)
        world = random_warehouse(rng, EnvParameters.WORLD_SIZE if size is None else size)
        cfg = make_config(1, world.shape[0], world.shape[1],
                          num_agents=EnvParameters.N_AGENTS if num_agents is None else num_agents,
                          fov=fov, human_mode="random", goal_mode="random", fix_choice=1,
                          seed=int(rng.integers(1, 2 ** 63)))
        self._init_batched(cfg)
        self.obstacleMap = world
        self.num_channel = cfg.num_channel
        self.use_hp = self.use_da = False
        self._env.reset_seeded(world)
