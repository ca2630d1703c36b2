"""mapf_amd -- MI355X-native batched MAPF gridworld + PPO rollout engine.

Host-side mirror of the reference's env/runner API (Nielsencu/primal-ppo
mapf_gym.py / runner.py) over the HIP C ABI in ../lib/libmapf.so
(include/mapf.h).  The GPU path is the only path: if libmapf.so is missing
or no GPU is visible, calls fail loudly -- there is no CPU fallback.
"""
from .config import EnvParameters, TrainingParameters, NetParameters, make_config  # noqa: F401

__all__ = ["EnvParameters", "TrainingParameters", "NetParameters", "make_config"]
