"""mapf_amd -- MI355X-native batched MAPF gridworld + PPO rollout engine.

Host-side mirror of the reference's env/runner API (Nielsencu/primal-ppo
mapf_gym.py / runner.py) over the HIP C ABI in ../lib/libmapf.so
(include/mapf.h).  The GPU path is the only path: if libmapf.so is missing
or no GPU is visible, calls fail loudly -- there is no CPU fallback.

Graph capture mode.  ROCm 7's HIP runtime records a hipGraph capture as
prebuilt AQL packets by default (DEBUG_CLR_GRAPH_PACKET_CAPTURE=1).  In that
mode a captured hipMemsetAsync takes effect on the first replay only
(a captured memset(0) + add(1) replays to 1, then to garbage: profiles/r05_diag20_packet_capture_on.log;
tests/test_gpu_graph_capture_mode.py pins it), so
every captured multi-block torch reduction -- its semaphores are zeroed by a
captured memset -- returns stale partial sums from the second replay on: the
captured PPO update's bias gradients, grad norm and loss means.
The runtime reads the flag at its first HIP call, so it is switched off here,
before torch or libmapf touch the GPU; an explicit setting in the environment
is kept, and Model checks captured reductions before it captures an update
(model.captured_reductions_ok).
"""
import os as _os

GRAPH_CAPTURE_FLAG = "DEBUG_CLR_GRAPH_PACKET_CAPTURE"
_flag_was_set = GRAPH_CAPTURE_FLAG in _os.environ
_os.environ.setdefault(GRAPH_CAPTURE_FLAG, "0")


def _warn_if_runtime_started():
    """Import order: the flag only takes effect if mapf_amd is imported before the
    process's first HIP call.  If torch already started the runtime, say so: captured updates then
    self-check (model.captured_reductions_ok) and may run eagerly."""
    import sys
    torch = sys.modules.get("torch")
    if _flag_was_set or torch is None or not torch.cuda.is_initialized():
        return
    import warnings
    warnings.warn("mapf_amd was imported after the HIP runtime started: DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 does not "
                  "apply to this process (import mapf_amd before any GPU work, or set it in the environment); "
                  "captured PPO updates will check captured reductions first and may run eagerly", RuntimeWarning)


_warn_if_runtime_started()

from .config import EnvParameters, TrainingParameters, NetParameters, make_config  # noqa: F401,E402

__all__ = ["EnvParameters", "TrainingParameters", "NetParameters", "make_config", "GRAPH_CAPTURE_FLAG"]
