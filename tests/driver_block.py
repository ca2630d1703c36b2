"""The reference's training-data block, driver.py:97-134 (Nielsencu/primal-ppo), restated
statement for statement so tests can run it unchanged over DeviceRunner results.

Test infrastructure only.  It keeps every construct the drop-in has to survive: the
attribute walk over `dir(BatchValues())` with list appends (:101-107), np.nanmean over the
`dir(performance)` fields (:110-117), np.concatenate(..., axis=0) of every attribute
(:119-121) and the minibatch loop over `inds = np.arange(N_STEPS)` shuffled by the global
numpy RNG (:124-134).  The classes and the model are parameters: the reference imports
BatchValues / OneEpPerformance from util.py and a Model from model.py.
"""
import numpy as np


def run_driver_block(job_results, global_model, BatchValues, OneEpPerformance, TrainingParameters,
                     curr_steps=0, curr_episodes=0):
    done_len = len(job_results)
    # get reinforcement learning data                                       (driver.py:97-121)
    curr_steps += done_len * TrainingParameters.N_STEPS
    mb = BatchValues()
    performance = OneEpPerformance()
    for results in range(done_len):
        for value in dir(BatchValues()):
            if not value.startswith('__'):
                temp = getattr(mb, value)
                temp.append(getattr(job_results[results][0], value))
                setattr(mb, value, temp)
        curr_episodes += 1
        for i in dir(performance):
            if not i.startswith('__'):
                setattr(performance, i, np.nanmean(getattr(job_results[results][-1], i)))
    for i in dir(performance):
        if not i.startswith('__'):
            setattr(performance, i, np.nanmean(getattr(performance, i)))
    for value in dir(BatchValues()):
        if not value.startswith('__'):
            setattr(mb, value, np.concatenate(getattr(mb, value), axis=0))

    # training of reinforcement learning                                    (driver.py:123-134)
    mb_loss = []
    inds = np.arange(TrainingParameters.N_STEPS)
    for _ in range(TrainingParameters.N_EPOCHS):
        np.random.shuffle(inds)
        for start in range(0, TrainingParameters.N_STEPS, TrainingParameters.MINIBATCH_SIZE):
            end = start + TrainingParameters.MINIBATCH_SIZE
            mb_inds = inds[start:end]
            mb_loss.append(global_model.train(mb.observations[mb_inds], mb.vectors[mb_inds], mb.returns[mb_inds],
                                              mb.costReturns[mb_inds], mb.values[mb_inds], mb.costValues[mb_inds],
                                              mb.actions[mb_inds], mb.ps[mb_inds],
                                              mb.hiddenState[mb_inds], mb.trainValid[mb_inds],
                                              performance.episodeCostReward))
    return mb, performance, mb_loss, curr_steps, curr_episodes


class ReferenceBatchValues:
    """util.py:41-54: the reference's collector -- twelve empty lists, nothing else."""

    def __init__(self):
        for k in ("observations", "vectors", "rewards", "values", "ps", "actions", "hiddenState", "returns",
                  "trainValid", "costRewards", "costValues", "costReturns"):
            setattr(self, k, list())


class ReferenceOneEpPerformance:
    """util.py:56-65: eight zero counters."""

    def __init__(self):
        for k in ("totalGoals", "shadowGoals", "episodeReward", "staticCollide", "humanCollide", "agentCollide",
                  "episodeCostReward", "constraintViolations"):
            setattr(self, k, 0)


def expected_minibatches(seed, TrainingParameters):
    """The mb_inds run_driver_block draws after np.random.seed(seed)."""
    np.random.seed(seed)
    inds = np.arange(TrainingParameters.N_STEPS)
    out = []
    for _ in range(TrainingParameters.N_EPOCHS):
        np.random.shuffle(inds)
        for start in range(0, TrainingParameters.N_STEPS, TrainingParameters.MINIBATCH_SIZE):
            out.append(inds[start:start + TrainingParameters.MINIBATCH_SIZE].copy())
    return out


class HostGuard:
    """Context manager: any Tensor.cpu / numpy / __array__ / tolist while active raises, i.e. a
    buffer being copied to the host.  `allow()` lifts it (for the model's own stats copy)."""

    NAMES = ("cpu", "numpy", "__array__", "tolist")

    def __init__(self):
        import torch
        self.torch = torch
        self.saved = {}
        self.active = False
        self.hits = []

    def __enter__(self):
        T = self.torch.Tensor
        for n in self.NAMES:
            orig = getattr(T, n)
            self.saved[n] = orig

            def guarded(t, *a, _orig=orig, _n=n, **k):
                if self.active and t.device.type != "cpu":
                    self.hits.append((_n, tuple(t.shape)))
                    raise AssertionError(f"device tensor {tuple(t.shape)} copied to the host via .{_n}")
                return _orig(t, *a, **k)
            setattr(T, n, guarded)
        self.active = True
        return self

    def __exit__(self, *exc):
        for n, orig in self.saved.items():
            setattr(self.torch.Tensor, n, orig)
        self.active = False
        return False

    def allow(self):
        guard = self

        class _Lift:
            def __enter__(self):
                self.was = guard.active
                guard.active = False

            def __exit__(self, *exc):
                guard.active = self.was
                return False
        return _Lift()
