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
from .env import BatchedMapfGym, episode_sum, gae


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


PERF_FIELDS = ("totalGoals", "shadowGoals", "episodeReward", "staticCollide", "humanCollide", "agentCollide",
               "episodeCostReward", "constraintViolations")
BATCH_FIELDS = ("observations", "vectors", "rewards", "values", "ps", "actions", "hiddenState", "returns",
                "trainValid", "costRewards", "costValues", "costReturns")


class OneEpPerformance:
    """util.py:56-65: the counters of ONE env's rollout (runner.py:66-99 sums them over one
    env's steps).  DeviceRunner.run() returns the mean over its B envs: driver.py:108-117
    passes one runner's object on (its loop overwrites `performance` with each result in
    turn), and Model.train feeds performance.episodeCostReward to the Lagrangian
    (model.py:180, lagrange.py) -- a per-env quantity.  performance_per_env() has all B.
    Like the reference's class it has no public attribute but the 8 counters: driver.py
    walks `dir(performance)` and np.nanmean()s every name not starting with '__'."""

    def __init__(self):
        for f in PERF_FIELDS:
            setattr(self, f, 0)


def _row_index(idx, n, device):
    """A driver-style row index (int, slice, int array/list/tensor, bool mask) over n rows ->
    (int64 rows in [0, n), True if idx was a scalar).  Host indices (what driver.py passes:
    numpy mb_inds) are checked and wrapped on the host and come back as a host array --
    no device synchronisation; device tensors stay on the device (their bounds check reads
    two scalars back)."""
    if isinstance(idx, (int, np.integer)):
        if not -n <= int(idx) < n:
            raise IndexError(f"row {int(idx)} out of range for {n} rows")
        return np.array([int(idx) % n], np.int64), True
    if isinstance(idx, slice):
        return np.arange(*idx.indices(n), dtype=np.int64), False
    if isinstance(idx, torch.Tensor) and idx.device.type == "cpu":
        idx = idx.numpy()
    if not isinstance(idx, torch.Tensor):
        idx = np.asarray(idx)
        if idx.dtype == np.bool_:
            if idx.shape != (n,):
                raise IndexError(f"boolean index of shape {idx.shape} for {n} rows")
            idx = np.flatnonzero(idx)
        elif idx.size and not np.issubdtype(idx.dtype, np.integer):
            raise IndexError(f"row indices must be integers, not {idx.dtype}")
        idx = idx.astype(np.int64, copy=False).reshape(-1)
        if idx.size and (idx.min() < -n or idx.max() >= n):
            raise IndexError("row index out of range")
        return (idx % n if n else idx), False
    if idx.dtype == torch.bool:
        if tuple(idx.shape) != (n,):
            raise IndexError(f"boolean index of shape {tuple(idx.shape)} for {n} rows")
        idx = idx.nonzero().squeeze(1)
    elif idx.is_floating_point():
        raise IndexError(f"row indices must be integers, not {idx.dtype}")
    idx = idx.to(device=device, dtype=torch.int64).reshape(-1)
    if idx.numel() and (int(idx.min()) < -n or int(idx.max()) >= n):
        raise IndexError("row index out of range")
    return (idx % n if n else idx), False


class _IndexCache:
    """driver.py:131-134 indexes twelve attributes with the same mb_inds: the device copy of
    a host index array (and its (step, env) split) is made once per minibatch, not per
    attribute.  Keyed by the array's bytes; one entry."""

    def __init__(self):
        self.key, self.val = None, None

    def get(self, rows, tag, device, make):
        key = (rows.tobytes(), tag, str(device))
        if key != self.key:
            self.key, self.val = key, make()
        return self.val


_INDEX_CACHE = _IndexCache()


class _DeviceRows:
    """Row views of rollout buffers that stay on the device.  driver.py:119-121 hands a list of
    them (one per runner result) to np.concatenate(..., axis=0): __array_function__ answers
    with a lazy ConcatRows (runner k's rows after runner k-1's) instead of letting numpy
    coerce the rows one by one to the host; any other numpy function, and __array__,
    refuse -- a buffer never leaves the device behind the caller's back."""

    def __len__(self):
        return self.shape[0]

    def __array__(self, *args, **kwargs):
        raise TypeError(f"{type(self).__name__} holds device rows; index it (rows[mb_inds]) or materialize()")

    def __array_function__(self, func, types, args, kwargs):
        if func is not np.concatenate:
            return NotImplemented
        seq = args[0] if args else kwargs.get("arrays")
        axis = kwargs.get("axis", args[1] if len(args) > 1 else 0)
        if axis != 0 or set(kwargs) - {"axis", "arrays"}:
            return NotImplemented
        return concat_rows(list(seq))

    def __getitem__(self, idx):
        rows, scalar = _row_index(idx, self.shape[0], self.device)
        out = self._gather(rows)
        return out[0] if scalar else out


class EnvMajorRows(_DeviceRows):
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

    def _gather(self, rows):
        T = self.T
        if isinstance(rows, np.ndarray):       # host rows: one H2D copy of (step, env) per minibatch
            ts, bs = _INDEX_CACHE.get(rows, ("env-major", T), self.device, lambda: tuple(
                torch.from_numpy(np.stack([rows % T, rows // T])).to(self.device, non_blocking=True)))
            return self.buf[ts, bs]
        return self.buf[rows % T, rows // T]

    def materialize(self):
        return self.buf.transpose(0, 1).reshape(self.shape)


class ZeroRows(_DeviceRows):
    """hiddenState rows: all zeros in the reference (runner.py:47-48, never read by the
    net), handed out as expanded zero views, never materialised."""

    def __init__(self, n, row_shape, device):
        self.shape = torch.Size((n,) + tuple(row_shape))
        self.dtype, self.device = torch.float32, torch.device(device)

    def _gather(self, rows):
        k = rows.size if isinstance(rows, np.ndarray) else rows.numel()
        return torch.zeros((), device=self.device).expand((k,) + tuple(self.shape[1:]))

    def materialize(self):
        return torch.zeros(self.shape, device=self.device)


class ConcatRows(_DeviceRows):
    """np.concatenate(parts, axis=0) of device row views, kept lazy: row r belongs to the part
    whose row range holds it.  Indexing gathers each part's share of the rows on the device
    and scatters it into one output in the order asked for."""

    def __init__(self, parts):
        self.parts = parts
        self.offsets = [0]
        for p in parts:
            self.offsets.append(self.offsets[-1] + p.shape[0])
        self.shape = torch.Size((self.offsets[-1],) + tuple(parts[0].shape[1:]))
        self.dtype, self.device = parts[0].dtype, parts[0].device
        self._bounds = torch.tensor(self.offsets[1:], device=self.device)

    def _gather(self, rows):
        if isinstance(rows, np.ndarray):       # host rows: split by part on the host
            part = np.searchsorted(np.asarray(self.offsets[1:]), rows, side="right")
            if (part == part[:1]).all() if rows.size else True:   # one part (driver.py: runner 0's rows)
                k = int(part[0]) if rows.size else 0
                return self.parts[k]._gather(rows - self.offsets[k])
            out = torch.empty((rows.size,) + tuple(self.shape[1:]), dtype=self.dtype, device=self.device)
            for k, p in enumerate(self.parts):
                sel = np.flatnonzero(part == k)
                if sel.size:
                    out[torch.from_numpy(sel).to(self.device)] = p._gather(rows[sel] - self.offsets[k])
            return out
        part = torch.bucketize(rows, self._bounds, right=True)
        out = torch.empty((rows.numel(),) + tuple(self.shape[1:]), dtype=self.dtype, device=self.device)
        for k, p in enumerate(self.parts):
            sel = (part == k).nonzero().squeeze(1)
            if sel.numel():
                out.index_copy_(0, sel, p._gather(rows[sel] - self.offsets[k]))
        return out

    def materialize(self):
        return torch.cat([p.materialize() for p in self.parts], dim=0)


def concat_rows(parts):
    """np.concatenate(parts, axis=0) for device row views (driver.py:119-121)."""
    flat = []
    for p in parts:
        if isinstance(p, ConcatRows):
            flat.extend(p.parts)
        elif isinstance(p, _DeviceRows):
            flat.append(p)
        else:
            raise TypeError(f"np.concatenate of device rows with {type(p).__name__}: every part must stay "
                            "on the device (DeviceRunner results only)")
    if not flat:
        raise ValueError("need at least one array to concatenate")
    first = flat[0]
    for p in flat[1:]:
        if tuple(p.shape[1:]) != tuple(first.shape[1:]) or p.dtype != first.dtype or p.device != first.device:
            raise ValueError(f"row shape/dtype/device mismatch in concatenate: {tuple(first.shape[1:])} "
                             f"{first.dtype} {first.device} vs {tuple(p.shape[1:])} {p.dtype} {p.device}")
    if len(flat) == 1:
        return first
    if all(isinstance(p, ZeroRows) for p in flat):
        return ZeroRows(sum(p.shape[0] for p in flat), first.shape[1:], first.device)
    return ConcatRows(flat)


class BatchValues:
    """util.py:41-54: the rollout's arrays by the reference's attribute names (driver.py reads
    them with getattr over `dir(BatchValues())`), each a device row view; mb["name"] works
    too.  BatchValues() with no arguments is the reference's empty collector (12 lists), so
    driver.py:99-121 runs unchanged whichever of the two classes it imports: there is no
    public attribute besides the 12 fields."""

    def __init__(self, **fields):
        unknown = set(fields) - set(BATCH_FIELDS)
        if unknown:
            raise TypeError(f"unknown BatchValues fields {sorted(unknown)}")
        for k in BATCH_FIELDS:
            setattr(self, k, fields[k] if k in fields else list())

    def __getitem__(self, name):
        return getattr(self, name)


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
            # np.sum over each step's float32 rewards (pairwise order), accumulated from the python
            # int 0 -- which stays np.float32 (NEP 50): float32 over the steps (runner.py:95-96)
            "episodeReward": episode_sum(self.rewards),
            "episodeCostReward": episode_sum(self.cost_rewards),
            "totalGoals": self.goals.sum(dim=(0, 2)), "constraintViolations": self.constraints.sum(dim=(0, 2))}
        return {k: v.double().cpu().numpy() for k, v in per.items()}

    def performance(self):
        """The mean over envs of performance_per_env() (see OneEpPerformance)."""
        p = OneEpPerformance()
        for k, v in self.performance_per_env().items():
            setattr(p, k, float(np.mean(v)))
        return p
