"""BatchedMapfGym: B lockstep MAPF environments resident on one MI355X.

Python face of libmapf.so (include/mapf.h).  Every call is asynchronous on
the current torch HIP stream; inputs and outputs are torch tensors in HBM.
Reference API it batches: mapf_gym.MapfGym / FixedMapfGym (mapf_gym.py:163-669).
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .config import MapfConfig, make_config


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _check(t, dtype, numel, device, name):
    """Every buffer handed to the kernels as a raw pointer: right dtype, contiguous,
    the element count the kernel writes, on the handle's GPU (a wrong one would be
    an out-of-bounds device write, not an error)."""
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor, got {type(t).__name__}")
    if t.dtype != dtype:
        raise TypeError(f"{name}: dtype {t.dtype}, expected {dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: not contiguous")
    if t.numel() != numel:
        raise ValueError(f"{name}: {t.numel()} elements, expected {numel}")
    if device is not None and t.device != device:
        raise ValueError(f"{name}: on {t.device}, expected {device}")
    return t


def parse_tuning(text):
    """ "roll_fair=2,wide_obs=1" -> {"roll_fair": 2, "wide_obs": 1} (mapf_tuning fields)."""
    out = {}
    for kv in (text or "").split(","):
        if kv.strip():
            k, v = kv.split("=")
            out[k.strip()] = int(v)
    return out


class BatchedMapfGym:
    """B environments x N agents on one GPU (one handle per process/GPU)."""

    def __init__(self, cfg: MapfConfig = None, device=None, tuning=None, **kw):
        """tuning: optional mapf_tuning fields (include/mapf.h) as a dict or a "k=v,k=v" string --
        which form of a kernel the launches take; results are identical for every value
        (see set_tuning)."""
        if isinstance(tuning, str):
            tuning = parse_tuning(tuning)
        if cfg is None:
            cfg = make_config(**kw)
        if not torch.cuda.is_available():
            raise RuntimeError("BatchedMapfGym needs a GPU (MI355X); there is no CPU fallback")
        self.cfg = cfg
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device("cuda", dev.index if dev.index is not None else torch.cuda.current_device())
        self.B, self.N, self.H, self.W = cfg.num_envs, cfg.num_agents, cfg.height, cfg.width
        self.F, self.C = cfg.fov, cfg.num_channel
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(_lib.lib().mapf_create(ctypes.byref(cfg), self.device.index, ctypes.byref(h)))
        self.h = h
        self.path_capacity = _lib.lib().mapf_path_capacity(self.h)
        if tuning:
            self.set_tuning(**tuning)
        else:
            self._query_forms()
        dev = self.device
        B, N = self.B, self.N
        self.out = dict(
            status=torch.zeros(B, N, dtype=torch.int8, device=dev),
            reward=torch.zeros(B, N, dtype=torch.float32, device=dev),
            shadow_goals=torch.zeros(B, dtype=torch.int32, device=dev),
            cost=torch.zeros(B, N, dtype=torch.float32, device=dev),
            train_valid=torch.zeros(B, N, 5, dtype=torch.float32, device=dev),
            actions_fixed=torch.zeros(B, N, dtype=torch.int32, device=dev),
            goals_reached=torch.zeros(B, N, dtype=torch.float32, device=dev),
            constraints=torch.zeros(B, N, dtype=torch.float32, device=dev),
            reward_total=torch.zeros(B, N, dtype=torch.float32, device=dev))
        self._stepout = self._make_stepout(self.out)
        self.obs = torch.zeros(B, N, self.C, self.F, self.F, dtype=torch.float32, device=dev)
        self.vec = torch.zeros(B, N, 4, dtype=torch.float32, device=dev)
        self.actions = torch.zeros(B, N, dtype=torch.int32, device=dev)

    def _query_forms(self):
        self.fused = bool(_lib.lib().mapf_step_observe_fused(self.h))   # step_observe = one launch
        # rollout_random = one launch: 1 pair-lane kernel (c2), 2 one wave per env (c4, c5); 0 per-step launches
        self.rollout_kernel = int(_lib.lib().mapf_rollout_random_fused(self.h))
        self.rollout_fused = self.rollout_kernel != 0
        self._roll_fast = None

    @staticmethod
    def default_tuning():
        """mapf_tuning_default as a dict (include/mapf.h: mapf_tuning)."""
        t = _lib.Tuning()
        _lib.lib().mapf_tuning_default(ctypes.byref(t))
        return {n: int(getattr(t, n)) for n in _lib.TUNING_FIELDS}

    def tuning(self):
        t = _lib.Tuning()
        _lib.check(_lib.lib().mapf_get_tuning(self.h, ctypes.byref(t)))
        return {n: int(getattr(t, n)) for n in _lib.TUNING_FIELDS}

    def set_tuning(self, **fields):
        """Change launch-form fields of mapf_tuning (unknown names raise, bad values raise
        through the library's validation); the next launch takes the new form."""
        t = _lib.Tuning()
        _lib.check(_lib.lib().mapf_get_tuning(self.h, ctypes.byref(t)))
        for k, v in fields.items():
            if k not in _lib.TUNING_FIELDS:
                raise KeyError(f"unknown tuning field {k!r}")
            setattr(t, k, int(v))
        _lib.check(_lib.lib().mapf_set_tuning(self.h, ctypes.byref(t)))
        self._query_forms()

    def rollout_plan(self, slots=False):
        """The kernel (template instantiation + form) mapf_rollout_random launches now, as text."""
        buf = ctypes.create_string_buffer(512)
        kind = _lib.lib().mapf_rollout_plan(self.h, 1 if slots else 0, buf, 512)
        if kind < 0:
            _lib.check(kind)
        return buf.value.decode()

    def rollout_kernel_name(self, slots=False):
        """The template instantiation alone, e.g. 'rollout_wide3_kernel<u64,1,false>'."""
        return self.rollout_plan(slots).split(" ")[0]

    @staticmethod
    def _make_stepout(out):
        so = _lib.StepOut()
        for name, _ in _lib.StepOut._fields_:
            t = out.get(name)
            setattr(so, name, t.data_ptr() if t is not None else None)
        return so

    def close(self):
        if getattr(self, "h", None):
            _lib.lib().mapf_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- reset
    def _maps_array(self, maps):
        maps = np.ascontiguousarray(maps, dtype=np.int8)
        if self.cfg.shared_map:
            maps = maps.reshape(1, self.H, self.W)
        else:
            maps = maps.reshape(self.B, self.H, self.W)
        return maps

    def reset_fixed(self, maps, seqs, human_start=None, human_goal=None, human_seq=None):
        """FixedMapfGym (mapf_gym.py:648-669) for every env.

        seqs: [B][N] lists of (row, col) -- start then goals (util.Sequence).
        human_start/goal: [B, 2] (LoopingHuman) or human_seq: [B] lists (FixedPathHuman)."""
        m = self._maps_array(maps)
        S = self.cfg.max_seq
        seq = np.zeros((self.B, self.N, S, 2), np.int32)
        sl = np.zeros((self.B, self.N), np.int32)
        for b in range(self.B):
            for i in range(self.N):
                s = np.asarray(seqs[b][i], np.int32).reshape(-1, 2)
                if len(s) > S:
                    raise ValueError(f"sequence of {len(s)} cells exceeds max_seq={S}")
                seq[b, i, :len(s)] = s
                sl[b, i] = len(s)
        spec = _lib.ResetSpec()
        spec.mode = 0
        keep = [m, seq, sl]
        spec.maps = m.ctypes.data
        spec.seq = seq.ctypes.data
        spec.seq_len = sl.ctypes.data
        if human_seq is not None:
            HS = self.cfg.max_human_seq
            hs = np.zeros((self.B, HS, 2), np.int32)
            hl = np.zeros(self.B, np.int32)
            for b in range(self.B):
                q = np.asarray(human_seq[b], np.int32).reshape(-1, 2)
                hs[b, :len(q)] = q
                hl[b] = len(q)
            keep += [hs, hl]
            spec.human_seq = hs.ctypes.data
            spec.human_seq_len = hl.ctypes.data
        else:
            a = np.ascontiguousarray(np.asarray(human_start, np.int32).reshape(self.B, 2))
            g = np.ascontiguousarray(np.asarray(human_goal, np.int32).reshape(self.B, 2))
            keep += [a, g]
            spec.human_start = a.ctypes.data
            spec.human_goal = g.ctypes.data
        with torch.cuda.device(self.device):
            _lib.check(_lib.lib().mapf_reset(self.h, ctypes.byref(spec), _stream(self.device)))
        del keep

    def reset_seeded(self, maps, seed=0):
        """MapfGym (mapf_gym.py:164-184): human entrance/goal and agent starts/goals drawn on device."""
        m = self._maps_array(maps)
        spec = _lib.ResetSpec()
        spec.mode = 1
        spec.maps = m.ctypes.data
        spec.seed = seed
        with torch.cuda.device(self.device):
            _lib.check(_lib.lib().mapf_reset(self.h, ctypes.byref(spec), _stream(self.device)))

    def reset_generated(self, kind="warehouse", lo=None, hi=None, density=0.3, largest=False, epoch=0, seed=0,
                        return_maps=False):
        """MapfGym() on maps generated on the device (mapf_reset_generated): kind "warehouse"
        draws each env's generateWarehouse length in [lo, hi] (default EnvParameters.WORLD_SIZE,
        mapf_gym.py:166; the H x W stack must hold the longest), "random" fills H x W with
        -(rand < density); largest keeps the largest 4-connected free component.  Then the
        seeded reset (agents, goals, human) as reset_seeded.  Asynchronous; return_maps gives
        the int8 maps as a device tensor [shared_map ? 1 : B, H, W]."""
        from .config import EnvParameters
        spec = _lib.MapGenSpec()
        spec.kind = {"warehouse": _lib.MAPS_WAREHOUSE, "random": _lib.MAPS_RANDOM}[kind]
        ws = EnvParameters.WORLD_SIZE
        spec.lo = ws[0] if lo is None else lo
        spec.hi = ws[1] if hi is None else hi
        spec.largest, spec.density, spec.epoch, spec.seed = int(largest), float(density), int(epoch), int(seed)
        maps = None
        if return_maps:
            maps = torch.empty(1 if self.cfg.shared_map else self.B, self.H, self.W, dtype=torch.int8,
                               device=self.device)
        with torch.cuda.device(self.device):
            _lib.check(_lib.lib().mapf_reset_generated(self.h, ctypes.byref(spec), _ptr(maps),
                                                       _stream(self.device)))
        return maps

    # ----------------------------------------------------------------- step
    def step(self, actions=None, commit=True):
        """One lockstep step (runner.py:64-100 order).  actions: int32 [B, N] on device.
        Returns the dict of output tensors (reused between calls).

        Graph capture: steps and observes may be captured into a hipGraph and
        replayed, provided a captured sequence holds a multiple of 3 committed
        steps (the device work lists rotate over 3 slots)."""
        if actions is None:
            actions = self.actions
        _check(actions, torch.int32, self.B * self.N, self.device, "actions")
        _lib.check(_lib.lib().mapf_step(self.h, _ptr(actions), ctypes.byref(self._stepout),
                                        1 if commit else 0, _stream(self.device)))
        return self.out

    def step_random(self, actions=None, commit=True):
        """Random-policy step: actions drawn on device (written to `actions`), then stepped, one launch."""
        if actions is None:
            actions = self.actions
        _check(actions, torch.int32, self.B * self.N, self.device, "actions")
        _lib.check(_lib.lib().mapf_step_random(self.h, _ptr(actions), ctypes.byref(self._stepout),
                                               1 if commit else 0, _stream(self.device)))
        return self.out

    def observe(self, obs=None, vec=None):
        """getAllObservations for all envs: obs [B, N, C, F, F], vec [B, N, 4] (float32)."""
        obs = self.obs if obs is None else obs
        vec = self.vec if vec is None else vec
        _check(obs, torch.float32, self.B * self.N * self.C * self.F * self.F, self.device, "obs")
        _check(vec, torch.float32, self.B * self.N * 4, self.device, "vec")
        _lib.check(_lib.lib().mapf_observe(self.h, _ptr(obs), _ptr(vec), _stream(self.device)))
        return obs, vec

    def step_observe(self, actions=None, obs=None, vec=None, random_policy=False, out=None):
        """Committed step + getAllObservations in one launch (mapf_step_observe): the same
        outputs as step() followed by observe().  random_policy: draw the actions on device
        into `actions` first (mapf_step_observe_random).  out: optional dict of output
        tensors (the keys of self.out, any subset; missing = not written) to write the step's
        outputs into instead of self.out, e.g. slices of rollout buffers.
        Returns (out, obs, vec)."""
        if actions is None:
            actions = self.actions
        obs = self.obs if obs is None else obs
        vec = self.vec if vec is None else vec
        _check(actions, torch.int32, self.B * self.N, self.device, "actions")
        _check(obs, torch.float32, self.B * self.N * self.C * self.F * self.F, self.device, "obs")
        _check(vec, torch.float32, self.B * self.N * 4, self.device, "vec")
        fn =_lib.lib().mapf_step_observe_random if random_policy else _lib.lib().mapf_step_observe
        so = self._stepout if out is None else self._make_stepout(self._check_out(out))
        _lib.check(fn(self.h, _ptr(actions), ctypes.byref(so), _ptr(obs), _ptr(vec), _stream(self.device)))
        return (self.out if out is None else out), obs, vec

    def rollout_random(self, T, slots=False, actions=None, obs=None, vec=None, out=None):
        """T x step_observe(random_policy=True) -- runner.py:64-100 with the uniform random
        policy, T times -- as ONE launch where mapf_rollout_random_fused (each wave owns an
        env and loops step -> observe -> its search work).  slots: step t writes slot t of
        [T]-leading buffers (actions [T, B, N], obs [T, B, N, C, F, F], vec [T, B, N, 4],
        out[k] [T, ...]); otherwise every step overwrites the [B]-leading buffers.
        Returns (out, obs, vec)."""
        if not slots and actions is None and obs is None and vec is None and out is None:
            # the default [B]-leading buffers (checked at construction): the call's arguments are
            # built once -- a 20-step rollout takes ~300 us on the GPU, so the host's ~8 us of
            # argument checks and ctypes wrapping per call were 2-3 % of it
            key = (id(self.h), id(self.actions), id(self.obs), id(self.vec), id(self._stepout))
            fast = self._roll_fast
            if fast is None or fast[0] != key:
                fast = self._roll_fast = (key, _lib.lib().mapf_rollout_random, self.h, ctypes.byref(self._stepout),
                                          _ptr(self.actions), _ptr(self.obs), _ptr(self.vec))
            _, fn, h, so, pa, po, pv = fast
            _lib.check(fn(h, int(T), 0, pa, so, po, pv, _stream(self.device)))
            return self.out, self.obs, self.vec
        k = T if slots else 1
        actions = self.actions if actions is None else actions
        obs = self.obs if obs is None else obs
        vec = self.vec if vec is None else vec
        _check(actions, torch.int32, k * self.B * self.N, self.device, "actions")
        _check(obs, torch.float32, k * self.B * self.N * self.C * self.F * self.F, self.device, "obs")
        _check(vec, torch.float32, k * self.B * self.N * 4, self.device, "vec")
        if out is None:
            if slots:
                raise ValueError("slots=True needs [T]-leading output buffers (out=...)")
            so, out = self._stepout, self.out
        else:
            for key, t in out.items():
                ref = self.out[key]
                _check(t, ref.dtype, k * ref.numel(), self.device, key)
            so = self._make_stepout(out)
        _lib.check(_lib.lib().mapf_rollout_random(self.h, int(T), 1 if slots else 0, _ptr(actions), ctypes.byref(so),
                                                  _ptr(obs), _ptr(vec), _stream(self.device)))
        return out, obs, vec

    def rollout_launcher(self, T, slots=False, actions=None, obs=None, vec=None, out=None):
        """rollout_random(T, slots, ...) prepared once: the buffers are checked and the C call's
        arguments built now, on the current stream; the returned callable issues the launch with
        no per-call host work beyond one ctypes call (a 20-step rollout is ~350 us on the GPU, the
        checks and wrapping ~60 us of host time).  The buffers must outlive the launcher."""
        k = T if slots else 1
        actions = self.actions if actions is None else actions
        obs = self.obs if obs is None else obs
        vec = self.vec if vec is None else vec
        _check(actions, torch.int32, k * self.B * self.N, self.device, "actions")
        _check(obs, torch.float32, k * self.B * self.N * self.C * self.F * self.F, self.device, "obs")
        _check(vec, torch.float32, k * self.B * self.N * 4, self.device, "vec")
        if out is None:
            if slots:
                raise ValueError("slots=True needs [T]-leading output buffers (out=...)")
            out = self.out
        for key, t in out.items():
            _check(t, self.out[key].dtype, k * self.out[key].numel(), self.device, key)
        so = self._make_stepout(out)
        args = (self.h, int(T), 1 if slots else 0, _ptr(actions), ctypes.byref(so), _ptr(obs), _ptr(vec),
                _stream(self.device))
        fn = _lib.lib().mapf_rollout_random
        keep = (so, actions, obs, vec, out)

        def launch():
            _lib.check(fn(*args))
            return keep[4], keep[2], keep[3]
        return launch

    def _check_out(self, out):
        for k, t in out.items():
            ref = self.out[k]
            _check(t, ref.dtype, ref.numel(), self.device, k)
        return out

    def flush(self):
        """Run pending search work (BFS maps, next human paths) now, in its own launch."""
        _lib.check(_lib.lib().mapf_flush(self.h, _stream(self.device)))

    def release_captures(self):
        """Free the argument slots captured rollouts of this env took (mapf_release_captures):
        only after every hipGraph holding one has been destroyed."""
        _lib.check(_lib.lib().mapf_release_captures(self.h))

    def random_actions(self, out=None):
        out = self.actions if out is None else out
        _check(out, torch.int32, self.B * self.N, self.device, "actions")
        _lib.check(_lib.lib().mapf_random_actions(self.h, _ptr(out), _stream(self.device)))
        return out

    def bfs(self):
        d = torch.empty(self.B, self.N, self.H, self.W, dtype=torch.int16, device=self.device)
        _lib.check(_lib.lib().mapf_bfs(self.h, _ptr(d), _stream(self.device)))
        return d

    def render(self, envs=None, scale=20):
        """renderWorld (util.py:189-232) of the given envs (default all) on the device:
        uint8 RGB frames [n, H*scale, W*scale, 3] on this env's device."""
        idx = torch.arange(self.B, dtype=torch.int32) if envs is None else torch.as_tensor(envs, dtype=torch.int32)
        if idx.numel() and (int(idx.min()) < 0 or int(idx.max()) >= self.B):
            raise IndexError(f"env index out of range 0..{self.B - 1}")
        idx = idx.to(self.device).contiguous()
        out = torch.empty(idx.numel(), self.H * scale, self.W * scale, 3, dtype=torch.uint8, device=self.device)
        _lib.check(_lib.lib().mapf_render(self.h, _ptr(idx), idx.numel(), int(scale), _ptr(out),
                                          _stream(self.device)))
        return out

    def counters(self):
        c = np.zeros(16, np.uint32)
        _lib.check(_lib.lib().mapf_get_counters(self.h, ctypes.c_void_p(c.ctypes.data), _stream(self.device)))
        return c

    def profile(self, reset=True):
        """Phase-cycle sums of the MAPF_STAMPS diagnostic build (zeros otherwise)."""
        c = np.zeros(16, np.uint64)
        _lib.check(_lib.lib().mapf_get_profile(self.h, ctypes.c_void_p(c.ctypes.data), int(reset),
                                               _stream(self.device)))
        return c

    def wave_profile(self, nwaves):
        """Diagnostic (stamps) build: per-wave phase cycles of the last step launch, uint64 [nwaves, 8]."""
        out = np.zeros((nwaves, 8), dtype=np.uint64)
        _lib.check(_lib.lib().mapf_get_wave_profile(self.h, out.ctypes.data_as(ctypes.c_void_p), nwaves,
                                                     _stream(self.device)))
        return out

    def timeline(self, nblocks):
        """Diagnostic (stamps) build: per-workgroup timeline of the last fused launch,
        uint64 [nblocks, 8] (realtime stamps 0-3 at 100 MHz, HW_ID, XCC_ID)."""
        out = np.zeros((nblocks, 8), dtype=np.uint64)
        _lib.check(_lib.lib().mapf_get_timeline(self.h, out.ctypes.data_as(ctypes.c_void_p), nblocks,
                                                 _stream(self.device)))
        return out

    def get_state(self):
        B, N, L = self.B, self.N, self.path_capacity
        st = dict(pos=np.zeros((B, N, 2), np.int32), goal=np.zeros((B, N, 2), np.int32),
                  last_action=np.zeros((B, N), np.int32), seq_cursor=np.zeros((B, N), np.int32),
                  human=np.zeros((B, 10), np.int32), human_path=np.zeros((B, L, 2), np.int32),
                  clock=np.zeros(B, np.uint32))
        s = _lib.State(*[st[n].ctypes.data for n, _ in _lib.State._fields_])
        _lib.check(_lib.lib().mapf_get_state(self.h, ctypes.byref(s), _stream(self.device)))
        return st

    def set_state(self, **kw):
        keep = {}
        s = _lib.State()
        for n, _ in _lib.State._fields_:
            if n in kw and kw[n] is not None:
                dt = np.uint32 if n == "clock" else np.int32
                a = np.ascontiguousarray(kw[n], dtype=dt)
                keep[n] = a
                setattr(s, n, a.ctypes.data)
        _lib.check(_lib.lib().mapf_set_state(self.h, ctypes.byref(s), _stream(self.device)))


def gae(rewards, values, last_values, gamma=0.95, lam=0.95):
    """runner.py:117-149 on device: rewards/values [T, ...] float32, last_values [...]."""
    T = rewards.shape[0]
    M = rewards[0].numel()
    dev = rewards.device
    if dev.type != "cuda":
        raise ValueError("gae: tensors must be on the GPU")
    _check(rewards, torch.float32, T * M, dev, "rewards")
    _check(values, torch.float32, T * M, dev, "values")
    _check(last_values, torch.float32, M, dev, "last_values")
    adv = torch.empty_like(rewards)
    ret = torch.empty_like(rewards)
    _lib.check(_lib.lib().mapf_gae(_ptr(rewards), _ptr(values), _ptr(last_values), _ptr(adv), _ptr(ret), T, M,
                                   gamma, lam, _stream(rewards.device)))
    return adv, ret


def normalize_advantages(returns, values, cost_returns, cost_values, lagrange=0.0, mix=False):
    """model.py:106-113 on device; returns (advantage, cost_advantage)."""
    dev, M = returns.device, returns.numel()
    if dev.type != "cuda":
        raise ValueError("normalize_advantages: tensors must be on the GPU")
    for name, t in (("returns", returns), ("values", values), ("cost_returns", cost_returns),
                    ("cost_values", cost_values)):
        _check(t, torch.float32, M, dev, name)
    adv = torch.empty_like(returns)
    cadv = torch.empty_like(returns)
    _lib.check(_lib.lib().mapf_normalize_advantages(
        _ptr(returns), _ptr(values), _ptr(cost_returns), _ptr(cost_values), _ptr(adv), _ptr(cadv),
        returns.numel(), float(lagrange), int(mix), _stream(returns.device)))
    return adv, cadv


def normalize_advantages_dlam(returns, values, cost_returns, cost_values, lam2, mix=False):
    """normalize_advantages with the multiplier in device memory: lam2 = float32 [2] on the GPU,
    {f32(lagrange), f32(lagrange + 1)} (mapf_normalize_advantages_dlam) -- capturable once and
    replayed with a new multiplier written into lam2."""
    dev, M = returns.device, returns.numel()
    for name, t in (("returns", returns), ("values", values), ("cost_returns", cost_returns),
                    ("cost_values", cost_values)):
        _check(t, torch.float32, M, dev, name)
    _check(lam2, torch.float32, 2, dev, "lam2")
    adv = torch.empty_like(returns)
    cadv = torch.empty_like(returns)
    _lib.check(_lib.lib().mapf_normalize_advantages_dlam(
        _ptr(returns), _ptr(values), _ptr(cost_returns), _ptr(cost_values), _ptr(adv), _ptr(cadv), M, _ptr(lam2),
        int(mix), _stream(dev)))
    return adv, cadv


def normalize_advantages_distributed(returns, values, cost_returns, cost_values, lagrange=0.0, mix=False, group=None,
                                     lam2=None):
    """normalize_advantages over a minibatch split across the ranks of torch.distributed: this
    rank's rows in, this rank's rows out, normalised with the GLOBAL mean and unbiased std
    (model.py:106-113 on the whole minibatch).  Two-pass fp64 moments on the device
    (mapf_advantage_moments), each pass all-reduced (2 small all-reduces), then
    mapf_normalize_advantages_stats.  lam2: the multiplier in device memory instead of
    `lagrange` (float32 [2] = {f32(lagrange), f32(lagrange + 1)}, as normalize_advantages_dlam;
    mapf_normalize_advantages_stats_dlam) -- Model.train's distributed device update."""
    if returns.device.type != "cuda":
        raise ValueError("normalize_advantages_distributed: tensors must be on the GPU")
    if lam2 is not None:
        _check(lam2, torch.float32, 2, returns.device, "lam2")
    stats = advantage_stats_distributed(returns, values, cost_returns, cost_values, group=group)
    return normalize_advantages_with_stats(returns, values, cost_returns, cost_values, stats, lagrange, mix, lam2)


def advantage_stats_distributed(returns, values, cost_returns, cost_values, group=None, out=None):
    """The GLOBAL advantage statistics of normalize_advantages_distributed: float64 [4] = {mean(r - v),
    mean(cr - cv), unbiased var(r - v), unbiased var(cr - cv)} over every rank's rows (two-pass fp64
    moments, each pass all-reduced).  out: a float64 [4] device tensor to write them into (the
    segmented captured update keeps them in a static buffer its graph reads)."""
    import torch.distributed as dist
    dev, M = returns.device, returns.numel()
    for name, t in (("returns", returns), ("values", values), ("cost_returns", cost_returns),
                    ("cost_values", cost_values)):
        _check(t, torch.float32, M, dev, name)
    st, L = _stream(dev), _lib.lib()
    ptrs = [_ptr(t) for t in (returns, values, cost_returns, cost_values)]
    buf = torch.zeros(3, dtype=torch.float64, device=dev)          # sum x, sum c, rows
    buf[2] = M
    _lib.check(L.mapf_advantage_moments(*ptrs, M, None, _ptr(buf), st))
    dist.all_reduce(buf, group=group)
    mean = (buf[:2] / buf[2]).contiguous()
    q = torch.zeros(2, dtype=torch.float64, device=dev)
    _lib.check(L.mapf_advantage_moments(*ptrs, M, _ptr(mean), _ptr(q), st))
    dist.all_reduce(q, group=group)
    stats = torch.cat([mean, q / (buf[2] - 1).clamp_min(1)])
    if out is None:
        return stats.contiguous()
    _check(out, torch.float64, 4, dev, "out")
    return out.copy_(stats)


def normalize_advantages_with_stats(returns, values, cost_returns, cost_values, stats, lagrange=0.0, mix=False,
                                    lam2=None):
    """model.py:106-113 with given statistics (advantage_stats_distributed's float64 [4]): this rank's
    rows normalised (mapf_normalize_advantages_stats[_dlam]); no collective, so capturable."""
    dev, M = returns.device, returns.numel()
    for name, t in (("returns", returns), ("values", values), ("cost_returns", cost_returns),
                    ("cost_values", cost_values)):
        _check(t, torch.float32, M, dev, name)
    _check(stats, torch.float64, 4, dev, "stats")
    if lam2 is not None:
        _check(lam2, torch.float32, 2, dev, "lam2")
    st, L = _stream(dev), _lib.lib()
    ptrs = [_ptr(t) for t in (returns, values, cost_returns, cost_values)]
    adv = torch.empty_like(returns)
    cadv = torch.empty_like(returns)
    if lam2 is None:
        _lib.check(L.mapf_normalize_advantages_stats(*ptrs, _ptr(stats), _ptr(adv), _ptr(cadv), M, float(lagrange),
                                                     int(mix), st))
    else:
        _lib.check(L.mapf_normalize_advantages_stats_dlam(*ptrs, _ptr(stats), _ptr(adv), _ptr(cadv), M, _ptr(lam2),
                                                          int(mix), st))
    return adv, cadv


def episode_sum(x):
    """OneEpPerformance.episodeReward-style sums (runner.py:95-96) of every env: x [T, B, N] float32
    on the GPU -> [B] float32, each step's numpy float32 np.sum over N accumulated in float32."""
    T, B, N = x.shape
    _check(x, torch.float32, T * B * N, x.device, "x")
    out = torch.empty(B, dtype=torch.float32, device=x.device)
    _lib.check(_lib.lib().mapf_episode_sum(_ptr(x), T, B, N, _ptr(out), _stream(x.device)))
    return out


def sample_actions(ps, seed, step, out32=None, out64=None):
    """model.py:38-40 on device: ps [..., 5] float32 -> actions."""
    ps2 = ps.reshape(-1, ps.shape[-1])
    if ps2.dtype != torch.float32 or ps2.stride(1) != 1 or ps2.shape[-1] != 5 or ps2.device.type != "cuda":
        raise ValueError("sample_actions: ps must be float32 [..., 5] on the GPU with unit stride in the last dim")
    M = ps2.shape[0]
    if out32 is None and out64 is None:
        raise ValueError("sample_actions: give out32 and/or out64")
    if out32 is not None:
        _check(out32, torch.int32, M, ps2.device, "out32")
    if out64 is not None:
        _check(out64, torch.int64, M, ps2.device, "out64")
    _lib.check(_lib.lib().mapf_sample_actions(_ptr(ps2), ps2.stride(0), _ptr(out32), _ptr(out64), M, seed, step,
                                              _stream(ps.device)))
    return out32 if out32 is not None else out64
