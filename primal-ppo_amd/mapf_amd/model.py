"""Model: action sampling, value bootstrap and the PPO-Lagrangian update.

Mirrors the reference's Model (model.py:13-231) and Lagrangian multipliers
(lagrange.py:26-88), with the device-resident pieces of the hot path:
  * step(): the policy forward + on-device categorical sampling (mapf_sample_actions
    in place of np.random.choice, model.py:38-40);
  * train(): advantage normalisation by the HIP kernels (mapf_normalize_advantages_dlam,
    model.py:106-113) -- statistics over the GLOBAL minibatch when distributed (two-pass
    fp64 moments all-reduced, mapf_normalize_advantages_stats_dlam; _DeviceUpdate.body) --
    then the reference's loss (:115-170), AMP GradScaler, and between backward and
    unscale the RCCL all-reduce of the flattened gradient bucket (SURVEY.md §3.4:
    the only exchange step of the path).  Every rank then holds the same gradient, so
    found-inf, clipping, Adam and the loss scale agree across ranks; the returned stats are
    averaged over the ranks (the global minibatch's means when the shards are equal).
"""
import ctypes

import numpy as np
import torch
import torch.distributed as dist
import torch.nn.functional as F

from .config import EnvParameters, LagrangianParameters, NetParameters, TrainingParameters
from .net import SCRIMPNet


class _FusedPPOLoss(torch.autograd.Function):
    """model.py:115-175's loss terms and their gradient in one HIP launch
    (csrc/mapf_ppo.hip, mapf_ppo_loss).  Returns (all_loss, terms[7] = policy, entropy,
    critic, valid, cost critic, cost, clip_frac); only all_loss carries a gradient."""

    @staticmethod
    def forward(ctx, new_ps, new_v, new_cv, policy_sig, old_ps, action, old_v, returns, old_cv, cost_returns,
                advantage, cost_advantage, train_valid, coef):
        from . import _lib
        A = new_ps.shape[-1]
        R = new_ps.numel() // A
        f = lambda t, *shape: t.detach().float().reshape(*shape).contiguous()
        ins = [f(new_ps, R, A), f(old_ps, R, A), action.detach().long().reshape(R).contiguous()]
        vecs = [f(t, R) for t in (new_v, old_v, returns, new_cv, old_cv, cost_returns, advantage, cost_advantage)]
        sig, tv = f(policy_sig, R, A), f(train_valid, R, A)
        loss = torch.empty((), device=new_ps.device)
        terms = torch.empty(7, device=new_ps.device)
        grads = [torch.empty(R, A, device=new_ps.device), torch.empty(R, device=new_ps.device),
                 torch.empty(R, device=new_ps.device), torch.empty(R, A, device=new_ps.device)]
        p = lambda t: ctypes.c_void_p(t.data_ptr())
        st = ctypes.c_void_p(torch.cuda.current_stream(new_ps.device).cuda_stream)
        if isinstance(coef, torch.Tensor):     # device coefficients (the captured update)
            fn, c = _lib.lib().mapf_ppo_loss_dcoef, p(coef)
        else:
            fn, c = _lib.lib().mapf_ppo_loss, (ctypes.c_float * 6)(*coef)
        _lib.check(fn(*[p(t) for t in ins], *[p(t) for t in vecs[:6]], p(vecs[6]), p(vecs[7]), p(sig),
                      int(policy_sig.dtype == torch.float16), p(tv), R, A, c, p(loss), p(terms),
                      *[p(g) for g in grads], st))
        ctx.save_for_backward(*grads)
        ctx.meta = [(t.shape, t.dtype) for t in (new_ps, new_v, new_cv, policy_sig)]
        ctx.mark_non_differentiable(terms)
        return loss, terms

    @staticmethod
    def backward(ctx, g_loss, g_terms):
        out = [(g * g_loss).reshape(shape).to(dtype) for g, (shape, dtype) in zip(ctx.saved_tensors, ctx.meta)]
        return (*out,) + (None,) * 10


class Lagrangian:
    """lagrange.py:26-53: softplus-parameterised multiplier trained by Adam."""

    def __init__(self, cost_limit):
        self.cost_limit = cost_limit
        self.lagrangian_param = torch.tensor(max(0.0, LagrangianParameters.INIT_VALUE), requires_grad=True).float()
        self.lagrangian_optimizer = torch.optim.Adam([self.lagrangian_param], lr=LagrangianParameters.LR)

    def get_lagrangian_param(self):
        return F.softplus(self.lagrangian_param).detach().item()

    def update_lagrangian_multiplier(self, ep_cost_avg):
        loss = -self.lagrangian_param * (ep_cost_avg - self.cost_limit)
        self.lagrangian_optimizer.zero_grad()
        loss.backward()
        self.lagrangian_optimizer.step()
        self.lagrangian_param.data.clamp_(0.0, LagrangianParameters.UPPER_BOUND)


class PIDLagrangian:
    """lagrange.py:55-88: PID-controlled multiplier (CPPO-PID)."""

    def __init__(self, cost_limit):
        self.cost_limit = cost_limit
        self.i_term = max(0.0, LagrangianParameters.INIT_VALUE)
        self.lagrangian_param = 0.0
        self.delta_moving_avg = 0.0
        self.cost_moving_avg = 0.0
        self.cost_moving_avg_prev = 0.0

    def get_lagrangian_param(self):
        return self.lagrangian_param

    def update_lagrangian_multiplier(self, ep_cost_avg):
        P = LagrangianParameters
        delta = ep_cost_avg - self.cost_limit
        self.delta_moving_avg = self.delta_moving_avg * P.DELTA_MOVING_AVG_ALPHA + (1 - P.DELTA_MOVING_AVG_ALPHA) * delta
        self.cost_moving_avg = self.cost_moving_avg * P.COST_MOVING_AVG_ALPHA + (1 - P.COST_MOVING_AVG_ALPHA) * ep_cost_avg
        d_term = max(0.0, self.cost_moving_avg - self.cost_moving_avg_prev)
        self.i_term = max(0.0, self.i_term + delta * P.KI)
        self.lagrangian_param = max(0.0, P.KP * self.delta_moving_avg + self.i_term + P.KD * d_term)
        self.cost_moving_avg_prev = self.cost_moving_avg


def get_lagrangian(kind, cost_limit):
    return Lagrangian(cost_limit) if kind == 0 else PIDLagrangian(cost_limit)


def _normalize(x):
    """model.py:106: (x - mean) / (std_unbiased + 1e-6); global statistics across ranks."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        s = torch.stack([x.sum(), (x * x).sum(), torch.tensor(float(x.numel()), device=x.device)]).double()
        dist.all_reduce(s)
        n = s[2]
        mean = s[0] / n
        var = (s[1] - n * mean * mean) / (n - 1)
        return (x - mean.float()) / (var.clamp_min(0).sqrt().float() + 1e-6)
    return (x - x.mean()) / (x.std() + 1e-6)


class Model:
    # PyTorch TunableOp with the shipped per-shape GEMM solutions (gemm_tuning.py).  PROCESS-WIDE: once a
    # CUDA Model is built, every later GEMM of the process whose shape is in the file (user code too)
    # takes the listed hipBLASLt solution.  Set Model.tuned_gemms = False before the first Model to keep
    # torch's defaults (or set PYTORCH_TUNABLEOP_ENABLED yourself).
    tuned_gemms = True

    def __init__(self, env_id, device, global_model=False, numChannel=None, num_agents=None, fov=None):
        self.ID = env_id
        self.device = torch.device(device)
        self.network = SCRIMPNet(numChannel=numChannel, num_agents=num_agents, fov=fov).to(self.device)
        if self.device.type == "cuda":     # NHWC convolutions: no layout transposes around MIOpen's kernels
            self.network = self.network.to(memory_format=torch.channels_last)
            if self.tuned_gemms:
                from .gemm_tuning import use_tuned_gemms
                use_tuned_gemms()          # the measured-best hipBLASLt solution per GEMM shape (gemm_tuning.py)
            # MIOpen find mode: the per-shape conv solver is measured once and cached
            # (c3 policy forward 23.1 -> 20.7 ms at 32,768 agents)
            torch.backends.cudnn.benchmark = True
        self.num_agents = num_agents or EnvParameters.N_AGENTS
        self._flat = None
        self.fused_loss = True        # GPU: the loss terms + their gradient in one launch (_FusedPPOLoss)
        self.graph_update = True      # GPU: the update replayed from captured hipGraphs (_DeviceUpdate)
        # GPU: unscale + clip + Adam as mapf_optim_unscale_clip_adam (_DeviceUpdate._fused_tail) instead of torch's
        # passes: tested equal, but not faster in its current form (profiles/r06zk_ab_optim*.txt), so off
        self.fused_optim = False
        self.distributed_update = None  # None: the all-reduced update when world size > 1; True / False: forced
        self._updates = {}
        if global_model:
            # fused Adam on the GPU: one launch for every parameter, and the AMP found-inf skip taken
            # on the device (optimizer.found_inf), so the update has no host synchronisation
            gpu = self.device.type == "cuda"
            self.net_optimizer = torch.optim.Adam(self.network.parameters(), lr=TrainingParameters.lr, fused=gpu,
                                                  capturable=gpu)
            self.lagrange = get_lagrangian(LagrangianParameters.LAGRANGIAN_TYPE, TrainingParameters.COST_LIMIT_PER_AGENT)
            self.net_scaler = torch.amp.GradScaler(self.device.type, enabled=self.device.type == "cuda")
            self.broadcast_weights()

    def broadcast_weights(self, src=0):
        """SURVEY.md §8(e) "weights broadcast at init": when torch.distributed is initialised with
        more than one rank, every rank takes rank `src`'s parameters and buffers (one RCCL / gloo
        broadcast per dtype bucket), so ranks constructed with different seeds hold one model
        before the first all-reduced update (the reference has one global model, driver.py:50).
        Collective: every rank must construct its global Model (or call this) in the same order.
        Returns True if a broadcast ran."""
        if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
            return False
        tensors = list(self.network.parameters()) + list(self.network.buffers())
        for dtype in sorted({t.dtype for t in tensors}, key=str):
            group = [t for t in tensors if t.dtype == dtype]
            flat = torch.cat([t.detach().reshape(-1) for t in group])
            dist.broadcast(flat, src)
            off = 0
            with torch.no_grad():
                for t in group:      # copy_ bumps the version: the fp16 weight cache (_half) re-reads
                    t.copy_(flat[off:off + t.numel()].view_as(t))
                    off += t.numel()
        return True

    # ------------------------------------------------------------ acting
    @torch.no_grad()
    def step(self, observation, vector, input_state=None, seed=0, step=0, actions_out=None, actions32_out=None):
        """model.py:26-41 on device: returns (actions int64, ps, v, block, output_state, cv) as tensors.
        Sampling: inverse CDF with a Philox uniform (mapf_sample_actions); actions32_out: also
        write the actions as int32 (the env's action format) in the same launch."""
        ps, v, block, _, out_state, _, cv = self.network(observation, vector, input_state)
        ps32 = ps.float().contiguous()
        if self.device.type == "cuda":
            from .env import sample_actions
            a = actions_out if actions_out is not None else torch.empty(ps32.shape[:-1], dtype=torch.int64,
                                                                         device=self.device)
            sample_actions(ps32, seed, step, out32=actions32_out, out64=a)
        else:
            a = torch.multinomial(ps32.reshape(-1, ps32.shape[-1]), 1).reshape(ps32.shape[:-1])
        return a, ps32, v.float(), block.float(), out_state, cv.float()

    @torch.no_grad()
    def value(self, obs, vector, input_state=None):
        """model.py:62-69."""
        _, v, _, _, _, _, cv = self.network(obs, vector, input_state)
        return v.float(), cv.float()

    def set_weights(self, weights):
        self.network.load_state_dict(weights)

    # ------------------------------------------------------------ learning
    def _allreduce_grads(self):
        """One bucketed all-reduce (RCCL over xGMI) of every gradient, averaged over ranks."""
        if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
            return
        params = [p for p in self.network.parameters() if p.grad is not None]
        flat = torch.cat([p.grad.reshape(-1) for p in params])
        dist.all_reduce(flat)
        flat.div_(dist.get_world_size())
        off = 0
        for p in params:
            n = p.grad.numel()
            p.grad.copy_(flat[off:off + n].view_as(p.grad))
            off += n

    def train(self, observation, vector, returns, cost_returns, old_v, old_cv, action, old_ps, input_state,
              train_valid, episode_cost):
        """model.py:78-199.  Inputs may be numpy arrays (reference contract) or device tensors."""
        dev = self.device
        t = lambda x: (torch.from_numpy(x) if isinstance(x, np.ndarray) else x).to(dev)
        observation, vector = t(observation), t(vector)
        returns, old_v, cost_returns, old_cv = t(returns).float(), t(old_v).float(), t(cost_returns).float(), t(old_cv).float()
        action = t(action).long().unsqueeze(-1)
        old_ps, train_valid = t(old_ps).float(), t(train_valid).float()

        lam = self.lagrange.get_lagrangian_param()
        distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        if self.distributed_update is not None:     # forced (measurement: the c4 path at world size 1)
            distributed = bool(self.distributed_update) and dist.is_available() and dist.is_initialized()
        if dev.type == "cuda" and self.fused_loss:      # the device update (fused loss, captured graph)
            return self._train_device(observation, vector, returns, cost_returns, old_v, old_cv, action, old_ps,
                                      input_state, train_valid, episode_cost, lam, distributed)
        if dev.type == "cuda":
            # the HIP normalisation; distributed: global two-pass moments all-reduced into it
            from .env import normalize_advantages, normalize_advantages_distributed
            fn = normalize_advantages_distributed if distributed else normalize_advantages
            advantage, cost_advantage = fn(returns.contiguous(), old_v.contiguous(), cost_returns.contiguous(),
                                           old_cv.contiguous(), lagrange=lam, mix=TrainingParameters.MINUS_ADV_WITH_CADV)
        else:                   # CPU (the gloo tests' host path): torch, global statistics when distributed
            advantage = _normalize(returns - old_v)
            cost_advantage = _normalize(cost_returns - old_cv)
            if TrainingParameters.MINUS_ADV_WITH_CADV:
                advantage = (advantage - lam * cost_advantage) / (lam + 1)

        self.net_optimizer.zero_grad()
        with torch.autocast(device_type=dev.type, enabled=dev.type == "cuda"):
            new_ps, new_v, block, policy_sig, _, _, new_cv = self.network(observation, vector, input_state)
            new_p = new_ps.gather(-1, action)
            old_p = old_ps.gather(-1, action)
            ratio = torch.exp(torch.log(torch.clamp(new_p, 1e-6, 1.0)) - torch.log(torch.clamp(old_p, 1e-6, 1.0)))
            entropy = torch.mean(-torch.sum(new_ps * torch.log(torch.clamp(new_ps, 1e-6, 1.0)), dim=-1, keepdim=True))
            clip = TrainingParameters.CLIP_RANGE
            new_v = torch.squeeze(new_v)
            v_clip = old_v + torch.clamp(new_v - old_v, -clip, clip)
            critic_loss = torch.mean(torch.maximum(torch.square(new_v - returns), torch.square(v_clip - returns)))
            new_cv = torch.squeeze(new_cv)
            cv_clip = old_cv + torch.clamp(new_cv - old_cv, -clip, clip)
            cost_critic_loss = torch.mean(torch.maximum(torch.square(new_cv - cost_returns),
                                                        torch.square(cv_clip - cost_returns)))
            ratio = torch.squeeze(ratio)
            policy_loss = torch.mean(torch.min(advantage * ratio, advantage * torch.clamp(ratio, 1.0 - clip, 1.0 + clip)))
            valid_loss = -torch.mean(torch.log(torch.clamp(policy_sig, 1e-6, 1.0 - 1e-6)) * train_valid +
                                     torch.log(torch.clamp(1 - policy_sig, 1e-6, 1.0 - 1e-6)) * (1 - train_valid))
            cost_loss = torch.mean(ratio * cost_advantage)
            all_loss = (-policy_loss - entropy * TrainingParameters.ENTROPY_COEF
                        + TrainingParameters.VALUE_COEF * critic_loss + TrainingParameters.VALID_COEF * valid_loss
                        + TrainingParameters.COST_VALUE_COEF * cost_critic_loss
                        + TrainingParameters.COST_COEF * lam * cost_loss)
        clip_frac = torch.mean(torch.greater(torch.abs(ratio - 1.0), clip).float())
        return self._finish_update(all_loss, policy_loss, entropy, critic_loss, valid_loss, cost_critic_loss,
                                   cost_loss, clip_frac, advantage, cost_advantage, episode_cost, distributed)

    # ------------------------------------------------------------ the device update
    def _train_device(self, observation, vector, returns, cost_returns, old_v, old_cv, action, old_ps, input_state,
                      train_valid, episode_cost, lam, distributed):
        """model.py:78-199 on the GPU with no host synchronisation inside the update: HIP
        normalisation (multiplier in device memory), autocast forward, the fused loss (its
        coefficients in device memory), backward, [RCCL all-reduce of the gradient bucket],
        AMP unscale + found-inf on the device, clip, fused Adam skipping on found-inf, loss-scale
        update -- GradScaler's semantics (init 2^16, x2 every 2000 finite steps, x0.5 on inf).
        After two eager updates of a minibatch shape the body is captured and every later update of
        that shape replays it (the host launched ~1,500 small ops per update): one hipGraph on one
        rank; distributed, two graph segments with the collectives between them run eagerly -- the
        advantage moments' two all-reduces (global statistics) before segment A (normalise ->
        forward -> loss -> backward into a static gradient bucket), the bucket's all-reduce between
        backward and unscale (model.py:177-185), segment B (unscale -> clip -> Adam -> scale update),
        then the stats' all-reduce (_DeviceUpdate.run).  input_state is ignored, as the network ignores it (net.py:102-155 never
        reads it): driver.py passes the rollout's zero hiddenState rows, never None.
        The loss scale and its growth tracker are net_scaler's own tensors (one AMP state per
        model, as the reference's one GradScaler, shared by every minibatch shape and by the
        eager path)."""
        key = (tuple(observation.shape), tuple(vector.shape), tuple(old_ps.shape), tuple(train_valid.shape))
        sc = self.net_scaler
        if sc._scale is None:
            sc._lazy_init_scale_growth_tracker(self.device)
        upd = self._updates.get(key)
        if upd is not None and not upd.uses(sc):
            upd = None                        # net_scaler replaced or reconfigured: re-capture
        if upd is None:
            upd = self._updates[key] = _DeviceUpdate(self, observation, vector, returns, old_ps, train_valid, action)
        T = TrainingParameters
        upd.load(observation, vector, returns, cost_returns, old_v, old_cv, action, old_ps, train_valid,
                 coef=(T.CLIP_RANGE, T.ENTROPY_COEF, T.VALUE_COEF, T.VALID_COEF, T.COST_VALUE_COEF, T.COST_COEF * lam),
                 lam=lam)
        upd.run(graph=self.graph_update, allreduce=distributed)
        # the Lagrangian step (host, model.py:180) depends only on the episode cost
        if distributed:   # every rank must update the multiplier with the same episode cost
            c = torch.tensor([float(episode_cost)], dtype=torch.float64, device=self.device)
            dist.all_reduce(c)
            episode_cost = c.item() / dist.get_world_size()
        self.lagrange.update_lagrangian_multiplier(episode_cost / EnvParameters.N_AGENTS)
        self.network.weights_updated()        # replays bump no tensor version: drop the fp16 acting copies
        stats = upd.stats.cpu().numpy()       # one device -> host copy
        return [np.asarray(v) for v in stats] + [self.lagrange.get_lagrangian_param()]

    def _finish_update(self, all_loss, policy_loss, entropy, critic_loss, valid_loss, cost_critic_loss, cost_loss,
                       clip_frac, advantage, cost_advantage, episode_cost, distributed):
        """model.py:177-199: backward, gradient exchange, Lagrangian step, clip, Adam, stats."""
        dev = self.device
        self.net_scaler.scale(all_loss).backward()
        self._allreduce_grads()
        self.net_scaler.unscale_(self.net_optimizer)
        if distributed:   # every rank must update the multiplier with the same episode cost
            c = torch.tensor([float(episode_cost)], dtype=torch.float64, device=dev)
            dist.all_reduce(c)
            episode_cost = c.item() / dist.get_world_size()
        self.lagrange.update_lagrangian_multiplier(episode_cost / EnvParameters.N_AGENTS)
        grad_norm = torch.nn.utils.clip_grad_norm_(self.network.parameters(), TrainingParameters.MAX_GRAD_NORM)
        self.net_scaler.step(self.net_optimizer)
        self.net_scaler.update()
        stats = torch.stack([t.detach().float().reshape(()) for t in (
            all_loss, policy_loss, entropy, critic_loss, valid_loss, cost_critic_loss, cost_loss, clip_frac, grad_norm,
            torch.mean(advantage), torch.mean(cost_advantage))]).cpu().numpy()       # one device -> host copy
        return [np.asarray(v) for v in stats] + [self.lagrange.get_lagrangian_param()]


_REDUCTIONS_OK = {}


def captured_reductions_ok(device):
    """Whether a captured multi-block torch reduction gives the right sum on every replay in this
    process (mapf_amd/__init__.py: with the HIP runtime's packet capture on, the captured memset that
    zeroes the reduction's semaphores takes effect on the first replay only).  One exact fp32 sum of
    1088 x 1536 ones, captured, its output poisoned with NaN before each of three replays."""
    dev = torch.device(device)
    key = (dev.type, dev.index if dev.index is not None else torch.cuda.current_device())
    if key not in _REDUCTIONS_OK:
        x = torch.ones(1088, 1536, device=dev)
        want = float(x.numel())                   # < 2^24: exact in fp32 whatever the order
        g, s = torch.cuda.CUDAGraph(), torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                y = x.sum().reshape(1)
        torch.cuda.current_stream(dev).wait_stream(s)
        got = []
        for _ in range(3):
            y.fill_(float("nan"))
            g.replay()
            got.append(y.item())
        del g
        _REDUCTIONS_OK[key] = all(v == want for v in got)
        if not _REDUCTIONS_OK[key]:
            import warnings
            warnings.warn(f"captured torch reductions replay wrong on this HIP runtime ({got}, want {want}; "
                          f"is DEBUG_CLR_GRAPH_PACKET_CAPTURE=1?): the PPO update runs eagerly", RuntimeWarning)
    return _REDUCTIONS_OK[key]


class _DeviceUpdate:
    """The static buffers and the body of one minibatch shape's device update (Model._train_device)."""

    WARMUP = 2          # eager updates before the capture (allocator, MIOpen find, Adam state)

    def __init__(self, model, observation, vector, returns, old_ps, train_valid, action):
        dev = model.device
        self.model = model
        e = lambda x, dt=torch.float32: torch.zeros(tuple(x.shape), dtype=dt, device=dev)   # noqa: E731
        self.obs, self.vec = e(observation), e(vector)
        self.ret, self.cret, self.v, self.cv = e(returns), e(returns), e(returns), e(returns)
        self.action = e(action, torch.int64)
        self.old_ps, self.tv = e(old_ps), e(train_valid)
        self.dyn = torch.zeros(8, dtype=torch.float32, device=dev)     # coef[6], lam, f32(lam + 1)
        sc = model.net_scaler                  # its live state and settings (GradScaler: 2^16, x2 / 2000, x0.5)
        self.scaler = sc
        self.scale, self.growth = sc._scale, sc._growth_tracker        # 0-dim device tensors, updated in place
        self.amp = self._amp_settings(sc)
        self.found_inf = torch.zeros((), dtype=torch.float32, device=dev)
        self.stats = torch.zeros(11, dtype=torch.float32, device=dev)
        self.nstats = torch.zeros(4, dtype=torch.float64, device=dev)    # global advantage statistics (distributed)
        self.grad_params, self.flat = None, None                          # the gradient bucket (distributed)
        self.live = None
        self.graph = None                    # one CUDAGraph, or (segment A, segment B) when distributed
        self.graph_allreduce = False
        self.eager_runs = 0

    @staticmethod
    def _amp_settings(sc):
        return float(sc._growth_factor), float(sc._backoff_factor), int(sc._growth_interval)

    def uses(self, sc):
        """True while this update's captured AMP state is `sc`'s (same tensors, same settings)."""
        return (self.scaler is sc and self.scale is sc._scale and self.growth is sc._growth_tracker
                and self.amp == self._amp_settings(sc))

    def load(self, observation, vector, returns, cost_returns, old_v, old_cv, action, old_ps, train_valid, coef, lam):
        for dst, src in ((self.obs, observation), (self.vec, vector), (self.ret, returns), (self.cret, cost_returns),
                         (self.v, old_v), (self.cv, old_cv), (self.old_ps, old_ps), (self.tv, train_valid)):
            dst.copy_(src.reshape(dst.shape), non_blocking=True)
        self.action.copy_(action.reshape(self.action.shape), non_blocking=True)
        # host double -> f32 exactly as the host-argument kernels round them
        h = torch.tensor(list(coef) + [lam, lam + 1.0], dtype=torch.float64).float()
        self.dyn.copy_(h.pin_memory() if torch.cuda.is_available() else h, non_blocking=True)

    def _front(self, allreduce):
        """normalise -> forward -> fused loss -> backward (graph segment A when distributed); with
        allreduce, the normalisation reads the global statistics in self.nstats (computed and
        all-reduced by _moments before the segment) and the gradients end in the static bucket"""
        net, opt = self.model.network, self.model.net_optimizer
        T = TrainingParameters
        opt.zero_grad(set_to_none=True)
        from .env import normalize_advantages_dlam, normalize_advantages_with_stats
        ins = (self.ret.reshape(-1), self.v.reshape(-1), self.cret.reshape(-1), self.cv.reshape(-1))
        if allreduce:    # model.py:106-113 over the GLOBAL minibatch: moments all-reduced
            adv, cadv = normalize_advantages_with_stats(*ins, self.nstats, mix=T.MINUS_ADV_WITH_CADV,
                                                        lam2=self.dyn[6:8])
        else:
            adv, cadv = normalize_advantages_dlam(*ins, self.dyn[6:8], T.MINUS_ADV_WITH_CADV)
        adv, cadv = adv.view(self.ret.shape), cadv.view(self.ret.shape)
        with torch.autocast(device_type="cuda", cache_enabled=False):
            new_ps, new_v, block, policy_sig, _, _, new_cv = net(self.obs, self.vec, None)
        all_loss, terms = _FusedPPOLoss.apply(new_ps, new_v, new_cv, policy_sig, self.old_ps, self.action.unsqueeze(-1),
                                              self.v, self.ret, self.cv, self.cret, adv, cadv, self.tv, self.dyn[:6])
        (all_loss * self.scale).backward()
        self.live = (all_loss, terms, adv, cadv)       # read by _back (kept alive: graph A writes them)
        if allreduce:    # the flattened gradient bucket (model.py:177-185: all-reduced between backward and unscale)
            gp = [p for p in net.parameters() if p.grad is not None]
            if self.grad_params is None:
                self.grad_params = gp
                self.flat = torch.empty(sum(p.numel() for p in gp), dtype=torch.float32, device=self.model.device)
            assert len(gp) == len(self.grad_params) and all(a is b for a, b in zip(gp, self.grad_params))
            # each gradient's elements in memory order (AccumulateGrad lays a dense parameter's gradient out
            # like the parameter: contiguous or channels_last), so _back's views of the bucket take the
            # parameter's own strides -- fused Adam wants parameter and gradient alike
            assert all(p.grad.stride() == p.stride() for p in gp)
            torch.cat([p.grad.as_strided((p.numel(),), (1,)) for p in gp], out=self.flat)

    def _back(self, allreduce):
        """[bucket averaged over the ranks] -> unscale + found-inf -> clip -> fused Adam -> loss-scale
        update -> stats (graph segment B when distributed)"""
        net, opt = self.model.network, self.model.net_optimizer
        T = TrainingParameters
        if allreduce:    # the parameters' gradients become views of the all-reduced bucket (no copy back)
            self.flat.div_(dist.get_world_size())
            off = 0
            for p in self.grad_params:
                p.grad = self.flat.as_strided(p.shape, p.stride(), off)
                off += p.numel()
        params = [p for p in net.parameters() if p.grad is not None]
        self.found_inf.zero_()
        if self._fused_tail_ok(opt, params):
            grad_norm = self._fused_tail(opt, params)
        else:
            torch._amp_foreach_non_finite_check_and_unscale_([p.grad for p in params], self.found_inf,
                                                             self.scale.double().reciprocal().float())
            grad_norm = torch.nn.utils.clip_grad_norm_(params, T.MAX_GRAD_NORM)
            opt.grad_scale, opt.found_inf = None, self.found_inf     # fused Adam: skipped on the device when inf
            opt.step()
            opt.grad_scale = opt.found_inf = None
        torch._amp_update_scale_(self.scale, self.growth, self.found_inf, *self.amp)
        all_loss, terms, adv, cadv = self.live
        self.stats.copy_(torch.stack([t.detach().float().reshape(()) for t in (
            all_loss, terms[0], terms[1], terms[2], terms[3], terms[4], terms[5], terms[6], grad_norm,
            torch.mean(adv), torch.mean(cadv))]))

    def _fused_tail_ok(self, opt, params):
        """the optimizer tail can run as mapf_optim_unscale_clip_adam: Model.fused_optim, one plain Adam group
        (no weight decay / amsgrad / maximize), fp32 CUDA parameters whose gradients share their dense layout"""
        if not (self.model.fused_optim and isinstance(opt, torch.optim.Adam) and len(opt.param_groups) == 1 and
                params):
            return False
        grp = opt.param_groups[0]
        if grp["weight_decay"] or grp["amsgrad"] or grp.get("maximize") or len(grp["params"]) != len(params):
            return False
        from .net import _CastParams

        def state_ok(p):          # none yet, or torch's fused / capturable layout (device fp32 step, moments like p)
            st = opt.state.get(p, {})
            if not st:
                return True
            return (set(st) == {"step", "exp_avg", "exp_avg_sq"} and st["step"].is_cuda and
                    st["step"].dtype == torch.float32 and st["step"].numel() == 1 and
                    all(st[k].dtype == torch.float32 and st[k].stride() == p.stride() for k in ("exp_avg", "exp_avg_sq")))
        return all(p.is_cuda and p.dtype == torch.float32 and p.grad is not None and p.grad.dtype == torch.float32
                   and p.grad.stride() == p.stride() and _CastParams.dense(p) and state_ok(p) for p in params)

    def _fused_tail(self, opt, params):
        """unscale + found-inf, clip_grad_norm_(MAX_GRAD_NORM) and the Adam step in three launches
        (mapf_optim_unscale_clip_adam) on the optimizer's own state, which it creates as torch's
        fused / capturable Adam does (zero moments, a zero fp32 step per parameter); returns the grad norm
        (a device scalar)"""
        from . import _lib
        grp = opt.param_groups[0]
        for p in params:
            st = opt.state[p]
            if len(st) == 0:
                st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        k = len(params)
        arr = lambda ts: (ctypes.c_void_p * k)(*[t.data_ptr() for t in ts])  # noqa: E731
        sts = [opt.state[p] for p in params]
        blocks = sum((p.numel() + 8191) // 8192 for p in params)
        if getattr(self, "_tail_work", None) is None or self._tail_work.numel() < blocks:
            self._tail_work = torch.empty(blocks, dtype=torch.float32, device=params[0].device)
            self._tail_norm = torch.empty((), dtype=torch.float32, device=params[0].device)
        b1, b2 = grp["betas"]
        st = ctypes.c_void_p(torch.cuda.current_stream(params[0].device).cuda_stream)
        _lib.check(_lib.lib().mapf_optim_unscale_clip_adam(
            arr(params), arr([p.grad for p in params]), arr([x["exp_avg"] for x in sts]),
            arr([x["exp_avg_sq"] for x in sts]), (ctypes.c_int64 * k)(*[p.numel() for p in params]),
            arr([x["step"] for x in sts]), k, ctypes.c_void_p(self.scale.data_ptr()),
            float(TrainingParameters.MAX_GRAD_NORM), float(grp["lr"]), float(b1), float(b2), float(grp["eps"]),
            ctypes.c_void_p(self.found_inf.data_ptr()), ctypes.c_void_p(self._tail_norm.data_ptr()),
            ctypes.c_void_p(self._tail_work.data_ptr()), self._tail_work.numel(), st))
        return self._tail_norm

    def _moments(self):
        """eager, before segment A: the global advantage statistics (two all-reduced moment passes)"""
        from .env import advantage_stats_distributed
        advantage_stats_distributed(self.ret.reshape(-1), self.v.reshape(-1), self.cret.reshape(-1),
                                    self.cv.reshape(-1), out=self.nstats)

    def _exchange(self):
        """eager, between the segments: the gradient bucket's all-reduce (RCCL over xGMI)"""
        dist.all_reduce(self.flat)

    def _exchange_stats(self):
        """eager, after segment B: the loss terms' and advantages' means over the global minibatch"""
        dist.all_reduce(self.stats)
        self.stats.div_(dist.get_world_size())

    def body(self, allreduce=False):
        """one whole update, eagerly (or captured whole when not distributed)"""
        if allreduce:
            self._moments()
        self._front(allreduce)
        if allreduce:
            self._exchange()
        self._back(allreduce)
        if allreduce:
            self._exchange_stats()

    @staticmethod
    def _capture(fn):
        """fn captured into a hipGraph on a side stream.  thread_local capture mode: the process group's
        watchdog thread keeps querying the events of earlier RCCL work while the capture runs, which the
        default (global) mode forbids -- it killed the process (hipErrorStreamCaptureUnsupported) in the
        c4-shaped distributed update on a 1-rank RCCL group.  The eager collectives are also drained
        (synchronize) before the capture begins."""
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                fn()
        torch.cuda.current_stream().wait_stream(s)
        return g

    def run(self, graph=True, allreduce=False):
        """graph: after WARMUP eager updates of this shape, replay captured graphs -- one graph for the
        whole update on one rank; distributed, two segments (A: normalise -> backward into the static
        gradient bucket; B: unscale -> clip -> Adam -> scale update -> stats) with the collectives run
        eagerly around and between them (moments before A, the bucket all-reduce between, the stats
        after B), so the c4 update replays its ~1,500 small ops too."""
        if graph and self.graph is None and not captured_reductions_ok(self.model.device):
            graph = False                   # the runtime would replay the update wrong: eager
        if not graph or self.eager_runs < self.WARMUP:
            if graph:                       # warm-up on a side stream, as capture wants
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    self.body(allreduce=allreduce)
                torch.cuda.current_stream().wait_stream(s)
            else:
                self.body(allreduce=allreduce)
            self.eager_runs += 1
            return
        if self.graph is None:
            self.graph = (self._capture(lambda: self._front(True)), self._capture(lambda: self._back(True))) \
                if allreduce else self._capture(self.body)
            self.graph_allreduce = allreduce
        if self.graph_allreduce != allreduce:
            raise RuntimeError("a minibatch shape's captured update switched between one rank and distributed")
        if allreduce:
            self._moments()
            self.graph[0].replay()
            self._exchange()
            self.graph[1].replay()
            self._exchange_stats()
        else:
            self.graph.replay()
