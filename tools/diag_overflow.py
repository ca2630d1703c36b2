import copy, sys
sys.path.insert(0, "tests"); sys.path.insert(0, "primal-ppo_amd")
import numpy as np, torch
from test_gpu_update_graph import _batch
from mapf_amd.model import Model, _DeviceUpdate, _FusedPPOLoss
from mapf_amd.config import TrainingParameters as T
torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
orig = _DeviceUpdate.body
def body(self, allreduce=False):
    m, net, opt = self.model, self.model.network, self.model.net_optimizer
    opt.zero_grad(set_to_none=True)
    from mapf_amd.env import normalize_advantages_dlam
    adv, cadv = normalize_advantages_dlam(self.ret.reshape(-1), self.v.reshape(-1), self.cret.reshape(-1),
                                          self.cv.reshape(-1), self.dyn[6:8], T.MINUS_ADV_WITH_CADV)
    adv, cadv = adv.view(self.ret.shape), cadv.view(self.ret.shape)
    with torch.autocast(device_type="cuda", cache_enabled=False):
        new_ps, new_v, block, policy_sig, _, _, new_cv = net(self.obs, self.vec, None)
    all_loss, terms = _FusedPPOLoss.apply(new_ps, new_v, new_cv, policy_sig, self.old_ps, self.action.unsqueeze(-1),
                                          self.v, self.ret, self.cv, self.cret, adv, cadv, self.tv, self.dyn[:6])
    (all_loss * self.scale).backward()
    params = [p for p in net.parameters() if p.grad is not None]
    torch.cuda.synchronize()
    bad = [(i, tuple(p.shape), p.grad.dtype) for i, p in enumerate(params) if not torch.isfinite(p.grad).all()]
    self.found_inf.zero_()
    torch._amp_foreach_non_finite_check_and_unscale_([p.grad for p in params], self.found_inf,
                                                     self.scale.double().reciprocal().float())
    torch.cuda.synchronize()
    print("  nonfinite grads:", bad[:5], "n", len(bad), "found_inf", float(self.found_inf), "scale", float(self.scale),
          "nparams", len(params), "dtypes", sorted({str(p.grad.dtype) for p in params}),
          "devices", sorted({str(p.grad.device) for p in params}), "contig", all(p.grad.is_contiguous() for p in params),
          flush=True)
    grad_norm = torch.nn.utils.clip_grad_norm_(params, T.MAX_GRAD_NORM)
    opt.grad_scale, opt.found_inf = None, self.found_inf
    opt.step()
    opt.grad_scale = opt.found_inf = None
    torch._amp_update_scale_(self.scale, self.growth, self.found_inf, *self.amp)
    self.stats.copy_(torch.stack([t.detach().float().reshape(()) for t in (
        all_loss, terms[0], terms[1], terms[2], terms[3], terms[4], terms[5], terms[6], grad_norm,
        torch.mean(adv), torch.mean(cadv))]))
_DeviceUpdate.body = body
torch.manual_seed(0)
m2 = Model(0, "cuda", global_model=True, numChannel=6, num_agents=8, fov=9)
m2.graph_update = False
m2.network.eval()
m2.net_scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 8)
g = torch.Generator(device="cuda").manual_seed(1)
batches = [_batch(g) for _ in range(6)]
for k, b in enumerate(batches):
    obs, vec, ret, cret, v, cv, act, ps, tv = b
    print("update", k, flush=True)
    s = m2.train(obs, vec, ret, cret, v, cv, act, ps, None, tv, 1.0)
    print("  grad_norm", float(s[8]))
