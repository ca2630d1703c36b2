// primal-ppo_amd/csrc/mapf_ppo.hip -- the PPO loss terms of one minibatch update as one
// kernel (learner-side fusion), forward and backward together.
//
// Reference: model.py:115-175 (Model.train under autocast):
//   ratio       = exp(log(clamp(new_p, 1e-6, 1)) - log(clamp(old_p, 1e-6, 1)))   :117-119
//   entropy     = mean(-sum_a new_ps * log(clamp(new_ps, 1e-6, 1)))                :121
//   critic      = mean(max((v - R)^2, (old_v + clamp(v - old_v, -c, c) - R)^2))    :124-129
//   cost critic = the same on (cv, old_cv, cost returns)                            :131-136
//   policy      = mean(min(adv * ratio, adv * clamp(ratio, 1 - c, 1 + c)))          :139-143
//   valid       = -mean(log(clamp(sig, 1e-6, 1 - 1e-6)) * tv
//                       + log(clamp(1 - sig, 1e-6, 1 - 1e-6)) * (1 - tv))           :146-148
//   cost        = mean(ratio * cost_adv)                                            :154
//   all         = -policy - ENT * entropy + VC * critic + VALID * valid
//                 + CVC * cost critic + COST * lambda * cost                        :158-162
//   clip_frac   = mean(|ratio - 1| > c)                                             :175
// over R = rows x agents elements (A actions each).  The gradient of `all` with respect
// to new_ps, v, cv and sig is written in the same pass, with torch's conventions:
// clamp passes the gradient on its closed range, min / max split it in half on ties.
// policy_sig comes out of the autocast net in fp16, so with sig_fp16 the clamp bounds
// and 1 - sig are rounded to fp16 as torch does there (log itself autocasts to fp32).
//
// One workgroup of 1024 threads walks the rows; the sums reduce in a fixed order
// (deterministic).  R is small (one minibatch: 256 x 8 rows in the c4 update).
#include <hip/hip_fp16.h>

#include "mapf.h"
#include "mapf_common.h"

namespace mapf {
namespace ppo {

struct Args {
    const float *new_ps, *old_ps, *new_v, *old_v, *ret, *new_cv, *old_cv, *cret, *adv, *cadv, *sig, *tv;
    const int64_t *action;
    float *loss, *terms, *g_ps, *g_v, *g_cv, *g_sig;
    long R;
    int A, sig_fp16;
    float clip, ent, vc, valid, cvc, costlam;
    const float *coefd;      // non-null: the six coefficients read from device memory (graph replays)
};

__device__ inline float r16(float x) { return __half2float(__float2half_rn(x)); }
__device__ inline float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
__device__ inline float in_range(float x, float lo, float hi) { return (x >= lo && x <= hi) ? 1.f : 0.f; }

// d max(a, b) / d a  and  d max(a, b) / d b  (torch.maximum: halves on a tie)
__device__ inline void dmax(float a, float b, float &da, float &db) {
    da = a > b ? 1.f : (a == b ? 0.5f : 0.f);
    db = b > a ? 1.f : (a == b ? 0.5f : 0.f);
}

// clipped value loss term and its gradient with respect to v (the coefficient / R outside)
__device__ inline float value_term(float v, float ov, float r, float c, float &gv) {
    const float dv = v - ov;
    const float vc = ov + clampf(dv, -c, c);
    const float l1 = (v - r) * (v - r), l2 = (vc - r) * (vc - r);
    float d1, d2;
    dmax(l1, l2, d1, d2);
    gv = d1 * 2.f * (v - r) + d2 * 2.f * (vc - r) * in_range(dv, -c, c);
    return fmaxf(l1, l2);
}

__global__ __launch_bounds__(1024) void ppo_loss_kernel(Args a) {
    if (a.coefd) {
        a.clip = a.coefd[0]; a.ent = a.coefd[1]; a.vc = a.coefd[2];
        a.valid = a.coefd[3]; a.cvc = a.coefd[4]; a.costlam = a.coefd[5];
    }
    constexpr int NS = 7;              // policy, entropy, critic, valid, cost critic, cost, clipped
    float s[NS] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const float invR = 1.f / (float)a.R, invRA = 1.f / ((float)a.R * (float)a.A);
    int bad = 0;
    const float slo = a.sig_fp16 ? r16(1e-6f) : 1e-6f, shi = a.sig_fp16 ? r16(1.f - 1e-6f) : 1.f - 1e-6f;
    for (long r = threadIdx.x; r < a.R; r += blockDim.x) {
        const float *np = a.new_ps + r * a.A, *sg = a.sig + r * a.A, *tv = a.tv + r * a.A;
        float *gp = a.g_ps + r * a.A, *gs = a.g_sig + r * a.A;
        int act = (int)a.action[r];
        if (act < 0 || act >= a.A) {       // torch.gather would raise: poison the loss instead
            bad = 1;
            act = 0;
        }
        // entropy and the valid loss, per action
        for (int k = 0; k < a.A; ++k) {
            const float p = np[k], cp = clampf(p, 1e-6f, 1.f);
            s[1] -= p * logf(cp);
            gp[k] = a.ent * invR * (logf(cp) + p * in_range(p, 1e-6f, 1.f) / cp);
            const float x = sg[k], om = a.sig_fp16 ? r16(1.f - x) : 1.f - x;
            const float c1 = clampf(x, slo, shi), c2 = clampf(om, slo, shi), t = tv[k];
            s[3] += logf(c1) * t + logf(c2) * (1.f - t);
            // d/dx of -(log c1 * t + log c2 * (1 - t)), with d om / dx = -1
            gs[k] = -a.valid * invRA * (t * in_range(x, slo, shi) / c1 - (1.f - t) * in_range(om, slo, shi) / c2);
        }
        // ratio terms
        const float p = np[act], op = a.old_ps[r * a.A + act];
        const float cp = clampf(p, 1e-6f, 1.f), cop = clampf(op, 1e-6f, 1.f);
        const float ratio = expf(logf(cp) - logf(cop));
        const float ad = a.adv[r], cad = a.cadv[r];
        const float rc = clampf(ratio, 1.f - a.clip, 1.f + a.clip);
        const float x1 = ad * ratio, x2 = ad * rc;
        s[0] += fminf(x1, x2);
        s[5] += ratio * cad;
        s[6] += fabsf(ratio - 1.f) > a.clip ? 1.f : 0.f;
        // d min(x1, x2) / d ratio  (torch.minimum: halves on a tie)
        const float d1 = x1 < x2 ? 1.f : (x1 == x2 ? 0.5f : 0.f), d2 = x2 < x1 ? 1.f : (x1 == x2 ? 0.5f : 0.f);
        const float dpol = d1 * ad + d2 * ad * in_range(ratio, 1.f - a.clip, 1.f + a.clip);
        const float gratio = (-dpol + a.costlam * cad) * invR;
        gp[act] += gratio * ratio * in_range(p, 1e-6f, 1.f) / cp;
        // value heads
        float gv, gcv;
        s[2] += value_term(a.new_v[r], a.old_v[r], a.ret[r], a.clip, gv);
        s[4] += value_term(a.new_cv[r], a.old_cv[r], a.cret[r], a.clip, gcv);
        a.g_v[r] = a.vc * invR * gv;
        a.g_cv[r] = a.cvc * invR * gcv;
    }
    // fixed-order reduction: waves by xor shuffles, then wave 0 over the 16 wave sums
    __shared__ float part[16][NS];
    const int lane = (int)(threadIdx.x & 63), w = (int)(threadIdx.x >> 6);
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        float v = s[q];
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
        if (lane == 0) part[w][q] = v;
    }
    bad = __syncthreads_or(bad);
    if (threadIdx.x == 0) {
        float t[NS];
        for (int q = 0; q < NS; ++q) {
            t[q] = 0.f;
            for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t[q] += part[i][q];
        }
        const float pol = t[0] * invR, ent = t[1] * invR, cr = t[2] * invR, val = -t[3] * invRA, ccr = t[4] * invR,
                    cost = t[5] * invR, clipf = t[6] * invR;
        a.loss[0] = bad ? __builtin_nanf("")
                        : -pol - a.ent * ent + a.vc * cr + a.valid * val + a.cvc * ccr + a.costlam * cost;
        a.terms[0] = pol;
        a.terms[1] = ent;
        a.terms[2] = cr;
        a.terms[3] = val;
        a.terms[4] = ccr;
        a.terms[5] = cost;
        a.terms[6] = clipf;
    }
}

}  // namespace ppo
}  // namespace mapf

using namespace mapf;

extern "C" {

static int ppo_loss(const float *new_ps, const float *old_ps, const int64_t *action, const float *new_v,
                    const float *old_v, const float *returns, const float *new_cv, const float *old_cv,
                    const float *cost_returns, const float *advantage, const float *cost_advantage,
                    const float *policy_sig, int32_t sig_fp16, const float *train_valid, int64_t R, int32_t A,
                    const float *coef, bool coef_on_device, float *loss, float *terms, float *grad_ps, float *grad_v,
                    float *grad_cv, float *grad_sig, void *stream) {
    if (!new_ps || !old_ps || !action || !new_v || !old_v || !returns || !new_cv || !old_cv || !cost_returns ||
        !advantage || !cost_advantage || !policy_sig || !train_valid || !coef || !loss || !terms || !grad_ps || !grad_v ||
        !grad_cv || !grad_sig || R < 1 || A < 1 || A > 64)
        return MAPF_EINVAL;
    const float h[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const float *c = coef_on_device ? h : coef;
    ppo::Args a{new_ps, old_ps, new_v, old_v, returns, new_cv, old_cv, cost_returns, advantage, cost_advantage,
                policy_sig, train_valid, action, loss, terms, grad_ps, grad_v, grad_cv, grad_sig, (long)R, (int)A,
                sig_fp16 ? 1 : 0, c[0], c[1], c[2], c[3], c[4], c[5], coef_on_device ? coef : nullptr};
    hipLaunchKernelGGL(ppo::ppo_loss_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, a);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_ppo_loss(const float *new_ps, const float *old_ps, const int64_t *action, const float *new_v,
                  const float *old_v, const float *returns, const float *new_cv, const float *old_cv,
                  const float *cost_returns, const float *advantage, const float *cost_advantage,
                  const float *policy_sig, int32_t sig_fp16, const float *train_valid, int64_t R, int32_t A,
                  const float *coef, float *loss, float *terms, float *grad_ps, float *grad_v, float *grad_cv,
                  float *grad_sig, void *stream) {
    return ppo_loss(new_ps, old_ps, action, new_v, old_v, returns, new_cv, old_cv, cost_returns, advantage,
                    cost_advantage, policy_sig, sig_fp16, train_valid, R, A, coef, false, loss, terms, grad_ps, grad_v,
                    grad_cv, grad_sig, stream);
}

int mapf_ppo_loss_dcoef(const float *new_ps, const float *old_ps, const int64_t *action, const float *new_v,
                        const float *old_v, const float *returns, const float *new_cv, const float *old_cv,
                        const float *cost_returns, const float *advantage, const float *cost_advantage,
                        const float *policy_sig, int32_t sig_fp16, const float *train_valid, int64_t R, int32_t A,
                        const float *coef_dev, float *loss, float *terms, float *grad_ps, float *grad_v,
                        float *grad_cv, float *grad_sig, void *stream) {
    return ppo_loss(new_ps, old_ps, action, new_v, old_v, returns, new_cv, old_cv, cost_returns, advantage,
                    cost_advantage, policy_sig, sig_fp16, train_valid, R, A, coef_dev, true, loss, terms, grad_ps,
                    grad_v, grad_cv, grad_sig, stream);
}

}  // extern "C"
