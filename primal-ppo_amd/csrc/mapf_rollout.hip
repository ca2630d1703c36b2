// primal-ppo_amd/csrc/mapf_rollout.hip -- rollout-side kernels next to the policy.
//
//  gae_kernel        Runner.run GAE (runner.py:117-149): numpy float32 semantics
//                    -- the python-float constants are rounded to f32 (gamma and
//                    gamma*lam), every multiply and add rounds separately (no
//                    FMA contraction), nonterminal == 1, returns = adv + values.
//                    One lane per column, reverse scan over T; 16 B per (t, col).
//  normalize_kernel  Model.train (model.py:106-113): x - mean over the minibatch,
//                    divided by (unbiased std + 1e-6); optional Lagrangian mix
//                    adv = (adv - lam * cadv) / (lam + 1).  Sums in f64.
//  sample_kernel     Model.step (model.py:38-40): np.random.choice(5, p) as an
//                    inverse CDF with a Philox uniform.
#include "mapf_common.h"
#include "mapf_kernels.h"

namespace mapf {

#pragma clang fp contract(off)

__global__ __launch_bounds__(256) void gae_kernel(const float *__restrict__ r, const float *__restrict__ v,
                                                  const float *__restrict__ vl, float *__restrict__ adv,
                                                  float *__restrict__ ret, int T, int M, float g, float gl) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= M) return;
    float next_v = vl[m];
    float last = 0.f;
    for (int t = T - 1; t >= 0; --t) {
        const size_t k = (size_t)t * M + m;
        const float vt = v[k];
        const float gv = __fmul_rn(g, next_v);
        const float delta = __fsub_rn(__fadd_rn(r[k], gv), vt);
        last = __fadd_rn(delta, __fmul_rn(gl, last));
        adv[k] = last;
        ret[k] = __fadd_rn(last, vt);
        next_v = vt;
    }
}

__device__ inline double block_sum(double x, double *sh) {
    for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o, 64);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) sh[w] = x;
    __syncthreads();
    double t = 0.0;
    const int nw = blockDim.x >> 6;
    for (int k = 0; k < nw; ++k) t += sh[k];
    return t;
}

__global__ __launch_bounds__(1024) void normalize_kernel(const float *__restrict__ ret, const float *__restrict__ v,
                                                         const float *__restrict__ cret, const float *__restrict__ cv,
                                                         float *__restrict__ adv, float *__restrict__ cadv, int M,
                                                         float lam, float lam1, int mix) {
    __shared__ double sh[16];
    double s0 = 0.0, s1 = 0.0;
    for (int k = threadIdx.x; k < M; k += blockDim.x) {
        s0 += (double)__fsub_rn(ret[k], v[k]);
        s1 += (double)__fsub_rn(cret[k], cv[k]);
    }
    const double m0 = block_sum(s0, sh) / M;
    const double m1 = block_sum(s1, sh) / M;
    double q0 = 0.0, q1 = 0.0;
    for (int k = threadIdx.x; k < M; k += blockDim.x) {
        const double a = (double)__fsub_rn(ret[k], v[k]) - m0, c = (double)__fsub_rn(cret[k], cv[k]) - m1;
        q0 += a * a;
        q1 += c * c;
    }
    const double v0 = block_sum(q0, sh) / (M > 1 ? M - 1 : 1);
    const double v1 = block_sum(q1, sh) / (M > 1 ? M - 1 : 1);
    const float mean0 = (float)m0, mean1 = (float)m1;
    const float den0 = __fadd_rn((float)sqrt(v0), 1e-6f), den1 = __fadd_rn((float)sqrt(v1), 1e-6f);
    for (int k = threadIdx.x; k < M; k += blockDim.x) {
        float a = __fdiv_rn(__fsub_rn(__fsub_rn(ret[k], v[k]), mean0), den0);
        const float c = __fdiv_rn(__fsub_rn(__fsub_rn(cret[k], cv[k]), mean1), den1);
        if (mix) a = __fdiv_rn(__fsub_rn(a, __fmul_rn(lam, c)), lam1);   // lam1 = f32(lam + 1) in f64
        adv[k] = a;
        cadv[k] = c;
    }
}

__global__ __launch_bounds__(256) void sample_kernel(const float *__restrict__ ps, int stride, int32_t *a32,
                                                     int64_t *a64, int M, uint64_t seed, uint32_t step) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= M) return;
    const float *p = ps + (size_t)m * stride;
    float cdf[NA];
    float acc = 0.f;
#pragma unroll
    for (int a = 0; a < NA; ++a) { acc = __fadd_rn(acc, p[a]); cdf[a] = acc; }
    const u32x4 o = philox((uint32_t)m, P_SAMPLE, step, 0u, seed);
    const float u = __fmul_rn((float)(o.x >> 8) * (1.0f / 16777216.0f), acc);
    int pick = NA - 1;
#pragma unroll
    for (int a = NA - 1; a >= 0; --a)
        if (u < cdf[a]) pick = a;                 // searchsorted(cdf, u, side='right')
    if (a32) a32[m] = pick;
    if (a64) a64[m] = pick;
}

void launch_gae(const float *r, const float *v, const float *vl, float *adv, float *ret, int T, int M, float g,
                float gl, hipStream_t s) {
    hipLaunchKernelGGL(gae_kernel, dim3((M + 255) / 256), dim3(256), 0, s, r, v, vl, adv, ret, T, M, g, gl);
}

void launch_normalize(const float *ret, const float *v, const float *cret, const float *cv, float *adv, float *cadv,
                      int M, float lam, float lam1, int mix, hipStream_t s) {
    hipLaunchKernelGGL(normalize_kernel, dim3(1), dim3(1024), 0, s, ret, v, cret, cv, adv, cadv, M, lam, lam1, mix);
}

void launch_sample(const float *ps, int stride, int32_t *a32, int64_t *a64, int M, uint64_t seed, uint32_t step,
                   hipStream_t s) {
    hipLaunchKernelGGL(sample_kernel, dim3((M + 255) / 256), dim3(256), 0, s, ps, stride, a32, a64, M, seed, step);
}

}  // namespace mapf
