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
//  moments_kernel /  the same statistics over a minibatch split across ranks: sums (then
//  normalize_stats_  sums of squares about the global mean) to be all-reduced, then the
//  kernel            normalisation with the global mean and unbiased variance.
//  episode_sum_kernel  OneEpPerformance.episodeReward / episodeCostReward (runner.py:95-96):
//                    each step's np.sum of the env's N float32 values (numpy's pairwise
//                    order), accumulated in float32 over the T steps.
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
                                                         float lam, float lam1, int mix, const float *lamd) {
    __shared__ double sh[16];
    if (lamd) { lam = lamd[0]; lam1 = lamd[1]; }     // {lam, f32(lam + 1)} in device memory (graph replays)
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

// Two-pass moments of x = ret - v and c = cret - cv over this rank's M rows, in fp64:
// mean == nullptr: out = {sum x, sum c}; else out = {sum (x - mean[0])^2, sum (c - mean[1])^2}.
__global__ __launch_bounds__(1024) void moments_kernel(const float *__restrict__ ret, const float *__restrict__ v,
                                                       const float *__restrict__ cret, const float *__restrict__ cv,
                                                       int M, const double *__restrict__ mean, double *__restrict__ out) {
    __shared__ double sh[16];
    const double m0 = mean ? mean[0] : 0.0, m1 = mean ? mean[1] : 0.0;
    double s0 = 0.0, s1 = 0.0;
    for (int k = threadIdx.x; k < M; k += blockDim.x) {
        const double a = (double)__fsub_rn(ret[k], v[k]) - m0, c = (double)__fsub_rn(cret[k], cv[k]) - m1;
        s0 += mean ? a * a : a;
        s1 += mean ? c * c : c;
    }
    s0 = block_sum(s0, sh);
    s1 = block_sum(s1, sh);
    if (threadIdx.x == 0) { out[0] = s0; out[1] = s1; }
}

// stats = {mean x, mean c, unbiased var x, unbiased var c} (global, fp64) -> the normalisation of
// normalize_kernel with those statistics
__global__ __launch_bounds__(256) void normalize_stats_kernel(const float *__restrict__ ret, const float *__restrict__ v,
                                                              const float *__restrict__ cret,
                                                              const float *__restrict__ cv,
                                                              const double *__restrict__ stats, float *__restrict__ adv,
                                                              float *__restrict__ cadv, int M, float lam, float lam1,
                                                              int mix, const float *__restrict__ lamd) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= M) return;
    if (lamd) { lam = lamd[0]; lam1 = lamd[1]; }     // {lam, f32(lam + 1)} in device memory
    const float mean0 = (float)stats[0], mean1 = (float)stats[1];
    const float den0 = __fadd_rn((float)sqrt(stats[2]), 1e-6f), den1 = __fadd_rn((float)sqrt(stats[3]), 1e-6f);
    float a = __fdiv_rn(__fsub_rn(__fsub_rn(ret[k], v[k]), mean0), den0);
    const float c = __fdiv_rn(__fsub_rn(__fsub_rn(cret[k], cv[k]), mean1), den1);
    if (mix) a = __fdiv_rn(__fsub_rn(a, __fmul_rn(lam, c)), lam1);
    adv[k] = a;
    cadv[k] = c;
}

// np.sum over a float32 [1, N] array (numpy's pairwise_sum, N <= 128: sequential below 8
// elements, else 8 strided accumulators combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then the
// remainder in order; the reduction's identity 0 added first)
__device__ inline float np_sum_f32(const float *a, int n) {
    float res;
    if (n < 8) {
        res = 0.f;
        for (int i = 0; i < n; ++i) res = __fadd_rn(res, a[i]);
    } else {
        float r[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        int i = 8;
        for (; i < n - (n % 8); i += 8)
#pragma unroll
            for (int j = 0; j < 8; ++j) r[j] = __fadd_rn(r[j], a[i + j]);
        res = __fadd_rn(__fadd_rn(__fadd_rn(r[0], r[1]), __fadd_rn(r[2], r[3])),
                        __fadd_rn(__fadd_rn(r[4], r[5]), __fadd_rn(r[6], r[7])));
        for (; i < n; ++i) res = __fadd_rn(res, a[i]);
    }
    return __fadd_rn(0.f, res);
}

// x [T][B][N]: out[b] = sum over t (float32, in order) of np_sum_f32(x[t][b][:]) -- the python
// accumulator starts at int 0, and 0 + np.float32 stays np.float32 (NEP 50)
__global__ __launch_bounds__(256) void episode_sum_kernel(const float *__restrict__ x, int T, int B, int N,
                                                          float *__restrict__ out) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    float acc = 0.f;
    for (int t = 0; t < T; ++t) acc = __fadd_rn(acc, np_sum_f32(x + ((size_t)t * B + b) * N, N));
    out[b] = acc;
}

void launch_moments(const float *ret, const float *v, const float *cret, const float *cv, int M, const double *mean,
                    double *out, hipStream_t s) {
    hipLaunchKernelGGL(moments_kernel, dim3(1), dim3(1024), 0, s, ret, v, cret, cv, M, mean, out);
}

void launch_normalize_stats(const float *ret, const float *v, const float *cret, const float *cv, const double *stats,
                            float *adv, float *cadv, int M, float lam, float lam1, int mix, const float *lamd,
                            hipStream_t s) {
    hipLaunchKernelGGL(normalize_stats_kernel, dim3((M + 255) / 256), dim3(256), 0, s, ret, v, cret, cv, stats, adv,
                       cadv, M, lam, lam1, mix, lamd);
}

void launch_episode_sum(const float *x, int T, int B, int N, float *out, hipStream_t s) {
    hipLaunchKernelGGL(episode_sum_kernel, dim3((B + 255) / 256), dim3(256), 0, s, x, T, B, N, out);
}

void launch_gae(const float *r, const float *v, const float *vl, float *adv, float *ret, int T, int M, float g,
                float gl, hipStream_t s) {
    hipLaunchKernelGGL(gae_kernel, dim3((M + 255) / 256), dim3(256), 0, s, r, v, vl, adv, ret, T, M, g, gl);
}

void launch_normalize(const float *ret, const float *v, const float *cret, const float *cv, float *adv, float *cadv,
                      int M, float lam, float lam1, int mix, const float *lamd, hipStream_t s) {
    hipLaunchKernelGGL(normalize_kernel, dim3(1), dim3(1024), 0, s, ret, v, cret, cv, adv, cadv, M, lam, lam1, mix,
                       lamd);
}

void launch_sample(const float *ps, int stride, int32_t *a32, int64_t *a64, int M, uint64_t seed, uint32_t step,
                   hipStream_t s) {
    hipLaunchKernelGGL(sample_kernel, dim3((M + 255) / 256), dim3(256), 0, s, ps, stride, a32, a64, M, seed, step);
}

}  // namespace mapf
