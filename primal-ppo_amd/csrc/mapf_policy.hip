// primal-ppo_amd/csrc/mapf_policy.hip -- fused elementwise kernels of the
// SCRIMPNet acting forward (net.py:101-155 run under torch.autocast with no
// grad: Model.step / Model.value, model.py:26-69).
//
// Every kernel here is HBM-bound and replaces two or three of PyTorch's
// elementwise passes over the same tensor (the rollout forward moves tensors of
// 32,768 agents x 17 tokens x 512):
//   nhwc_bias_relu          conv bias + ReLU on an NHWC fp16 conv output (in place)
//   nhwc_bias_relu_pool2    conv bias + ReLU + 2x2 max-pool (nn.MaxPool2d(2), floor)
//   layernorm_f16           LayerNorm of the fp32 residual stream, written as the fp16
//                           the next autocast linear would cast it to
//   dropout_residual        x(fp32) += dropout(y(fp16))      (PreNorm residual, do1/do2)
//   dropout_residual_layernorm   the residual above + the next PreNorm's LayerNorm, one pass
//   gelu_dropout_f16        h = dropout(gelu(h))  in place   (MLP_Block af1 + do1)
//   tokens                  x = dropout(cat(cls, A * VV) + pos_embedding)   (net.py:124-131)
//   tokens_layernorm        tokens + the first block's LayerNorm, one pass
//   attention_f16           softmax(q k^T * scale) v over the 17 tokens, 16 heads of 32 (MFMA)
// The training forward (autograd) uses the conv epilogues and LayerNorm here too, with their
// backward kernels below (relu_bias_bwd, relu_bias_pool_bwd, layernorm_bwd_f16, colsum, casts,
// attention_bwd_f16).  ReLU and max-pool keep torch's NaN semantics (relu_nan / max_nan).
//
// Dropout: keep with probability 1 - p, kept values scaled by 1 / (1 - p) (torch's
// inverted dropout); the mask bits come from a counter hash (keep4: murmur3's finaliser of
// the element index, keyed by `seed`) -- a different stream than torch's own generator; the
// reference's masks are random anyway (the net is never eval()-ed, net.py:50-51).
#include <vector>
#include <hip/hip_fp16.h>

#include "mapf.h"
#include "mapf_common.h"

namespace mapf {
namespace pol {

__device__ inline float h2f(uint32_t h) { return __half2float(__ushort_as_half((unsigned short)(h & 0xFFFFu))); }
__device__ inline uint32_t f2h(float f) { return (uint32_t)__half_as_ushort(__float2half_rn(f)); }
__device__ inline uint2 pack4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return make_uint2(a | (b << 16), c | (d << 16));
}

// murmur3's 32-bit finaliser: a bijection with full avalanche, 2 multiplies
__device__ inline uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}
// 4 keep decisions for float4 index i (bit k: element 4*i + k kept): one fmix32 per element of the
// element counter keyed by the seed (the key is wave-uniform: scalar ALU).  8 multiplies per 4
// draws where Philox4x32-10 takes 40 (integer multiplies are quarter rate): at p > 0 the masks
// of a 32,768-agent acting forward (~1.7e8 float4s) were ~0.3 ms of each fused linear launch.
__device__ inline unsigned keep4(uint64_t seed, uint64_t i, uint32_t thr) {
    const uint32_t key = fmix32((uint32_t)seed ^ fmix32((uint32_t)(seed >> 32) ^ 0x5EEDD0u));
    const uint32_t c = ((uint32_t)i << 2) ^ key ^ ((uint32_t)(i >> 30) * 0x9E3779B9u);
    return (fmix32(c) >= thr ? 1u : 0u) | (fmix32(c ^ 1u) >= thr ? 2u : 0u) | (fmix32(c ^ 2u) >= thr ? 4u : 0u) |
           (fmix32(c ^ 3u) >= thr ? 8u : 0u);
}
// bits k0 and k0 + 1 of keep4(seed, i, thr) (k0 in 0..2), as bits 0 and 1: the same draws, two hashes
__device__ inline unsigned keep2(uint64_t seed, uint64_t i, uint32_t thr, unsigned k0) {
    const uint32_t key = fmix32((uint32_t)seed ^ fmix32((uint32_t)(seed >> 32) ^ 0x5EEDD0u));
    const uint32_t c = ((uint32_t)i << 2) ^ key ^ ((uint32_t)(i >> 30) * 0x9E3779B9u);
    return (fmix32(c ^ k0) >= thr ? 1u : 0u) | (fmix32(c ^ (k0 + 1u)) >= thr ? 2u : 0u);
}
// the training forward's dropout seed: a counter in device memory (SCRIMPNet._train_seed) and a per-site salt
__device__ inline uint64_t dev_seed(const uint64_t *__restrict__ p, uint32_t salt) {
    return p[0] * 0x9E3779B97F4A7C15ull + (uint64_t)salt * 0xD1B54A32D192ED03ull;
}
inline uint32_t drop_threshold(float p) {
    const double t = (double)p * 4294967296.0;
    return t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
}

// ---- conv epilogues (NHWC fp16, C % 4 == 0, C <= 1024) -------------------------
// torch: the conv's fp16 output + fp16 bias (rounded to fp16), then ReLU
__global__ __launch_bounds__(256) void nhwc_bias_relu(uint16_t *__restrict__ x, const uint16_t *__restrict__ bias,
                                                      long rows, int C) {
    const int c4n = C >> 2;
    const int per = 256 / c4n;                      // rows per block pass
    const int tr = (int)threadIdx.x / c4n, c4 = (int)threadIdx.x - tr * c4n;
    if (tr >= per) return;
    const uint2 bb = *reinterpret_cast<const uint2 *>(bias + 4 * c4);
    const float b0 = h2f(bb.x), b1 = h2f(bb.x >> 16), b2 = h2f(bb.y), b3 = h2f(bb.y >> 16);
    for (long r = (long)blockIdx.x * per + tr; r < rows; r += (long)gridDim.x * per) {
        uint2 *p = reinterpret_cast<uint2 *>(x + r * C) + c4;
        const uint2 v = *p;
        *p = pack4(f2h(relu_nan(h2f(f2h(h2f(v.x) + b0)))), f2h(relu_nan(h2f(f2h(h2f(v.x >> 16) + b1)))),
                   f2h(relu_nan(h2f(f2h(h2f(v.y) + b2)))), f2h(relu_nan(h2f(f2h(h2f(v.y >> 16) + b3)))));
    }
}

// in [B][H][W][C] -> out [B][H/2][W/2][C]: relu(round(max(window) + b)) equals the
// max over the window of relu(round(x + b)) (both maps are monotone)
__global__ __launch_bounds__(256) void nhwc_bias_relu_pool2(const uint16_t *__restrict__ x,
                                                            const uint16_t *__restrict__ bias,
                                                            uint16_t *__restrict__ out, int B, int H, int W, int C) {
    const int Ho = H / 2, Wo = W / 2;
    const long rows = (long)B * Ho * Wo;
    const int c4n = C >> 2;
    const int per = 256 / c4n;
    const int tr = (int)threadIdx.x / c4n, c4 = (int)threadIdx.x - tr * c4n;
    if (tr >= per) return;
    const uint2 bb = *reinterpret_cast<const uint2 *>(bias + 4 * c4);
    const float bv[4] = {h2f(bb.x), h2f(bb.x >> 16), h2f(bb.y), h2f(bb.y >> 16)};
    for (long r = (long)blockIdx.x * per + tr; r < rows; r += (long)gridDim.x * per) {
        const long b = r / (Ho * Wo);
        const int rem = (int)(r - b * Ho * Wo), i = rem / Wo, j = rem - i * Wo;
        float m[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
        for (int di = 0; di < 2; ++di)
#pragma unroll
            for (int dj = 0; dj < 2; ++dj) {
                const uint2 v =
                    *(reinterpret_cast<const uint2 *>(x + ((b * H + 2 * i + di) * (long)W + 2 * j + dj) * C) + c4);
                m[0] = max_nan(m[0], h2f(v.x));
                m[1] = max_nan(m[1], h2f(v.x >> 16));
                m[2] = max_nan(m[2], h2f(v.y));
                m[3] = max_nan(m[3], h2f(v.y >> 16));
            }
        uint32_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = f2h(relu_nan(h2f(f2h(m[k] + bv[k]))));
        *(reinterpret_cast<uint2 *>(out + r * C) + c4) = pack4(o[0], o[1], o[2], o[3]);
    }
}

// ---- LayerNorm: one wave per row of D = 512 fp32 (8 per lane) -> fp16 ---------
__device__ inline float wave_sum(float v) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s, 64);
    return v;
}

// LayerNorm of one 512-wide row held by a wave as a = elements 4l..4l+3, c = 256+4l..
__device__ inline void ln_row(float4 a, float4 c, int lane, const float *__restrict__ gamma,
                              const float *__restrict__ beta, float eps, uint16_t *__restrict__ y) {
    constexpr int D = 512;
    const float mean = wave_sum(a.x + a.y + a.z + a.w + c.x + c.y + c.z + c.w) * (1.f / D);
    const float d[8] = {a.x - mean, a.y - mean, a.z - mean, a.w - mean, c.x - mean, c.y - mean, c.z - mean, c.w - mean};
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) ss += d[k] * d[k];
    const float rstd = 1.f / sqrtf(wave_sum(ss) * (1.f / D) + eps);
    const float4 g0 = reinterpret_cast<const float4 *>(gamma)[lane], g1 = reinterpret_cast<const float4 *>(gamma)[64 + lane];
    const float4 e0 = reinterpret_cast<const float4 *>(beta)[lane], e1 = reinterpret_cast<const float4 *>(beta)[64 + lane];
    const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    const float e[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
    uint32_t o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = f2h(d[k] * rstd * g[k] + e[k]);
    uint2 *yr = reinterpret_cast<uint2 *>(y);
    yr[lane] = pack4(o[0], o[1], o[2], o[3]);
    yr[64 + lane] = pack4(o[4], o[5], o[6], o[7]);
}

// ln_row for R rows a wave holds at once: every row's sums in ln_row's order, the R
// cross-lane reductions interleaved step by step (independent shuffles in flight together
// instead of one dependent chain per row); bit-identical to R ln_row calls.  Rows with
// live[r] false are computed but not stored.
template <int R>
__device__ inline void ln_rows(const float4 *a, const float4 *c, const bool *live, int lane,
                               const float *__restrict__ gamma, const float *__restrict__ beta, float eps,
                               uint16_t *const *y) {
    constexpr int D = 512;
    float sm[R];
#pragma unroll
    for (int r = 0; r < R; ++r) sm[r] = a[r].x + a[r].y + a[r].z + a[r].w + c[r].x + c[r].y + c[r].z + c[r].w;
#pragma unroll
    for (int st = 32; st >= 1; st >>= 1)
#pragma unroll
        for (int r = 0; r < R; ++r) sm[r] += __shfl_xor(sm[r], st, 64);
    float d[R][8], ss[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const float mean = sm[r] * (1.f / D);
        d[r][0] = a[r].x - mean; d[r][1] = a[r].y - mean; d[r][2] = a[r].z - mean; d[r][3] = a[r].w - mean;
        d[r][4] = c[r].x - mean; d[r][5] = c[r].y - mean; d[r][6] = c[r].z - mean; d[r][7] = c[r].w - mean;
        ss[r] = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) ss[r] += d[r][k] * d[r][k];
    }
#pragma unroll
    for (int st = 32; st >= 1; st >>= 1)
#pragma unroll
        for (int r = 0; r < R; ++r) ss[r] += __shfl_xor(ss[r], st, 64);
    const float4 g0 = reinterpret_cast<const float4 *>(gamma)[lane], g1 = reinterpret_cast<const float4 *>(gamma)[64 + lane];
    const float4 e0 = reinterpret_cast<const float4 *>(beta)[lane], e1 = reinterpret_cast<const float4 *>(beta)[64 + lane];
    const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    const float e[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const float rstd = 1.f / sqrtf(ss[r] * (1.f / D) + eps);
        uint32_t o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = f2h(d[r][k] * rstd * g[k] + e[k]);
        if (live[r]) {
            uint2 *yr = reinterpret_cast<uint2 *>(y[r]);
            yr[lane] = pack4(o[0], o[1], o[2], o[3]);
            yr[64 + lane] = pack4(o[4], o[5], o[6], o[7]);
        }
    }
}

__global__ __launch_bounds__(256) void layernorm_f16(const float *__restrict__ x, long xstride,
                                                     const float *__restrict__ gamma, const float *__restrict__ beta,
                                                     uint16_t *__restrict__ y, long rows, float eps) {
    const int lane = (int)(threadIdx.x & 63);
    const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const float4 *xr = reinterpret_cast<const float4 *>(x + row * xstride);
    ln_row(xr[lane], xr[64 + lane], lane, gamma, beta, eps, y + row * 512);
}

// ---- LayerNorm backward (the training forward's PreNorm, transformer.py:7-24) ------------
// z = fp16(LayerNorm(x)) is what the next fp16 linear reads under autocast (layernorm_f16); given
// dz (fp16), with mean / rstd recomputed from x exactly as layernorm_f16 computes them:
//   xhat = (x - mean) rstd, g = dz gamma,
//   dx = rstd (g - mean_k(g) - xhat mean_k(g xhat))       (fp32, one wave per row)
//   dgamma = sum_rows dz xhat, dbeta = sum_rows dz        (per-workgroup partials, then ln_bwd_colsum)
constexpr int LNB_WG = 512;                                 // partial rows of the gamma / beta gradients
// dy16 (training dropout + residual + LayerNorm, drln_fwd): also the gradient of the dropped branch,
// dy = fp16(fp16(dx) * scale) where drln_fwd kept the element, 0 where it dropped it -- autograd's fp16
// cast at the mixed-precision add, then torch's dropout backward (masked_scale)
__global__ __launch_bounds__(256) void layernorm_bwd_f16(const float *__restrict__ x, long xstride,
                                                         const float *__restrict__ gamma,
                                                         const uint16_t *__restrict__ dz,
                                                         const float *__restrict__ dres, float *__restrict__ dx,
                                                         float *__restrict__ part, long rows, float eps,
                                                         uint16_t *__restrict__ dy16, uint32_t thr, float scale,
                                                         const uint64_t *__restrict__ seedp, uint32_t salt) {
    constexpr int D = 512;
    __shared__ float red[2][4][D];
    const int lane = (int)(threadIdx.x & 63), wave = (int)(threadIdx.x >> 6);
    const float4 g0 = reinterpret_cast<const float4 *>(gamma)[lane], g1 = reinterpret_cast<const float4 *>(gamma)[64 + lane];
    const float gm[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    float ag[8], ab[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) ag[k] = ab[k] = 0.f;
    for (long row = (long)blockIdx.x * 4 + wave; row < rows; row += (long)gridDim.x * 4) {
        const float4 *xr = reinterpret_cast<const float4 *>(x + row * xstride);
        const float4 a = xr[lane], c = xr[64 + lane];
        const uint2 z0 = reinterpret_cast<const uint2 *>(dz + row * D)[lane];
        const uint2 z1 = reinterpret_cast<const uint2 *>(dz + row * D)[64 + lane];
        const float dzv[8] = {h2f(z0.x), h2f(z0.x >> 16), h2f(z0.y), h2f(z0.y >> 16),
                              h2f(z1.x), h2f(z1.x >> 16), h2f(z1.y), h2f(z1.y >> 16)};
        float sm = a.x + a.y + a.z + a.w + c.x + c.y + c.z + c.w;          // layernorm_f16's order
#pragma unroll
        for (int st = 32; st >= 1; st >>= 1) sm += __shfl_xor(sm, st, 64);
        const float mean = sm * (1.f / D);
        const float d[8] = {a.x - mean, a.y - mean, a.z - mean, a.w - mean, c.x - mean, c.y - mean, c.z - mean, c.w - mean};
        float ss = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) ss += d[k] * d[k];
#pragma unroll
        for (int st = 32; st >= 1; st >>= 1) ss += __shfl_xor(ss, st, 64);
        const float rstd = 1.f / sqrtf(ss * (1.f / D) + eps);
        float xh[8], gg[8], s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            xh[k] = d[k] * rstd;
            gg[k] = dzv[k] * gm[k];
            s1 += gg[k];
            s2 += gg[k] * xh[k];
            ag[k] += dzv[k] * xh[k];
            ab[k] += dzv[k];
        }
#pragma unroll
        for (int st = 32; st >= 1; st >>= 1) {
            s1 += __shfl_xor(s1, st, 64);
            s2 += __shfl_xor(s2, st, 64);
        }
        const float m1 = s1 * (1.f / D), m2 = s2 * (1.f / D);
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = rstd * (gg[k] - m1 - xh[k] * m2);
        if (dres) {                                         // + the residual path's gradient (x + fn(LN(x)))
            const float4 *rr = reinterpret_cast<const float4 *>(dres + row * D);
            const float4 r0 = rr[lane], r1 = rr[64 + lane];
            o[0] += r0.x; o[1] += r0.y; o[2] += r0.z; o[3] += r0.w;
            o[4] += r1.x; o[5] += r1.y; o[6] += r1.z; o[7] += r1.w;
        }
        float4 *dr = reinterpret_cast<float4 *>(dx + row * D);
        dr[lane] = make_float4(o[0], o[1], o[2], o[3]);
        dr[64 + lane] = make_float4(o[4], o[5], o[6], o[7]);
        if (dy16) {
            const uint64_t seed = thr ? dev_seed(seedp, salt) : 0;
            const unsigned k0 = thr ? keep4(seed, (uint64_t)(row * 128 + lane), thr) : 15u;
            const unsigned k1 = thr ? keep4(seed, (uint64_t)(row * 128 + 64 + lane), thr) : 15u;
            uint32_t h[8];
#pragma unroll
            for (int e = 0; e < 8; ++e)
                h[e] = (((e < 4 ? k0 : k1) >> (e & 3)) & 1u) ? f2h(h2f(f2h(o[e])) * scale) : 0u;
            uint2 *yr = reinterpret_cast<uint2 *>(dy16 + row * D);
            yr[lane] = pack4(h[0], h[1], h[2], h[3]);
            yr[64 + lane] = pack4(h[4], h[5], h[6], h[7]);
        }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int col = (k < 4 ? 4 * lane : 256 + 4 * lane) + (k & 3);
        red[0][wave][col] = ag[k];
        red[1][wave][col] = ab[k];
    }
    __syncthreads();
    for (int i = (int)threadIdx.x; i < 2 * D; i += 256) {
        const int w = i / D, col = i - w * D;
        part[((long)w * gridDim.x + blockIdx.x) * D + col] =
            (red[w][0][col] + red[w][1][col]) + (red[w][2][col] + red[w][3][col]);
    }
}

// column sums of the [2][G][512] partials -> dgamma, dbeta (fixed order: deterministic).  A block
// takes 8 of the 1,024 columns (128 blocks); its 32 x 8 threads sum 32 slices of the G rows (4 chains
// each), then the 32 slices are added in order.
__global__ __launch_bounds__(256) void ln_bwd_colsum(const float *__restrict__ part, int G, float *__restrict__ dgamma,
                                                     float *__restrict__ dbeta) {
    __shared__ float sl[32][9];
    const int t = (int)threadIdx.x, cl = t & 7, slice = t >> 3;
    const int i = (int)blockIdx.x * 8 + cl;                // 0 .. 1023: [gamma | beta] x 512 columns
    const int w = i >> 9, col = i & 511;
    const float *p = part + (long)w * G * 512 + col;
    const int per = (G + 31) / 32, g0 = slice * per, g1 = g0 + per < G ? g0 + per : G;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int gi = g0;
    for (; gi + 4 <= g1; gi += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[u] += p[(long)(gi + u) * 512];
    }
    for (; gi < g1; ++gi) acc[0] += p[(long)gi * 512];
    sl[slice][cl] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    __syncthreads();
    if (slice == 0) {
        float v = 0.f;
        for (int k = 0; k < 32; ++k) v += sl[k][cl];
        (w ? dbeta : dgamma)[col] = v;
    }
}

// ---- bias + ReLU backward (the training forward's conv layers: y = relu(conv(x) + b), NHWC fp16) --
// dx = dy where y > 0 (torch's threshold_backward on the ReLU output), and per-workgroup partial
// sums of dx over the rows for the bias gradient (then colsum_to_f16: fixed order).
constexpr int RB_WG = 512;
__global__ __launch_bounds__(256) void relu_bias_bwd(const uint16_t *__restrict__ y, const uint16_t *__restrict__ dy,
                                                     uint16_t *__restrict__ dx, float *__restrict__ part, long rows,
                                                     int C) {
    __shared__ float acc_s[256][4];
    const int c4n = C >> 2;
    const int per = 256 / c4n;                              // rows per block pass
    const int tr = (int)threadIdx.x / c4n, c4 = (int)threadIdx.x - tr * c4n;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    if (tr < per) {
        // four rows' loads in flight per step (the loop is latency-bound otherwise); the sums keep
        // the row order, so results do not depend on the unrolling
        const long step = (long)gridDim.x * per;
        constexpr int U = 4;
        for (long r0 = (long)blockIdx.x * per + tr; r0 < rows; r0 += U * step) {
            uint2 yv[U], gv[U];
#pragma unroll
            for (int q = 0; q < U; ++q) {
                const long r = r0 + q * step;
                yv[q] = r < rows ? reinterpret_cast<const uint2 *>(y + r * C)[c4] : make_uint2(0u, 0u);
                gv[q] = r < rows ? reinterpret_cast<const uint2 *>(dy + r * C)[c4] : make_uint2(0u, 0u);
            }
#pragma unroll
            for (int q = 0; q < U; ++q) {
                const long r = r0 + q * step;
                if (r >= rows) break;
                const uint32_t yy[4] = {yv[q].x & 0xFFFFu, yv[q].x >> 16, yv[q].y & 0xFFFFu, yv[q].y >> 16};
                const uint32_t gg[4] = {gv[q].x & 0xFFFFu, gv[q].x >> 16, gv[q].y & 0xFFFFu, gv[q].y >> 16};
                uint32_t o[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    o[k] = h2f(yy[k]) <= 0.f ? 0u : gg[k];       // threshold_backward: NaN passes
                    a[k] += h2f(o[k]);
                }
                reinterpret_cast<uint2 *>(dx + r * C)[c4] = pack4(o[0], o[1], o[2], o[3]);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) acc_s[threadIdx.x][k] = a[k];
    __syncthreads();
    for (int c = (int)threadIdx.x; c < C; c += 256) {       // channel c: threads (tr, c >> 2), tr in order
        float v = 0.f;
        for (int t = 0; t < per; ++t) v += acc_s[t * c4n + (c >> 2)][c & 3];
        part[(long)blockIdx.x * C + c] = v;
    }
}

// backward of p = maxpool2x2(relu(fp16(r + bias))) over NHWC fp16 (the training forward's pooled conv
// layers; forward nhwc_bias_relu_pool2 from the raw conv output r): per window and channel, the
// gradient dp goes to the window's first strictly greatest activation in (row, column) order --
// torch's max_pool2d argmax -- if that activation is > 0 (the ReLU mask); every other position,
// and the rows / columns no window covers (odd H / W), get 0.  Bias-gradient partial sums per block
// as relu_bias_bwd.
__global__ __launch_bounds__(256) void relu_bias_pool_bwd(const uint16_t *__restrict__ r,
                                                          const uint16_t *__restrict__ bias,
                                                          const uint16_t *__restrict__ dp, uint16_t *__restrict__ dr,
                                                          float *__restrict__ part, int B, int H, int W, int C) {
    __shared__ float acc_s[256][4];
    const int Ho = H / 2, Wo = W / 2;
    const int E = H * W - 4 * Ho * Wo;                      // uncovered positions per image
    const long units = (long)B * Ho * Wo + (long)B * E;
    const int c4n = C >> 2;
    const int per = 256 / c4n;
    const int tr = (int)threadIdx.x / c4n, c4 = (int)threadIdx.x - tr * c4n;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    if (tr < per) {
        const uint2 bb = *reinterpret_cast<const uint2 *>(bias + 4 * c4);
        const float bv[4] = {h2f(bb.x), h2f(bb.x >> 16), h2f(bb.y), h2f(bb.y >> 16)};
        const long nwin = (long)B * Ho * Wo;
        for (long u = (long)blockIdx.x * per + tr; u < units; u += (long)gridDim.x * per) {
            if (u < nwin) {
                const long b = u / (Ho * Wo);
                const int rem = (int)(u - b * Ho * Wo), i = rem / Wo, j = rem - i * Wo;
                const uint2 g = *(reinterpret_cast<const uint2 *>(dp + u * C) + c4);
                const float gv[4] = {h2f(g.x & 0xFFFFu), h2f(g.x >> 16), h2f(g.y & 0xFFFFu), h2f(g.y >> 16)};
                float m[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
                int am[4] = {0, 0, 0, 0};
                long pos[4];
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    pos[w] = ((b * H + 2 * i + (w >> 1)) * (long)W + 2 * j + (w & 1)) * C;
                    const uint2 v = *(reinterpret_cast<const uint2 *>(r + pos[w]) + c4);
                    const uint32_t vv[4] = {v.x & 0xFFFFu, v.x >> 16, v.y & 0xFFFFu, v.y >> 16};
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const float act = relu_nan(h2f(f2h(h2f(vv[k]) + bv[k])));
                        if (act > m[k] || act != act) {     // torch's argmax: a NaN wins (the last one)
                            m[k] = act;
                            am[k] = w;
                        }
                    }
                }
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    uint32_t o[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const bool hit = am[k] == w && !(m[k] <= 0.f);
                        o[k] = hit ? (uint32_t)f2h(gv[k]) : 0u;
                        if (hit) a[k] += gv[k];
                    }
                    *(reinterpret_cast<uint2 *>(dr + pos[w]) + c4) = pack4(o[0], o[1], o[2], o[3]);
                }
            } else {                                        // an uncovered position: last column, then last row
                const long e = u - nwin;
                const long b = e / E;
                const int k = (int)(e - b * E);
                const int colE = (W & 1) ? H : 0;
                int h, w;
                if (k < colE) {
                    h = k;
                    w = W - 1;
                } else {
                    h = H - 1;
                    w = k - colE;
                }
                *(reinterpret_cast<uint2 *>(dr + ((b * H + h) * (long)W + w) * C) + c4) = make_uint2(0u, 0u);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) acc_s[threadIdx.x][k] = a[k];
    __syncthreads();
    for (int c = (int)threadIdx.x; c < C; c += 256) {
        float v = 0.f;
        for (int t = 0; t < per; ++t) v += acc_s[t * c4n + (c >> 2)][c & 3];
        part[(long)blockIdx.x * C + c] = v;
    }
}

// per-workgroup partial column sums of an fp16 [rows][C] matrix (a linear's bias gradient: the
// output gradient summed over the rows); blockIdx.y takes 1,024-column chunks (C % 4 == 0)
__global__ __launch_bounds__(256) void colsum_partial_f16(const uint16_t *__restrict__ g, float *__restrict__ part,
                                                          long rows, int C) {
    __shared__ float acc_s[256][4];
    const int c0 = (int)blockIdx.y * 1024, Cc = C - c0 < 1024 ? C - c0 : 1024;
    const int c4n = Cc >> 2;
    const int per = 256 / c4n;
    const int tr = (int)threadIdx.x / c4n, c4 = (int)threadIdx.x - tr * c4n;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    if (tr < per) {
        const long step = (long)gridDim.x * per;
        constexpr int U = 8;                                // eight rows' loads in flight per step
        for (long r0 = (long)blockIdx.x * per + tr; r0 < rows; r0 += U * step) {
            uint2 v[U];
#pragma unroll
            for (int q = 0; q < U; ++q) {
                const long r = r0 + q * step;
                v[q] = r < rows ? reinterpret_cast<const uint2 *>(g + r * C + c0)[c4] : make_uint2(0u, 0u);
            }
#pragma unroll
            for (int q = 0; q < U; ++q) {               // (zero rows past the end add nothing)
                a[0] += h2f(v[q].x & 0xFFFFu);
                a[1] += h2f(v[q].x >> 16);
                a[2] += h2f(v[q].y & 0xFFFFu);
                a[3] += h2f(v[q].y >> 16);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) acc_s[threadIdx.x][k] = a[k];
    __syncthreads();
    for (int c = (int)threadIdx.x; c < Cc; c += 256) {
        float v = 0.f;
        for (int t = 0; t < per; ++t) v += acc_s[t * c4n + (c >> 2)][c & 3];
        part[(long)blockIdx.x * C + c0 + c] = v;
    }
}

// column sums of a short fp16 [rows][C] matrix in ONE launch (the bias gradient of the training forward's
// 2-D linears, rows <= COLSUM_SHORT_ROWS): a block takes 32 columns -- 4 groups of 8 (16-B loads) x 64 row
// lanes, each lane its rows in order, then the 64 lanes in order (a fixed order: deterministic); fp16 out.
constexpr long COLSUM_SHORT_ROWS = 8192;
__global__ __launch_bounds__(256) void colsum_short_f16(const uint16_t *__restrict__ g, long rows, int C,
                                                        uint16_t *__restrict__ out) {
    __shared__ float sl[64][33];
    const int t = (int)threadIdx.x, cg = t & 3, rl = t >> 2;
    const int c0 = (int)blockIdx.x * 32 + cg * 8;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (c0 < C) {
        long r = rl;
        constexpr int U = 8;                                // eight rows' loads in flight
        for (; r + (U - 1) * 64 < rows; r += U * 64) {
            uint4 v[U];
#pragma unroll
            for (int q = 0; q < U; ++q) v[q] = *reinterpret_cast<const uint4 *>(g + (r + q * 64) * C + c0);
#pragma unroll
            for (int q = 0; q < U; ++q) {
                const uint32_t w[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    a[2 * k] += h2f(w[k] & 0xFFFFu);
                    a[2 * k + 1] += h2f(w[k] >> 16);
                }
            }
        }
        for (; r < rows; r += 64) {
            const uint4 v = *reinterpret_cast<const uint4 *>(g + r * C + c0);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                a[2 * k] += h2f(w[k] & 0xFFFFu);
                a[2 * k + 1] += h2f(w[k] >> 16);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) sl[rl][cg * 8 + k] = a[k];
    __syncthreads();
    const int c = (int)blockIdx.x * 32 + t;
    if (t < 32 && c < C) {
        float v = 0.f;
        for (int l = 0; l < 64; ++l) v += sl[l][t];
        out[c] = (uint16_t)f2h(v);
    }
}

// out[c] = fp16(sum_g part[g][c]) over G partial rows in a fixed order: a block takes 8 columns, its
// 32 slices of the rows 4 chains each, then the slices in order (C / 8 blocks: 16 at C = 128, where
// 32-column blocks left 4 CUs to read the partials)
__global__ __launch_bounds__(256) void colsum_to_f16(const float *__restrict__ part, int G, int C,
                                                     uint16_t *__restrict__ out) {
    __shared__ float sl[32][9];
    const int t = (int)threadIdx.x, cl = t & 7, slice = t >> 3;
    const int c = (int)blockIdx.x * 8 + cl;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    if (c < C) {
        const int per = (G + 31) / 32, g0 = slice * per, g1 = g0 + per < G ? g0 + per : G;
        int gi = g0;
        for (; gi + 4 <= g1; gi += 4) {
#pragma unroll
            for (int u = 0; u < 4; ++u) acc[u] += part[(long)(gi + u) * C + c];
        }
        for (; gi < g1; ++gi) acc[0] += part[(long)gi * C + c];
    }
    sl[slice][cl] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    __syncthreads();
    if (slice == 0 && c < C) {
        float v = 0.f;
        for (int k = 0; k < 32; ++k) v += sl[k][cl];
        out[c] = (uint16_t)f2h(v);
    }
}

// ---- multi-tensor casts (the training forward's fp16 weight copies and their gradients) --
constexpr int CAST_MAX = 64, CAST_PER_BLOCK = 4096;         // tensors per launch, elements per block
struct CastList {
    const void *src[CAST_MAX];
    void *dst[CAST_MAX];
    long n[CAST_MAX];
    int blk0[CAST_MAX + 1];                                 // first block of tensor i; blk0[count] = grid
    int cout[CAST_MAX], ks[CAST_MAX];                       // cout > 0: the flipped, transposed conv weight
    int count;
};
template <bool TO_F16>
__global__ __launch_bounds__(256) void cast_multi(CastList L) {
    const int b = (int)blockIdx.x;
    int t = 0;
    while (t + 1 < L.count && L.blk0[t + 1] <= b) ++t;      // uniform scan over <= 64 entries
    const long base = (long)(b - L.blk0[t]) * CAST_PER_BLOCK, n = L.n[t];
    const int co = TO_F16 ? L.cout[t] : 0, ks = TO_F16 ? L.ks[t] : 1;
    for (int e = (int)threadIdx.x; e < CAST_PER_BLOCK; e += 256) {
        const long i = base + e;
        if (i >= n) break;
        if (TO_F16) {
            long j = i;
            if (co > 0) {       // dst [Cin][ky][kx][Cout] = src [Cout][ks-1-ky][ks-1-kx][Cin] (channels_last storage)
                const int cin = (int)(n / ((long)co * ks * ks));
                const int o = (int)(i % co);
                long r = i / co;
                const int kx = (int)(r % ks);
                r /= ks;
                const int ky = (int)(r % ks), ci = (int)(r / ks);
                j = (((long)o * ks + (ks - 1 - ky)) * ks + (ks - 1 - kx)) * cin + ci;
            }
            static_cast<uint16_t *>(L.dst[t])[i] = (uint16_t)f2h(static_cast<const float *>(L.src[t])[j]);
        } else {
            static_cast<float *>(L.dst[t])[i] = h2f(static_cast<const uint16_t *>(L.src[t])[i]);
        }
    }
}

template <bool TO_F16>
static int cast_multi_api(const void *const *src, void *const *dst, const int64_t *n, int32_t count, void *stream,
                          const int32_t *cout = nullptr, const int32_t *ks = nullptr) {
    if (!src || !dst || !n || count < 0 || count > CAST_MAX || (!cout) != (!ks)) return MAPF_EINVAL;
    CastList L{};
    long blocks = 0;
    for (int i = 0; i < count; ++i) {
        if (n[i] < 0 || (n[i] > 0 && (!src[i] || !dst[i]))) return MAPF_EINVAL;
        if (cout && cout[i] > 0 && (ks[i] <= 0 || n[i] % ((int64_t)cout[i] * ks[i] * ks[i]))) return MAPF_EINVAL;
        L.cout[i] = cout && cout[i] > 0 ? cout[i] : 0;
        L.ks[i] = cout && cout[i] > 0 ? ks[i] : 1;
        L.src[i] = src[i];
        L.dst[i] = dst[i];
        L.n[i] = (long)n[i];
        L.blk0[i] = (int)blocks;
        blocks += (n[i] + CAST_PER_BLOCK - 1) / CAST_PER_BLOCK;
        if (blocks > (1L << 30)) return MAPF_EINVAL;
    }
    L.blk0[count] = (int)blocks;
    L.count = count;
    if (blocks == 0) return MAPF_OK;
    hipLaunchKernelGGL(cast_multi<TO_F16>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, L);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

// ---- the update's optimizer tail (model._DeviceUpdate._back): AMP unscale + found-inf, the grad-norm
// clip and Adam in three launches over up to OPT_MAX fp32 tensors each, in place of torch's unscale,
// foreach-norm, stack / norm / clamp, foreach-mul and fused-Adam passes.  p, g, m, v of a tensor share
// one dense layout, so element k of each is the same parameter entry.
constexpr int OPT_MAX = 64, OPT_PER_BLOCK = 8192;
struct OptList {
    float *p[OPT_MAX];
    float *g[OPT_MAX];
    float *m[OPT_MAX];
    float *v[OPT_MAX];
    long n[OPT_MAX];
    int blk0[OPT_MAX + 1];                                  // first block of tensor i; blk0[count] = the chunk's grid
    int count;
};
__device__ inline int opt_tensor(const OptList &L, int b) {
    int t = 0;
    while (t + 1 < L.count && L.blk0[t + 1] <= b) ++t;      // uniform scan over <= 64 entries
    return t;
}
__device__ inline float opt_inv_scale(const float *scale) { return (float)(1.0 / (double)scale[0]); }

// pass 1: per block, the sum of squares of the unscaled gradients (fp32, the block's elements in a
// fixed order) -> part[part0 + block]; any non-finite gradient sets found_inf = 1
__global__ __launch_bounds__(256) void optim_sumsq(OptList L, const float *__restrict__ scale, float *__restrict__ part,
                                                   int part0, float *__restrict__ found_inf) {
    __shared__ float red[4];
    __shared__ int bad;
    const int b = (int)blockIdx.x, t = opt_tensor(L, b);
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    const float inv = opt_inv_scale(scale);
    const long base = (long)(b - L.blk0[t]) * OPT_PER_BLOCK, n = L.n[t];
    float acc = 0.f;
    bool nf = false;
    for (int e0 = (int)threadIdx.x; e0 < OPT_PER_BLOCK; e0 += 4 * 256) {   // four independent loads in flight
        float gv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long i = base + e0 + u * 256;
            gv[u] = (e0 + u * 256 < OPT_PER_BLOCK && i < n) ? L.g[t][i] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            nf |= !isfinite(gv[u]);
            const float x = gv[u] * inv;
            acc += x * x;
        }
    }
    if (nf) bad = 1;
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        part[part0 + b] = (red[0] + red[1]) + (red[2] + red[3]);
        if (bad) found_inf[0] = 1.f;
    }
}

// the total gradient norm from the G partials, in one fixed order (every block computes the same value)
__device__ inline float opt_total_norm(const float *__restrict__ part, int G) {
    __shared__ float red[4];
    float a = 0.f;
    for (int k = (int)threadIdx.x; k < G; k += 256) a += part[k];
    a = wave_sum(a);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
    __syncthreads();
    const float tot = (red[0] + red[1]) + (red[2] + red[3]);
    __syncthreads();
    return sqrtf(tot);
}

// pass 2: g' = (g / scale) * min(max_norm / (norm + 1e-6), 1) (torch's unscale_ then clip_grad_norm_'s
// in-place scaling, two roundings), written back to g as torch leaves it; then, unless found_inf, torch's
// fused Adam step (no weight decay, no amsgrad) with step = the stored step + 1.  Block 0 writes the norm.
__global__ __launch_bounds__(256) void optim_adam(OptList L, const float *__restrict__ part, int G,
                                                  const float *__restrict__ scale, const float *__restrict__ found_inf,
                                                  const float *__restrict__ step, float max_norm, float lr, float beta1,
                                                  float beta2, float eps, float *__restrict__ grad_norm) {
    const int b = (int)blockIdx.x, t = opt_tensor(L, b);
    const float norm = opt_total_norm(part, G);
    if (b == 0 && threadIdx.x == 0 && grad_norm) grad_norm[0] = norm;
    const float inv = opt_inv_scale(scale);
    const float coef = fminf(max_norm / (norm + 1e-6f), 1.f);
    const long base0 = (long)(b - L.blk0[t]) * OPT_PER_BLOCK, n0 = L.n[t];
    if (found_inf[0] != 0.f) {                              // the step is skipped; g as torch leaves it
        for (int e = (int)threadIdx.x; e < OPT_PER_BLOCK && base0 + e < n0; e += 256)
            L.g[t][base0 + e] = (L.g[t][base0 + e] * inv) * coef;
        return;
    }
    const float s = step[0] + 1.f;
    const float bc1 = 1.f - powf(beta1, s), bc2s = sqrtf(1.f - powf(beta2, s));
    const float step_size = lr / bc1;
    const long base = (long)(b - L.blk0[t]) * OPT_PER_BLOCK, n = L.n[t];
    for (int e0 = (int)threadIdx.x; e0 < OPT_PER_BLOCK; e0 += 4 * 256) {   // four entries' loads in flight
        float gv[4], mv[4], vv[4], pv[4];
        bool ok[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long i = base + e0 + u * 256;
            ok[u] = e0 + u * 256 < OPT_PER_BLOCK && i < n;
            gv[u] = ok[u] ? L.g[t][i] : 0.f;
            mv[u] = ok[u] ? L.m[t][i] : 0.f;
            vv[u] = ok[u] ? L.v[t][i] : 0.f;
            pv[u] = ok[u] ? L.p[t][i] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (!ok[u]) continue;
            const long i = base + e0 + u * 256;
            const float g = (gv[u] * inv) * coef;
            const float m = beta1 * mv[u] + (1.f - beta1) * g;
            const float v = beta2 * vv[u] + (1.f - beta2) * g * g;
            L.g[t][i] = g;
            L.m[t][i] = m;
            L.v[t][i] = v;
            L.p[t][i] = pv[u] - step_size * m / (sqrtf(v) / bc2s + eps);
        }
    }
}

// pass 3: every tensor's step += 1 unless found_inf (torch's capturable Adam keeps one per parameter)
struct OptSteps {
    float *s[OPT_MAX];
    int count;
};
__global__ void optim_steps(OptSteps S, const float *__restrict__ found_inf) {
    const int i = (int)threadIdx.x;
    if (i < S.count && found_inf[0] == 0.f) S.s[i][0] += 1.f;
}

// ---- dropout epilogues -----------------------------------------------------------
__device__ inline float4 add_dropped(float4 a, uint2 v, unsigned k, float scale) {
    a.x += (k & 1u) ? h2f(f2h(h2f(v.x) * scale)) : 0.f;
    a.y += (k & 2u) ? h2f(f2h(h2f(v.x >> 16) * scale)) : 0.f;
    a.z += (k & 4u) ? h2f(f2h(h2f(v.y) * scale)) : 0.f;
    a.w += (k & 8u) ? h2f(f2h(h2f(v.y >> 16) * scale)) : 0.f;
    return a;
}

// x[i] += dropout(y[i]); torch: dropout on the fp16 tensor (y * scale rounded to fp16),
// then fp16 + fp32 -> fp32
__global__ __launch_bounds__(256) void dropout_residual(float *__restrict__ x, const uint16_t *__restrict__ y, long n4,
                                                        uint32_t thr, float scale, uint64_t seed) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
        const unsigned k = thr ? keep4(seed, (uint64_t)i, thr) : 15u;
        reinterpret_cast<float4 *>(x)[i] =
            add_dropped(reinterpret_cast<float4 *>(x)[i], reinterpret_cast<const uint2 *>(y)[i], k, scale);
    }
}

// x += dropout(y); z = LayerNorm(x) -> fp16: dropout_residual then layernorm_f16 in one
// pass over the residual stream (same mask bits, same arithmetic -- bit-identical to the
// two launches), one wave per 512-wide row of contiguous x, y
__global__ __launch_bounds__(256) void dropout_residual_layernorm(float *__restrict__ x, const uint16_t *__restrict__ y,
                                                                  const float *__restrict__ gamma,
                                                                  const float *__restrict__ beta,
                                                                  uint16_t *__restrict__ z, long rows, uint32_t thr,
                                                                  float scale, float eps, uint64_t seed) {
    const int lane = (int)(threadIdx.x & 63);
    const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const long i0 = row * 128 + lane, i1 = i0 + 64;          // float4 indices, as dropout_residual's
    float4 *xr = reinterpret_cast<float4 *>(x);
    const uint2 *yr = reinterpret_cast<const uint2 *>(y);
    const float4 a = add_dropped(xr[i0], yr[i0], thr ? keep4(seed, (uint64_t)i0, thr) : 15u, scale);
    const float4 c = add_dropped(xr[i1], yr[i1], thr ? keep4(seed, (uint64_t)i1, thr) : 15u, scale);
    xr[i0] = a;
    xr[i1] = c;
    ln_row(a, c, lane, gamma, beta, eps, z + row * 512);
}

// h = dropout(gelu(h)) in place: exact (erf) GELU in fp32 rounded to fp16 like torch's
// fp16 GELU, then dropout on the fp16 values
__global__ __launch_bounds__(256) void gelu_dropout_f16(uint16_t *__restrict__ h, long n4, uint32_t thr, float scale,
                                                        uint64_t seed) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
        const unsigned k = thr ? keep4(seed, (uint64_t)i, thr) : 15u;
        uint2 *p = reinterpret_cast<uint2 *>(h) + i;
        const uint2 v = *p;
        const uint32_t in[4] = {v.x, v.x >> 16, v.y, v.y >> 16};
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float a = h2f(in[q]);
            const float g = h2f(f2h(0.5f * a * (1.f + erff(a * 0.70710678118654752f))));
            o[q] = ((k >> q) & 1u) ? f2h(g * scale) : 0u;
        }
        *p = pack4(o[0], o[1], o[2], o[3]);
    }
}

// ---- the TRAINING forward's dropout (round 6): the same hash masks, the seed in device memory ------
// A captured update replays its kernels with the arguments they were captured with, so a seed passed
// by value would drop the same elements in every replay.  These kernels read a counter the training
// forward increments on the device (SCRIMPNet._train_seed, captured with the update) and mix in a
// per-site salt: every replay, and every dropout site, draws its own mask.

// x_out = res + dropout(y) (fp32; res may be a strided view: rstride floats per row), z = LayerNorm(x_out)
// fp16: dropout_residual_layernorm's arithmetic without writing over the residual (autograd keeps it)
__global__ __launch_bounds__(256) void drln_fwd(const float *__restrict__ res, long rstride, const uint16_t *__restrict__ y,
                                                float *__restrict__ xo, const float *__restrict__ gamma,
                                                const float *__restrict__ beta, uint16_t *__restrict__ z, long rows,
                                                uint32_t thr, float scale, float eps, const uint64_t *__restrict__ seedp,
                                                uint32_t salt) {
    const int lane = (int)(threadIdx.x & 63);
    const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const uint64_t seed = thr ? dev_seed(seedp, salt) : 0;
    const long i0 = row * 128 + lane, i1 = i0 + 64;
    const float4 *rr = reinterpret_cast<const float4 *>(res + row * rstride);
    const uint2 *yr = reinterpret_cast<const uint2 *>(y);
    const float4 a = add_dropped(rr[lane], yr[i0], thr ? keep4(seed, (uint64_t)i0, thr) : 15u, scale);
    const float4 c = add_dropped(rr[64 + lane], yr[i1], thr ? keep4(seed, (uint64_t)i1, thr) : 15u, scale);
    float4 *xr = reinterpret_cast<float4 *>(xo);
    xr[i0] = a;
    xr[i1] = c;
    ln_row(a, c, lane, gamma, beta, eps, z + row * 512);
}

__device__ inline float gelu_exact(float a) { return 0.5f * a * (1.f + erff(a * 0.70710678118654752f)); }

// out = dropout(gelu(h)) (h kept for the backward): gelu_dropout_f16's arithmetic, out of place
__global__ __launch_bounds__(256) void gelu_dropout_train(const uint16_t *__restrict__ h, uint16_t *__restrict__ out, long n4,
                                                          uint32_t thr, float scale, const uint64_t *__restrict__ seedp,
                                                          uint32_t salt) {
    const uint64_t seed = thr ? dev_seed(seedp, salt) : 0;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
        const unsigned k = thr ? keep4(seed, (uint64_t)i, thr) : 15u;
        const uint2 v = reinterpret_cast<const uint2 *>(h)[i];
        const uint32_t in[4] = {v.x, v.x >> 16, v.y, v.y >> 16};
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = ((k >> q) & 1u) ? f2h(h2f(f2h(gelu_exact(h2f(in[q])))) * scale) : 0u;
        reinterpret_cast<uint2 *>(out)[i] = pack4(o[0], o[1], o[2], o[3]);
    }
}

// dh = gelu'(h) * dropout_backward(dout): torch's masked_scale (fp16(dout * scale) where kept) then its
// exact GeluBackward in fp32 (0.5 (1 + erf(x / sqrt 2)) + x exp(-x^2 / 2) / sqrt(2 pi)), rounded to fp16
__global__ __launch_bounds__(256) void gelu_dropout_bwd(const uint16_t *__restrict__ h, const uint16_t *__restrict__ dout,
                                                        uint16_t *__restrict__ dh, long n4, uint32_t thr, float scale,
                                                        const uint64_t *__restrict__ seedp, uint32_t salt) {
    const uint64_t seed = thr ? dev_seed(seedp, salt) : 0;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
        const unsigned k = thr ? keep4(seed, (uint64_t)i, thr) : 15u;
        const uint2 v = reinterpret_cast<const uint2 *>(h)[i], gv = reinterpret_cast<const uint2 *>(dout)[i];
        const uint32_t in[4] = {v.x, v.x >> 16, v.y, v.y >> 16}, gi[4] = {gv.x, gv.x >> 16, gv.y, gv.y >> 16};
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float t = ((k >> q) & 1u) ? h2f(f2h(h2f(gi[q]) * scale)) : 0.f;
            const float x = h2f(in[q]);
            const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
            const float pdf = expf(-0.5f * x * x) * 0.39894228040143268f;
            o[q] = f2h(t * __builtin_fmaf(x, pdf, cdf));     // torch's kernel, compiled with contraction
        }
        reinterpret_cast<uint2 *>(dh)[i] = pack4(o[0], o[1], o[2], o[3]);
    }
}

// x[b][0][:] = cls + pos[0];  x[b][1+t][:] = A[b][t] * VV[b][:] + pos[1+t];  then dropout
// (all fp32: softmax output A is fp32 under autocast, the fp16 VV promotes).
// A fp32 [B][L], VV fp16 [B][D], cls fp32 [D], pos fp32 [L+1][D]; D % 4 == 0.
__device__ inline float4 token4(const float *__restrict__ A, const uint16_t *__restrict__ VV,
                                const float *__restrict__ cls, const float *__restrict__ pos, long b, int t, int d4,
                                int L, int D, long i, uint32_t thr, float scale, uint64_t seed) {
    const float4 pp = reinterpret_cast<const float4 *>(pos + (long)t * D)[d4];
    float4 v;
    if (t == 0) {
        const float4 c = reinterpret_cast<const float4 *>(cls)[d4];
        v = make_float4(c.x + pp.x, c.y + pp.y, c.z + pp.z, c.w + pp.w);
    } else {
        const float a = A[b * L + t - 1];
        const uint2 w = reinterpret_cast<const uint2 *>(VV + b * D)[d4];
        v = make_float4(a * h2f(w.x) + pp.x, a * h2f(w.x >> 16) + pp.y, a * h2f(w.y) + pp.z, a * h2f(w.y >> 16) + pp.w);
    }
    if (thr) {
        const unsigned k = keep4(seed, (uint64_t)i, thr);
        v.x = (k & 1u) ? v.x * scale : 0.f;
        v.y = (k & 2u) ? v.y * scale : 0.f;
        v.z = (k & 4u) ? v.z * scale : 0.f;
        v.w = (k & 8u) ? v.w * scale : 0.f;
    }
    return v;
}

__global__ __launch_bounds__(256) void tokens(float *__restrict__ x, const float *__restrict__ A,
                                              const uint16_t *__restrict__ VV, const float *__restrict__ cls,
                                              const float *__restrict__ pos, long B, int L, int D, uint32_t thr,
                                              float scale, uint64_t seed) {
    const int d4n = D >> 2;
    const long n4 = B * (L + 1) * d4n;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
        const long row = i / d4n;
        const int d4 = (int)(i - row * d4n);
        const long b = row / (L + 1);
        reinterpret_cast<float4 *>(x)[i] =
            token4(A, VV, cls, pos, b, (int)(row - b * (L + 1)), d4, L, D, i, thr, scale, seed);
    }
}

// tokens + the first PreNorm's LayerNorm (z fp16) in one pass, one wave per 512-wide
// row; bit-identical to tokens followed by layernorm_f16
__global__ __launch_bounds__(256) void tokens_layernorm(float *__restrict__ x, const float *__restrict__ A,
                                                        const uint16_t *__restrict__ VV, const float *__restrict__ cls,
                                                        const float *__restrict__ pos, long B, int L, uint32_t thr,
                                                        float scale, uint64_t seed, const float *__restrict__ gamma,
                                                        const float *__restrict__ beta, float eps,
                                                        uint16_t *__restrict__ z) {
    // four rows per wave (ln_rows: their reductions interleaved), 16 per block
    constexpr int R = 4;
    const int lane = (int)(threadIdx.x & 63);
    const long rows = B * (L + 1);
    const long row0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
    if (row0 >= rows) return;
    float4 av[R], cv[R];
    bool live[R];
    uint16_t *zr[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const long row = row0 + r;
        live[r] = row < rows;
        zr[r] = z + (live[r] ? row : 0) * 512;
        if (!live[r]) {
            av[r] = cv[r] = make_float4(0.f, 0.f, 0.f, 0.f);
            continue;
        }
        const long b = row / (L + 1);
        const int t = (int)(row - b * (L + 1));
        av[r] = token4(A, VV, cls, pos, b, t, lane, L, 512, row * 128 + lane, thr, scale, seed);
        cv[r] = token4(A, VV, cls, pos, b, t, 64 + lane, L, 512, row * 128 + 64 + lane, thr, scale, seed);
        if (x) {                                    // (null: the next fused linear recomputes the tokens)
            float4 *xr = reinterpret_cast<float4 *>(x) + row * 128;
            xr[lane] = av[r];
            xr[64 + lane] = cv[r];
        }
    }
    ln_rows<R>(av, cv, live, lane, gamma, beta, eps, zr);
}

// ---- the TRAINING forward's tokens (net._TokensLN; SCRIMPNet.forward's tokeniser, net.py:124-130) ----
// x = dropout(cat(cls, A * VV) + pos) fp32 as torch's ops compute it -- the product and the sum rounded
// separately (no contraction), the dropout as x * scale where kept -- with the mask from the device seed
// (dev_seed: graph-safe), and z = fp16(LayerNorm(x)).  A: [B][16] fp32, VV: [B][512] fp16.
constexpr int TOK_L = 16, TOK_T = TOK_L + 1;
constexpr long TOK_BWD_WG = 512;                            // tokens_train_bwd's blocks at most (2 per CU)
__device__ inline float4 token4_train(const float *__restrict__ A, const uint16_t *__restrict__ VV,
                                      const float *__restrict__ cls, const float *__restrict__ pos, long b, int t,
                                      int d4, long i, uint32_t thr, float scale, uint64_t seed) {
    const float4 pp = reinterpret_cast<const float4 *>(pos + (long)t * 512)[d4];
    float4 v;
    if (t == 0) {
        const float4 c = reinterpret_cast<const float4 *>(cls)[d4];
        v = make_float4(__fadd_rn(c.x, pp.x), __fadd_rn(c.y, pp.y), __fadd_rn(c.z, pp.z), __fadd_rn(c.w, pp.w));
    } else {
        const float a = A[b * TOK_L + t - 1];
        const uint2 w = reinterpret_cast<const uint2 *>(VV + b * 512)[d4];
        v = make_float4(__fadd_rn(__fmul_rn(a, h2f(w.x)), pp.x), __fadd_rn(__fmul_rn(a, h2f(w.x >> 16)), pp.y),
                        __fadd_rn(__fmul_rn(a, h2f(w.y)), pp.z), __fadd_rn(__fmul_rn(a, h2f(w.y >> 16)), pp.w));
    }
    if (thr) {
        const unsigned k = keep4(seed, (uint64_t)i, thr);
        v.x = (k & 1u) ? __fmul_rn(v.x, scale) : 0.f;
        v.y = (k & 2u) ? __fmul_rn(v.y, scale) : 0.f;
        v.z = (k & 4u) ? __fmul_rn(v.z, scale) : 0.f;
        v.w = (k & 8u) ? __fmul_rn(v.w, scale) : 0.f;
    }
    return v;
}

__global__ __launch_bounds__(256) void tokens_ln_train(float *__restrict__ x, const float *__restrict__ A,
                                                       const uint16_t *__restrict__ VV, const float *__restrict__ cls,
                                                       const float *__restrict__ pos, long B, uint32_t thr, float scale,
                                                       const uint64_t *__restrict__ seedp, uint32_t salt,
                                                       const float *__restrict__ gamma, const float *__restrict__ beta,
                                                       float eps, uint16_t *__restrict__ z) {
    constexpr int R = 4;                                    // four rows per wave, 16 per block (tokens_layernorm)
    const int lane = (int)(threadIdx.x & 63);
    const long rows = B * TOK_T;
    const long row0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
    if (row0 >= rows) return;
    const uint64_t seed = thr ? dev_seed(seedp, salt) : 0;
    float4 av[R], cv[R];
    bool live[R];
    uint16_t *zr[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const long row = row0 + r;
        live[r] = row < rows;
        zr[r] = z + (live[r] ? row : 0) * 512;
        if (!live[r]) {
            av[r] = cv[r] = make_float4(0.f, 0.f, 0.f, 0.f);
            continue;
        }
        const long b = row / TOK_T;
        const int t = (int)(row - b * TOK_T);
        av[r] = token4_train(A, VV, cls, pos, b, t, lane, row * 128 + lane, thr, scale, seed);
        cv[r] = token4_train(A, VV, cls, pos, b, t, 64 + lane, row * 128 + 64 + lane, thr, scale, seed);
        float4 *xr = reinterpret_cast<float4 *>(x) + row * 128;
        xr[lane] = av[r];
        xr[64 + lane] = cv[r];
    }
    ln_rows<R>(av, cv, live, lane, gamma, beta, eps, zr);
}

// backward of tokens_ln_train's tokens, given dx = dL/dx fp32 [B][17][512] (LayerNorm's backward with the
// residual's gradient already added): g = dx * scale where the forward kept, else 0 (torch's dropout
// backward); dA[b][t] = sum_c g[b][t+1][c] VV[b][c] (fp32); dVV[b][c] = fp16(sum_t g[b][t+1][c] A[b][t]), the
// products rounded before the sums as torch's mul then sum; and per-block partial sums of g over the block's
// sequences (dpos; its token-0 row is dcls) for tokens_bwd_colsum, in a fixed order.  256 threads per block,
// 2 columns each; sequences two at a time (both rows' 34 loads in flight).
__device__ inline void tok_bwd_row(const float *__restrict__ dx, long b, int c0, uint32_t thr, float scale,
                                   uint64_t seed, float2 (&g)[TOK_T]) {
#pragma unroll
    for (int t = 0; t < TOK_T; ++t) g[t] = *reinterpret_cast<const float2 *>(dx + (b * TOK_T + t) * 512 + c0);
    if (thr) {
#pragma unroll
        for (int t = 0; t < TOK_T; ++t) {
            const long i = (b * TOK_T + t) * 512 + c0;
            const unsigned k = keep2(seed, (uint64_t)(i >> 2), thr, (unsigned)(c0 & 3));
            g[t].x = (k & 1u) ? __fmul_rn(g[t].x, scale) : 0.f;
            g[t].y = (k & 2u) ? __fmul_rn(g[t].y, scale) : 0.f;
        }
    }
}

__global__ __launch_bounds__(256) void tokens_train_bwd(const float *__restrict__ dx, const float *__restrict__ A,
                                                        const uint16_t *__restrict__ VV, long B, int per, uint32_t thr,
                                                        float scale, const uint64_t *__restrict__ seedp, uint32_t salt,
                                                        float *__restrict__ dA, uint16_t *__restrict__ dVV,
                                                        float *__restrict__ part) {
    __shared__ float red[2][4][TOK_L];
    const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6, c0 = 2 * tid;
    const uint64_t seed = thr ? dev_seed(seedp, salt) : 0;
    float2 acc[TOK_T];
#pragma unroll
    for (int t = 0; t < TOK_T; ++t) acc[t] = make_float2(0.f, 0.f);
    const long b0 = (long)blockIdx.x * per, b1 = b0 + per < B ? b0 + per : B;
    for (long b = b0; b < b1; b += 2) {
        const int nb = b + 1 < b1 ? 2 : 1;
        float2 g[2][TOK_T];
        tok_bwd_row(dx, b, c0, thr, scale, seed, g[0]);
        if (nb == 2) tok_bwd_row(dx, b + 1, c0, thr, scale, seed, g[1]);
        float pa[2][TOK_L];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            if (q >= nb) {
#pragma unroll
                for (int t = 0; t < TOK_L; ++t) pa[q][t] = 0.f;
                continue;
            }
            const long bb = b + q;
#pragma unroll
            for (int t = 0; t < TOK_T; ++t) {               // dpos partials in sequence order
                acc[t].x += g[q][t].x;
                acc[t].y += g[q][t].y;
            }
            const uint32_t vv = *reinterpret_cast<const uint32_t *>(VV + bb * 512 + c0);
            const float v0 = h2f(vv & 0xFFFFu), v1 = h2f(vv >> 16);
            float s0 = 0.f, s1 = 0.f;
#pragma unroll
            for (int t = 0; t < TOK_L; ++t) {
                const float a = A[bb * TOK_L + t];
                s0 = __fadd_rn(s0, __fmul_rn(g[q][t + 1].x, a));
                s1 = __fadd_rn(s1, __fmul_rn(g[q][t + 1].y, a));
                pa[q][t] = __fadd_rn(__fmul_rn(g[q][t + 1].x, v0), __fmul_rn(g[q][t + 1].y, v1));
            }
            *reinterpret_cast<uint32_t *>(dVV + bb * 512 + c0) = (uint32_t)f2h(s0) | ((uint32_t)f2h(s1) << 16);
        }
        // dA: 2 x 16 sums over the 512 columns -- interleaved wave reductions, then the 4 waves in order
#pragma unroll
        for (int s = 32; s >= 1; s >>= 1)
#pragma unroll
            for (int q = 0; q < 2; ++q)
#pragma unroll
                for (int t = 0; t < TOK_L; ++t) pa[q][t] += __shfl_xor(pa[q][t], s, 64);
        if (lane == 0) {
#pragma unroll
            for (int q = 0; q < 2; ++q)
#pragma unroll
                for (int t = 0; t < TOK_L; ++t) red[q][wv][t] = pa[q][t];
        }
        __syncthreads();
        if (tid < 2 * TOK_L && tid / TOK_L < nb) {
            const int q = tid / TOK_L, t = tid % TOK_L;
            dA[(b + q) * TOK_L + t] = (red[q][0][t] + red[q][1][t]) + (red[q][2][t] + red[q][3][t]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int t = 0; t < TOK_T; ++t)
        *reinterpret_cast<float2 *>(part + ((long)blockIdx.x * TOK_T + t) * 512 + c0) = acc[t];
}

// dpos[c] = sum_g part[g][c] over G partial rows in a fixed order (colsum_to_f16's, fp32 out); dcls = its
// first 512 columns (the cls token's gradient: token 0's)
__global__ __launch_bounds__(256) void tokens_bwd_colsum(const float *__restrict__ part, int G, int C,
                                                         float *__restrict__ dpos, float *__restrict__ dcls) {
    __shared__ float sl[8][32];
    const int t = (int)threadIdx.x, cl = t & 31, slice = t >> 5;
    const int c = (int)blockIdx.x * 32 + cl;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    if (c < C) {
        const int per = (G + 7) / 8, g0 = slice * per, g1 = g0 + per < G ? g0 + per : G;
        int gi = g0;
        for (; gi + 4 <= g1; gi += 4) {
#pragma unroll
            for (int u = 0; u < 4; ++u) acc[u] += part[(long)(gi + u) * C + c];
        }
        for (; gi < g1; ++gi) acc[0] += part[(long)gi * C + c];
    }
    sl[slice][cl] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    __syncthreads();
    if (slice == 0 && c < C) {
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) v += sl[k][cl];
        dpos[c] = v;
        if (c < 512) dcls[c] = v;
    }
}

// ---- attention over a short token axis (transformer.py:48-85; n <= 32 tokens) -----
// softmax(q k^T * scale) v per head (head_dim 32), fp16 in, fp32 scores / softmax,
// P rounded to fp16 for the P.V product (as the flash SDPA kernel it replaces does),
// fp16 out.  MFMA v_mfma_f32_16x16x32_f16, one contraction step = one head's 32 dims:
//   S^T[key][query] = K Q^T   A = K rows (16-B loads), B = Q rows (16-B loads); keys and
//                             queries padded to 2 tiles of 16 (n = 17: CLS + 16 cells)
//   softmax over keys         the accumulator holds a query column on each lane, its keys
//                             in registers + the 4 lanes l, l^16, l^32, l^48
//   O^T[dh][query] = V^T P^T  the accumulator is the B operand as is (its k order is
//                             (r>>2)*16 + 4*(l>>4) + (r&3)); V^T comes from an LDS image of
//                             V read with ds_read_b64_tr_b16 in that same key order
// One workgroup per sequence, 4 waves x 4 heads; all of a wave's loads issue up front.
// Strides in fp16 elements: token (row) and sequence.
typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
typedef short s4_t __attribute__((ext_vector_type(4)));
typedef float f4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4_t lds_s4_t;

// V image of one head: 32 key rows x 64 B; 16-B chunk c of row r sits at chunk
// c ^ 2*((r >> 2) & 1), so the transposed reads' rows r and r + 4 use different banks
__device__ inline int vimg_off(int r, int c) { return r * 64 + ((c ^ (((r >> 2) & 1) << 1)) << 4); }

__device__ inline uint4 ld16(const uint16_t *p, bool ok) {
    return ok ? *reinterpret_cast<const uint4 *>(p) : make_uint4(0u, 0u, 0u, 0u);
}
__device__ inline h8_t as_h8(uint4 u) { return __builtin_bit_cast(h8_t, u); }

template <int QT>
__global__ __launch_bounds__(256) void attention_f16(const uint16_t *__restrict__ q, const uint16_t *__restrict__ k,
                                                     const uint16_t *__restrict__ v, uint16_t *__restrict__ out,
                                                     int n, int q_rows, long q_ts, long q_bs, long kv_ts, long kv_bs,
                                                     float scale_log2e) {
    constexpr int HW = 4;                                     // heads per wave
    __shared__ __attribute__((aligned(16))) uint8_t vimg[4][HW][2048];
    const int lane = (int)(threadIdx.x & 63), w = (int)(threadIdx.x >> 6);
    const int g = lane >> 4, i = lane & 15;
    const long b = blockIdx.x;
    const uint16_t *qb = q + b * q_bs, *kb = k + b * kv_bs, *vb = v + b * kv_bs;
    uint4 kf[HW][2], vf[HW][2], qf[HW][QT];
#pragma unroll
    for (int hh = 0; hh < HW; ++hh) {
        const int col = (w * HW + hh) * 32 + 8 * g;           // this lane's 8 dims of the head
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int key = 16 * t + i;
            kf[hh][t] = ld16(kb + key * kv_ts + col, key < n);
            vf[hh][t] = ld16(vb + key * kv_ts + col, key < n);
        }
#pragma unroll
        for (int t = 0; t < QT; ++t) qf[hh][t] = ld16(qb + (16 * t + i) * q_ts + col, 16 * t + i < q_rows);
    }
#pragma unroll
    for (int hh = 0; hh < HW; ++hh)
#pragma unroll
        for (int t = 0; t < 2; ++t) *reinterpret_cast<uint4 *>(&vimg[w][hh][vimg_off(16 * t + i, g)]) = vf[hh][t];
    __syncthreads();
#pragma unroll
    for (int hh = 0; hh < HW; ++hh) {
        const int h = w * HW + hh;
        f4_t s[2][QT];
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
                s[kt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h8(kf[hh][kt]), as_h8(qf[hh][qt]),
                                                                   f4_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        h8_t pf[QT];
        float inv[QT];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            float x[8], m = -INFINITY;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int key = (e >> 2) * 16 + 4 * g + (e & 3);
                x[e] = key < n ? s[e >> 2][qt][e & 3] * scale_log2e : -INFINITY;
                m = fmaxf(m, x[e]);
            }
            m = fmaxf(m, __shfl_xor(m, 16, 64));
            m = fmaxf(m, __shfl_xor(m, 32, 64));
            float sum = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float pe = exp2f(x[e] - m);
                sum += pe;
                pf[qt][e] = (_Float16)pe;
            }
            sum += __shfl_xor(sum, 16, 64);
            sum += __shfl_xor(sum, 32, 64);
            inv[qt] = 1.f / sum;
        }
        const int rq = i >> 2, cp = i & 3;                    // this lane's address in its tr-read block
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
            const uint8_t *img = vimg[w][hh];
            const int c = 2 * dt + (cp >> 1), hb = 8 * (cp & 1);
            const s4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t *)(img + vimg_off(4 * g + rq, c) + hb));
            const s4_t hi =
                __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t *)(img + vimg_off(16 + 4 * g + rq, c) + hb));
            const h8_t vt = __builtin_bit_cast(h8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                const f4_t o = __builtin_amdgcn_mfma_f32_16x16x32_f16(vt, pf[qt], f4_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                const int qr = 16 * qt + i;
                if (qr < q_rows)
                    *reinterpret_cast<uint2 *>(out + (b * q_rows + qr) * 512 + h * 32 + 16 * dt + 4 * g) =
                        pack4(f2h(o[0] * inv[qt]), f2h(o[1] * inv[qt]), f2h(o[2] * inv[qt]), f2h(o[3] * inv[qt]));
            }
        }
    }
}

inline int grid_for(long items, int per_block) {
    long g = (items + per_block - 1) / per_block;
    if (g > 16384) g = 16384;
    return (int)(g < 1 ? 1 : g);
}

// ---- 512 x 512 linear layers with their epilogues on the MFMA -------------------------
// y = A W^T + b (torch Linear under autocast: fp16 operands, fp32 accumulation, the bias added
// before the ONE rounding to fp16, as hipBLASLt's bias epilogue does), N = K = 512, then
//   EPI 0  out = dropout(gelu(y))                  (MLP_Block af1 + do1: gelu_dropout_f16's arithmetic)
//   EPI 1  x += dropout(y); z = LayerNorm(x) fp16  (Residual do1 / do2 + the next PreNorm:
//          dropout_residual_layernorm's arithmetic)
// with the same mask bits (float4 index row * 128 + col / 4 of the [M, 512] tensor) as the
// separate launches, so only the GEMM's summation order differs from lin() + the epilogue kernel;
// the linear's fp16 output never goes to HBM.  Workgroup: 64 rows x all 512 columns, 8 waves
// as 2 (rows) x 4 (columns), 32 x 128 per wave (4 accumulators of v_mfma_f32_32x32x16_f16).  K in
// chunks of 32 staged by LDS-DMA (A: 64 rows x 64 B, W: 512 rows x 64 B; two buffers, 72 KiB, so
// two workgroups share a CU and one's elementwise epilogue overlaps the other's GEMM).  64-B LDS
// rows, 16-B pieces XOR-swizzled by (row >> 2) & 3 on the source side: a ds_read_b128 16-lane group
// reads 16 distinct rows at one piece and a 256-B bank row holds 4 rows, so every lane of a group
// gets its own slot.  Then the fp16 y tile goes through LDS and each wave takes whole rows for the
// elementwise epilogue (ln_row).
typedef _Float16 gh8_t __attribute__((ext_vector_type(8)));
typedef float gf16_t __attribute__((ext_vector_type(16)));
constexpr int GL_BM = 64, GL_D = 512;
// MT = 64-row tiles per workgroup sharing each staged W chunk (round 5: MT = 2 halves the W bytes
// per row -- 32 KiB of W per 32-deep chunk were 8 of every 9 bytes the kernel DMA'd at MT = 1)
// S = LDS stages of the K ring (round 5): S - 1 chunks in flight when a chunk is waited for, one
// raw s_barrier per chunk (S = 2: one in flight -- two workgroups per CU at MT = 1; S = 3, 4: one
// workgroup per CU whose DMA latency the ring itself covers)
// BK = K per chunk (round 6): 32 (64-B LDS rows: a DMA instruction fills 16 rows x 64 B, half-line
// fragments), or 64 -- full 128-B lines, 8 rows per DMA instruction, half the barriers; with MT = 2
// and S = 2 that is 2 x (16 + 64) KiB = all 160 KiB of the CU's LDS (one workgroup per CU)
template <int MT, int S = 2, int BK = 32>
struct GL {
    static constexpr int ABYTES = MT * GL_BM * BK * 2, BBYTES = GL_D * BK * 2, BUF = ABYTES + BBYTES;
    static constexpr int LDS = S * BUF;
    static constexpr int ROWB = BK * 2;                       // LDS bytes per staged row
    static constexpr int RPI = 1024 / ROWB;                   // rows one DMA instruction fills (64 lanes x 16 B)
    static_assert(BK == 32 || BK == 64, "chunk depth");
    static_assert(GL_BM * GL_D * 2 <= LDS, "epilogue tile");
    static_assert(LDS <= 163840, "LDS per workgroup");
};

__device__ __attribute__((aligned(16))) uint4 g_lin_zero[1];    // source of the rows past M

// s_waitcnt immediate: vmcnt(n) (6 bits: [3:0] and [15:14]) and lgkmcnt(0), expcnt unconstrained
constexpr int vm_lgkm0(int n) { return (n & 15) | ((n >> 4) << 14) | 0x0070; }

// byte offset of 16-B piece q of staged row r: 64-B rows XOR-keyed by (r >> 2) & 3 (4 rows per 256-B
// bank row), 128-B rows by (r >> 1) & 7 (2 rows per bank row) -- a ds_read_b128 16-lane group reads
// 16 consecutive rows at one logical piece and gets 16 distinct bank slots either way
template <int BK>
__device__ inline int gl_swz(int r, int q) {
    if constexpr (BK == 32) return r * 64 + ((q ^ ((r >> 2) & 3)) << 4);
    else return r * 128 + ((q ^ ((r >> 1) & 7)) << 4);
}
__device__ inline void gl_dma16(const void *src, void *lds) {
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void *)lds, 16, 0, 0);
}
// byte offset of column n (fp16) of row r in the swizzled [64][512] fp16 epilogue tile
__device__ inline int gl_tile(int r, int n) {
    const int byte = n * 2;
    return r * 1024 + (byte >> 7) * 128 + ((((byte >> 4) & 7) ^ (r & 7)) << 4) + (byte & 15);
}

// EPI 1 with tok.VV set: the residual stream's input rows are the tokens (mapf_tokens' token4,
// same mask bits) recomputed here instead of read back from x -- x is only written
struct TokSrc {
    const float *A;
    const uint16_t *VV;
    const float *cls, *pos;
    int L;
    uint32_t thr;
    float scale;
    uint64_t seed;
    int x_every;        // > 1: write back only rows g with g % x_every == 0 (token 0 of each sequence)
};

// DBG (diagnostic builds, -DMAPF_LIN_DEBUG): 1 = the GEMM with a plain fp16 store as the epilogue, 2 = the
// epilogue without the GEMM (acc = 0)
template <int EPI, int MT, int S, int DBG = 0, int BK = 32>
__global__ __launch_bounds__(512) void linear512_kernel(const uint16_t *__restrict__ A, const uint16_t *__restrict__ W,
                                                        const uint16_t *__restrict__ bias, long M,
                                                        uint16_t *__restrict__ out, float *__restrict__ x,
                                                        const float *__restrict__ gamma, const float *__restrict__ beta,
                                                        uint16_t *__restrict__ z, float eps, uint32_t thr, float scale,
                                                        uint64_t seed, TokSrc tok) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int t = (int)threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    using G = GL<MT, S, BK>;
    constexpr int RPI = G::RPI, ROWB = G::ROWB;
    // A rows MT * 64, W rows 512: DMA instructions of RPI rows; instruction g of A / W goes to wave
    // g % 8 (BK = 32: waves 0..4 MT - 1 fill one A instruction each; BK = 64: 8 MT A + 64 W
    // instructions, MT + 8 per wave)
    constexpr int JA = (MT * GL_BM / RPI + 7) / 8, JW = GL_D / RPI / 8;
    constexpr int NA = MT * GL_BM / RPI;                       // A instructions in all
    const long mt0 = (long)blockIdx.x * GL_BM * MT;
    // one DMA instruction fills RPI rows lane-linearly: lane l -> row RPI g + l / (64 / RPI), physical
    // piece l % (64 / RPI); the source is pre-swizzled: the lane fetches the logical piece that lands in
    // its physical slot (gl_swz), which depends on g only through its parity (BK = 64) or not (BK = 32)
    const int lpr = 64 / RPI;                                  // lanes per row: 4 or 8
    auto logical_piece = [&](int g) {
        const int r = RPI * g + lane / lpr, ph = lane % lpr;
        return BK == 32 ? (ph ^ ((r >> 2) & 3)) : (ph ^ ((r >> 1) & 7));
    };
    const int q0 = logical_piece(0), q1 = logical_piece(1);
    const uint16_t *srcA[JA];
#pragma unroll
    for (int j = 0; j < JA; ++j) {
        const int g = wave + 8 * j;
        const long rowA = mt0 + RPI * g + lane / lpr;
        srcA[j] = (g < NA && rowA < M) ? A + rowA * GL_D + ((g & 1) ? q1 : q0) * 8 : nullptr;
    }
    auto issue = [&](int c, int buf) {
        char *As = smem + buf * G::BUF;
        char *Bs = As + G::ABYTES;
#pragma unroll
        for (int j = 0; j < JA; ++j) {
            const int g = wave + 8 * j;
            if (g < NA)
                gl_dma16(srcA[j] ? (const void *)(srcA[j] + c * BK) : (const void *)g_lin_zero, As + RPI * g * ROWB);
        }
#pragma unroll
        for (int j = 0; j < JW; ++j) {                         // BK 32: wave w fills W rows 64w..64w+63
            const int g = JW * wave + j;
            const int n = RPI * g + lane / lpr;
            gl_dma16(W + (size_t)n * GL_D + c * BK + ((g & 1) ? q1 : q0) * 8, Bs + RPI * g * ROWB);
        }
    };
    const int wm = wave & 1, wn = wave >> 1, fr = lane & 31, fh = lane >> 5;
    gf16_t acc[MT][4];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int b = 0; b < 4; ++b)
            for (int r = 0; r < 16; ++r) acc[i][b][r] = 0.f;
    constexpr int NCH = GL_D / BK;
    // ring: chunks 0 .. S-2 in flight; at chunk c wait until only the chunks after it (at most S - 2)
    // are outstanding -- each wave's DMAs per chunk: DA (the waves that fill an A instruction) or DB
    // -- then ONE raw barrier (every wave's copies of chunk c have landed, every wave is done reading
    // chunk c - 1), then refill chunk c - 1's buffer with chunk c + S - 1 and compute chunk c.
    // lgkmcnt(0) before the barrier: chunk c - 1's LDS reads have returned before its buffer is restaged.
    constexpr int DB = JW, DA = JW + JA;                       // (BK = 32, MT = 1: 4 / 5)
    const bool fills_a = wave < NA;                            // (waves with JA A instructions: NA >= 8 fills all)
#pragma unroll
    for (int c = 0; c < S - 1; ++c) if (DBG != 2) issue(c, c);
    for (int c = 0; c < (DBG == 2 ? 0 : NCH); ++c) {
        const int ahead = (NCH - 1 - c) < (S - 2) ? (NCH - 1 - c) : (S - 2);
        if (ahead >= 2) {
            if (fills_a) __builtin_amdgcn_s_waitcnt(vm_lgkm0(2 * DA));
            else __builtin_amdgcn_s_waitcnt(vm_lgkm0(2 * DB));
        } else if (ahead == 1) {
            if (fills_a) __builtin_amdgcn_s_waitcnt(vm_lgkm0(DA));
            else __builtin_amdgcn_s_waitcnt(vm_lgkm0(DB));
        } else {
            __builtin_amdgcn_s_waitcnt(vm_lgkm0(0));
        }
        __builtin_amdgcn_s_barrier();
        if (c + S - 1 < NCH) issue(c + S - 1, (c + S - 1) % S);
        const char *As = smem + (c % S) * G::BUF;
        const char *Bs = As + G::ABYTES;
        // every fragment of a 32-deep half-chunk read first (the waits then retire them progressively
        // under the MFMAs; reading each MFMA's operands just before it left the MFMA pipe waiting on LDS
        // latency); BK = 64 takes two such halves
#pragma unroll
        for (int h = 0; h < BK / 32; ++h) {
            constexpr int KS = 2;
            gh8_t af[KS][MT], bf[KS][4];
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const int qq = 2 * (2 * h + s) + fh;
#pragma unroll
                for (int i = 0; i < MT; ++i)
                    af[s][i] = *reinterpret_cast<const gh8_t *>(As + gl_swz<BK>(64 * i + 32 * wm + fr, qq));
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    bf[s][b] = *reinterpret_cast<const gh8_t *>(Bs + gl_swz<BK>(128 * wn + 32 * b + fr, qq));
            }
#pragma unroll
            for (int s = 0; s < KS; ++s)
#pragma unroll
                for (int b = 0; b < 4; ++b)
#pragma unroll
                    for (int i = 0; i < MT; ++i)
                        acc[i][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[s][i], bf[s][b], acc[i][b], 0, 0, 0);
            // pin that order against the scheduler's register-saving interleave (read, wait, MFMA)
            __builtin_amdgcn_sched_group_barrier(0x100, KS * (MT + 4), 0);
            __builtin_amdgcn_sched_group_barrier(0x008, KS * 4 * MT, 0);
        }
    }
    static_assert(S <= 4 && 2 * DA <= 63, "the waits above count at most two chunks ahead (6-bit vmcnt)");
    __builtin_amdgcn_s_waitcnt(0xC07F);                        // every wave done reading the last chunk
    __builtin_amdgcn_s_barrier();
    // the 64-row tiles one after the other through one LDS tile
#pragma unroll
    for (int i = 0; i < MT; ++i) {
    const long m0 = mt0 + (long)GL_BM * i;
    if (i > 0) __syncthreads();                                 // the previous tile's epilogue is done with it
    // y = fp16(acc + bias) -> LDS tile
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int n = 128 * wn + 32 * b + fr;
        const float bv = h2f(bias[n]);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * fh;
            *reinterpret_cast<uint16_t *>(smem + gl_tile(row, n)) = (uint16_t)f2h(acc[i][b][r] + bv);
        }
    }
    __syncthreads();
    if (DBG == 1) {
        for (int row = wave; row < GL_BM; row += 8) {
            const long g = m0 + row;
            if (g >= M) break;
            uint16_t *dst = EPI == 0 ? out : z;
            reinterpret_cast<uint4 *>(dst)[g * 64 + lane] = *reinterpret_cast<const uint4 *>(smem + gl_tile(row, 8 * lane));
        }
        continue;
    }
    if (EPI == 1) {
        // wave w takes rows w, w + 8, ..., four at a time (ln_rows: their reductions interleaved)
        constexpr int R = 4;
        for (int row0 = wave; row0 < GL_BM; row0 += 8 * R) {
            float4 av[R], cv[R];
            bool live[R];
            uint16_t *zr[R];
            float4 *xr = reinterpret_cast<float4 *>(x);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int row = row0 + 8 * r;
                const long g = m0 + row;
                live[r] = row < GL_BM && g < M;
                zr[r] = z + (live[r] ? g : 0) * 512;
                if (!live[r]) {
                    av[r] = cv[r] = make_float4(0.f, 0.f, 0.f, 0.f);
                    continue;
                }
                const uint2 y0 = *reinterpret_cast<const uint2 *>(smem + gl_tile(row, 4 * lane));
                const uint2 y1 = *reinterpret_cast<const uint2 *>(smem + gl_tile(row, 256 + 4 * lane));
                const long i0 = g * 128 + lane, i1 = i0 + 64;
                const unsigned k0 = thr ? keep4(seed, (uint64_t)i0, thr) : 15u;
                const unsigned k1 = thr ? keep4(seed, (uint64_t)i1, thr) : 15u;
                float4 x0, x1;
                if (tok.VV) {
                    const long tb = g / (tok.L + 1);
                    const int tt = (int)(g - tb * (tok.L + 1));
                    x0 = token4(tok.A, tok.VV, tok.cls, tok.pos, tb, tt, lane, tok.L, 512, i0, tok.thr, tok.scale,
                                tok.seed);
                    x1 = token4(tok.A, tok.VV, tok.cls, tok.pos, tb, tt, 64 + lane, tok.L, 512, i1, tok.thr,
                                tok.scale, tok.seed);
                } else {
                    x0 = xr[i0];
                    x1 = xr[i1];
                }
                av[r] = add_dropped(x0, y0, k0, scale);
                cv[r] = add_dropped(x1, y1, k1, scale);
                if (tok.x_every <= 1 || g % tok.x_every == 0) {
                    xr[i0] = av[r];
                    xr[i1] = cv[r];
                }
            }
            ln_rows<R>(av, cv, live, lane, gamma, beta, eps, zr);
        }
        continue;
    }
    // EPI 0 (GELU + dropout): wave w takes rows w, w + 8, ...; lane holds columns 4l..4l+3 and 256+4l..
    for (int row = wave; row < GL_BM; row += 8) {
        const long g = m0 + row;
        if (g >= M) break;
        const uint2 y0 = *reinterpret_cast<const uint2 *>(smem + gl_tile(row, 4 * lane));
        const uint2 y1 = *reinterpret_cast<const uint2 *>(smem + gl_tile(row, 256 + 4 * lane));
        const long i0 = g * 128 + lane, i1 = i0 + 64;          // float4 indices of the [M, 512] tensor
        const unsigned k0 = thr ? keep4(seed, (uint64_t)i0, thr) : 15u, k1 = thr ? keep4(seed, (uint64_t)i1, thr) : 15u;
        if (EPI == 0) {
            uint2 o[2];
            const uint2 yv[2] = {y0, y1};
            const unsigned kk[2] = {k0, k1};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t in[4] = {yv[h].x, yv[h].x >> 16, yv[h].y, yv[h].y >> 16};
                uint32_t r4[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float a = h2f(in[e]);
                    const float gl = h2f(f2h(0.5f * a * (1.f + erff(a * 0.70710678118654752f))));
                    r4[e] = ((kk[h] >> e) & 1u) ? f2h(gl * scale) : 0u;
                }
                o[h] = pack4(r4[0], r4[1], r4[2], r4[3]);
            }
            reinterpret_cast<uint2 *>(out)[i0] = o[0];
            reinterpret_cast<uint2 *>(out)[i1] = o[1];
        }
    }
    }
}

// MT row tiles per workgroup (mapf_linear512_select): 2 (80 KiB of LDS at S = 2), 1, or 0 (default: 1);
// S ring stages (mapf_linear512_stages): 2, 3, 4 or 0 (default: 2).  Measured at the c3 shape
// (tools/bench_lin_impl.py, profiles/r05_lin_forms.jsonl): 64-row, 2-stage workgroups -- two per CU --
// are the fastest or within 1 % for the GELU, rows and tokens forms; deeper rings cost the second
// workgroup per CU and lose 10-25 %.
static int g_lin_mt = 0, g_lin_stages = 0, g_lin_kdepth = 0;
#ifndef MAPF_LIN_DEBUG
#define MAPF_LIN_DEBUG 0     // diagnostic builds: make variant V=lindbg1 VFLAGS=-DMAPF_LIN_DEBUG=1
#endif
static constexpr int lin_debug() { return MAPF_LIN_DEBUG; }
template <int EPI, int MT, int S, int BK = 32, class... Args>
static void launch_linear512_form(long rows, hipStream_t s, Args... args) {
    constexpr int lds = GL<MT, S, BK>::LDS;
    const dim3 grid((unsigned)((rows + MT * GL_BM - 1) / (MT * GL_BM)));
    if (S == 2 && lin_debug() == 1)
        hipLaunchKernelGGL((linear512_kernel<EPI, MT, S, 1, BK>), grid, dim3(512), lds, s, args...);
    else if (S == 2 && lin_debug() == 2)
        hipLaunchKernelGGL((linear512_kernel<EPI, MT, S, 2, BK>), grid, dim3(512), lds, s, args...);
    else
        hipLaunchKernelGGL((linear512_kernel<EPI, MT, S, 0, BK>), grid, dim3(512), lds, s, args...);
}
template <int EPI, class... Args>
static void launch_linear512(long rows, hipStream_t s, Args... args) {
    const int mt = g_lin_mt ? g_lin_mt : 1;
    const int st = g_lin_stages ? g_lin_stages : 2;
    if (g_lin_kdepth == 64) {           // full-line K chunks: two stages (the LDS holds no more at MT = 2)
        if (mt == 2) launch_linear512_form<EPI, 2, 2, 64>(rows, s, args...);
        else launch_linear512_form<EPI, 1, 2, 64>(rows, s, args...);
        return;
    }
    if (mt == 2) {
        if (st == 4) launch_linear512_form<EPI, 2, 4>(rows, s, args...);
        else if (st == 3) launch_linear512_form<EPI, 2, 3>(rows, s, args...);
        else launch_linear512_form<EPI, 2, 2>(rows, s, args...);
    } else {
        if (st == 4) launch_linear512_form<EPI, 1, 4>(rows, s, args...);
        else if (st == 3) launch_linear512_form<EPI, 1, 3>(rows, s, args...);
        else launch_linear512_form<EPI, 1, 2>(rows, s, args...);
    }
}

// ---- attention backward (the training forward's attention, transformer.py:48-85) ---------
// For SDPA's flash backward the 17-token sequences are all overhead (0.31 ms per layer at 2,048
// agents x 16 heads).  One workgroup per sequence, wave w takes heads w, w + 4, ...; per head,
// with P recomputed in fp32 from q, k (as flash does) and D = rowsum(dO o) from the forward's
// fp16 output:
//   row pass, lane i < rows:    S_i. = scale q_i k^T, P_i. = softmax, dP_ij = dO_i v_j,
//                               dS_ij = P_ij (dP_ij - D_i), dq_i = scale sum_j dS_ij k_j
//   column pass, lane j < n:    dv_j = sum_i P_ij dO_i, dk_j = scale sum_i dS_ij q_i
// K, V, Q, dO staged as fp16 rows in LDS (every lane of a row pass reads the same K / V row:
// broadcasts), P and dS as fp32 [i][j]; fp16 gradients out.  n <= 32, head_dim 32, 16 heads.
constexpr int AB_ROW = 64;                                  // bytes per fp16 head row
// One workgroup of ONE wave per (sequence, head group) (round 5: was one workgroup per sequence, four
// waves looping over four heads each with workgroup barriers between the passes): n <= 20 packs three
// heads side by side in the wave (21 lanes each: 51 of 64 lanes carry a row instead of 17).  NC = row capacity: 20
// (n <= 20, the 17-token layers) or 32.  LDS per wave: Q, dO, K, V rows + P, dS in fp32.
// P / dS element (i, j): NC = 32 at i * 32 + (j ^ i) -- the row pass (lanes = i, one j) and the column
// pass (lanes = j, one i) both hit distinct banks; NC = 20 at i * 21 + j (odd stride: distinct banks
// for both passes too).
template <int NC> struct AB {
    static constexpr int PS = NC == 32 ? 32 : NC + 1;
    static constexpr int LDS = 4 * NC * AB_ROW + 2 * NC * PS * 4;
    static __device__ inline int pij(int i, int j) { return NC == 32 ? i * 32 + (j ^ (i & 31)) : i * PS + j; }
};
static_assert(AB<32>::LDS <= 65536 && AB<20>::LDS <= 65536, "attention_bwd_f16 LDS");
__device__ inline void ab_row_to_f32(const char *src, float *f) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint4 u = reinterpret_cast<const uint4 *>(src)[c];
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            f[8 * c + 2 * e] = h2f(w[e]);
            f[8 * c + 2 * e + 1] = h2f(w[e] >> 16);
        }
    }
}
typedef _Float16 ab_h2_t __attribute__((ext_vector_type(2)));
// a . row over 32 fp16 pairs with v_dot2_f32_f16 (fp16 products exact in fp32, fp32 sums)
__device__ inline float ab_dot(const uint32_t *a, const char *row) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};               // four independent chains (latency, not issue, bound)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint4 u = reinterpret_cast<const uint4 *>(row)[c];
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
            acc[e] = __builtin_amdgcn_fdot2(__builtin_bit_cast(ab_h2_t, a[4 * c + e]), __builtin_bit_cast(ab_h2_t, w[e]),
                                            acc[e], false);
    }
    return (acc[0] + acc[1]) + (acc[2] + acc[3]);
}
__device__ inline void ab_load_h(const char *src, uint32_t *a) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint4 u = reinterpret_cast<const uint4 *>(src)[c];
        a[4 * c] = u.x;
        a[4 * c + 1] = u.y;
        a[4 * c + 2] = u.z;
        a[4 * c + 3] = u.w;
    }
}
__device__ inline void ab_axpy(float *acc, float s, const char *row) {
    float f[32];
    ab_row_to_f32(row, f);
#pragma unroll
    for (int d = 0; d < 32; ++d) acc[d] = fmaf(s, f[d], acc[d]);
}
__device__ inline void ab_store(uint16_t *dst, const float *f, float scale) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
        reinterpret_cast<uint4 *>(dst)[c] =
            make_uint4(f2h(f[8 * c] * scale) | (f2h(f[8 * c + 1] * scale) << 16),
                       f2h(f[8 * c + 2] * scale) | (f2h(f[8 * c + 3] * scale) << 16),
                       f2h(f[8 * c + 4] * scale) | (f2h(f[8 * c + 5] * scale) << 16),
                       f2h(f[8 * c + 6] * scale) | (f2h(f[8 * c + 7] * scale) << 16));
}

template <int NC, int HPW>
__global__ __launch_bounds__(64) void attention_bwd_f16(const uint16_t *__restrict__ q, const uint16_t *__restrict__ k,
                                                         const uint16_t *__restrict__ v, const uint16_t *__restrict__ o,
                                                         const uint16_t *__restrict__ dout, uint16_t *__restrict__ dq,
                                                         uint16_t *__restrict__ dk, uint16_t *__restrict__ dv, int n,
                                                         int rows, long q_ts, long q_ss, long kv_ts, long kv_ss,
                                                         long o_ts, long o_ss, float scale) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    using G = AB<NC>;
    constexpr int GLN = 64 / HPW;                          // lanes per head: HPW heads side by side
    const int lane = (int)threadIdx.x, g = lane / GLN, r = lane - g * GLN;
    const int h = (int)blockIdx.y * HPW + g;
    const bool hv = g < HPW && h < 16;                     // lanes past the last head group idle
    const long b = blockIdx.x;
    char *Qh = smem + (hv ? g : 0) * G::LDS, *dOh = Qh + NC * AB_ROW, *Kh = dOh + NC * AB_ROW, *Vh = Kh + NC * AB_ROW;
    float *P = reinterpret_cast<float *>(Vh + NC * AB_ROW), *dS = P + NC * G::PS;
    {
        if (hv && r < n) {
            const uint4 *ks = reinterpret_cast<const uint4 *>(k + b * kv_ss + r * kv_ts + h * 32);
            const uint4 *vs = reinterpret_cast<const uint4 *>(v + b * kv_ss + r * kv_ts + h * 32);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                reinterpret_cast<uint4 *>(Kh + r * AB_ROW)[c] = ks[c];
                reinterpret_cast<uint4 *>(Vh + r * AB_ROW)[c] = vs[c];
            }
        }
        uint32_t qh[16], gh[16];                           // this row's q and dO, fp16 pairs
        float D = 0.f;
        if (hv && r < rows) {
            ab_load_h(reinterpret_cast<const char *>(q + b * q_ss + r * q_ts + h * 32), qh);
            ab_load_h(reinterpret_cast<const char *>(dout + b * o_ss + r * o_ts + h * 32), gh);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                reinterpret_cast<uint4 *>(Qh + r * AB_ROW)[c] = make_uint4(qh[4 * c], qh[4 * c + 1], qh[4 * c + 2], qh[4 * c + 3]);
                reinterpret_cast<uint4 *>(dOh + r * AB_ROW)[c] = make_uint4(gh[4 * c], gh[4 * c + 1], gh[4 * c + 2], gh[4 * c + 3]);
            }
            D = ab_dot(gh, reinterpret_cast<const char *>(o + b * o_ss + r * o_ts + h * 32));
        }
        __syncthreads();
        if (hv && r < rows) {                              // row pass
            float sv[NC];
            float m = -INFINITY;
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                sv[j] = j < n ? scale * ab_dot(qh, Kh + j * AB_ROW) : -INFINITY;
                m = fmaxf(m, sv[j]);
            }
            float l = 0.f;
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                sv[j] = j < n ? __expf(sv[j] - m) : 0.f;
                l += sv[j];
            }
            const float rl = 1.f / l;
            float gq[32];
#pragma unroll
            for (int d = 0; d < 32; ++d) gq[d] = 0.f;
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                if (j < n) {
                    const float pj = sv[j] * rl;
                    const float ds = pj * (ab_dot(gh, Vh + j * AB_ROW) - D);
                    P[G::pij(r, j)] = pj;
                    dS[G::pij(r, j)] = ds;
                    ab_axpy(gq, ds, Kh + j * AB_ROW);
                }
            }
            ab_store(dq + b * q_ss + r * q_ts + h * 32, gq, scale);
        }
        __syncthreads();
        if (hv && r < n) {                                 // column pass
            float gk[32], gv[32];
#pragma unroll
            for (int d = 0; d < 32; ++d) gk[d] = gv[d] = 0.f;
            for (int i = 0; i < rows; ++i) {
                ab_axpy(gv, P[G::pij(i, r)], dOh + i * AB_ROW);
                ab_axpy(gk, dS[G::pij(i, r)], Qh + i * AB_ROW);
            }
            ab_store(dk + b * kv_ss + r * kv_ts + h * 32, gk, scale);
            ab_store(dv + b * kv_ss + r * kv_ts + h * 32, gv, 1.f);
        }
        __syncthreads();
    }
}

// ---- attention backward on the MFMA (round 6) ------------------------------------------------
// One wave per (sequence, head); the 16 x 16 x 32 f16 MFMA with one contraction step = the head's 32
// dims or 32 (padded) tokens.  Two register layouts of the score matrix, as the forward kernel:
//   T (keys x queries): S^T = K Q^T and dP^T = V dO^T; the softmax over keys per query column (4 lanes
//     l, l^16, l^32, l^48), its max / sum and D_q = rowsum(dO o O) kept in LDS;
//     dS^T = P^T (dP^T - D); dQ^T = K^T dS^T: the accumulators are the B operand as they are (their k
//     order (j >> 2) * 16 + 4 (l >> 4) + (j & 3)), K^T read in that order from an LDS image of K with
//     ds_read_b64_tr_b16 -- attention_f16's O^T = V^T P^T;
//   N (queries x keys): S = Q K^T and dP = dO V^T recomputed, P from the stored max / sum, dS;
//     dV^T = dO^T P and dK^T = Q^T dS, dO^T and Q^T from their LDS images.
// P and dS are rounded to fp16 as MFMA operands (flash SDPA's backward does the same); sums in fp32.
// 28 MFMAs per (sequence, head); the kernel moves K, V, Q, dO, O in and dQ, dK, dV out (HBM-bound).
// QT = query tiles of 16: 2 (rows <= 32) or 1 (rows <= 16: the token-0 query).
constexpr int ABM_WAVES = 4;
constexpr int ABM_LDS_WAVE = 3 * 2048 + 3 * 32 * 4;        // K, Q, dO images + max, sum, D per query
template <int QT>
__global__ __launch_bounds__(256) void attention_bwd_mfma(const uint16_t *__restrict__ q, const uint16_t *__restrict__ k,
                                                          const uint16_t *__restrict__ v, const uint16_t *__restrict__ o,
                                                          const uint16_t *__restrict__ dout, uint16_t *__restrict__ dq,
                                                          uint16_t *__restrict__ dk, uint16_t *__restrict__ dv, int n,
                                                          int rows, long q_ts, long q_ss, long kv_ts, long kv_ss,
                                                          long o_ts, long o_ss, float scale) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[ABM_WAVES][ABM_LDS_WAVE];
    const int lane = (int)(threadIdx.x & 63), w = (int)(threadIdx.x >> 6);
    const int g = lane >> 4, i = lane & 15;
    const int h = (int)blockIdx.y * ABM_WAVES + w;             // head
    const long b = blockIdx.x;
    uint8_t *Kimg = lds[w], *Qimg = Kimg + 2048, *Gimg = Qimg + 2048;
    float *Mq = reinterpret_cast<float *>(Gimg + 2048), *Lq = Mq + 32, *Dq = Lq + 32;
    const uint16_t *qb = q + b * q_ss + h * 32 + 8 * g, *kb = k + b * kv_ss + h * 32 + 8 * g;
    const uint16_t *vb = v + b * kv_ss + h * 32 + 8 * g, *ob = o + b * o_ss + h * 32 + 8 * g;
    const uint16_t *gb = dout + b * o_ss + h * 32 + 8 * g;
    // fragments: lane (i, g) holds token row 16 t + i, dims 8 g .. 8 g + 7 (zeros past n / rows)
    uint4 kf[2], vf[2], qf[QT], gf[QT], of[QT];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        kf[t] = ld16(kb + (16 * t + i) * kv_ts, 16 * t + i < n);
        vf[t] = ld16(vb + (16 * t + i) * kv_ts, 16 * t + i < n);
    }
#pragma unroll
    for (int t = 0; t < QT; ++t) {
        const bool ok = 16 * t + i < rows;
        qf[t] = ld16(qb + (16 * t + i) * q_ts, ok);
        gf[t] = ld16(gb + (16 * t + i) * o_ts, ok);
        of[t] = ld16(ob + (16 * t + i) * o_ts, ok);
    }
    // LDS images (32 token rows x 64 B, vimg_off's swizzle), zero rows where no token is
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        *reinterpret_cast<uint4 *>(Kimg + vimg_off(16 * t + i, g)) = kf[t];
        *reinterpret_cast<uint4 *>(Qimg + vimg_off(16 * t + i, g)) = t < QT ? qf[t < QT ? t : 0] : make_uint4(0u, 0u, 0u, 0u);
        *reinterpret_cast<uint4 *>(Gimg + vimg_off(16 * t + i, g)) = t < QT ? gf[t < QT ? t : 0] : make_uint4(0u, 0u, 0u, 0u);
    }
    // D_q = sum_d dO o O for query 16 qt + i (all four lanes of the column get it)
    float Dv[QT];
#pragma unroll
    for (int t = 0; t < QT; ++t) {
        const h8_t a = as_h8(gf[t]), c = as_h8(of[t]);
        float d = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) d += (float)a[e] * (float)c[e];
        d += __shfl_xor(d, 16, 64);
        d += __shfl_xor(d, 32, 64);
        Dv[t] = d;
    }
    // ---- layout T: rows = keys (16 kt + 4 g + e), columns = queries (16 qt + i)
    const f4_t zero4 = {0.f, 0.f, 0.f, 0.f};
    h8_t dsT[QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        f4_t s[2], dp[2];
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
            s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h8(kf[kt]), as_h8(qf[qt]), zero4, 0, 0, 0);
            dp[kt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h8(vf[kt]), as_h8(gf[qt]), zero4, 0, 0, 0);
        }
        float x[8], m = -INFINITY;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int key = (e >> 2) * 16 + 4 * g + (e & 3);
            x[e] = key < n ? s[e >> 2][e & 3] * scale : -INFINITY;
            m = fmaxf(m, x[e]);
        }
        m = fmaxf(m, __shfl_xor(m, 16, 64));
        m = fmaxf(m, __shfl_xor(m, 32, 64));
        float l = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            x[e] = __expf(x[e] - m);
            l += x[e];
        }
        l += __shfl_xor(l, 16, 64);
        l += __shfl_xor(l, 32, 64);
        const float rl = 1.f / l;
#pragma unroll
        for (int e = 0; e < 8; ++e) dsT[qt][e] = (_Float16)(x[e] * rl * (dp[e >> 2][e & 3] - Dv[qt]));
        if (g == 0) {
            Mq[16 * qt + i] = m;
            Lq[16 * qt + i] = rl;
            Dq[16 * qt + i] = Dv[qt];
        }
    }
    if (QT == 1 && g == 0) {                                   // queries 16..31 do not exist: P = dS = 0 there
        Mq[16 + i] = 0.f;
        Lq[16 + i] = 0.f;
        Dq[16 + i] = 0.f;
    }
    __syncthreads();                                           // the images and the per-query stats are written
    // the transposed A operand X^T (row = dim 16 dt + i, k = token in the accumulators' order) from image X
    auto trX = [&](const uint8_t *img, int dt) {
        const int rq = i >> 2, cp = i & 3;
        const int c = 2 * dt + (cp >> 1), hb = 8 * (cp & 1);
        const s4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t *)(img + vimg_off(4 * g + rq, c) + hb));
        const s4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t *)(img + vimg_off(16 + 4 * g + rq, c) + hb));
        return __builtin_bit_cast(h8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    // dQ^T = scale K^T dS^T: lane -> dims 16 dt + 4 g + e of query 16 qt + i
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
        const h8_t kt_ = trX(Kimg, dt);
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            const f4_t r = __builtin_amdgcn_mfma_f32_16x16x32_f16(kt_, dsT[qt], zero4, 0, 0, 0);
            const int qr = 16 * qt + i;
            if (qr < rows)
                *reinterpret_cast<uint2 *>(dq + b * q_ss + qr * q_ts + h * 32 + 16 * dt + 4 * g) =
                    pack4(f2h(r[0] * scale), f2h(r[1] * scale), f2h(r[2] * scale), f2h(r[3] * scale));
        }
    }
    // ---- layout N: rows = queries (16 qt + 4 g + e), columns = keys (16 kt + i)
    h8_t pN[2], dsN[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
        const int key = 16 * kt + i;
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
            if (qt < QT) {
                const f4_t s = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h8(qf[qt < QT ? qt : 0]), as_h8(kf[kt]), zero4, 0, 0, 0);
                const f4_t dp = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h8(gf[qt < QT ? qt : 0]), as_h8(vf[kt]), zero4, 0, 0, 0);
                const float4 mq = *reinterpret_cast<const float4 *>(Mq + 16 * qt + 4 * g);
                const float4 lq = *reinterpret_cast<const float4 *>(Lq + 16 * qt + 4 * g);
                const float4 dq4 = *reinterpret_cast<const float4 *>(Dq + 16 * qt + 4 * g);
                const float mm[4] = {mq.x, mq.y, mq.z, mq.w}, ll[4] = {lq.x, lq.y, lq.z, lq.w};
                const float dd[4] = {dq4.x, dq4.y, dq4.z, dq4.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float p = key < n ? __expf(s[e] * scale - mm[e]) * ll[e] : 0.f;
                    pN[kt][4 * qt + e] = (_Float16)p;
                    dsN[kt][4 * qt + e] = (_Float16)(p * (dp[e] - dd[e]));
                }
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) pN[kt][4 * qt + e] = dsN[kt][4 * qt + e] = (_Float16)0.f;
            }
        }
    }
    // dV^T = dO^T P, dK^T = scale Q^T dS: lane -> dims 16 dt + 4 g + e of key 16 kt + i
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
        const h8_t gt = trX(Gimg, dt), qt_ = trX(Qimg, dt);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
            const int key = 16 * kt + i;
            const f4_t rv = __builtin_amdgcn_mfma_f32_16x16x32_f16(gt, pN[kt], zero4, 0, 0, 0);
            const f4_t rk = __builtin_amdgcn_mfma_f32_16x16x32_f16(qt_, dsN[kt], zero4, 0, 0, 0);
            if (key < n) {
                *reinterpret_cast<uint2 *>(dv + b * kv_ss + key * kv_ts + h * 32 + 16 * dt + 4 * g) =
                    pack4(f2h(rv[0]), f2h(rv[1]), f2h(rv[2]), f2h(rv[3]));
                *reinterpret_cast<uint2 *>(dk + b * kv_ss + key * kv_ts + h * 32 + 16 * dt + 4 * g) =
                    pack4(f2h(rk[0] * scale), f2h(rk[1] * scale), f2h(rk[2] * scale), f2h(rk[3] * scale));
            }
        }
    }
}

// 1 (default): attention_bwd_mfma; 0: the VALU kernel above (attention_bwd_f16)
static int g_attn_bwd_form = 1;

}  // namespace pol
}  // namespace mapf

using namespace mapf;

extern "C" {

int mapf_nhwc_bias_relu(uint16_t *x, const uint16_t *bias, int64_t rows, int32_t C, void *stream) {
    if (!x || !bias || rows < 0 || C <= 0 || (C & 3) || C > 1024) return MAPF_EINVAL;
    if (rows == 0) return MAPF_OK;
    const int per = 256 / (C / 4);
    hipLaunchKernelGGL(pol::nhwc_bias_relu, dim3(pol::grid_for(rows, per)), dim3(256), 0, (hipStream_t)stream, x, bias,
                       (long)rows, (int)C);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_nhwc_bias_relu_pool2(const uint16_t *x, const uint16_t *bias, uint16_t *out, int32_t B, int32_t H, int32_t W,
                              int32_t C, void *stream) {
    if (!x || !bias || !out || B < 0 || H < 2 || W < 2 || C <= 0 || (C & 3) || C > 1024) return MAPF_EINVAL;
    if (B == 0) return MAPF_OK;
    const int per = 256 / (C / 4);
    const long rows = (long)B * (H / 2) * (W / 2);
    hipLaunchKernelGGL(pol::nhwc_bias_relu_pool2, dim3(pol::grid_for(rows, per)), dim3(256), 0, (hipStream_t)stream, x,
                       bias, out, (int)B, (int)H, (int)W, (int)C);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_layernorm_f16(const float *x, int64_t x_row_stride, const float *gamma, const float *beta, uint16_t *y,
                       int64_t rows, int32_t dim, float eps, void *stream) {
    if (!x || !gamma || !beta || !y || rows < 0 || dim != 512 || (x_row_stride & 3)) return MAPF_EINVAL;
    if (rows == 0) return MAPF_OK;
    hipLaunchKernelGGL(pol::layernorm_f16, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, x,
                       (long)x_row_stride, gamma, beta, y, (long)rows, eps);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_cast_f32_to_f16_multi(const float *const *src, uint16_t *const *dst, const int64_t *n, int32_t count,
                               void *stream) {
    return pol::cast_multi_api<true>(reinterpret_cast<const void *const *>(src), reinterpret_cast<void *const *>(dst),
                                     n, count, stream);
}

int mapf_cast_f32_to_f16_multi_flip(const float *const *src, uint16_t *const *dst, const int64_t *n,
                                    const int32_t *cout, const int32_t *ks, int32_t count, void *stream) {
    if (!cout || !ks) return MAPF_EINVAL;
    return pol::cast_multi_api<true>(reinterpret_cast<const void *const *>(src), reinterpret_cast<void *const *>(dst),
                                     n, count, stream, cout, ks);
}

int mapf_optim_unscale_clip_adam(float *const *p, float *const *g, float *const *m, float *const *v,
                                 const int64_t *n, float *const *steps, int32_t count, const float *scale,
                                 float max_norm, float lr, float beta1, float beta2, float eps, float *found_inf,
                                 float *grad_norm, float *work, int64_t work_floats, void *stream) {
    if (!p || !g || !m || !v || !n || !steps || !scale || !found_inf || !work || count <= 0) return MAPF_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    // the chunks of <= OPT_MAX tensors and their blocks (partials for every chunk in one array)
    std::vector<pol::OptList> chunks;
    long G = 0;
    for (int c0 = 0; c0 < count; c0 += pol::OPT_MAX) {
        pol::OptList L{};
        L.count = count - c0 < pol::OPT_MAX ? count - c0 : pol::OPT_MAX;
        long blocks = 0;
        for (int k = 0; k < L.count; ++k) {
            const int i = c0 + k;
            if (n[i] <= 0 || !p[i] || !g[i] || !m[i] || !v[i] || !steps[i]) return MAPF_EINVAL;
            L.p[k] = p[i];
            L.g[k] = g[i];
            L.m[k] = m[i];
            L.v[k] = v[i];
            L.n[k] = (long)n[i];
            L.blk0[k] = (int)blocks;
            blocks += (n[i] + pol::OPT_PER_BLOCK - 1) / pol::OPT_PER_BLOCK;
        }
        L.blk0[L.count] = (int)blocks;
        G += blocks;
        chunks.push_back(L);
    }
    if (G > work_floats || G > (1L << 24)) return MAPF_EINVAL;
    long off = 0;
    for (const auto &L : chunks) {
        hipLaunchKernelGGL(pol::optim_sumsq, dim3((unsigned)L.blk0[L.count]), dim3(256), 0, s, L, scale, work, (int)off,
                           found_inf);
        off += L.blk0[L.count];
    }
    for (size_t k = 0; k < chunks.size(); ++k)
        hipLaunchKernelGGL(pol::optim_adam, dim3((unsigned)chunks[k].blk0[chunks[k].count]), dim3(256), 0, s,
                           chunks[k], work, (int)G, scale, found_inf, steps[0], max_norm, lr, beta1, beta2, eps,
                           k == 0 ? grad_norm : nullptr);
    for (int c0 = 0; c0 < count; c0 += pol::OPT_MAX) {
        pol::OptSteps S{};
        S.count = count - c0 < pol::OPT_MAX ? count - c0 : pol::OPT_MAX;
        for (int k = 0; k < S.count; ++k) S.s[k] = steps[c0 + k];
        hipLaunchKernelGGL(pol::optim_steps, dim3(1), dim3(64), 0, s, S, found_inf);
    }
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_cast_f16_to_f32_multi(const uint16_t *const *src, float *const *dst, const int64_t *n, int32_t count,
                               void *stream) {
    return pol::cast_multi_api<false>(reinterpret_cast<const void *const *>(src), reinterpret_cast<void *const *>(dst), n,
                                 count, stream);
}

int mapf_colsum_f16(const uint16_t *g, uint16_t *out, float *work, int64_t rows, int32_t C, void *stream) {
    if ((!g && rows > 0) || !out || !work || rows < 0 || C <= 0 || (C & 3) || C > 4096 || ((uintptr_t)g & 7))
        return MAPF_EINVAL;
    if (rows <= pol::COLSUM_SHORT_ROWS && !(C & 7) && !((uintptr_t)g & 15)) {
        hipLaunchKernelGGL(pol::colsum_short_f16, dim3((unsigned)((C + 31) / 32)), dim3(256), 0, (hipStream_t)stream, g,
                           (long)rows, (int)C, out);
        return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
    }
    const int per = 256 / ((C < 1024 ? C : 1024) / 4);
    const long need = (rows + per - 1) / per;
    const int G = (int)(need < pol::RB_WG ? need : pol::RB_WG);
    if (G > 0)
        hipLaunchKernelGGL(pol::colsum_partial_f16, dim3((unsigned)G, (unsigned)((C + 1023) / 1024)), dim3(256), 0,
                           (hipStream_t)stream, g, work, (long)rows, (int)C);
    hipLaunchKernelGGL(pol::colsum_to_f16, dim3((unsigned)((C + 7) / 8)), dim3(256), 0, (hipStream_t)stream, work, G,
                       (int)C, out);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_relu_bias_pool_bwd_f16(const uint16_t *r, const uint16_t *bias, const uint16_t *dp, uint16_t *dr,
                                uint16_t *dbias, float *work, int32_t B, int32_t H, int32_t W, int32_t C,
                                void *stream) {
    if (!r || !bias || !dp || !dr || !dbias || !work || B < 0 || H < 2 || W < 2 || C <= 0 || (C & 3) || C > 1024 ||
        (((uintptr_t)r | (uintptr_t)dp | (uintptr_t)dr | (uintptr_t)bias) & 7))
        return MAPF_EINVAL;
    const int per = 256 / (C / 4);
    const long units = (long)B * (H / 2) * (W / 2) + (long)B * (H * W - 4 * (H / 2) * (W / 2));
    const long need = (units + per - 1) / per;
    const int G = (int)(need < pol::RB_WG ? need : pol::RB_WG);
    if (G > 0)
        hipLaunchKernelGGL(pol::relu_bias_pool_bwd, dim3((unsigned)G), dim3(256), 0, (hipStream_t)stream, r, bias, dp,
                           dr, work, (int)B, (int)H, (int)W, (int)C);
    hipLaunchKernelGGL(pol::colsum_to_f16, dim3((unsigned)((C + 7) / 8)), dim3(256), 0, (hipStream_t)stream, work, G,
                       (int)C, dbias);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_relu_bias_bwd_f16(const uint16_t *y, const uint16_t *dy, uint16_t *dx, uint16_t *dbias, float *work,
                           int64_t rows, int32_t C, void *stream) {
    if (!y || !dy || !dx || !dbias || !work || rows < 0 || C <= 0 || (C & 3) || C > 1024 ||
        (((uintptr_t)y | (uintptr_t)dy | (uintptr_t)dx) & 7))
        return MAPF_EINVAL;
    const int per = 256 / (C / 4);
    const long need = (rows + per - 1) / per;
    const int G = (int)(need < pol::RB_WG ? need : pol::RB_WG);
    if (G > 0)
        hipLaunchKernelGGL(pol::relu_bias_bwd, dim3((unsigned)G), dim3(256), 0, (hipStream_t)stream, y, dy, dx, work,
                           (long)rows, (int)C);
    hipLaunchKernelGGL(pol::colsum_to_f16, dim3((unsigned)((C + 7) / 8)), dim3(256), 0, (hipStream_t)stream, work, G,
                       (int)C, dbias);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_layernorm_bwd_f16(const float *x, int64_t x_row_stride, const float *gamma, const uint16_t *dz,
                           const float *dres, float *dx, float *dgamma, float *dbeta, float *work, int64_t rows,
                           int32_t dim, float eps, void *stream) {
    if (!x || !gamma || !dz || !dx || !dgamma || !dbeta || !work || rows < 0 || dim != 512 || (x_row_stride & 3) ||
        (((uintptr_t)x | (uintptr_t)gamma | (uintptr_t)dx | (uintptr_t)dres) & 15) || ((uintptr_t)dz & 7))
        return MAPF_EINVAL;
    const int G = (int)(rows < 4 * pol::LNB_WG ? (rows + 3) / 4 : pol::LNB_WG);
    if (G > 0)
        hipLaunchKernelGGL(pol::layernorm_bwd_f16, dim3((unsigned)G), dim3(256), 0, (hipStream_t)stream, x,
                           (long)x_row_stride, gamma, dz, dres, dx, work, (long)rows, eps, nullptr, 0u, 1.f, nullptr, 0u);
    hipLaunchKernelGGL(pol::ln_bwd_colsum, dim3(128), dim3(256), 0, (hipStream_t)stream, work, G, dgamma, dbeta);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_layernorm_dropout_bwd_f16(const float *x, const float *gamma, const uint16_t *dz, const float *dres, float *dx,
                                   uint16_t *dy, float *dgamma, float *dbeta, float *work, int64_t rows, int32_t dim,
                                   float eps, float p, const uint64_t *seed_dev, uint32_t salt, void *stream) {
    if (!x || !gamma || !dz || !dx || !dy || !dgamma || !dbeta || !work || !seed_dev || rows < 0 || dim != 512 ||
        !(p >= 0.f && p < 1.f) ||
        (((uintptr_t)x | (uintptr_t)gamma | (uintptr_t)dx | (uintptr_t)dres) & 15) || (((uintptr_t)dz | (uintptr_t)dy) & 7))
        return MAPF_EINVAL;
    const int G = (int)(rows < 4 * pol::LNB_WG ? (rows + 3) / 4 : pol::LNB_WG);
    if (G > 0)
        hipLaunchKernelGGL(pol::layernorm_bwd_f16, dim3((unsigned)G), dim3(256), 0, (hipStream_t)stream, x, (long)512,
                           gamma, dz, dres, dx, work, (long)rows, eps, dy, pol::drop_threshold(p), 1.f / (1.f - p),
                           seed_dev, salt);
    hipLaunchKernelGGL(pol::ln_bwd_colsum, dim3(128), dim3(256), 0, (hipStream_t)stream, work, G, dgamma, dbeta);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_dropout_residual_layernorm_train(const float *res, int64_t res_row_stride, const uint16_t *y, float *x_out,
                                          const float *gamma, const float *beta, uint16_t *z, int64_t rows, int32_t dim,
                                          float eps, float p, const uint64_t *seed_dev, uint32_t salt, void *stream) {
    if (!res || !y || !x_out || !gamma || !beta || !z || !seed_dev || rows < 0 || dim != 512 || (res_row_stride & 3) ||
        !(p >= 0.f && p < 1.f) ||
        (((uintptr_t)res | (uintptr_t)x_out | (uintptr_t)gamma | (uintptr_t)beta) & 15) || (((uintptr_t)y | (uintptr_t)z) & 7))
        return MAPF_EINVAL;
    if (rows == 0) return MAPF_OK;
    hipLaunchKernelGGL(pol::drln_fwd, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, res,
                       (long)res_row_stride, y, x_out, gamma, beta, z, (long)rows, pol::drop_threshold(p),
                       1.f / (1.f - p), eps, seed_dev, salt);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_gelu_dropout_train_f16(const uint16_t *h, uint16_t *out, int64_t n, float p, const uint64_t *seed_dev,
                                uint32_t salt, void *stream) {
    if (!h || !out || !seed_dev || n < 0 || (n & 3) || !(p >= 0.f && p < 1.f) || (((uintptr_t)h | (uintptr_t)out) & 7))
        return MAPF_EINVAL;
    if (n == 0) return MAPF_OK;
    hipLaunchKernelGGL(pol::gelu_dropout_train, dim3(pol::grid_for(n / 4, 256)), dim3(256), 0, (hipStream_t)stream, h, out,
                       (long)(n / 4), pol::drop_threshold(p), 1.f / (1.f - p), seed_dev, salt);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_gelu_dropout_bwd_f16(const uint16_t *h, const uint16_t *dout, uint16_t *dh, int64_t n, float p,
                              const uint64_t *seed_dev, uint32_t salt, void *stream) {
    if (!h || !dout || !dh || !seed_dev || n < 0 || (n & 3) || !(p >= 0.f && p < 1.f) ||
        (((uintptr_t)h | (uintptr_t)dout | (uintptr_t)dh) & 7))
        return MAPF_EINVAL;
    if (n == 0) return MAPF_OK;
    hipLaunchKernelGGL(pol::gelu_dropout_bwd, dim3(pol::grid_for(n / 4, 256)), dim3(256), 0, (hipStream_t)stream, h, dout,
                       dh, (long)(n / 4), pol::drop_threshold(p), 1.f / (1.f - p), seed_dev, salt);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_dropout_residual(float *x, const uint16_t *y, int64_t n, float p, uint64_t seed, void *stream) {
    if (!x || !y || n < 0 || (n & 3) || !(p >= 0.f && p < 1.f)) return MAPF_EINVAL;
    if (n == 0) return MAPF_OK;
    hipLaunchKernelGGL(pol::dropout_residual, dim3(pol::grid_for(n / 4, 256)), dim3(256), 0, (hipStream_t)stream, x, y,
                       (long)(n / 4), pol::drop_threshold(p), 1.f / (1.f - p), seed);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_dropout_residual_layernorm(float *x, const uint16_t *y, const float *gamma, const float *beta, uint16_t *z,
                                    int64_t rows, int32_t dim, float eps, float p, uint64_t seed, void *stream) {
    if (!x || !y || !gamma || !beta || !z || rows < 0 || dim != 512 || !(p >= 0.f && p < 1.f)) return MAPF_EINVAL;
    if (rows == 0) return MAPF_OK;
    hipLaunchKernelGGL(pol::dropout_residual_layernorm, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, x, y, gamma, beta, z, (long)rows, pol::drop_threshold(p), 1.f / (1.f - p),
                       eps, seed);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_gelu_dropout_f16(uint16_t *h, int64_t n, float p, uint64_t seed, void *stream) {
    if (!h || n < 0 || (n & 3) || !(p >= 0.f && p < 1.f)) return MAPF_EINVAL;
    if (n == 0) return MAPF_OK;
    hipLaunchKernelGGL(pol::gelu_dropout_f16, dim3(pol::grid_for(n / 4, 256)), dim3(256), 0, (hipStream_t)stream, h,
                       (long)(n / 4), pol::drop_threshold(p), 1.f / (1.f - p), seed);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_linear512_select(int32_t row_tiles) {
    if (row_tiles < 0 || row_tiles > 2) return MAPF_EINVAL;
    pol::g_lin_mt = row_tiles;
    return MAPF_OK;
}

int mapf_linear512_stages(int32_t stages) {
    if (stages != 0 && (stages < 2 || stages > 4)) return MAPF_EINVAL;
    pol::g_lin_stages = stages;
    return MAPF_OK;
}

int mapf_linear512_kdepth(int32_t k) {
    if (k != 0 && k != 32 && k != 64) return MAPF_EINVAL;
    pol::g_lin_kdepth = k;
    return MAPF_OK;
}

int mapf_linear512_gelu_dropout(const uint16_t *a, const uint16_t *w, const uint16_t *bias, uint16_t *out, int64_t rows,
                                float p, uint64_t seed, void *stream) {
    if (!a || !w || !bias || !out || rows < 0 || !(p >= 0.f && p < 1.f)) return MAPF_EINVAL;
    if (rows == 0) return MAPF_OK;
    pol::launch_linear512<0>((long)rows, (hipStream_t)stream, a, w, bias, (long)rows, out, nullptr, nullptr, nullptr,
                       nullptr, 0.f, pol::drop_threshold(p), 1.f / (1.f - p), seed, pol::TokSrc{});
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_linear512_residual_layernorm(const uint16_t *a, const uint16_t *w, const uint16_t *bias, float *x,
                                      const float *gamma, const float *beta, uint16_t *z, int64_t rows, float eps,
                                      float p, uint64_t seed, void *stream) {
    if (!a || !w || !bias || !x || !gamma || !beta || !z || rows < 0 || !(p >= 0.f && p < 1.f)) return MAPF_EINVAL;
    if (rows == 0) return MAPF_OK;
    pol::launch_linear512<1>((long)rows, (hipStream_t)stream, a, w, bias, (long)rows, nullptr, x, gamma, beta, z, eps,
                       pol::drop_threshold(p), 1.f / (1.f - p), seed, pol::TokSrc{});
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_linear512_residual_layernorm_rows(const uint16_t *a, const uint16_t *w, const uint16_t *bias, float *x,
                                           const float *gamma, const float *beta, uint16_t *z, int64_t rows, float eps,
                                           float p, uint64_t seed, int32_t x_every, void *stream) {
    if (!a || !w || !bias || !x || !gamma || !beta || !z || rows < 0 || x_every < 1 || !(p >= 0.f && p < 1.f))
        return MAPF_EINVAL;
    if (rows == 0) return MAPF_OK;
    pol::TokSrc tok{};
    tok.x_every = x_every;
    pol::launch_linear512<1>((long)rows, (hipStream_t)stream, a, w, bias, (long)rows, nullptr, x, gamma, beta, z, eps,
                       pol::drop_threshold(p), 1.f / (1.f - p), seed, tok);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_linear512_tokens_residual_layernorm(const uint16_t *a, const uint16_t *w, const uint16_t *bias, float *x,
                                             const float *gamma, const float *beta, uint16_t *z, int64_t B, int32_t L,
                                             float eps, float p, uint64_t seed, const float *tok_A,
                                             const uint16_t *tok_VV, const float *tok_cls, const float *tok_pos,
                                             float tok_p, uint64_t tok_seed, void *stream) {
    if (!a || !w || !bias || !x || !gamma || !beta || !z || !tok_A || !tok_VV || !tok_cls || !tok_pos || B < 0 ||
        L < 1 || !(p >= 0.f && p < 1.f) || !(tok_p >= 0.f && tok_p < 1.f))
        return MAPF_EINVAL;
    if (B == 0) return MAPF_OK;
    const long rows = (long)B * (L + 1);
    const pol::TokSrc tok{tok_A, tok_VV, tok_cls, tok_pos, (int)L, pol::drop_threshold(tok_p), 1.f / (1.f - tok_p),
                          tok_seed, 1};
    pol::launch_linear512<1>((long)rows, (hipStream_t)stream, a, w, bias, rows, nullptr, x, gamma, beta, z, eps,
                       pol::drop_threshold(p), 1.f / (1.f - p), seed, tok);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_tokens(float *x, const float *A, const uint16_t *VV, const float *cls, const float *pos, int64_t B, int32_t L,
                int32_t D, float p, uint64_t seed, void *stream) {
    if (!x || !A || !VV || !cls || !pos || B < 0 || L < 1 || D <= 0 || (D & 3) || !(p >= 0.f && p < 1.f))
        return MAPF_EINVAL;
    if (B == 0) return MAPF_OK;
    const long n4 = (long)B * (L + 1) * (D / 4);
    hipLaunchKernelGGL(pol::tokens, dim3(pol::grid_for(n4, 256)), dim3(256), 0, (hipStream_t)stream, x, A, VV, cls,
                       pos, (long)B, (int)L, (int)D, pol::drop_threshold(p), 1.f / (1.f - p), seed);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_tokens_layernorm(float *x, const float *A, const uint16_t *VV, const float *cls, const float *pos, int64_t B,
                          int32_t L, int32_t D, float p, uint64_t seed, const float *gamma, const float *beta,
                          float eps, uint16_t *z, void *stream) {
    if (!A || !VV || !cls || !pos || !gamma || !beta || !z || B < 0 || L < 1 || D != 512 || !(p >= 0.f && p < 1.f))
        return MAPF_EINVAL;
    if (B == 0) return MAPF_OK;
    const long rows = (long)B * (L + 1);
    hipLaunchKernelGGL(pol::tokens_layernorm, dim3((unsigned)((rows + 15) / 16)), dim3(256), 0, (hipStream_t)stream, x, A,
                       VV, cls, pos, (long)B, (int)L, pol::drop_threshold(p), 1.f / (1.f - p), seed, gamma, beta, eps,
                       z);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_tokens_layernorm_train(float *x, const float *A, const uint16_t *VV, const float *cls, const float *pos,
                                int64_t B, int32_t L, float p, const uint64_t *seed_dev, uint32_t salt, const float *gamma,
                                const float *beta, float eps, uint16_t *z, void *stream) {
    if (!x || !A || !VV || !cls || !pos || !seed_dev || !gamma || !beta || !z || B < 0 || L != pol::TOK_L ||
        !(p >= 0.f && p < 1.f) ||
        (((uintptr_t)x | (uintptr_t)cls | (uintptr_t)pos | (uintptr_t)gamma | (uintptr_t)beta) & 15) ||
        (((uintptr_t)VV | (uintptr_t)z) & 7))
        return MAPF_EINVAL;
    if (B == 0) return MAPF_OK;
    const long rows = (long)B * pol::TOK_T;
    hipLaunchKernelGGL(pol::tokens_ln_train, dim3((unsigned)((rows + 15) / 16)), dim3(256), 0, (hipStream_t)stream, x,
                       A, VV, cls, pos, (long)B, pol::drop_threshold(p), 1.f / (1.f - p), seed_dev, salt, gamma, beta,
                       eps, z);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_tokens_train_bwd(const float *dx, const float *A, const uint16_t *VV, float *dA, uint16_t *dVV, float *dpos,
                          float *dcls, float *work, int64_t B, int32_t L, float p, const uint64_t *seed_dev,
                          uint32_t salt, void *stream) {
    if (!dx || !A || !VV || !dA || !dVV || !dpos || !dcls || !work || !seed_dev || B < 0 || L != pol::TOK_L ||
        !(p >= 0.f && p < 1.f) || (((uintptr_t)dx | (uintptr_t)work) & 7) || (((uintptr_t)VV | (uintptr_t)dVV) & 3))
        return MAPF_EINVAL;
    constexpr int C = pol::TOK_T * 512;
    const long per = B > 0 ? (B + pol::TOK_BWD_WG - 1) / pol::TOK_BWD_WG : 1;   // <= TOK_BWD_WG blocks
    const int G = (int)((B + per - 1) / per);
    if (G > 0)
        hipLaunchKernelGGL(pol::tokens_train_bwd, dim3((unsigned)G), dim3(256), 0, (hipStream_t)stream, dx, A, VV,
                           (long)B, (int)per, pol::drop_threshold(p), 1.f / (1.f - p), seed_dev, salt, dA, dVV, work);
    hipLaunchKernelGGL(pol::tokens_bwd_colsum, dim3((unsigned)(C / 32)), dim3(256), 0, (hipStream_t)stream, work, G, C,
                       dpos, dcls);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_attention_f16(const uint16_t *q, const uint16_t *k, const uint16_t *v, uint16_t *out, int64_t B, int32_t n,
                       int32_t q_rows, int64_t q_token_stride, int64_t q_seq_stride, int64_t kv_token_stride,
                       int64_t kv_seq_stride, int32_t heads, int32_t head_dim, float scale, void *stream) {
    // 16-B operand loads: 8-element aligned strides and 16-B aligned bases
    if (!q || !k || !v || !out || B < 0 || n < 1 || n > 32 || q_rows < 1 || q_rows > n || heads != 16 ||
        head_dim != 32 || ((q_token_stride | q_seq_stride | kv_token_stride | kv_seq_stride) & 7) ||
        (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v) & 15) || ((uintptr_t)out & 7))
        return MAPF_EINVAL;
    if (B == 0) return MAPF_OK;
    const float sl2e = scale * 1.4426950408889634f;
    if (q_rows <= 16)
        hipLaunchKernelGGL(pol::attention_f16<1>, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, q, k, v, out,
                           (int)n, (int)q_rows, (long)q_token_stride, (long)q_seq_stride, (long)kv_token_stride,
                           (long)kv_seq_stride, sl2e);
    else
        hipLaunchKernelGGL(pol::attention_f16<2>, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, q, k, v, out,
                           (int)n, (int)q_rows, (long)q_token_stride, (long)q_seq_stride, (long)kv_token_stride,
                           (long)kv_seq_stride, sl2e);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_attention_bwd_f16(const uint16_t *q, const uint16_t *k, const uint16_t *v, const uint16_t *out,
                           const uint16_t *dout, uint16_t *dq, uint16_t *dk, uint16_t *dv, int64_t B, int32_t n,
                           int32_t q_rows, int64_t q_token_stride, int64_t q_seq_stride, int64_t kv_token_stride,
                           int64_t kv_seq_stride, int64_t out_token_stride, int64_t out_seq_stride, int32_t heads,
                           int32_t head_dim, float scale, void *stream) {
    if (!q || !k || !v || !out || !dout || !dq || !dk || !dv || B < 0 || n < 1 || n > 32 || q_rows < 1 ||
        q_rows > n || heads != 16 || head_dim != 32 ||
        ((q_token_stride | q_seq_stride | kv_token_stride | kv_seq_stride | out_token_stride | out_seq_stride) & 7) ||
        (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)out | (uintptr_t)dout | (uintptr_t)dq |
          (uintptr_t)dk | (uintptr_t)dv) & 15))
        return MAPF_EINVAL;
    if (B == 0) return MAPF_OK;
    if (pol::g_attn_bwd_form == 1) {   // one wave per (sequence, head), four heads per workgroup
        if (q_rows <= 16)
            hipLaunchKernelGGL((pol::attention_bwd_mfma<1>), dim3((unsigned)B, 4), dim3(256), 0, (hipStream_t)stream, q, k,
                               v, out, dout, dq, dk, dv, (int)n, (int)q_rows, (long)q_token_stride, (long)q_seq_stride,
                               (long)kv_token_stride, (long)kv_seq_stride, (long)out_token_stride, (long)out_seq_stride,
                               scale);
        else
            hipLaunchKernelGGL((pol::attention_bwd_mfma<2>), dim3((unsigned)B, 4), dim3(256), 0, (hipStream_t)stream, q, k,
                               v, out, dout, dq, dk, dv, (int)n, (int)q_rows, (long)q_token_stride, (long)q_seq_stride,
                               (long)kv_token_stride, (long)kv_seq_stride, (long)out_token_stride, (long)out_seq_stride,
                               scale);
        return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
    }
    if (n <= 20)        // three heads per wave (21 lanes each), six workgroups per sequence
        hipLaunchKernelGGL((pol::attention_bwd_f16<20, 3>), dim3((unsigned)B, 6), dim3(64), 3 * pol::AB<20>::LDS,
                           (hipStream_t)stream, q, k, v, out, dout, dq, dk, dv, (int)n, (int)q_rows, (long)q_token_stride,
                           (long)q_seq_stride, (long)kv_token_stride, (long)kv_seq_stride, (long)out_token_stride,
                           (long)out_seq_stride, scale);
    else
        hipLaunchKernelGGL((pol::attention_bwd_f16<32, 1>), dim3((unsigned)B, 16), dim3(64), pol::AB<32>::LDS,
                           (hipStream_t)stream, q, k, v, out, dout, dq, dk, dv, (int)n, (int)q_rows, (long)q_token_stride,
                           (long)q_seq_stride, (long)kv_token_stride, (long)kv_seq_stride, (long)out_token_stride,
                           (long)out_seq_stride, scale);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_attention_bwd_select(int32_t form) {
    if (form < 0 || form > 1) return MAPF_EINVAL;
    pol::g_attn_bwd_form = form;
    return MAPF_OK;
}

}  // extern "C"
