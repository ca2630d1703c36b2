// primal-ppo_amd/csrc/mapf_conv.hip -- SCRIMPNet's 3x3 convolutions on the 9x9 FOV
// (conv1a, conv1b: 128 -> 128 channels, padding 1; net.py:101-122) as an MFMA
// implicit GEMM with the bias + ReLU (+ 2x2 max-pool) epilogue fused.
//
//   out[p][co] = relu(round16(round16(sum_{tap, ci} in[p + tap][ci] * W[tap][co][ci]) + b[co]))
//
// -- the rounding points of the autocast path it replaces (fp16 conv output, fp16 bias
// add, ReLU; MIOpen accumulates in fp32 as this kernel does).
//
// One workgroup = 3 images (243 output pixels = M, padded to 16 MFMA tiles of 16),
// all 128 output channels (N = 8 tiles), K = 9 taps x 128 channels, 4 waves x 4 M-tiles.
//  * the 3 input images sit in LDS with a zero halo, [img][11][11][128] fp16 (93 KB);
//    16-B chunk c of padded pixel Q is stored at chunk c ^ (Q & 15), so the 16 lanes
//    of an A-fragment read (16 consecutive pixels, one chunk) hit 16 different banks;
//  * the weights stream one tap at a time ([co][ci] fp16, 32 KB, chunk c of row co at
//    c ^ (co & 15)); the next tap's weights are loaded into registers while the MFMAs
//    of the current one run (register staging);
//  * v_mfma_f32_16x16x32_f16: A = 16 pixels x 32 channels of one tap, B = 32 channels x
//    16 output channels; 32 fp32 accumulators of 4 per lane (4 M x 8 N tiles);
//  * epilogue through LDS: bias + ReLU as fp16 into a [m][co] image, then coalesced
//    16-B stores -- or the 2x2 max-pool (floor, nn.MaxPool2d(2)) of that image.
// Status: correct (GPU tests) but 1.54 ms for 32,768 images vs 1.10 ms for MIOpen's CK
// kernel + 0.17 ms for its epilogue pass, so SCRIMPNet.own_conv is off by default.  With
// the MFMAs replaced by one VALU op the launch still takes 1.25 ms (tools/conv_exp.py,
// tools/conv_variants.sh): at one 158 KB workgroup per CU the staging, the per-tap
// barriers and the epilogue never overlap the MFMAs.  Next: two workgroups per CU or a
// persistent, pipelined version.
#include <hip/hip_fp16.h>

#include "mapf.h"
#include "mapf_common.h"

namespace mapf {
namespace conv {

typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
typedef float f4_t __attribute__((ext_vector_type(4)));

constexpr int C = 128, H = 9, HP = 11, IMG = 3, M = IMG * H * H, MT = 16;
constexpr int IN_BYTES = IMG * HP * HP * C * 2;        // 92,928
constexpr int W_BYTES = C * C * 2;                     // 32,768

__device__ inline float h2f(uint32_t h) { return __half2float(__ushort_as_half((unsigned short)(h & 0xFFFFu))); }
__device__ inline uint32_t f2h(float f) { return (uint32_t)__half_as_ushort(__float2half_rn(f)); }
__device__ inline int in_off(int Q, int c) { return (Q * 16 + (c ^ (Q & 15))) * 16; }
__device__ inline int w_off(int co, int c) { return (co * 16 + (c ^ (co & 15))) * 16; }

template <bool POOL>
__global__ __launch_bounds__(256) void conv3x3_c128_9x9(const uint16_t *__restrict__ x,
                                                        const uint16_t *__restrict__ w,
                                                        const uint16_t *__restrict__ bias,
                                                        uint16_t *__restrict__ out, int B) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[IN_BYTES + W_BYTES];
    uint8_t *lin = lds, *lw = lds + IN_BYTES;
    const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int img0 = (int)blockIdx.x * IMG;
    const int nimg = min(IMG, B - img0);

    // one tap's weights -> registers: chunk tid + 256 k = row 16 k + tid / 16, chunk tid % 16
    uint4 wr[8];
    auto wload = [&](int tap) {
        const uint4 *src = reinterpret_cast<const uint4 *>(w + (size_t)tap * C * C) + tid;
#pragma unroll
        for (int k = 0; k < 8; ++k) wr[k] = src[256 * k];
    };
    auto wstore = [&]() {
#pragma unroll
        for (int k = 0; k < 8; ++k) *reinterpret_cast<uint4 *>(lw + w_off(16 * k + (tid >> 4), tid & 15)) = wr[k];
    };
    wload(0);
    // input images with a zero halo (and zero images past B): all of a thread's loads
    // in flight at once, then the LDS stores
    constexpr int NCH = IMG * HP * HP * 16, PER = (NCH + 255) / 256;
    uint4 v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int i = tid + 256 * k, c = i & 15, Q = i >> 4;
        const int im = Q / (HP * HP), q = Q - im * HP * HP, py = q / HP, px = q - py * HP;
        v[k] = make_uint4(0u, 0u, 0u, 0u);
#ifndef MAPF_CONV_DIAG_NOIN
        if (i < NCH && im < nimg && py >= 1 && py <= H && px >= 1 && px <= H)
#else
        if (i < 0)
#endif
            v[k] = reinterpret_cast<const uint4 *>(x + ((size_t)(img0 + im) * H * H + (py - 1) * H + (px - 1)) * C)[c];
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int i = tid + 256 * k;
        if (i < NCH) *reinterpret_cast<uint4 *>(lin + in_off(i >> 4, i & 15)) = v[k];
    }
    wstore();
    __syncthreads();

    // this lane's pixels: M-tiles wv*4 + t, row (lane & 15)
    int qb[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        int m = (wv * 4 + t) * 16 + (lane & 15);
        if (m >= M) m = 0;                               // padded rows: any pixel, never stored
        const int im = m / (H * H), p = m - im * H * H, y = p / H, xx = p - y * H;
        qb[t] = im * HP * HP + (y + 1) * HP + (xx + 1);
    }
    const int g = lane >> 4;
    f4_t acc[4][8];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int n = 0; n < 8; ++n) acc[t][n] = f4_t{0.f, 0.f, 0.f, 0.f};

    for (int tap = 0; tap < 9; ++tap) {
#ifndef MAPF_CONV_DIAG_NOW
        if (tap < 8) wload(tap + 1);                     // in flight during this tap's MFMAs
#endif
        const int dq = (tap / 3 - 1) * HP + (tap % 3 - 1);
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) {
            const int c = kc * 4 + g;
            h8_t a[4], bf[8];
#pragma unroll
            for (int t = 0; t < 4; ++t)
                a[t] = *reinterpret_cast<const h8_t *>(lin + in_off(qb[t] + dq, c));
#pragma unroll
            for (int n = 0; n < 8; ++n) bf[n] = *reinterpret_cast<const h8_t *>(lw + w_off(n * 16 + (lane & 15), c));
#ifndef MAPF_CONV_DIAG_NOMFMA
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int n = 0; n < 8; ++n)
                    acc[t][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[t], bf[n], acc[t][n], 0, 0, 0);
#else
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int n = 0; n < 8; ++n) acc[t][n][0] += (float)a[t][0] * (float)bf[n][1];
#endif
        }
        __syncthreads();                                 // every wave is done with this tap's weights
        if (tap < 8) {
            wstore();
            __syncthreads();
        }
    }

    // epilogue: fp16 [m][co] image over the input area (all waves are past the last tap)
    uint16_t *img = reinterpret_cast<uint16_t *>(lin);
#pragma unroll
    for (int n = 0; n < 8; ++n) {
        const int co = n * 16 + (lane & 15);
        const float bv = h2f(bias[co]);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = (wv * 4 + t) * 16 + 4 * g + r;
                img[m * C + co] = (uint16_t)f2h(fmaxf(h2f(f2h(h2f(f2h(acc[t][n][r])) + bv)), 0.f));
            }
    }
    __syncthreads();
    if (!POOL) {
        for (int i = tid; i < nimg * H * H * 16; i += 256)
            reinterpret_cast<uint4 *>(out + (size_t)img0 * H * H * C)[i] = reinterpret_cast<const uint4 *>(img)[i];
    } else {
        constexpr int HO = H / 2;
        for (int i = tid; i < nimg * HO * HO * 16; i += 256) {
            const int c = i & 15, o = i >> 4;
            const int im = o / (HO * HO), r = o - im * HO * HO, oy = r / HO, ox = r - oy * HO;
            const int m0 = im * H * H + 2 * oy * H + 2 * ox;
            const uint4 *s = reinterpret_cast<const uint4 *>(img);
            const uint4 v0 = s[m0 * 16 + c], v1 = s[(m0 + 1) * 16 + c], v2 = s[(m0 + H) * 16 + c],
                        v3 = s[(m0 + H + 1) * 16 + c];
            const uint32_t *p0 = &v0.x, *p1 = &v1.x, *p2 = &v2.x, *p3 = &v3.x;
            uint32_t o4[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                uint32_t lo = 0, hi = 0;
                float mlo = -INFINITY, mhi = -INFINITY;
                const uint32_t ws[4] = {p0[k], p1[k], p2[k], p3[k]};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float fl = h2f(ws[j]), fh = h2f(ws[j] >> 16);
                    if (fl > mlo) { mlo = fl; lo = ws[j] & 0xFFFFu; }
                    if (fh > mhi) { mhi = fh; hi = ws[j] >> 16; }
                }
                o4[k] = lo | (hi << 16);
            }
            reinterpret_cast<uint4 *>(out + ((size_t)img0 * HO * HO) * C)[i] = make_uint4(o4[0], o4[1], o4[2], o4[3]);
        }
    }
}

}  // namespace conv
}  // namespace mapf

using namespace mapf;

extern "C" {

int mapf_conv3x3_c128_9x9(const uint16_t *x, const uint16_t *w_taps, const uint16_t *bias, uint16_t *out, int64_t B,
                          int32_t pool, void *stream) {
    if (!x || !w_taps || !bias || !out || B < 0 || B > (int64_t)1 << 30 ||
        (((uintptr_t)x | (uintptr_t)w_taps | (uintptr_t)out) & 15))
        return MAPF_EINVAL;
    if (B == 0) return MAPF_OK;
    const unsigned grid = (unsigned)((B + conv::IMG - 1) / conv::IMG);
    if (pool)
        hipLaunchKernelGGL(conv::conv3x3_c128_9x9<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, w_taps, bias,
                           out, (int)B);
    else
        hipLaunchKernelGGL(conv::conv3x3_c128_9x9<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, w_taps, bias,
                           out, (int)B);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

}  // extern "C"
