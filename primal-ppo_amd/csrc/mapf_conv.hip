// primal-ppo_amd/csrc/mapf_conv.hip -- SCRIMPNet's convolutions (net.py:101-112, under
// torch.autocast: fp16 operands, fp32 accumulation, fp16 output) as an implicit GEMM on the
// gfx950 matrix cores, for the acting forward (Model.step / Model.value, no grad).
//
//   out[img][oy][ox][n] = sum_{ky, kx, c} in[img][oy + ky - P][ox + kx - P][c] * w[n][ky][kx][c]
//
// GEMM view: M = images x Ho x Wo output pixels (NHWC rows), N = Cout, K = KS * KS * Cin,
// K ordered (ky, kx, c) so that one K-chunk of 64 is 64 consecutive channels of ONE input
// pixel: a row of the A tile is a contiguous 128-B run of the NHWC input (or zeros where the
// tap falls in the padding) -- the im2col matrix is never built.  The packed weight is
// [Cout][KS][KS][Cin] fp16 (torch's [Cout][Cin][KS][KS] permuted once, net.py caches it).
//
// Workgroup: WAVES waves, BM = 32 * WAVES output pixels x all Cout channels (the input of a
// pixel tile is read once per tap, from L2/L1: each input pixel is reused by KS^2 taps).  Each
// wave owns 32 rows x Cout: Cout/32 accumulators of v_mfma_f32_32x32x16_f16 (16 fp32 per lane
// each).  K loop over 64-wide chunks staged by LDS-DMA (global_load_lds_dwordx4: no staging
// registers) into two LDS buffers: chunk c + 1's copies are in flight while the matrix cores
// work on chunk c (a counted vmcnt retires only chunk c's, then a raw barrier).  LDS rows are
// 128 B with the 16-B pieces XOR-swizzled by (row >> 1) & 7 (swz below) -- on the SOURCE side: a
// DMA instruction writes its 64 lanes' 16 B linearly (8 rows x 8 pieces), so lane l fetches the
// logical piece that lands in its physical slot -- and each 16-lane group of a ds_read_b128
// fragment load gets 16 distinct bank slots.  Taps in the padding fetch 16 zero bytes (a zero block in the code object).
// Epilogue: fp32 accumulators -> fp16 (the conv's own rounding), optionally + bias (rounded
// again, as torch adds the bias to the fp16 conv output) and ReLU -- through an LDS transpose
// so every output row leaves as 16-B stores.
#include <hip/hip_fp16.h>

#include "mapf.h"
#include "mapf_common.h"

namespace mapf {
namespace conv {

typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
typedef float f16_t __attribute__((ext_vector_type(16)));

constexpr int BK = 64;              // K per chunk: 64 fp16 = one 128-B row per A / B row

__device__ __attribute__((aligned(16))) uint4 g_zero16[1];   // the padding taps' source (zero-initialised)

// byte offset of 16-B piece q of row r in a swizzled 128-B-row tile.  ds_read_b128 serves a wave in
// four 16-lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31} and the same +32), each conflict-free
// when its 16 lanes hit the 16 distinct 16-B slots of the 256-B bank row; a fragment load reads rows
// 0..31 (lane & 31) at one piece, and two 128-B rows share a bank row, so the XOR key is
// (r >> 1) & 7: with r & 1 it gives every row of a group its own slot ((r & 7) would pair rows
// r and r + 8 of a group on one slot: 2-way).
__device__ inline int swz_key(int r) { return (r >> 1) & 7; }
__device__ inline int swz(int r, int q) { return r * 128 + ((q ^ swz_key(r)) << 4); }
// the logical piece lane l fetches when one DMA instruction fills rows 8 g .. 8 g + 7 lane-linearly
__device__ inline int dma_piece(int lane, int g) { return (lane & 7) ^ swz_key(8 * g + (lane >> 3)); }

__device__ inline uint32_t f2h(float f) { return (uint32_t)__half_as_ushort(__float2half_rn(f)); }
__device__ inline float h2f(uint32_t h) { return __half2float(__ushort_as_half((unsigned short)(h & 0xFFFFu))); }

__device__ inline void dma16(const void *src, void *lds_base) {
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void *)lds_base, 16, 0, 0);
}

template <int CIN, int COUT, int KS, int WAVES>
struct Cfg {
    static constexpr int THREADS = 64 * WAVES;
    static constexpr int NT = COUT / 32;                  // accumulator tiles along N per wave
    static constexpr int BM = 32 * WAVES;                 // output pixels per workgroup
    static constexpr int K = KS * KS * CIN;
    static constexpr int CB = CIN / BK;                   // chunks per tap
    static constexpr int NCHUNK = KS * KS * CB;
    static constexpr int A_BYTES = BM * BK * 2, B_BYTES = COUT * BK * 2, BUF = A_BYTES + B_BYTES;
    static constexpr int JA = BM / 8 / WAVES;             // DMA instructions (8 rows each) per wave per chunk
    static constexpr int JB = COUT / 8 / WAVES;
    static constexpr int LDS = 2 * BUF > BM * COUT * 2 ? 2 * BUF : BM * COUT * 2;
    static_assert(CIN % BK == 0 && COUT % 32 == 0 && (COUT / 8) % WAVES == 0, "shape");
    static_assert(JA + JB <= 15, "vmcnt field");
};

// epi: 0 = raw fp16 conv output, 1 = + bias, ReLU
template <int CIN, int COUT, int KS, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void conv_igemm_kernel(const uint16_t *__restrict__ in,
                                                                const uint16_t *__restrict__ w,
                                                                const uint16_t *__restrict__ bias,
                                                                uint16_t *__restrict__ out, int M, int H, int W,
                                                                int Ho, int Wo, int pad, int epi) {
    using C = Cfg<CIN, COUT, KS, WAVES>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int t = (int)threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int m0 = (int)blockIdx.x * C::BM;
    const int HWo = Ho * Wo;
    // lane l of a DMA instruction filling rows 8 g .. 8 g + 7 writes row 8 g + (l >> 3), physical
    // piece l & 7 = logical piece dma_piece(l, g), which depends on g only through its parity
    const int q0 = dma_piece(lane, 0), q1 = dma_piece(lane, 1);
    // this lane's A rows (one per DMA instruction): the output pixel's input pixel index and (oy, ox)
    int apix[C::JA], ayx[C::JA];
#pragma unroll
    for (int j = 0; j < C::JA; ++j) {
        const int m = m0 + 8 * (wave * C::JA + j) + (lane >> 3);
        if (m < M) {
            const int img = m / HWo, pos = m - img * HWo, oy = pos / Wo, ox = pos - oy * Wo;
            apix[j] = img * H * W + oy * W + ox;
            ayx[j] = (oy << 16) | ox;
        } else {
            apix[j] = 0;
            ayx[j] = (int)0x80000000u;             // every tap out of range
        }
    }
    auto issue = [&](int c, int buf) {             // chunk c -> LDS buffer buf (DMA, in flight)
        const int tap = c / C::CB, cb = c - tap * C::CB;
        const int ky = tap / KS, kx = tap - ky * KS;
        char *A = smem + buf * C::BUF;
        char *B = A + C::A_BYTES;
        const int dpix = (ky - pad) * W + (kx - pad);
#pragma unroll
        for (int j = 0; j < C::JA; ++j) {
            const int iy = (ayx[j] >> 16) + ky - pad, ix = (ayx[j] & 0xFFFF) + kx - pad;
            const bool ok = ((unsigned)iy < (unsigned)H) & ((unsigned)ix < (unsigned)W);
            const int q = ((wave * C::JA + j) & 1) ? q1 : q0;
            const void *src = ok ? (const void *)(in + (size_t)(apix[j] + dpix) * CIN + cb * BK + q * 8)
                                 : (const void *)g_zero16;
            dma16(src, A + 8 * (wave * C::JA + j) * 128);
        }
#pragma unroll
        for (int j = 0; j < C::JB; ++j) {
            const int n = 8 * (wave * C::JB + j) + (lane >> 3);
            const int q = ((wave * C::JB + j) & 1) ? q1 : q0;
            dma16(w + (size_t)n * C::K + c * BK + q * 8, B + 8 * (wave * C::JB + j) * 128);
        }
    };

    f16_t acc[C::NT];
#pragma unroll
    for (int b = 0; b < C::NT; ++b)
        for (int r = 0; r < 16; ++r) acc[b][r] = 0.f;

    issue(0, 0);
    const int fr = lane & 31, fh = lane >> 5;     // fragment row within a 32-tile, K half
    for (int c = 0; c < C::NCHUNK; ++c) {
        if (c + 1 < C::NCHUNK) {
            issue(c + 1, (c + 1) & 1);            // buffer (c+1)&1 was last read in chunk c-1 (barrier since)
            // chunk c's copies (issued before chunk c + 1's) have landed: vmcnt(JA + JB)
            __builtin_amdgcn_s_waitcnt(0x0F70 | (C::JA + C::JB));
        } else {
            __builtin_amdgcn_s_waitcnt(0x0F70);
        }
        __builtin_amdgcn_s_barrier();             // ... in every wave
        const char *A = smem + (c & 1) * C::BUF;
        const char *B = A + C::A_BYTES;
#pragma unroll
        for (int s = 0; s < BK / 16; ++s) {       // 16-deep MFMA steps
            const int qq = 2 * s + fh;
            const h8_t af = *reinterpret_cast<const h8_t *>(A + swz(wave * 32 + fr, qq));
#pragma unroll
            for (int b = 0; b < C::NT; ++b) {
                const h8_t bf = *reinterpret_cast<const h8_t *>(B + swz(b * 32 + fr, qq));
                acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf, acc[b], 0, 0, 0);
            }
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);       // lgkmcnt(0): this wave's fragment reads are done
        __builtin_amdgcn_s_barrier();             // ... in every wave: buffer c&1 may be refilled
    }

    // epilogue: fp16 tile [BM][COUT] in LDS (row-major, 16-B pieces swizzled by row & 7 within
    // each 128-B group), then 16-B stores of whole output rows
    char *T = smem;
    constexpr int RB = COUT * 2;                  // bytes per tile row
#pragma unroll
    for (int b = 0; b < C::NT; ++b) {
        const int n = b * 32 + fr;
        const float bv = epi ? h2f(bias[n]) : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
            float v = h2f(f2h(acc[b][r]));                    // the conv's fp16 output
            if (epi) v = relu_nan(h2f(f2h(v + bv)));        // + bias (fp16), ReLU
            const int byte = n * 2, g = byte >> 7, pq = (byte >> 4) & 7;
            *reinterpret_cast<uint16_t *>(T + row * RB + g * 128 + ((pq ^ (row & 7)) << 4) + (byte & 15)) =
                (uint16_t)f2h(v);
        }
    }
    __syncthreads();
    constexpr int PIECES_ROW = RB / 16;
    for (int p = t; p < C::BM * PIECES_ROW; p += C::THREADS) {
        const int row = p / PIECES_ROW, pc = p - row * PIECES_ROW;
        const int m = m0 + row;
        if (m >= M) continue;
        const int g = pc >> 3, pq = pc & 7;
        const uint4 v = *reinterpret_cast<const uint4 *>(T + row * RB + g * 128 + ((pq ^ (row & 7)) << 4));
        *reinterpret_cast<uint4 *>(out + (size_t)m * COUT + pc * 8) = v;
    }
}

// The same implicit GEMM with K chunks of 32 (64-B LDS rows) in a ring of STAGES buffers: the
// same LDS as the 64-deep double buffer holds STAGES - 1 chunks in flight instead of one, with one
// barrier per chunk (the buffer refilled at chunk c is the one every wave finished reading before
// chunk c's barrier).  64-B rows: a DMA instruction fills 16 rows, lane l row 16 g + (l >> 2),
// physical piece l & 3; the XOR key (row >> 2) & 3 gives each lane of a ds_read_b128 16-lane group
// (16 distinct rows, 4 rows per 256-B bank row) its own slot.
__device__ inline int swz64(int r, int q) { return r * 64 + ((q ^ ((r >> 2) & 3)) << 4); }
template <int N>
__device__ inline void wait_vm() {
    static_assert(N >= 0 && N <= 63, "vmcnt");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}

template <int CIN, int COUT, int KS, int WAVES, int STAGES>
struct Cfg32 {
    static constexpr int THREADS = 64 * WAVES, NT = COUT / 32, BM = 32 * WAVES, K = KS * KS * CIN;
    static constexpr int CB = CIN / 32, NCHUNK = KS * KS * CB;
    static constexpr int A_BYTES = BM * 64, B_BYTES = COUT * 64, BUF = A_BYTES + B_BYTES;
    static constexpr int JA = BM / 16 / WAVES, JB = COUT / 16 / WAVES, J = JA + JB;
    static constexpr int LDS = STAGES * BUF > BM * COUT * 2 ? STAGES * BUF : BM * COUT * 2;
    static_assert(CIN % 32 == 0 && COUT % 32 == 0 && BM % (16 * WAVES) == 0 && COUT % (16 * WAVES) == 0, "shape");
    static_assert(STAGES >= 2 && (STAGES - 2) * J <= 63 && NCHUNK >= STAGES, "ring");
};

template <int CIN, int COUT, int KS, int WAVES, int STAGES>
__global__ __launch_bounds__(64 * WAVES) void conv_igemm32_kernel(const uint16_t *__restrict__ in,
                                                                  const uint16_t *__restrict__ w,
                                                                  const uint16_t *__restrict__ bias,
                                                                  uint16_t *__restrict__ out, int M, int H, int W,
                                                                  int Ho, int Wo, int pad, int epi, int ipt) {
    // ipt > 0: tiles of ipt whole images (ipt * Ho * Wo <= BM rows, the rest padding) and a pooled
    // epilogue: out = relu(fp16(max2x2(conv) + bias)), [img][Ho / 2][Wo / 2][COUT] (nhwc_bias_relu_pool2)
    using C = Cfg32<CIN, COUT, KS, WAVES, STAGES>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int t = (int)threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int HWo = Ho * Wo;
    const int rows_here = ipt ? ipt * HWo : C::BM;     // tile rows that are output pixels
    const int m0 = (int)blockIdx.x * rows_here;
    const int q = (lane & 3) ^ ((lane >> 4) & 3);          // logical piece of this lane's 16 B
    int apix[C::JA], ayx[C::JA];
#pragma unroll
    for (int j = 0; j < C::JA; ++j) {
        const int r = 16 * (wave * C::JA + j) + (lane >> 2), m = m0 + r;
        if (r < rows_here && m < M) {
            const int img = m / HWo, pos = m - img * HWo, oy = pos / Wo, ox = pos - oy * Wo;
            apix[j] = img * H * W + oy * W + ox;
            ayx[j] = (oy << 16) | ox;
        } else {
            apix[j] = 0;
            ayx[j] = (int)0x80000000u;                     // every tap out of range
        }
    }
    auto issue = [&](int c, int buf) {
        const int tap = c / C::CB, cb = c - tap * C::CB;
        const int ky = tap / KS, kx = tap - ky * KS;
        char *A = smem + buf * C::BUF;
        char *B = A + C::A_BYTES;
        const int dpix = (ky - pad) * W + (kx - pad);
#pragma unroll
        for (int j = 0; j < C::JA; ++j) {
            const int iy = (ayx[j] >> 16) + ky - pad, ix = (ayx[j] & 0xFFFF) + kx - pad;
            const bool ok = ((unsigned)iy < (unsigned)H) & ((unsigned)ix < (unsigned)W);
            const void *src = ok ? (const void *)(in + (size_t)(apix[j] + dpix) * CIN + cb * 32 + q * 8)
                                 : (const void *)g_zero16;
            dma16(src, A + 16 * (wave * C::JA + j) * 64);
        }
#pragma unroll
        for (int j = 0; j < C::JB; ++j) {
            const int n = 16 * (wave * C::JB + j) + (lane >> 2);
            dma16(w + (size_t)n * C::K + c * 32 + q * 8, B + 16 * (wave * C::JB + j) * 64);
        }
    };
    f16_t acc[C::NT];
#pragma unroll
    for (int b = 0; b < C::NT; ++b)
        for (int r = 0; r < 16; ++r) acc[b][r] = 0.f;
#pragma unroll
    for (int c = 0; c < STAGES - 1; ++c) issue(c, c);
    const int fr = lane & 31, fh = lane >> 5;
    for (int c = 0; c < C::NCHUNK; ++c) {
        // chunks c + 1 .. min(c + STAGES - 2, NCHUNK - 1) may stay in flight
        const int ahead = C::NCHUNK - 1 - c < STAGES - 2 ? C::NCHUNK - 1 - c : STAGES - 2;
        if (ahead >= STAGES - 2) wait_vm<(STAGES - 2) * C::J>();
        else if (STAGES > 3 && ahead == 1) wait_vm<(STAGES > 3 ? C::J : 0)>();
        else if (STAGES > 4 && ahead == 2) wait_vm<(STAGES > 4 ? 2 * C::J : 0)>();
        else wait_vm<0>();
        __builtin_amdgcn_s_barrier();
        if (c + STAGES - 1 < C::NCHUNK) issue(c + STAGES - 1, (c + STAGES - 1) % STAGES);
        const char *A = smem + (c % STAGES) * C::BUF;
        const char *B = A + C::A_BYTES;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int qq = 2 * s + fh;
            const h8_t af = *reinterpret_cast<const h8_t *>(A + swz64(wave * 32 + fr, qq));
#pragma unroll
            for (int b = 0; b < C::NT; ++b) {
                const h8_t bf = *reinterpret_cast<const h8_t *>(B + swz64(b * 32 + fr, qq));
                acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf, acc[b], 0, 0, 0);
            }
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
    }
    __syncthreads();                                  // every wave done with the ring: the tile reuses it
    char *T = smem;
    constexpr int RB = COUT * 2;
#pragma unroll
    for (int b = 0; b < C::NT; ++b) {
        const int n = b * 32 + fr;
        const float bv = epi ? h2f(bias[n]) : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
            float v = h2f(f2h(acc[b][r]));
            if (epi) v = relu_nan(h2f(f2h(v + bv)));
            const int byte = n * 2, g = byte >> 7, pq = (byte >> 4) & 7;
            *reinterpret_cast<uint16_t *>(T + row * RB + g * 128 + ((pq ^ (row & 7)) << 4) + (byte & 15)) =
                (uint16_t)f2h(v);
        }
    }
    __syncthreads();
    constexpr int PIECES_ROW = RB / 16;
    auto piece = [&](int row, int pc) {
        return *reinterpret_cast<const uint4 *>(T + row * RB + (pc >> 3) * 128 + (((pc & 7) ^ (row & 7)) << 4));
    };
    if (ipt) {                                        // 2x2 max-pool + bias + ReLU of whole images
        const int Hp = Ho >> 1, Wp = Wo >> 1, img0 = (int)blockIdx.x * ipt;
        const int nimg_here = min(ipt, M / HWo - img0);
        const int items = nimg_here * Hp * Wp * PIECES_ROW;
        for (int p = t; p < items; p += C::THREADS) {
            const int pc = p % PIECES_ROW, cell = p / PIECES_ROW;
            const int il = cell / (Hp * Wp), rem = cell - il * (Hp * Wp), pi = rem / Wp, pj = rem - pi * Wp;
            const int r00 = il * HWo + 2 * pi * Wo + 2 * pj;
            const uint4 v[4] = {piece(r00, pc), piece(r00 + 1, pc), piece(r00 + Wo, pc), piece(r00 + Wo + 1, pc)};
            const uint4 bb = *reinterpret_cast<const uint4 *>(bias + pc * 8);
            const uint32_t bw[4] = {bb.x, bb.y, bb.z, bb.w};
            uint32_t o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {                  // 2 channels per dword
                const uint32_t w0 = (&v[0].x)[e], w1 = (&v[1].x)[e], w2 = (&v[2].x)[e], w3 = (&v[3].x)[e];
                uint32_t h2[2];
#pragma unroll
                for (int hh = 0; hh < 2; ++hh) {
                    const int sh = 16 * hh;
                    const float m = max_nan(max_nan(max_nan(h2f(w0 >> sh), h2f(w1 >> sh)), h2f(w2 >> sh)), h2f(w3 >> sh));
                    h2[hh] = f2h(relu_nan(h2f(f2h(m + h2f(bw[e] >> sh)))));
                }
                o[e] = h2[0] | (h2[1] << 16);
            }
            *reinterpret_cast<uint4 *>(out + ((size_t)(img0 + il) * Hp * Wp + pi * Wp + pj) * COUT + pc * 8) =
                make_uint4(o[0], o[1], o[2], o[3]);
        }
        return;
    }
    for (int p = t; p < C::BM * PIECES_ROW; p += C::THREADS) {
        const int row = p / PIECES_ROW, pc = p - row * PIECES_ROW;
        const int m = m0 + row;
        if (m >= M) continue;
        *reinterpret_cast<uint4 *>(out + (size_t)m * COUT + pc * 8) = piece(row, pc);
    }
}

// ---- Image-resident implicit GEMM (round 5) ---------------------------------------------
// conv_igemm32 stages one A row per (output pixel, tap): every input pixel crosses L2 -> LDS KS^2
// times (9x for the 3x3 layers), 24 KiB of DMA per 32-deep K-chunk at 128 channels -- the kernel
// ran at ~37 GB/s per CU of LDS-DMA, about half what the CU can take in from L2, latency-bound on
// those copies.  Here a workgroup owns `ipt` WHOLE images (ipt * Ho * Wo <= 32 * WAVES rows) and
// each 32-channel slice of their input pixels is DMA'd into LDS once; every tap's A fragment is
// read from that image at a shifted pixel index.  K order (channel chunk cc, tap, 32 channels):
// per chunk only the weight slice (COUT x 32) streams, through a ring of S buffers; the next image
// chunk is DMA'd into the other image buffer while the current one is in use (issued at the
// current chunk's first tap, waited for T taps later).  For the 3x3 / 128-channel layers the
// L2 -> LDS bytes per tile fall from 864 to ~390 KiB.
//
// LDS image of one channel chunk: slot s (64 B = 32 fp16 channels of one pixel) at s * 64, the 16-B
// pieces XOR-swizzled by (s >> 2) & 3.  Input pixel (img, iy, ix) sits at slot
//     MARGIN + img * IS + (iy + pad) * Wo + ix          (rows of Wo slots, ix < W <= Wo)
// with zero slots for the pad rows; columns past W and the horizontal padding are never stored --
// the A fragment of a tap whose ix = ox + kx - pad falls outside [0, W) is zeroed in registers.
// The output row r = img * Ho * Wo + oy * Wo + ox of tap (ky, kx) reads slot
//     MARGIN + r + img * (IS - Ho * Wo) + ky * Wo + kx - pad,
// and IS = Ho * Wo + 16 k makes that r + const mod 16: the 16 rows a ds_read_b128 lane group
// reads ({0-3,12-15,20-27} / {4-11,16-19,28-31} of a wave's 32) are 16 distinct residues, i.e. 16
// distinct (s & 3, piece) bank slots -- conflict-free for every tap.  A DMA instruction fills 16
// consecutive slots lane-linearly (lane l: slot 16 g + (l >> 2), physical piece l & 3), the source
// pre-swizzled; slots that hold no input pixel (pad rows, gaps, the margin) fetch zeros.
constexpr int IMG_MARGIN = 16;

template <int CIN, int COUT, int KS, int WAVES, int S, int JI>
struct CfgImg {
    static constexpr int THREADS = 64 * WAVES, NT = COUT / 32, BM = 32 * WAVES, T = KS * KS, K = T * CIN;
    static constexpr int NCC = CIN / 32, NCH = NCC * T;
    static constexpr int IMG_SLOTS = 16 * JI * WAVES, IMG_BYTES = IMG_SLOTS * 64;
    static constexpr int B_BYTES = COUT * 64, JB = COUT / 16 / WAVES;
    static constexpr int RING = 2 * IMG_BYTES + S * B_BYTES;
    static constexpr int LDS = RING > BM * COUT * 2 ? RING : BM * COUT * 2;
    static_assert(CIN % 32 == 0 && COUT % 32 == 0 && COUT % (16 * WAVES) == 0, "shape");
    static_assert(S == 3 && T >= S && JB + JI <= 15, "ring / vmcnt");
};

__device__ inline int img_slot(int s, int q) { return s * 64 + ((q ^ ((s >> 2) & 3)) << 4); }

template <int CIN, int COUT, int KS, int WAVES, int S, int JI>
__global__ __launch_bounds__(64 * WAVES) void conv_img_kernel(const uint16_t *__restrict__ in,
                                                              const uint16_t *__restrict__ w,
                                                              const uint16_t *__restrict__ bias,
                                                              uint16_t *__restrict__ out, int nimg, int H, int W,
                                                              int pad, int ipt, int IS, int epi, int pool) {
    using C = CfgImg<CIN, COUT, KS, WAVES, S, JI>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int t = (int)threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int Ho = H + 2 * pad - KS + 1, Wo = W + 2 * pad - KS + 1, HWo = Ho * Wo;
    const int img0 = (int)blockIdx.x * ipt;
    const int nimg_here = min(ipt, nimg - img0);
    const int rows_here = nimg_here * HWo;
    char *IMG = smem;                                         // two image-chunk buffers
    char *BR = smem + 2 * C::IMG_BYTES;                       // the weight ring
    // image-chunk DMA: this lane's source (element offset of channel 0 of its pixel, or -1: zeros)
    // and logical piece, per instruction j (the same for every channel chunk)
    int isrc[JI];
#pragma unroll
    for (int j = 0; j < JI; ++j) {
        const int slot = 16 * (wave * JI + j) + (lane >> 2);
        const int u = slot - IMG_MARGIN;
        int src = -1;
        if (u >= 0 && u < nimg_here * IS) {
            const int il = u / IS, rem = u - il * IS, rr = rem / Wo, ix = rem - rr * Wo, iy = rr - pad;
            if ((unsigned)iy < (unsigned)H && ix < W) src = (((img0 + il) * H + iy) * W + ix) * CIN;
        }
        const int q = (lane & 3) ^ ((slot >> 2) & 3);
        isrc[j] = src < 0 ? -1 : src + q * 8;
    }
    auto issue_img = [&](int cc, int buf) {
        char *D = IMG + buf * C::IMG_BYTES;
#pragma unroll
        for (int j = 0; j < JI; ++j)
            dma16(isrc[j] >= 0 ? (const void *)(in + isrc[j] + cc * 32) : (const void *)g_zero16,
                  D + 16 * (wave * JI + j) * 64);
    };
    const int qw = (lane & 3) ^ ((lane >> 4) & 3);            // weight rows: key (n >> 2) & 3, n = 16 g + (l >> 2)
    auto issue_b = [&](int c, int slot) {
        const int cc = c / C::T, tap = c - cc * C::T;
        char *D = BR + slot * C::B_BYTES;
#pragma unroll
        for (int j = 0; j < C::JB; ++j) {
            const int n = 16 * (wave * C::JB + j) + (lane >> 2);
            dma16(w + (size_t)n * C::K + tap * CIN + cc * 32 + qw * 8, D + 16 * (wave * C::JB + j) * 64);
        }
    };
    // this lane's A row: slot of tap (0, 0) and its output column (for the horizontal padding mask)
    const int fr = lane & 31, fh = lane >> 5;
    const int r = wave * 32 + fr;
    int sbase, ox;
    if (r < rows_here) {
        const int il = r / HWo, p = r - il * HWo, oy = p / Wo;
        ox = p - oy * Wo;
        sbase = IMG_MARGIN + il * IS + oy * Wo + ox - pad;
    } else {                                                  // padding row: any slot of the same residue
        ox = 0x4000;                                          // every tap masked
        sbase = IMG_MARGIN + (r & 15);
    }
    f16_t acc[C::NT];
#pragma unroll
    for (int b = 0; b < C::NT; ++b)
        for (int e = 0; e < 16; ++e) acc[b][e] = 0.f;
    issue_img(0, 0);
#pragma unroll
    for (int c = 0; c < S - 1; ++c) issue_b(c, c);
    for (int c = 0; c < C::NCH; ++c) {
        const int cc = c / C::T, tap = c - cc * C::T;
        // weights of chunk c (and image chunk cc, DMA'd >= T >= S chunks earlier) have landed;
        // younger copies may stay in flight: the next weight slice, and the next image chunk if one
        // was issued in the last S - 1 chunks (at a chunk's tap 0)
        if (c + S - 2 >= C::NCH) wait_vm<0>();
        else if ((tap >= 1 && tap <= S - 1) && cc + 1 < C::NCC) wait_vm<(S - 2) * C::JB + JI>();
        else wait_vm<(S - 2) * C::JB>();
        __builtin_amdgcn_s_barrier();
        if (c + S - 1 < C::NCH) issue_b(c + S - 1, (c + S - 1) % S);
        if (tap == 0 && cc + 1 < C::NCC) issue_img(cc + 1, (cc + 1) & 1);   // its buffer was read in cc - 1
        const char *A = IMG + (cc & 1) * C::IMG_BYTES;
        const char *B = BR + (c % S) * C::B_BYTES;
        const int ky = tap / KS, kx = tap - ky * KS;
        const int sl = sbase + ky * Wo + kx;
        const bool ok = (unsigned)(ox + kx - pad) < (unsigned)W;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            const int qq = 2 * s2 + fh;
            h8_t af = *reinterpret_cast<const h8_t *>(A + img_slot(sl, qq));
            if (!ok) af = h8_t{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
            for (int b = 0; b < C::NT; ++b) {
                const h8_t bf = *reinterpret_cast<const h8_t *>(B + swz64(b * 32 + fr, qq));
                acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf, acc[b], 0, 0, 0);
            }
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
    }
    __syncthreads();                                  // every wave done with the images and the ring
    char *Tt = smem;
    constexpr int RB = COUT * 2;
#pragma unroll
    for (int b = 0; b < C::NT; ++b) {
        const int n = b * 32 + fr;
        const float bv = epi ? h2f(bias[n]) : 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int row = wave * 32 + (e & 3) + 8 * (e >> 2) + 4 * fh;
            float v = h2f(f2h(acc[b][e]));
            if (epi) v = relu_nan(h2f(f2h(v + bv)));
            const int byte = n * 2, g = byte >> 7, pq = (byte >> 4) & 7;
            *reinterpret_cast<uint16_t *>(Tt + row * RB + g * 128 + ((pq ^ (row & 7)) << 4) + (byte & 15)) =
                (uint16_t)f2h(v);
        }
    }
    __syncthreads();
    constexpr int PIECES_ROW = RB / 16;
    auto piece = [&](int row, int pc) {
        return *reinterpret_cast<const uint4 *>(Tt + row * RB + (pc >> 3) * 128 + (((pc & 7) ^ (row & 7)) << 4));
    };
    if (pool) {                                       // 2x2 max-pool + bias + ReLU of whole images
        const int Hp = Ho >> 1, Wp = Wo >> 1;
        const int items = nimg_here * Hp * Wp * PIECES_ROW;
        for (int p = t; p < items; p += C::THREADS) {
            const int pc = p % PIECES_ROW, cell = p / PIECES_ROW;
            const int il = cell / (Hp * Wp), rem = cell - il * (Hp * Wp), pi = rem / Wp, pj = rem - pi * Wp;
            const int r00 = il * HWo + 2 * pi * Wo + 2 * pj;
            const uint4 v[4] = {piece(r00, pc), piece(r00 + 1, pc), piece(r00 + Wo, pc), piece(r00 + Wo + 1, pc)};
            const uint4 bb = *reinterpret_cast<const uint4 *>(bias + pc * 8);
            const uint32_t bw[4] = {bb.x, bb.y, bb.z, bb.w};
            uint32_t o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t w0 = (&v[0].x)[e], w1 = (&v[1].x)[e], w2 = (&v[2].x)[e], w3 = (&v[3].x)[e];
                uint32_t h2[2];
#pragma unroll
                for (int hh = 0; hh < 2; ++hh) {
                    const int sh = 16 * hh;
                    const float m = max_nan(max_nan(max_nan(h2f(w0 >> sh), h2f(w1 >> sh)), h2f(w2 >> sh)), h2f(w3 >> sh));
                    h2[hh] = f2h(relu_nan(h2f(f2h(m + h2f(bw[e] >> sh)))));
                }
                o[e] = h2[0] | (h2[1] << 16);
            }
            *reinterpret_cast<uint4 *>(out + ((size_t)(img0 + il) * Hp * Wp + pi * Wp + pj) * COUT + pc * 8) =
                make_uint4(o[0], o[1], o[2], o[3]);
        }
        return;
    }
    const size_t m0 = (size_t)img0 * HWo;
    for (int p = t; p < rows_here * PIECES_ROW; p += C::THREADS) {
        const int row = p / PIECES_ROW, pc = p - row * PIECES_ROW;
        *reinterpret_cast<uint4 *>(out + (m0 + row) * COUT + pc * 8) = piece(row, pc);
    }
}

// the image-resident form's geometry for one layer, or false when it does not apply
struct ImgPlan {
    int ipt, IS, ji;
};
template <int WAVES>
static bool plan_img(int H, int W, int pad, int KS, ImgPlan &p) {
    const int Ho = H + 2 * pad - KS + 1, Wo = W + 2 * pad - KS + 1, HWo = Ho * Wo;
    if (Ho < 1 || Wo < W || HWo > 32 * WAVES || pad > 15) return false;
    const int need = (Ho + KS - 1) * Wo + KS;        // slots an image's taps can reach (+ slack)
    int IS = HWo;
    while (IS < need) IS += 16;
    p.ipt = (32 * WAVES) / HWo;
    const int slots = IMG_MARGIN + p.ipt * IS;
    // padding rows read slot MARGIN + (r & 15) + tap offset: keep every read inside the buffer
    const int reach = IMG_MARGIN + 32 * WAVES + (KS - 1) * Wo + KS;
    const int need_slots = slots > reach ? slots : reach;
    p.ji = (need_slots + 16 * WAVES - 1) / (16 * WAVES);
    p.IS = IS;
    return p.ji <= 4;
}

// 1 (default): the form measured faster per layer (tools/bench_conv_impl.py, profiles/r05_conv_ab.jsonl):
//   image-resident for the 3x3 layers and the pooled 2x2 layer, per-tap staged for the plain 2x2 layers;
// 2: image-resident wherever its geometry applies; 0: per-tap staged everywhere
static int g_conv_impl = 1;

template <int CIN, int COUT, int KS, int WAVES, int JI>
static void launch_img_ji(const uint16_t *in, const uint16_t *w, const uint16_t *bias, uint16_t *out, int nimg, int H,
                          int W, int pad, const ImgPlan &p, int epi, int pool, hipStream_t s) {
    using C = CfgImg<CIN, COUT, KS, WAVES, 3, JI>;
    hipLaunchKernelGGL((conv_img_kernel<CIN, COUT, KS, WAVES, 3, JI>), dim3((nimg + p.ipt - 1) / p.ipt), dim3(C::THREADS),
                       C::LDS, s, in, w, bias, out, nimg, H, W, pad, p.ipt, p.IS, epi, pool);
}
template <int CIN, int COUT, int KS, int WAVES>
static bool launch_img(const uint16_t *in, const uint16_t *w, const uint16_t *bias, uint16_t *out, int nimg, int H,
                       int W, int pad, int epi, int pool, hipStream_t s) {
    ImgPlan p;
    if (g_conv_impl == 0 || (g_conv_impl == 1 && KS == 2 && !pool) || !plan_img<WAVES>(H, W, pad, KS, p))
        return false;
    if (pool && ((H + 2 * pad - KS + 1) < 2 || (W + 2 * pad - KS + 1) < 2)) return false;
    if (p.ji <= 3) launch_img_ji<CIN, COUT, KS, WAVES, 3>(in, w, bias, out, nimg, H, W, pad, p, epi, pool, s);
    else launch_img_ji<CIN, COUT, KS, WAVES, 4>(in, w, bias, out, nimg, H, W, pad, p, epi, pool, s);
    return true;
}

#ifndef MAPF_CONV_STAGES
#define MAPF_CONV_STAGES 3                            // 0: the 64-deep double buffer (conv_igemm_kernel)
#endif

template <int CIN, int COUT, int KS, int WAVES>
static void launch(const uint16_t *in, const uint16_t *w, const uint16_t *bias, uint16_t *out, int M, int H, int W,
                   int Ho, int Wo, int pad, int epi, hipStream_t s, bool pool = false) {
#if MAPF_CONV_STAGES
    using C = Cfg32<CIN, COUT, KS, WAVES, MAPF_CONV_STAGES>;
    if (pool) {                                   // whole images per tile (the caller checked Ho * Wo <= BM)
        const int ipt = C::BM / (Ho * Wo), nimg = M / (Ho * Wo);
        hipLaunchKernelGGL((conv_igemm32_kernel<CIN, COUT, KS, WAVES, MAPF_CONV_STAGES>), dim3((nimg + ipt - 1) / ipt),
                           dim3(C::THREADS), C::LDS, s, in, w, bias, out, M, H, W, Ho, Wo, pad, 0, ipt);
        return;
    }
    hipLaunchKernelGGL((conv_igemm32_kernel<CIN, COUT, KS, WAVES, MAPF_CONV_STAGES>), dim3((M + C::BM - 1) / C::BM),
                       dim3(C::THREADS), C::LDS, s, in, w, bias, out, M, H, W, Ho, Wo, pad, epi, 0);
#else
    using C = Cfg<CIN, COUT, KS, WAVES>;
    hipLaunchKernelGGL((conv_igemm_kernel<CIN, COUT, KS, WAVES>), dim3((M + C::BM - 1) / C::BM), dim3(C::THREADS),
                       C::LDS, s, in, w, bias, out, M, H, W, Ho, Wo, pad, epi);
#endif
}

// The first convolution (conv1, net.py:104: Cin = num_channel <= 7, 3x3, padding 1) straight from
// the fp32 NCHW observation: K = Cin * 9 <= 63 (torch's (c, ky, kx) order, zero-padded to 64: the
// packed weight is [Cout][64] fp16) is ONE chunk.  A workgroup of 128 output pixels copies the
// (at most (127 / HW) + 2) images they lie in, cast to fp16 as autocast does, into an LDS image
// with a zero border, and the weight into a swizzled LDS tile; builds its 128 im2col rows from the
// image (a thread per (row, 16-B piece of 8 k): 8 LDS reads at offsets fixed per thread, one
// 16-B write); multiplies; and writes relu(fp16(fp16(acc) + bias)) as NHWC fp16 from registers
// (the weight is the MFMA row operand, so the accumulators hold C^T: 4 consecutive channels of a
// pixel per 8-B store) -- the MIOpen path's NHWC copy and cast, the conv and the bias / ReLU pass
// in one launch.  ~100 VGPRs and ~37 KiB of LDS: four workgroups per CU overlap each other's
// load -> build -> MFMA -> store phases.
__device__ inline int div_small(int a, int b, float rb) {    // a / b for 0 <= a < 2^22, b > 0 (rb = 1 / b)
    int q = (int)((float)a * rb);
    q += (a - q * b >= b) ? 1 : 0;
    q -= (a - q * b < 0) ? 1 : 0;
    return q;
}

template <int COUT>
__global__ __launch_bounds__(256) void conv_first_kernel(const float *__restrict__ in, const uint16_t *__restrict__ w,
                                                         const uint16_t *__restrict__ bias, uint16_t *__restrict__ out,
                                                         int M, int C, int H, int W, int nimg) {
    constexpr int BM = 128, NT = COUT / 32;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char *As = smem;                                   // [128][64] fp16 im2col rows, swizzled
    char *Bs = smem + BM * 128;                        // [COUT][64] fp16 weight, swizzled
    uint16_t *Img = reinterpret_cast<uint16_t *>(smem + BM * 128 + COUT * 128);   // [n][C][H + 2][W + 2]
    const int t = (int)threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int fr = lane & 31, fh = lane >> 5;
    const int m0 = (int)blockIdx.x * BM;
    const int HW = H * W, K = C * 9, PW = W + 2, PP = (H + 2) * PW;
    const float rHW = 1.f / (float)HW, rW = 1.f / (float)W;
    const int img_lo = m0 / HW;
    int img_hi = (m0 + BM - 1) / HW;
    if (img_hi > nimg - 1) img_hi = nimg - 1;
    const int n = img_hi - img_lo + 1;
    // the weight -> LDS (its loads overlap the image staging below)
    uint4 wv[COUT * 8 / 256];
#pragma unroll
    for (int j = 0; j < COUT * 8 / 256; ++j) {
        const int p = t + 256 * j;
        wv[j] = *reinterpret_cast<const uint4 *>(w + (size_t)(p >> 3) * 64 + (p & 7) * 8);
    }
    // 1. zero the LDS images (the border stays zero), 2. copy the interior, cast to fp16
    const int img_words = (n * C * PP + 1) >> 1;
    for (int e = t; e < img_words; e += 256) reinterpret_cast<uint32_t *>(Img)[e] = 0u;
#pragma unroll
    for (int j = 0; j < COUT * 8 / 256; ++j) {
        const int p = t + 256 * j;
        *reinterpret_cast<uint4 *>(Bs + swz(p >> 3, p & 7)) = wv[j];
    }
    __syncthreads();
    const float *src = in + (size_t)img_lo * C * HW;
    const int count = n * C * HW;
    for (int e = t; e < count; e += 256) {
        const int ic = div_small(e, HW, rHW), rem = e - ic * HW, y = div_small(rem, W, rW), x = rem - y * W;
        Img[ic * PP + (y + 1) * PW + x + 1] = (uint16_t)f2h(src[e]);
    }
    __syncthreads();
    // 3. im2col: thread t builds piece t & 7 (k = 8 (t & 7) .. + 7) of rows (t >> 3) + 32 i
    {
        const int pc = t & 7;
        int koff[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int k = 8 * pc + e, c = (k * 57) >> 9, tap = k - 9 * c, ky = (tap * 11) >> 5, kx = tap - 3 * ky;
            koff[e] = k < K ? c * PP + ky * PW + kx : -1;           // (k * 57) >> 9 == k / 9 for k < 64
        }
#pragma unroll
        for (int i = 0; i < BM / 32; ++i) {
            const int r = (t >> 3) + 32 * i, m = m0 + r;
            uint32_t hv[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
            if (m < M) {
                const int img = m / HW, pos = m - img * HW, oy = div_small(pos, W, rW), ox = pos - oy * W;
                const uint16_t *base = Img + (img - img_lo) * C * PP + oy * PW + ox;
#pragma unroll
                for (int e = 0; e < 8; ++e) hv[e] = koff[e] >= 0 ? (uint32_t)base[koff[e]] : 0u;
            }
            *reinterpret_cast<uint4 *>(As + swz(r, pc)) =
                make_uint4(hv[0] | (hv[1] << 16), hv[2] | (hv[3] << 16), hv[4] | (hv[5] << 16), hv[6] | (hv[7] << 16));
        }
    }
    __syncthreads();
    f16_t acc[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i)
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const h8_t pf = *reinterpret_cast<const h8_t *>(As + swz(wave * 32 + fr, 2 * s + fh));
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            const h8_t wf = *reinterpret_cast<const h8_t *>(Bs + swz(32 * i + fr, 2 * s + fh));
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wf, pf, acc[i], 0, 0, 0);
        }
    }
    // epilogue from registers: acc[i] register 4 gq + e = channel 32 i + 8 gq + 4 fh + e of pixel
    // m0 + 32 wave + fr
    const int m = m0 + wave * 32 + fr;
    if (m < M) {
#pragma unroll
        for (int i = 0; i < NT; ++i)
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                const int n0 = 32 * i + 8 * gq + 4 * fh;
                const uint2 bb = *reinterpret_cast<const uint2 *>(bias + n0);
                const float bv[4] = {h2f(bb.x), h2f(bb.x >> 16), h2f(bb.y), h2f(bb.y >> 16)};
                uint32_t hv[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) hv[e] = f2h(relu_nan(h2f(f2h(h2f(f2h(acc[i][4 * gq + e])) + bv[e]))));
                *reinterpret_cast<uint2 *>(out + (size_t)m * COUT + n0) =
                    make_uint2(hv[0] | (hv[1] << 16), hv[2] | (hv[3] << 16));
            }
    }
}

}  // namespace conv
}  // namespace mapf

using namespace mapf;

extern "C" {

int mapf_conv_nhwc_f16(const uint16_t *x, const uint16_t *w_packed, const uint16_t *bias, uint16_t *y, int64_t nimg,
                       int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t ks, int32_t pad, int32_t relu,
                       void *stream) {
    if (!x || !w_packed || !y || (relu && !bias)) return MAPF_EINVAL;
    if (nimg < 1 || H < 1 || W < 1 || pad < 0 || pad >= ks) return MAPF_EINVAL;
    const int Ho = H + 2 * pad - ks + 1, Wo = W + 2 * pad - ks + 1;
    if (Ho < 1 || Wo < 1) return MAPF_EINVAL;
    const int64_t M64 = nimg * Ho * Wo;
    if (M64 > (int64_t)0x7FFFFFFF - 1024 || nimg * H * W > (int64_t)0x7FFFFFFF / 512) return MAPF_EINVAL;
    const int M = (int)M64, epi = relu ? 1 : 0;
    hipStream_t s = (hipStream_t)stream;
    if (Cin == 128 && Cout == 128 && ks == 3 && conv::launch_img<128, 128, 3, 8>(x, w_packed, bias, y, (int)nimg, H, W, pad, epi, 0, s));
    else if (Cin == 128 && Cout == 256 && ks == 2 && conv::launch_img<128, 256, 2, 8>(x, w_packed, bias, y, (int)nimg, H, W, pad, epi, 0, s));
    else if (Cin == 256 && Cout == 256 && ks == 2 && conv::launch_img<256, 256, 2, 8>(x, w_packed, bias, y, (int)nimg, H, W, pad, epi, 0, s));
    else if (Cin == 128 && Cout == 128 && ks == 3) conv::launch<128, 128, 3, 8>(x, w_packed, bias, y, M, H, W, Ho, Wo, pad, epi, s);
    else if (Cin == 128 && Cout == 256 && ks == 2) conv::launch<128, 256, 2, 8>(x, w_packed, bias, y, M, H, W, Ho, Wo, pad, epi, s);
    else if (Cin == 256 && Cout == 256 && ks == 2) conv::launch<256, 256, 2, 8>(x, w_packed, bias, y, M, H, W, Ho, Wo, pad, epi, s);
    // the data gradient of conv2 (128 -> 256, 2x2): 256 -> 128 over the flipped weight (net._HipConv;
    // MIOpen's backward-data kernel took 174 us for it at 2,048 images, profiles/r06f_update_profile.txt)
    else if (Cin == 256 && Cout == 128 && ks == 2) conv::launch<256, 128, 2, 8>(x, w_packed, bias, y, M, H, W, Ho, Wo, pad, epi, s);
    else return MAPF_EINVAL;
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

int mapf_conv_nhwc_pool_f16(const uint16_t *x, const uint16_t *w_packed, const uint16_t *bias, uint16_t *y, int64_t nimg,
                            int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t ks, int32_t pad, void *stream) {
#if MAPF_CONV_STAGES
    if (!x || !w_packed || !bias || !y) return MAPF_EINVAL;
    if (nimg < 1 || H < 1 || W < 1 || pad < 0 || pad >= ks) return MAPF_EINVAL;
    const int Ho = H + 2 * pad - ks + 1, Wo = W + 2 * pad - ks + 1;
    if (Ho < 2 || Wo < 2) return MAPF_EINVAL;
    const int64_t M64 = nimg * Ho * Wo;
    if (M64 > (int64_t)0x7FFFFFFF - 1024 || nimg * H * W > (int64_t)0x7FFFFFFF / 512) return MAPF_EINVAL;
    const int M = (int)M64;
    hipStream_t s = (hipStream_t)stream;
    // (8 waves for the 128-channel form too: 256-row tiles hold 3 whole 9 x 9 images, 5 % padding)
    if (Cin == 128 && Cout == 128 && ks == 3 && conv::launch_img<128, 128, 3, 8>(x, w_packed, bias, y, (int)nimg, H, W, pad, 0, 1, s));
    else if (Cin == 256 && Cout == 256 && ks == 2 && conv::launch_img<256, 256, 2, 8>(x, w_packed, bias, y, (int)nimg, H, W, pad, 0, 1, s));
    else if (Cin == 128 && Cout == 128 && ks == 3 && Ho * Wo <= conv::Cfg32<128, 128, 3, 8, MAPF_CONV_STAGES>::BM)
        conv::launch<128, 128, 3, 8>(x, w_packed, bias, y, M, H, W, Ho, Wo, pad, 0, s, true);
    else if (Cin == 256 && Cout == 256 && ks == 2 && Ho * Wo <= conv::Cfg32<256, 256, 2, 8, MAPF_CONV_STAGES>::BM)
        conv::launch<256, 256, 2, 8>(x, w_packed, bias, y, M, H, W, Ho, Wo, pad, 0, s, true);
    else return MAPF_EINVAL;
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
#else
    return MAPF_EINVAL;
#endif
}

int mapf_conv_select(int32_t impl) {
    if (impl < 0 || impl > 2) return MAPF_EINVAL;
    conv::g_conv_impl = impl;
    return MAPF_OK;
}

int mapf_conv_first_f32(const float *x_nchw, const uint16_t *w, const uint16_t *bias, uint16_t *y, int64_t nimg,
                        int32_t Cin, int32_t H, int32_t W, int32_t Cout, void *stream) {
    if (!x_nchw || !w || !bias || !y) return MAPF_EINVAL;
    if (nimg < 1 || Cin < 1 || Cin > 7 || H < 1 || W < 1 || Cout != 128) return MAPF_EINVAL;
    const int64_t M64 = nimg * H * W;
    if (M64 > (int64_t)0x7FFFFFFF - 1024) return MAPF_EINVAL;
    const int M = (int)M64;
    const int64_t HW = (int64_t)H * W;
    if ((int64_t)(H + 2) * (W + 2) * Cin > 16384) return MAPF_EINVAL;
    const int64_t nmax = 127 / HW + 2;                 // images one 128-pixel tile can touch
    const size_t lds = (size_t)128 * 128 + (size_t)Cout * 128 + (size_t)(nmax * Cin * (H + 2) * (W + 2) * 2 + 3) / 4 * 4;
    if (lds > 64 * 1024) return MAPF_EINVAL;
    hipLaunchKernelGGL(conv::conv_first_kernel<128>, dim3((M + 127) / 128), dim3(256), lds, (hipStream_t)stream, x_nchw,
                       w, bias, y, M, (int)Cin, (int)H, (int)W, (int)nimg);
    return hipGetLastError() == hipSuccess ? MAPF_OK : MAPF_EDEVICE;
}

}  // extern "C"
