// tools/fetch_calib.hip -- calibrate rocprofv3's FETCH_SIZE for the c5 BFS-channel read pattern
// (the guide's x2 correction is for 16-B/lane streaming reads only).
//
//   hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d OUT -o run -- tools/fetch_calib
//
// Two kernels over buffers far larger than the 256 MiB Infinity Cache, each launched once on cold
// data:
//   stream_kernel   16 B per lane, fully coalesced, over 1 GiB (the guide's reference: FETCH = bytes / 2)
//   window_kernel   the rollout kernels' BFS-channel reads (csrc/mapf_observe.h, phase 2, C = 7):
//                   B envs x N agents, agent maps [H/8][W/8][8][8] int16 (bfs_at), one lane per
//                   (agent, FOV row) task reading the row's window as aligned dwords from column
//                   tc & ~1 (ceil((F+1)/2) of them) plus the agent's own cell -- the same addresses
//                   as the kernel for the same seeded positions
// The host counts, for exactly those addresses, the algorithmic bytes (F*F*2 + 2 per agent), the
// distinct 32-, 64- and 128-B blocks touched, and prints them as JSON; FETCH_SIZE per dispatch
// (from the rocprofv3 csv) divided by each gives the calibration.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

#define CHK(x)                                                                                  \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

__host__ __device__ inline int tw(int W) { return (W + 7) >> 3; }
__host__ __device__ inline size_t cells(int H, int W) { return (size_t)((H + 7) >> 3) * tw(W) * 64; }
__host__ __device__ inline int at(int W, int r, int c) {
    return ((((r >> 3) * tw(W)) + (c >> 3)) << 6) | ((r & 7) << 3) | (c & 7);
}

__global__ __launch_bounds__(256) void stream_kernel(const uint4 *__restrict__ x, size_t n16, uint32_t *out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = x[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// one wave per env; pos[b][k] = r | c << 16 (in-map cells)
__global__ __launch_bounds__(64) void window_kernel(const int16_t *__restrict__ bfs, const uint32_t *__restrict__ pos,
                                                    int N, int H, int W, int F, uint32_t *out) {
    const int b = blockIdx.x, lane = threadIdx.x;
    const size_t bc = cells(H, W);
    const int half = F / 2, cmax = tw(W) * 8 - 2;
    uint32_t acc = 0;
    for (int task = lane; task < N * F; task += 64) {
        const int k = task / F, x = task - k * F;
        const uint32_t p = pos[(size_t)b * N + k];
        const int pr = (int)(p & 0xFFFF), pc = (int)(p >> 16);
        const int rr = pr - half + x, tc = pc - half;
        if (rr < 0 || rr >= H) continue;
        const int16_t *bm = bfs + ((size_t)b * N + k) * bc;
        acc += (uint32_t)bm[at(W, pr, pc)];
        const int c0 = tc & ~1;
        uint32_t wv[9];
#pragma unroll
        for (int w = 0; w < 9; ++w)
            if (2 * w < F + 1) wv[w] = *reinterpret_cast<const uint32_t *>(bm + at(W, rr, min(max(c0 + 2 * w, 0), cmax)));
#pragma unroll
        for (int w = 0; w < 9; ++w)
            if (2 * w < F + 1) acc ^= wv[w];
    }
    if (acc == 0x12345678u) out[b] = acc;
}

int main(int argc, char **argv) {
    const int B = argc > 1 ? std::atoi(argv[1]) : 2048, N = 64, H = 80, W = 80, F = 11;
    const size_t bc = cells(H, W);
    const size_t map_bytes = (size_t)B * N * bc * 2;
    int16_t *d_bfs;
    uint32_t *d_pos, *d_out;
    CHK(hipMalloc(&d_bfs, map_bytes));
    CHK(hipMemset(d_bfs, 1, map_bytes));
    std::vector<uint32_t> pos((size_t)B * N);
    uint64_t s = 12345;
    auto rnd = [&](int n) { s = s * 6364136223846793005ull + 1442695040888963407ull; return (int)((s >> 33) % n); };
    for (auto &p : pos) p = (uint32_t)rnd(H) | ((uint32_t)rnd(W) << 16);
    CHK(hipMalloc(&d_pos, pos.size() * 4));
    CHK(hipMemcpy(d_pos, pos.data(), pos.size() * 4, hipMemcpyHostToDevice));
    CHK(hipMalloc(&d_out, (size_t)B * 4));
    // host: the addresses window_kernel reads
    std::set<uint64_t> b32, b64, b128;
    double alg = 0, dw = 0;
    const int half = F / 2, cmax = tw(W) * 8 - 2;
    for (int b = 0; b < B; ++b)
        for (int k = 0; k < N; ++k) {
            const int pr = (int)(pos[(size_t)b * N + k] & 0xFFFF), pc = (int)(pos[(size_t)b * N + k] >> 16);
            const uint64_t base = ((uint64_t)b * N + k) * bc * 2;
            alg += F * F * 2 + 2;
            for (int x = 0; x < F; ++x) {
                const int rr = pr - half + x, tc = pc - half;
                if (rr < 0 || rr >= H) continue;
                std::vector<uint64_t> addrs{base + 2 * (uint64_t)at(W, pr, pc)};
                const int c0 = tc & ~1;
                for (int w = 0; 2 * w < F + 1; ++w) addrs.push_back(base + 2 * (uint64_t)at(W, rr, std::min(std::max(c0 + 2 * w, 0), cmax)));
                for (uint64_t a : addrs) {
                    b32.insert(a >> 5);
                    b64.insert(a >> 6);
                    b128.insert(a >> 7);
                    dw += 4;
                }
            }
        }
    // 1 GiB stream, cold: touch a 2 GiB scratch in between to evict the Infinity Cache
    const size_t sbytes = (size_t)1 << 30;
    uint4 *d_s, *d_evict;
    CHK(hipMalloc(&d_s, sbytes));
    CHK(hipMalloc(&d_evict, 2 * sbytes));
    CHK(hipMemset(d_s, 2, sbytes));
    CHK(hipMemset(d_evict, 3, 2 * sbytes));
    CHK(hipDeviceSynchronize());
    hipLaunchKernelGGL(stream_kernel, dim3(4096), dim3(256), 0, 0, d_s, sbytes / 16, d_out);
    CHK(hipMemset(d_evict, 4, 2 * sbytes));
    hipLaunchKernelGGL(window_kernel, dim3(B), dim3(64), 0, 0, d_bfs, d_pos, N, H, W, F, d_out);
    CHK(hipDeviceSynchronize());
    std::printf("{\"stream_kernel_bytes\": %zu, \"window_kernel\": {\"envs\": %d, \"agents\": %d, \"grid\": [%d, %d], "
                "\"fov\": %d, \"algorithmic_bytes\": %.0f, \"dword_bytes_requested\": %.0f, \"blocks32_bytes\": %zu, "
                "\"blocks64_bytes\": %zu, \"blocks128_bytes\": %zu, \"map_bytes\": %zu}}\n",
                sbytes, B, N, H, W, F, alg, dw, b32.size() * 32, b64.size() * 64, b128.size() * 128, map_bytes);
    return 0;
}
