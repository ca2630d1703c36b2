// primal-ppo_amd/csrc/mapf_search.hip -- standalone search launch and the
// human path planner.
//
// The search work of a step (agent BFS maps, the humans' next paths) normally
// rides inside the observe launch (mapf_observe.hip: extra workgroups beside
// the HBM-bound observation writes).  This file holds the standalone form
// (resets, num_channel 7 whose BFS channel needs the maps before observing,
// and a step followed by another step without an observe in between), and
// plan_kernel, which (re)derives each human's next-path endpoints from the
// state (reset, mapf_set_state).
#include "mapf_group.h"
#include "mapf_kernels.h"
#include "mapf_search.h"

namespace mapf {

template <class T, int RW>
__global__ __launch_bounds__(256) void search_kernel(DevEnv e, int parity, int all) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int wave = threadIdx.x >> 6;
    char *lds = smem + (size_t)wave * srch::wave_lds<T, RW>(e.H, e.W);
    srch::search_items<T, RW>(e, parity, all, lds, blockIdx.x * (blockDim.x >> 6) + wave, gridDim.x * (blockDim.x >> 6));
}

// promote = 1: the path just searched into buffer hcur^1 becomes current (reset).
// Then every env plans its next path from (clock, hlen, hstep): the end-step of
// the current path has clock + len - 1 - hstep (plan_next_path).
__global__ __launch_bounds__(256) void plan_kernel(DevEnv e, int promote) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= e.B) return;
    int cur = e.hcur[b];
    if (promote) {
        cur ^= 1;
        e.hcur[b] = cur;
        e.hstep[b] = 0;
    }
    const uint32_t *path = human_path(e, b, cur);
    const int L = e.hlen[b * 2 + cur], hs = e.hstep[b];
    e.hpos[b] = path[hs];
    e.hnext[b] = path[hs + 1 < L ? hs + 1 : L - 1];
    uint32_t ns, ng;
    const uint32_t epoch = e.clock[b] + (uint32_t)(L - 1 - hs);
    plan_next_path(e, b, e.env_offset + (uint32_t)b, epoch, e.hseq_idx[b], ns, ng, true);
    e.hnext_start[b] = ns;
    e.hnext_goal[b] = ng;
}

template <class T, int RW>
static void launch_search_t(const DevEnv &e, int parity, int all, hipStream_t s) {
    const size_t lds = 4 * srch::wave_lds<T, RW>(e.H, e.W);
    const long items = (long)e.B + (e.keep_bfs ? (long)e.B * e.N : 0);
    long grid = (items + 3) / 4;
    const long cap = (all == 1 || all == 2) ? 8192 : 128;
    if (grid > cap) grid = cap;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL((search_kernel<T, RW>), dim3((unsigned)grid), dim3(256), lds, s, e, parity, all);
}

void launch_search(const DevEnv &e, int parity, int all, hipStream_t s) {
    const bool two = e.H > 64;
    if (e.W <= 32) {
        if (two) launch_search_t<uint32_t, 2>(e, parity, all, s); else launch_search_t<uint32_t, 1>(e, parity, all, s);
    } else if (e.W <= 64) {
        if (two) launch_search_t<uint64_t, 2>(e, parity, all, s); else launch_search_t<uint64_t, 1>(e, parity, all, s);
    } else {
        if (two) launch_search_t<srch::Row2, 2>(e, parity, all, s); else launch_search_t<srch::Row2, 1>(e, parity, all, s);
    }
}

// the tiled maps (bfs_at) as row-major [B*N][H][W] int16
__global__ __launch_bounds__(256) void bfs_export_kernel(DevEnv e, int16_t *__restrict__ dist) {
    const size_t HW = (size_t)e.H * e.W, n = (size_t)e.B * e.N * HW, bc = bfs_cells(e.H, e.W);
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t ai = i / HW;
        const int cell = (int)(i - ai * HW), r = cell / e.W, c = cell - r * e.W;
        dist[i] = e.bfs[ai * bc + bfs_at(e.W, r, c)];
    }
}

void launch_bfs_export(const DevEnv &e, int16_t *dist, hipStream_t s) {
    const size_t n = (size_t)e.B * e.N * e.H * e.W;
    size_t grid = (n + 255) / 256;
    if (grid > 16384) grid = 16384;
    hipLaunchKernelGGL(bfs_export_kernel, dim3((unsigned)grid), dim3(256), 0, s, e, dist);
}

void launch_plan(const DevEnv &e, int promote, hipStream_t s) {
    hipLaunchKernelGGL(plan_kernel, dim3((e.B + 255) / 256), dim3(256), 0, s, e, promote);
}

}  // namespace mapf
