// primal-ppo_amd/csrc/mapf_observe.hip -- getAllObservations for B envs
// (mapf_gym.py:246-336); the per-workgroup work is in mapf_observe.h.
#include "mapf_common.h"
#include "mapf_kernels.h"
#include "mapf_observe.h"
#include "mapf_search.h"

namespace mapf {

// The first `nsearch` workgroups run the step's search work (agent BFS maps,
// humans' next paths -- mapf_search.h), the rest write observations: the
// latency-bound searches hide under the HBM-bound observation stores.
// Only the narrow-row search (W <= 32, H <= 64: configs c1-c3) is hosted: its
// register footprint matches the observation role's; wider grids search in
// their own launch so the observation workgroups keep their occupancy.
template <bool HOST>
__global__ __launch_bounds__(256) void observe_kernel(DevEnv e, float *__restrict__ obs, float *__restrict__ vec,
                                                      int nsearch, int parity) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    TL_STAMP(0);
    TL_HWID();
    if constexpr (HOST) {
        if ((int)blockIdx.x < nsearch) {
            const int wave = threadIdx.x >> 6;
            char *lds = smem + (size_t)wave * srch::wave_lds<uint32_t, 1>(e.H, e.W);
            srch::search_items<uint32_t, 1>(e, parity, 0, lds, blockIdx.x * (blockDim.x >> 6) + wave,
                                            nsearch * (blockDim.x >> 6));
            return;
        }
    } else {
        nsearch = 0;
    }
    const int E = e.obs_envs;
    const int b0 = ((int)blockIdx.x - nsearch) * E;
    const int nenv = min(E, e.B - b0);
    ObsLds L = obs_layout(e, E, smem);
    float4 *lut = reinterpret_cast<float4 *>(smem + ((obs_lds_bytes(e, E) + 15) & ~(size_t)15));
    obs_lut_init(lut);              // ordered before use by the barrier below
    L.lut = lut;
    obs_init(e, L, E, b0, nenv, obs_map_word(e, b0, nenv, threadIdx.x));
    obs_load_agents(e, L, b0, nenv);
    TL_STAMP(1);
    __syncthreads();
    TL_STAMP(2);
    obs_emit(e, L, obs, vec, obs_workgroup(L, nenv), b0);
    TL_STAMP(3);
}

// BFS channel (ch 6, C = 7) of the agents whose map the step's search rewrote
// (bfs_list[parity]).  The search runs concurrently with the observe launch
// (mapf_observe forks it onto a second stream), so the observe launch read
// those agents' maps while they were being written; after the join this
// launch rewrites exactly their channel 6 from the new maps -- the same
// expression as obs_emit's.  One wave per listed agent, grid-strided.
__global__ __launch_bounds__(256) void bfs_fixup_kernel(DevEnv e, int parity, float *__restrict__ obs) {
    const uint32_t n = e.counters[C_BFS_COUNT + parity];
    const int lane = lane_id(), F = e.F, FF = F * F, half = F / 2;
    const uint32_t nw = gridDim.x * (blockDim.x >> 6);
    for (uint32_t item = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); item < n; item += nw) {
        const uint32_t ai = e.bfs_list[(size_t)parity * e.B * e.N + item];
        const uint32_t p = e.pos[ai];
        const int pr = prow(p), pc = pcol(p);
        const int16_t *bm = e.bfs + (size_t)ai * bfs_cells(e.H, e.W);
        const int own = bm[bfs_at(e.W, pr, pc)];
        float *o = obs + (size_t)ai * e.C * FF + 6 * FF;
        for (int q = lane; q < FF; q += 64) {
            const int rr = pr - half + q / F, cc = pc - half + q % F;
            float v = 0.f;
            if (own >= 0 && rr >= 0 && rr < e.H && cc >= 0 && cc < e.W) {
                const int d = bm[bfs_at(e.W, rr, cc)];
                if (d >= 0 && d < own) v = 1.f;
            }
            o[q] = v;
        }
    }
}

void launch_bfs_fixup(const DevEnv &e, int parity, float *obs, hipStream_t s) {
    hipLaunchKernelGGL(bfs_fixup_kernel, dim3(64), dim3(256), 0, s, e, parity, obs);
}

size_t observe_lds(const DevEnv &e) { return ((obs_lds_bytes(e, e.obs_envs) + 15) & ~(size_t)15) + 256; }   // + nibble table

bool observe_hosts_search(const DevEnv &e) { return e.W <= 32 && e.H <= 64; }

void launch_observe(const DevEnv &e, float *obs, float *vec, int nsearch, int parity, hipStream_t s) {
    if (!observe_hosts_search(e)) nsearch = 0;
    const int grid = (e.B + e.obs_envs - 1) / e.obs_envs + nsearch;
    size_t lds = observe_lds(e);
    if (nsearch > 0) {
        const size_t sl = 4 * srch::wave_lds<uint32_t, 1>(e.H, e.W);
        if (sl > lds) lds = sl;
        hipLaunchKernelGGL(observe_kernel<true>, dim3(grid), dim3(256), lds, s, e, obs, vec, nsearch, parity);
    } else {
        hipLaunchKernelGGL(observe_kernel<false>, dim3(grid), dim3(256), lds, s, e, obs, vec, 0, parity);
    }
}

}  // namespace mapf
