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
