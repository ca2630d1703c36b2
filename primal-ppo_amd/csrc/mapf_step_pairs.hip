// primal-ppo_amd/csrc/mapf_step_pairs.hip -- launcher of the pair-lane step
// (N <= 8 agents per env; the env's work is step_pairs_env, mapf_step_pairs.h).
#include "mapf_step_pairs.h"

namespace mapf {

template <int NP>
__global__ __launch_bounds__(256) void step_pairs_kernel(DevEnv e, int32_t *__restrict__ actions, StepOut out,
                                                         uint32_t flags, int slot) {
    PairsDeferred dfr;
    step_pairs_env<NP, false>(e, actions, out, flags, slot, blockIdx.x * blockDim.x + threadIdx.x, ObsLds{}, 0,
                              RegMap{0u, false}, dfr);
    step_pairs_finish(e, dfr, slot);
}

bool launch_step_pairs(const DevEnv &e, int32_t *actions, const StepOut &out, uint32_t flags, int slot,
                       hipStream_t s) {
    const int np = e.G;
    if (np > 8) return false;
    const long threads = (long)e.B * np * np;
    const int blk = e.step_block;
    const int grid = (int)((threads + blk - 1) / blk);
    switch (np) {
        case 1: hipLaunchKernelGGL(step_pairs_kernel<1>, dim3(grid), dim3(blk), 0, s, e, actions, out, flags, slot); break;
        case 2: hipLaunchKernelGGL(step_pairs_kernel<2>, dim3(grid), dim3(blk), 0, s, e, actions, out, flags, slot); break;
        case 4: hipLaunchKernelGGL(step_pairs_kernel<4>, dim3(grid), dim3(blk), 0, s, e, actions, out, flags, slot); break;
        default: hipLaunchKernelGGL(step_pairs_kernel<8>, dim3(grid), dim3(blk), 0, s, e, actions, out, flags, slot); break;
    }
    return true;
}

}  // namespace mapf
