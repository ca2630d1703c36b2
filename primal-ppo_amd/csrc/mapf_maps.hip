// primal-ppo_amd/csrc/mapf_maps.hip -- obstacle maps on the device.
//
// Generators, one workgroup per map, int8 [nmaps][H][W] (0 free, -1 obstacle):
//  * warehouse: MapfGym()'s map (mapf_gym.py:166 -> generateWarehouse(num_block=
//    WORLD_SIZE), map_generator.py:127-138).  Length L uniform in [lo, hi]
//    (np.random.randint(lo, hi + 1) there; a Philox draw here), breadth
//    int(L / (2/3)), int((breadth * (1 - 1/3)) / 6) shelves of 5 cells on every
//    odd row 1..L-2 from column int((breadth - shelves * 6) / 2) -- the same
//    float64 expressions, so the map of a given L is the reference's bit for bit.
//    Placed at the top-left of the H x W stack, the rest obstacle (the padding
//    of maps.random_warehouse_batch: off-map and padding read alike).
//  * random: random_generator's rule -(rand < p) (map_generator.py:23) over the
//    whole H x W, one Philox word per cell.
//  * largest component (config c5): free cells outside the largest 4-connected
//    free component become obstacles -- spawns, goals and the human then always
//    have a path (astar_4 returns a ValueError otherwise, astar_4.py:109).  Label
//    propagation in LDS (min cell index per component, with pointer jumping),
//    sizes by LDS atomics, ties to the component whose first cell comes first in
//    raster order (scipy.ndimage.label's order: maps.keep_largest_component).
// Then the env's padded obstacle bitmaps and static-action masks are built from
// the int8 maps on the device (also for maps uploaded by mapf_reset).
//
// Philox (key = seed): warehouse length (env, P_MAPGEN, epoch, 0).x; random cell
// q: word q & 3 of (env, P_MAPGEN | 1 << 8, epoch, q >> 2), obstacle iff
// word * 2^-32 < p in float64.  oracle/mapf_oracle.c oc_gen_* restate both.
#include "mapf_kernels.h"

namespace mapf {

__device__ inline void warehouse_shape(int L, int &breadth, int &shelves, int &free0) {
    const double lb = 2.0 / 3.0, fs = 1.0 / 3.0;
    breadth = (int)((double)L / lb);
    shelves = (int)(((double)breadth * (1.0 - fs)) / 6.0);
    free0 = (int)((double)(breadth - shelves * 6) / 2.0);
}

__global__ __launch_bounds__(256) void mapgen_kernel(DevEnv e, MapGen g, int8_t *maps) {
    const int m = blockIdx.x;
    const uint32_t env_id = e.env_offset + (uint32_t)m;
    int8_t *out = maps + (size_t)m * e.H * e.W;
    const int cells = e.H * e.W;
    if (g.kind == 0) {
        const uint32_t span = (uint32_t)(g.hi - g.lo + 1);
        const int L = g.lo + (int)__umulhi(philox(env_id, P_MAPGEN, g.epoch, 0u, g.seed).x, span);
        int breadth, shelves, free0;
        warehouse_shape(L, breadth, shelves, free0);
        for (int q = threadIdx.x; q < cells; q += blockDim.x) {
            const int r = q / e.W, c = q % e.W;
            bool ob = r >= L || c >= breadth;
            if (!ob && (r & 1) && r <= L - 2 && c >= free0 && c < free0 + shelves * 6 && (c - free0) % 6 < 5) ob = true;
            out[q] = ob ? (int8_t)-1 : (int8_t)0;
        }
    } else {
        const double p = (double)g.density;
        for (int q = threadIdx.x; q < cells; q += blockDim.x) {
            const u32x4 o = philox(env_id, P_MAPGEN | (1u << 8), g.epoch, (uint32_t)(q >> 2), g.seed);
            const uint32_t w = (q & 3) == 0 ? o.x : (q & 3) == 1 ? o.y : (q & 3) == 2 ? o.z : o.w;
            out[q] = ((double)w * 0x1p-32 < p) ? (int8_t)-1 : (int8_t)0;
        }
    }
}

// one workgroup of 1024 threads per map, H * W <= LC_MAX_CELLS (uint16 labels, uint32 sizes)
__global__ __launch_bounds__(1024) void largest_component_kernel(DevEnv e, int8_t *maps) {
    __shared__ uint16_t lab[LC_MAX_CELLS];
    __shared__ uint32_t cnt[LC_MAX_CELLS];
    __shared__ uint32_t best;
    const int H = e.H, W = e.W, cells = H * W;
    int8_t *mp = maps + (size_t)blockIdx.x * cells;
    constexpr uint16_t OB = 0xFFFF;
    for (int q = threadIdx.x; q < cells; q += blockDim.x) {
        lab[q] = mp[q] == 0 ? (uint16_t)q : OB;
        cnt[q] = 0;
    }
    if (threadIdx.x == 0) best = 0;
    __syncthreads();
    for (;;) {
        int changed = 0;
        for (int q = threadIdx.x; q < cells; q += blockDim.x) {
            const uint16_t l0 = lab[q];
            if (l0 == OB) continue;
            const int r = q / W, c = q % W;
            uint16_t m = l0;
            if (r > 0) { const uint16_t v = lab[q - W]; if (v < m) m = v; }
            if (r + 1 < H) { const uint16_t v = lab[q + W]; if (v < m) m = v; }
            if (c > 0) { const uint16_t v = lab[q - 1]; if (v < m) m = v; }
            if (c + 1 < W) { const uint16_t v = lab[q + 1]; if (v < m) m = v; }
            const uint16_t j = lab[m];          // pointer jumping: m's own label is <= m
            if (j < m) m = j;
            if (m < l0) { lab[q] = m; changed = 1; }
        }
        if (!__syncthreads_or(changed)) break;
    }
    for (int q = threadIdx.x; q < cells; q += blockDim.x)
        if (lab[q] != OB) atomicAdd(&cnt[lab[q]], 1u);
    __syncthreads();
    for (int q = threadIdx.x; q < cells; q += blockDim.x)
        if (cnt[q]) atomicMax(&best, (cnt[q] << 16) | (0xFFFFu - (uint32_t)q));
    __syncthreads();
    const uint16_t keep = (uint16_t)(0xFFFFu - (best & 0xFFFFu));
    for (int q = threadIdx.x; q < cells; q += blockDim.x)
        if (lab[q] != OB && lab[q] != keep) mp[q] = -1;
}

// padded obstacle bitmap words (one thread per word) and per-cell static-action masks
__global__ __launch_bounds__(256) void build_bits_kernel(DevEnv e, const int8_t *maps, uint32_t *bits, int nmaps) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t per = (size_t)e.Hp * e.WW;
    if (t >= per * nmaps) return;
    const int m = (int)(t / per), r = (int)((t % per) / e.WW), w = (int)(t % e.WW);
    const int8_t *mp = maps + (size_t)m * e.H * e.W;
    uint32_t word = 0;
    for (int k = 0; k < 32; ++k) {
        const int mr = r - e.P, mc = w * 32 + k - e.P;
        const bool ob = mr < 0 || mr >= e.H || mc < 0 || mc >= e.W || mp[mr * e.W + mc] != 0;
        word |= (uint32_t)ob << k;
    }
    bits[t] = word;
}

// getInvalidActions' static list (mapf_gym.py:349-352) of every cell
__global__ __launch_bounds__(256) void build_smask_kernel(DevEnv e, const int8_t *maps, uint8_t *smask, int nmaps) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t cells = (size_t)e.H * e.W;
    if (t >= cells * nmaps) return;
    const int8_t *mp = maps + (t / cells) * cells;
    const int r = (int)((t % cells) / e.W), c = (int)(t % e.W);
    uint8_t mk = 0;
    for (int a = 0; a < NA; ++a) {
        const int rr = r + dr(a), cc = c + dc(a);
        if (rr < 0 || rr >= e.H || cc < 0 || cc >= e.W || mp[rr * e.W + cc] != 0) mk |= (uint8_t)(1u << a);
    }
    smask[t] = mk;
}

void launch_mapgen(const DevEnv &e, const MapGen &g, int8_t *maps, hipStream_t s) {
    const int nmaps = e.shared_map ? 1 : e.B;
    hipLaunchKernelGGL(mapgen_kernel, dim3(nmaps), dim3(256), 0, s, e, g, maps);
    if (g.largest) hipLaunchKernelGGL(largest_component_kernel, dim3(nmaps), dim3(1024), 0, s, e, maps);
}

void launch_build_maps(const DevEnv &e, const int8_t *maps, hipStream_t s) {
    const int nmaps = e.shared_map ? 1 : e.B;
    const size_t words = (size_t)nmaps * e.Hp * e.WW, cells = (size_t)nmaps * e.H * e.W;
    hipLaunchKernelGGL(build_bits_kernel, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, s, e, maps,
                       const_cast<uint32_t *>(e.map_bits), nmaps);
    hipLaunchKernelGGL(build_smask_kernel, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, s, e, maps,
                       const_cast<uint8_t *>(e.smask), nmaps);
}

}  // namespace mapf
