// primal-ppo_amd/csrc/mapf_diag.h -- profiling hooks of the diagnostic build.
//
// The product build (make) compiles every hook below to nothing.  `make stamps`
// (-DMAPF_STAMPS) builds ../lib/libmapf_stamps.so, whose kernels record phase
// cycles per wave and a per-workgroup timeline (tools/stamps.py, tools/timeline.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mapf {

// In-kernel phase stamps (diagnostic build only, -DMAPF_STAMPS): lane 0 of
// every wave adds the s_memtime delta of each phase into prof[k]; prof[15]
// counts the waves.  The product build compiles them out.
__device__ inline uint64_t stamp_now() {
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
__device__ inline uint64_t stamp_rt() {   // constant-rate 100 MHz counter
    uint64_t t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
#ifdef MAPF_STAMPS
// per-wave phase deltas kept in registers, one plain store per phase at the end
// (prof[wave * 8 + k]; no atomics, so the stamps do not contend)
#define STAMP_BEGIN() uint64_t _stamp_prev = stamp_now(); uint64_t _stamp_d[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define STAMP(k) do { __builtin_amdgcn_sched_barrier(0); const uint64_t _t = stamp_now(); \
    _stamp_d[k] += _t - _stamp_prev; _stamp_prev = _t; __builtin_amdgcn_sched_barrier(0); } while (0)
#define STAMP_END() do { if ((threadIdx.x & 63) == 0) { \
    const size_t _w = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; \
    if (_w < 65536) { for (int _k = 0; _k < 7; ++_k) e.prof[_w * 8 + _k] = _stamp_d[_k]; e.prof[_w * 8 + 7] = 1; } } } while (0)
// block timeline (fused kernel): thread 0 of block k writes the constant-rate
// (100 MHz) realtime counter of event t to prof[PROF_TL + k * 8 + t]; slot 6 =
// HW_ID, slot 7 = XCC_ID of the block's CU.
// (not in the wide rollout's unit, MAPF_WIDE_TU: its WSTAMP rows share that region)
#ifdef MAPF_WIDE_TU
#define TL_STAMP(t) do { } while (0)
#else
#define TL_STAMP(t) do { if (threadIdx.x == 0 && blockIdx.x < PROF_TL_BLOCKS) { uint64_t _r; \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_r)::"memory"); \
    e.prof[PROF_TL + (size_t)blockIdx.x * 8 + (t)] = _r; } } while (0)
#endif
#define TL_HWID() do { if (threadIdx.x == 0 && blockIdx.x < PROF_TL_BLOCKS) { uint32_t _h, _x; \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(_h)); \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(_x)); \
    e.prof[PROF_TL + (size_t)blockIdx.x * 8 + 6] = _h; e.prof[PROF_TL + (size_t)blockIdx.x * 8 + 7] = _x; } } while (0)
// wide rollout kernel: phase time (100 MHz ticks) per env summed over the launch's steps, written to
// prof[PROF_TL + row * 8 + k] (k < 6; slot 7 = 1) by lane 0 of env b's first wave (row b) and, in
// the pipelined form, of its observing wave (row B + b)
// (slot 4 = the wave's start, slot 5 = its end on the realtime counter, slot 6 = HW_ID | XCC_ID << 32)
#define WSTAMP_BEGIN() uint64_t _w_prev = stamp_rt(); uint64_t _w_d[6] = {0, 0, 0, 0, _w_prev, 0}
#define WSTAMP(k) do { __builtin_amdgcn_sched_barrier(0); const uint64_t _t = stamp_rt(); \
    _w_d[k] += _t - _w_prev; _w_prev = _t; __builtin_amdgcn_sched_barrier(0); } while (0)
#define WSTAMP_END(b, r) do { const size_t _row = (size_t)(b) + (size_t)(r) * (size_t)e.B; \
    if ((threadIdx.x & 63) == 0 && _row < PROF_TL_BLOCKS) { \
    uint32_t _h, _x; _w_d[5] = stamp_rt(); \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(_h)); \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(_x)); \
    for (int _k = 0; _k < 6; ++_k) e.prof[PROF_TL + _row * 8 + _k] = _w_d[_k]; \
    e.prof[PROF_TL + _row * 8 + 6] = (uint64_t)_h | ((uint64_t)_x << 32); \
    e.prof[PROF_TL + _row * 8 + 7] = 1; } } while (0)
// pair-lane rollout kernel: each env wave's start / end (realtime) and HW_ID | XCC_ID << 32 in
// prof[(RSTAMP_ROW0 + b) * 8 + 4..6], slot 7 = 1 (rows above the step kernels' per-wave rows)
constexpr size_t RSTAMP_ROW0 = 32768;
#define RSTAMP_BEGIN() const uint64_t _r_start = stamp_rt()
#define RSTAMP_END(b) do { if ((threadIdx.x & 63) == 0 && (size_t)(b) < RSTAMP_ROW0) { \
    uint32_t _h, _x; const uint64_t _r_end = stamp_rt(); \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(_h)); \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(_x)); \
    unsigned long long *_p = e.prof + (RSTAMP_ROW0 + (size_t)(b)) * 8; \
    _p[4] = _r_start; _p[5] = _r_end; _p[6] = (uint64_t)_h | ((uint64_t)_x << 32); _p[7] = 1; } } while (0)
#else
#define RSTAMP_BEGIN() do { } while (0)
#define RSTAMP_END(b) do { } while (0)
#define WSTAMP_BEGIN() do { } while (0)
#define WSTAMP(k) do { } while (0)
#define WSTAMP_END(b, r) do { } while (0)
#define TL_STAMP(t) do { } while (0)
#define TL_HWID() do { } while (0)
#define STAMP_BEGIN() do { } while (0)
#define STAMP(k) do { } while (0)
#define STAMP_END() do { } while (0)
#endif

}  // namespace mapf
