// orbx_device.h — wave64 / workgroup helpers for the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace orbx {

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Number of set bits of `mask` below this lane (v_mbcnt_lo/hi).
__device__ __forceinline__ int lanes_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}

__device__ __forceinline__ int wave_incl_scan(int v) {
    const int lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// Exclusive scan across a 256-thread workgroup (4 waves).  `tmp` = 4 ints of LDS.
// Every thread must call it (contains barriers).
__device__ __forceinline__ int block_excl_scan(int v, int* tmp, int& total) {
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    int incl = wave_incl_scan(v);
    if (lane == 63) tmp[wid] = incl;
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        int s = tmp[w];
        base += (w < wid) ? s : 0;
        tot += s;
    }
    __syncthreads();
    total = tot;
    return base + incl - v;
}

__device__ __forceinline__ int block_sum(int v, int* tmp) {
    int total;
    block_excl_scan(v, tmp, total);
    return total;
}

}  // namespace orbx
