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

// Exclusive scan across a workgroup of NW waves (default 4 = 256 threads).  `tmp` = NW ints
// of LDS.  Every thread must call it (contains barriers).
template <int NW = 4>
__device__ __forceinline__ int block_excl_scan(int v, int* tmp, int& total) {
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    int incl = wave_incl_scan(v);
    if (lane == 63) tmp[wid] = incl;
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        int s = tmp[w];
        base += (w < wid) ? s : 0;
        tot += s;
    }
    __syncthreads();
    total = tot;
    return base + incl - v;
}

template <int NW = 4>
__device__ __forceinline__ int block_sum(int v, int* tmp) {
    int total;
    block_excl_scan<NW>(v, tmp, total);
    return total;
}

}  // namespace orbx

namespace orbx {

// Stage a rows x ndw-dword window (row r at gsrc + r*gpitch, 4-byte aligned rows) into LDS
// (row r at lds + r*lpitch_dw dwords).  Each thread issues up to 8 loads before its first
// LDS store, so a workgroup keeps NT*8 loads in flight instead of one per thread.  Element
// (row, col) indices advance by NT per step incrementally: one division per thread, none
// per element.
template <int NT>
__device__ __forceinline__ void stage_dwords(const uint8_t* __restrict__ gsrc, size_t gpitch,
                                             int rows, int ndw, uint32_t* lds, int lpitch_dw,
                                             int tid) {
    const int n = rows * ndw;
    if (n <= 0) return;
    const int dr = NT / ndw, dc = NT - dr * ndw;
    int r = tid / ndw, c = tid - (tid / ndw) * ndw;
    for (int base = 0; base < n; base += NT * 8) {
        uint32_t v[8];
        int at[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            // unconditional loads (index clamped): a guarded load becomes a branch + vmcnt(0)
            const bool in = base + k * NT + tid < n;
            const int ra = in ? r : rows - 1, ca = in ? c : ndw - 1;
            v[k] = *(const uint32_t*)(gsrc + (size_t)ra * gpitch + 4 * ca);
            at[k] = in ? ra * lpitch_dw + ca : -1;
            c += dc;
            r += dr;
            if (c >= ndw) { c -= ndw; ++r; }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (at[k] >= 0) lds[at[k]] = v[k];
    }
}

// Same for an arbitrary byte window (no alignment), 16 loads in flight per thread.
template <int NT>
__device__ __forceinline__ void stage_bytes(const uint8_t* __restrict__ gsrc, size_t gpitch,
                                            int rows, int cols, uint8_t* lds, int lpitch,
                                            int tid) {
    const int n = rows * cols;
    if (n <= 0) return;
    const int dr = NT / cols, dc = NT - dr * cols;
    int r = tid / cols, c = tid - (tid / cols) * cols;
    for (int base = 0; base < n; base += NT * 16) {
        uint8_t v[16];
        int at[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const bool in = base + k * NT + tid < n;
            const int ra = in ? r : rows - 1, ca = in ? c : cols - 1;
            v[k] = gsrc[(size_t)ra * gpitch + ca];
            at[k] = in ? ra * lpitch + ca : -1;
            c += dc;
            r += dr;
            if (c >= cols) { c -= cols; ++r; }
        }
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (at[k] >= 0) lds[at[k]] = v[k];
    }
}

}  // namespace orbx
