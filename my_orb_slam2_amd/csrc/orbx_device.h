// orbx_device.h — wave64 / workgroup helpers for the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace orbx {
#define ORBX_XCD_REMAP 1
// Logical (x, y) block of a 2-D grid.  Consecutive linear blocks are dealt round-robin over
// the 8 XCDs (MI355X_MICROARCH.md §Workgroup dispatch: blocks b and b + 8 share an XCD), so
// linear block L runs logical block (L mod 8) * n/8 + L / 8: every XCD walks a contiguous
// eighth of the logical order, and blocks that share halo rows, patches or an image share
// that XCD's L2.  Results never depend on the mapping.
__device__ __forceinline__ void xcd_block(int& bx, int& by) {
    const uint32_t gx = gridDim.x, n = gx * gridDim.y;
    uint32_t L = blockIdx.y * gx + blockIdx.x;
    if (ORBX_XCD_REMAP && (n & 7u) == 0) L = (L & 7u) * (n >> 3) + (L >> 3);
    by = (int)(L / gx);
    bx = (int)(L - (uint32_t)by * gx);
}


__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Number of set bits of `mask` below this lane (v_mbcnt_lo/hi).
__device__ __forceinline__ int lanes_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
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

// An explicit s_waitcnt vmcnt(0) (expcnt / lgkmcnt left at their maxima).  The staging loops
// below wait for their loads only inside the guarded LDS stores, so on the path that skips a
// store the compiler's wait analysis still counts that load as pending, and it then inserts
// a vmcnt(0) at the next use of the register anywhere downstream -- for k_fast that was the
// head of the compass loop, which drained the next cell's prefetch on every iteration.
// Waiting once here (every load has landed by now anyway) clears that state.
__device__ __forceinline__ void vmem_drained() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// Stage a rows x ndw-dword window (row r at gsrc + r*gpitch, 4-byte aligned rows) into LDS
// (row r at lds + r*lpitch_dw dwords).  Each thread issues up to 8 loads before its first
// LDS store, so a workgroup keeps NT*8 loads in flight instead of one per thread.  The
// element position, its 32-bit source offset and its LDS index advance by NT elements
// incrementally: one division per thread, no multiply per element (a 64-bit or 32-bit
// v_mul is a quarter-rate instruction).
template <int NT>
__device__ __forceinline__ void stage_dwords(const uint8_t* __restrict__ gsrc, size_t gpitch,
                                             int rows, int ndw, uint32_t* lds, int lpitch_dw,
                                             int tid) {
    const int n = rows * ndw;
    if (n <= 0) return;
    const uint32_t gp = (uint32_t)gpitch;
    const int dr = NT / ndw, dc = NT - dr * ndw;
    int r = tid / ndw, c = tid - r * ndw;
    uint32_t go = (uint32_t)r * gp + 4u * (uint32_t)c;
    int lo = r * lpitch_dw + c;
    const uint32_t gstep = (uint32_t)dr * gp + 4u * (uint32_t)dc, gwrap = gp - 4u * (uint32_t)ndw;
    const int lstep = dr * lpitch_dw + dc, lwrap = lpitch_dw - ndw;
    const uint32_t glast = (uint32_t)(rows - 1) * gp + 4u * (uint32_t)(ndw - 1);
    for (int base = 0; base < n; base += NT * 8) {
        uint32_t v[8];
        int at[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            // unconditional loads (offset clamped): a guarded load becomes a branch + vmcnt(0)
            const bool in = base + k * NT + tid < n;
            v[k] = *(const uint32_t*)(gsrc + (in ? go : glast));
            at[k] = in ? lo : -1;
            c += dc;
            go += gstep;
            lo += lstep;
            if (c >= ndw) { c -= ndw; go += gwrap; lo += lwrap; }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (at[k] >= 0) lds[at[k]] = v[k];
    }
    vmem_drained();
}

// Column-owner form for windows of at most 64 dwords per row and 4*MAXK rows (256 threads):
// lane c of wave w owns column c and rows w, w + 4, ...  The per-lane source and LDS offsets
// are fixed; row k's base is a uniform (scalar) address, so an element costs one load and one
// LDS store and no per-element index arithmetic or exec-mask branch.  Returns false (nothing
// staged) when the window does not fit the form.
template <int MAXK>
__device__ __forceinline__ bool stage_dwords_cols(const uint8_t* __restrict__ gsrc, size_t gpitch,
                                                  int rows, int ndw, uint32_t* lds,
                                                  int lpitch_dw, int tid) {
    if (ndw > 64 || rows > 4 * MAXK) return false;
    if (rows <= 0 || ndw <= 0) return true;
    const int c = tid & 63, w = tid >> 6;
    const bool colok = c < ndw;
    const uint32_t voff = 4u * (uint32_t)(colok ? c : 0);
    uint32_t v[MAXK];
#pragma unroll
    for (int k = 0; k < MAXK; ++k) {
        // rows past the window re-read the last row (uniform clamp, no branch)
        const int r = min(w + 4 * k, rows - 1);
        v[k] = *(const uint32_t*)(gsrc + (size_t)r * gpitch + voff);
    }
    if (colok) {
        uint32_t* l = lds + w * lpitch_dw + c;
#pragma unroll
        for (int k = 0; k < MAXK; ++k)
            if (w + 4 * k < rows) l[4 * k * lpitch_dw] = v[k];
    }
    vmem_drained();
    return true;
}

}  // namespace orbx
