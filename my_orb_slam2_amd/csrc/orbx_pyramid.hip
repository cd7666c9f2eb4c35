// orbx_pyramid.hip — one fused kernel per pyramid level: level l from level l-1
// (ComputePyramid, src/ORBextractor.cc:1129-1154) and its 7x7 Gaussian (operator(),
// :1106-1108) in the same pass.
//
// A 256-thread workgroup owns a 128 x 32 output tile of level l.  It stages the source
// window of the tile + the 3-pixel blur halo (coordinates reflected as BORDER_REFLECT_101)
// in LDS with aligned dword loads (all loads of a thread in flight before its first LDS
// store), computes level l on tile + halo in groups of 4 adjacent pixels (the window bytes
// of a group come from 3 dword LDS reads per source row; OpenCV INTER_LINEAR fixed-point
// coefficients from per-group packed tables), writes the tile, then runs the separable
// blur on 4-pixel groups (3 dword reads per row pass, 7 b64 reads per column pass) and
// writes the blurred tile.  Level l is read from HBM once (by level l+1's launch).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "orbx_device.h"
#include "orbx_internal.h"
#include "orbx_kernels.h"

namespace orbx {


#define LT_GW (LT_W / 4)      // output groups per row

__device__ __forceinline__ int reflect101_i(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p;
        else p = 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

__device__ __forceinline__ int sat8(int v) { return min(max(v, 0), 255); }

typedef unsigned short us2 __attribute__((ext_vector_type(2)));
typedef float f2v __attribute__((ext_vector_type(2)));

// OpenCV INTER_LINEAR 8U value from the two horizontal sums (VResizeLinear + cast).
__device__ __forceinline__ int vresize(int h0, int h1, int b0, int b1, bool simd) {
    if (simd) {   // VResizeLinearVec_32s8u: packs(>>4), mulhi, adds, (+2)>>2, packus
        const int t0 = min(h0 >> 4, 32767), t1 = min(h1 >> 4, 32767);
        int m = (int)(__umul24(t0, b0) >> 16) + (int)(__umul24(t1, b1) >> 16);
        m = min(max(m, -32768), 32767);
        m = min(m + 2, 32767);
        return sat8(m >> 2);
    }
    return sat8((int)((__umul24(h0, b0) + __umul24(h1, b1) + (1u << 21)) >> 22));   // FixedPtCast<int, uchar, 22>
}

struct BlurTaps {
    uint32_t tapA, tapB;   // v_dot4 taps k0..k3 / k4..k6,0 (row pass)
    uint32_t K4, K5, K6;   // (k, k) u16 pairs (column pass)
    uint32_t k3;
};

// ---- 3. level tile out (output x = X0 + 4g  <->  halo group g + 1) ----
// ---- 4. blur row pass (RowFilter<uchar,int>: exact; sums <= 257*255 fit u16) ----
// pixel x = X0+4gq+j needs halo bytes 1+j .. 7+j: two v_dot4_u32_u8 over the byte runs
// 1+j..4+j (taps k0..k3) and 5+j..8+j (taps k4..k6, 0).  FULL: a 128 x 32 tile, fixed trip
// counts (no per-item bounds, whole-dword stores).
template <bool FULL>
__device__ __forceinline__ void tile_out_rows(const uint32_t* lvl, uint16_t* rows, int tid, int vw,
                                              int vh, uint8_t* dlev, int X0, int Y0, int pitch,
                                              const BlurTaps& tp) {
    const int ng = FULL ? LT_GW : (vw + 3) >> 2;
    const int n3 = FULL ? LT_H * LT_GW : vh * LT_GW;
    auto out_item = [&](int i) {
        const int r = i / LT_GW, gq = i - r * LT_GW;
        if (!FULL && gq >= ng) return;
        const uint32_t v = lvl[(r + 3) * LT_G + gq + 1];
        uint8_t* d = dlev + __umul24(Y0 + r, pitch) + X0 + 4 * gq;
        if (FULL || 4 * gq + 4 <= vw) *(uint32_t*)d = v;
        else
            for (int j = 0; 4 * gq + j < vw; ++j) d[j] = (uint8_t)(v >> (8 * j));
    };
    if constexpr (FULL) {
        static_assert((LT_H * LT_GW) % 256 == 0, "full-tile item count");
#pragma unroll
        for (int k = 0; k < LT_H * LT_GW / 256; ++k) out_item(tid + 256 * k);
    } else {
        for (int i = tid; i < n3; i += 256) out_item(i);
    }
    const int n4 = FULL ? (LT_H + 6) * LT_GW : (vh + 6) * LT_GW;
    auto row_item = [&](int i) {
        const int r = i / LT_GW, gq = i - r * LT_GW;
        if (!FULL && gq >= ng) return;
        const uint32_t* s = lvl + r * LT_G + gq;   // bytes of x = X0 + 4gq - 4 .. + 7
        const uint32_t d0 = s[0], d1 = s[1], d2 = s[2];
        uint32_t sum[4];
        sum[0] = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d1, d0, 1), tp.tapA,
                 __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d2, d1, 1), tp.tapB, 0u, false), false);
        sum[1] = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d1, d0, 2), tp.tapA,
                 __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d2, d1, 2), tp.tapB, 0u, false), false);
        sum[2] = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d1, d0, 3), tp.tapA,
                 __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d2, d1, 3), tp.tapB, 0u, false), false);
        sum[3] = __builtin_amdgcn_udot4(d1, tp.tapA, __builtin_amdgcn_udot4(d2, tp.tapB, 0u, false), false);
        const uint32_t lo = sum[0] | (sum[1] << 16), hi = sum[2] | (sum[3] << 16);
        *(uint2*)(rows + r * LT_W + 4 * gq) = make_uint2(lo, hi);
    };
    if constexpr (FULL) {
        constexpr int K4 = ((LT_H + 6) * LT_GW) / 256, R4 = ((LT_H + 6) * LT_GW) % 256;
#pragma unroll
        for (int k = 0; k < K4; ++k) row_item(tid + 256 * k);
        if (tid < R4) row_item(tid + 256 * K4);
    } else {
        for (int i = tid; i < n4; i += 256) row_item(i);
    }
}

// ---- 5. blur column pass (SymmColumnFilter / SymmColumnVec_32s8u) ----
// The SSE2 float form s = c0*f0 + p1*f1 + p2*f2 + p3*f3 (f = k/65536) is exact here:
// every product k*v is an integer < 2^24 scaled by a power of two, and every partial
// sum S = k3*c0 + k4*p1 + ... stays exact while S < 2^24 (partials only grow); at
// S >= 2^24 both forms give >= 256 and saturate to 255.  So rintf(S/65536) is
// round-half-even of the integer S, and the scalar tail is (S + 32768) >> 16.
// S_j = k3*c + k4*(r2+r4) + k5*(r1+r5) + k6*(r0+r6): per pixel three v_perm pair the
// symmetric rows' u16 sums and four v_dot2_u32_u16 accumulate (S < 2^24: exact).
template <bool FULL>
__device__ __forceinline__ void tile_columns(const uint16_t* rows, int tid, int vw, int vh,
                                             uint8_t* dblur, int X0, int Y0, int pitch, int bh,
                                             int bsimd_end, const BlurTaps& tp) {
    const int ng = FULL ? LT_GW : (vw + 3) >> 2;
    const int n5 = FULL ? LT_H * LT_GW : vh * LT_GW;
    const uint32_t K3lo = tp.k3, K3hi = tp.k3 << 16;
    auto col_item = [&](int i) {
        const int r = i / LT_GW, gq = i - r * LT_GW;
        if (!FULL && gq >= ng) return;
        uint2 v[7];
#pragma unroll
        for (int kk = 0; kk < 7; ++kk) v[kk] = *(const uint2*)(rows + (r + kk) * LT_W + 4 * gq);
        const int xg = X0 + 4 * gq;
        uint32_t packed = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            auto dw = [&](int kk) { return (j < 2) ? v[kk].x : v[kk].y; };
            const uint32_t sel = (j & 1) ? 0x07060302u : 0x05040100u;   // (a.hi, b.hi) / (a.lo, b.lo)
            const us2 p06 = __builtin_bit_cast(us2, __builtin_amdgcn_perm(dw(6), dw(0), sel));
            const us2 p15 = __builtin_bit_cast(us2, __builtin_amdgcn_perm(dw(5), dw(1), sel));
            const us2 p24 = __builtin_bit_cast(us2, __builtin_amdgcn_perm(dw(4), dw(2), sel));
            uint32_t S = __builtin_amdgcn_udot2(p06, __builtin_bit_cast(us2, tp.K6), 0u, false);
            S = __builtin_amdgcn_udot2(p15, __builtin_bit_cast(us2, tp.K5), S, false);
            S = __builtin_amdgcn_udot2(p24, __builtin_bit_cast(us2, tp.K4), S, false);
            S = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, dw(3)),
                                       __builtin_bit_cast(us2, (j & 1) ? K3hi : K3lo), S, false);
            const bool simd = xg + j < bsimd_end;
            const uint32_t val = (S + (simd ? 32767u + ((S >> 16) & 1u) : 32768u)) >> 16;
            packed |= min(val, 255u) << (8 * j);
        }
        uint8_t* d = dblur + blur_off(xg, Y0 + r, pitch, bh);
        if (FULL || 4 * gq + 4 <= vw) *(uint32_t*)d = packed;
        else
            for (int j = 0; 4 * gq + j < vw; ++j) d[j] = (uint8_t)(packed >> (8 * j));
    };
    if constexpr (FULL) {
#pragma unroll
        for (int k = 0; k < LT_H * LT_GW / 256; ++k) col_item(tid + 256 * k);
    } else {
        for (int i = tid; i < n5; i += 256) col_item(i);
    }
}

#define BLUR_SLIDE 4   // full tiles: output rows per thread in the column pass (0: one row per item)

// ---- 4'. blur row pass with float row sums ----
// Same v_dot4 sums as tile_out_rows; each sum (<= 257 * 255) is stored as an exact float.
template <bool FULL>
__device__ __forceinline__ void tile_out_rows_f(const uint32_t* lvl, float* rows, int tid, int vw,
                                                int vh, uint8_t* dlev, int X0, int Y0, int pitch,
                                                const BlurTaps& tp) {
    const int ng = FULL ? LT_GW : (vw + 3) >> 2;
    const int n3 = FULL ? LT_H * LT_GW : vh * LT_GW;
    auto out_item = [&](int i) {
        const int r = i / LT_GW, gq = i - r * LT_GW;
        if (!FULL && gq >= ng) return;
        const uint32_t v = lvl[(r + 3) * LT_G + gq + 1];
        uint8_t* d = dlev + __umul24(Y0 + r, pitch) + X0 + 4 * gq;
        if (FULL || 4 * gq + 4 <= vw) *(uint32_t*)d = v;
        else
            for (int j = 0; 4 * gq + j < vw; ++j) d[j] = (uint8_t)(v >> (8 * j));
    };
    if constexpr (FULL) {
#pragma unroll
        for (int k = 0; k < LT_H * LT_GW / 256; ++k) out_item(tid + 256 * k);
    } else {
        for (int i = tid; i < n3; i += 256) out_item(i);
    }
    const int n4 = FULL ? (LT_H + 6) * LT_GW : (vh + 6) * LT_GW;
    auto row_item = [&](int i) {
        const int r = i / LT_GW, gq = i - r * LT_GW;
        if (!FULL && gq >= ng) return;
        const uint32_t* s = lvl + r * LT_G + gq;
        const uint32_t d0 = s[0], d1 = s[1], d2 = s[2];
        float4 o;
        o.x = (float)__builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d1, d0, 1), tp.tapA,
                     __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d2, d1, 1), tp.tapB, 0u, false), false);
        o.y = (float)__builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d1, d0, 2), tp.tapA,
                     __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d2, d1, 2), tp.tapB, 0u, false), false);
        o.z = (float)__builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d1, d0, 3), tp.tapA,
                     __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d2, d1, 3), tp.tapB, 0u, false), false);
        o.w = (float)__builtin_amdgcn_udot4(d1, tp.tapA, __builtin_amdgcn_udot4(d2, tp.tapB, 0u, false), false);
        *(float4*)(rows + r * LT_W + 4 * gq) = o;
    };
    if constexpr (FULL) {
        constexpr int K4 = ((LT_H + 6) * LT_GW) / 256, R4 = ((LT_H + 6) * LT_GW) % 256;
#pragma unroll
        for (int k = 0; k < K4; ++k) row_item(tid + 256 * k);
        if (tid < R4) row_item(tid + 256 * K4);
    } else {
        for (int i = tid; i < n4; i += 256) row_item(i);
    }
}

// ---- 5'. blur column pass in float ----
// S = k3*c + k4*(r2+r4) + k5*(r1+r5) + k6*(r0+r6) with integer taps and integer row sums:
// every pairwise sum (< 2^17), product (< 2^23) and partial sum (< 2^24, see tile_columns)
// is exact in float, so Sf == S.  SSE2 pixels take rint(S / 65536) saturated to u8
// (v_cvt_pk_u8_f32 rounds to nearest even and clamps, as cvtps + packus do); the scalar
// tail takes (S + 32768) >> 16 from the exact integer.
template <bool FULL>
__device__ __forceinline__ void tile_columns_f(const float* rows, int tid, int vw, int vh,
                                               uint8_t* dblur, int X0, int Y0, int pitch, int bh,
                                               int bsimd_end, const BlurTaps& tp) {
    const int ng = FULL ? LT_GW : (vw + 3) >> 2;
    const int n5 = FULL ? LT_H * LT_GW : vh * LT_GW;
    // taps k / 65536 (the SSE2 path's own coefficients): power-of-two scaling keeps every
    // product and partial sum exact, so Sf = S / 65536 exactly
    const float inv = 1.0f / 65536.0f;
    const float f3 = (float)tp.k3 * inv, f4 = (float)(tp.K4 & 0xFFFF) * inv,
                f5 = (float)(tp.K5 & 0xFFFF) * inv, f6 = (float)(tp.K6 & 0xFFFF) * inv;
    // groups entirely left of bsimd_end take the SSE2 form only
    const bool tile_simd = X0 + 4 * ng <= bsimd_end;
    // S for the 4 pixels of one group from its 7 row sums v[0..6]
    auto col_sums = [&](const float4* v, float* S) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            auto c = [&](int kk) { return j == 0 ? v[kk].x : (j == 1 ? v[kk].y : (j == 2 ? v[kk].z : v[kk].w)); };
            float a = (c(0) + c(6)) * f6;
            a = __builtin_fmaf(c(1) + c(5), f5, a);
            a = __builtin_fmaf(c(2) + c(4), f4, a);
            S[j] = __builtin_fmaf(c(3), f3, a);
        }
    };
    auto col_store = [&](int r, int gq, const float* S) {
        const int xg = X0 + 4 * gq;
        uint32_t packed = 0;
        if (tile_simd || xg + 4 <= bsimd_end) {
#pragma unroll
            for (int j = 0; j < 4; ++j) packed = __builtin_amdgcn_cvt_pk_u8_f32(S[j], j, packed);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t Si = (uint32_t)(S[j] * 65536.0f);
                const bool simd = xg + j < bsimd_end;
                const uint32_t val = (Si + (simd ? 32767u + ((Si >> 16) & 1u) : 32768u)) >> 16;
                packed |= min(val, 255u) << (8 * j);
            }
        }
        uint8_t* d = dblur + blur_off(xg, Y0 + r, pitch, bh);
        if (FULL || 4 * gq + 4 <= vw) *(uint32_t*)d = packed;
        else
            for (int j = 0; 4 * gq + j < vw; ++j) d[j] = (uint8_t)(packed >> (8 * j));
    };
    auto col_item = [&](int i) {
        const int r = i / LT_GW, gq = i - r * LT_GW;
        if (!FULL && gq >= ng) return;
        float4 v[7];
#pragma unroll
        for (int kk = 0; kk < 7; ++kk) v[kk] = *(const float4*)(rows + (r + kk) * LT_W + 4 * gq);
        float S[4];
        col_sums(v, S);
        col_store(r, gq, S);
    };
    if constexpr (FULL) {
        // a thread owns one group and BLUR_SLIDE consecutive output rows: it reads their
        // BLUR_SLIDE + 6 row sums once (7 per output row in the item form)
        static_assert(LT_GW == 32 && LT_H * LT_GW == 256 * BLUR_SLIDE, "column-slide mapping");
        const int gq = tid & (LT_GW - 1), r0 = (tid >> 5) * BLUR_SLIDE;
        float4 v[BLUR_SLIDE + 6];
#pragma unroll
        for (int kk = 0; kk < BLUR_SLIDE + 6; ++kk)
            v[kk] = *(const float4*)(rows + (r0 + kk) * LT_W + 4 * gq);
#pragma unroll
        for (int o = 0; o < BLUR_SLIDE; ++o) {
            float S[4];
            col_sums(v + o, S);
            col_store(r0 + o, gq, S);
        }
    } else
    if constexpr (FULL) {
#pragma unroll
        for (int k = 0; k < LT_H * LT_GW / 256; ++k) col_item(tid + 256 * k);
    } else {
        for (int i = tid; i < n5; i += 256) col_item(i);
    }
}

#define STAGE_MAXK 12  // column-owner window staging: up to 48 rows (0: always the generic form)
#define LEVEL_WPE 1
// MODE (host-chosen per level, one instantiation each): 0 level 0 (copy of the input), 1 scale
// 1 copy, 2 exact 2:1 area, 3 INTER_LINEAR
template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LEVEL_WPE))) void k_level(const Geometry* __restrict__ g,
                                               const uint8_t* __restrict__ ltab,
                                               const uint8_t* __restrict__ in0,
                                               const uint8_t* __restrict__ in1, int split,
                                               size_t stride, size_t bstride,
                                               uint8_t* __restrict__ pyr,
                                               uint8_t* __restrict__ blur, int level) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    int bx, b;
    xcd_block(bx, b);
    const int tid = threadIdx.x;
    const LevelGeom& L = g->lv[level];
    const int tx = bx % L.ntx, ty = bx / L.ntx;
    const int X0 = tx * LT_W, Y0 = ty * LT_H;
    const int vw = min(LT_W, L.w - X0), vh = min(LT_H, L.h - Y0);

    uint8_t* p = smem;
    auto take = [&](size_t n) { uint8_t* r = p; p += (n + 15) & ~(size_t)15; return r; };
    uint32_t* lvl = (uint32_t*)take((size_t)LT_HR * LT_G * 4);      // [38][34] dwords
    // the blur's row sums (phases 3-4) share their LDS with the tables and the source window
    // (phases 1-2, dead after the barrier that ends phase 2): a smaller footprint, so more
    // workgroups -- and more window loads in flight -- per CU
    uint16_t* rows = (uint16_t*)p;                                   // [38][128] row sums
    uint2* cgrp = (uint2*)take((size_t)LT_G * 8);                    // per group: 4 x sx (u16)
    uint32_t* cinf = (uint32_t*)take((size_t)LT_G * 4);              // per group: flags
    uint4* calp = (uint4*)take((size_t)LT_G * 16);                   // per group: 4 x (a0, a1)
    uint4* csel = (uint4*)take((size_t)LT_G * 16);                   // per group: 4 x selector
    uint2* rinf = (uint2*)take((size_t)LT_HR * 8);                   // per row: ry0, ry1, b0, b1
    uint8_t* win = p;                                                // source window

    constexpr int mode = MODE;
    const LevelGeom& S = g->lv[level > 0 ? level - 1 : 0];
    // needed halo ranges (level coordinates, before reflection)
    const int nx0 = X0 - 3, nx1 = X0 + vw + 2, ny0 = Y0 - 3, ny1 = Y0 + vh + 2;

    // ---- 1. source window + tables (host-built per tile column / row, build_geometry) ----
    const LevelColTab* CT = (const LevelColTab*)(ltab + L.ctab) + tx;
    const LevelRowTab* RT = (const LevelRowTab*)(ltab + L.rowtab) + ty;
    const int wx0 = CT->x0, WWb = CT->ww, wy0 = RT->y0, WH = RT->wh;
    // table loads issued before the window loads, so both land in one round trip
    uint4 tc = make_uint4(0, 0, 0, 0), ta = make_uint4(0, 0, 0, 0), ts = ta;
    if (mode == 0) {
        // level 0 reads no tables
    } else if (tid < LT_G) {
        tc = make_uint4(CT->cgrp[2 * tid], CT->cgrp[2 * tid + 1], CT->cinf[tid], 0);
        ta = *(const uint4*)&CT->calp[4 * tid];
        ts = *(const uint4*)&CT->csel[4 * tid];
    } else if (tid >= 64 && tid < 64 + LT_HR) {
        tc = make_uint4(RT->rinf[2 * (tid - 64)], RT->rinf[2 * (tid - 64) + 1], 0, 0);
    }
    // window row pitch; modes 0/1 place x at column x - (X0 - 4) so that groups are dword-aligned
    const int WP = (mode == 3) ? ((WWb + 3) & ~3) : LT_G * 4;
    const int wcol0 = (mode == 3) ? 0 : wx0 - (X0 - 4);
    // level 0: the halo tile is the input itself, loaded straight into the level array: two
    // aligned dwords + v_alignbyte per 4-pixel group, or on border tiles four byte loads per
    // group (rows and columns reflected per item)
    constexpr bool direct = mode == 0;
    if (direct) {
        const uint8_t* src = (b < split ? in0 + (size_t)b * bstride : in1 + (size_t)(b - split) * bstride);
        const int W = L.w, H = L.h;
        constexpr int NI = (LT_HR * LT_G + 255) / 256;
        static_assert(256 / LT_G == 7 && 256 % LT_G == 18, "halo item stride");
        uint32_t d0[NI], d1[NI], sh[NI];
        // inner tiles: every group's aligned dword pair inside its image row (xg >= 4 keeps the
        // aligned base after the row start, xg + 8 <= W its second dword before the row end)
        const bool inner = X0 >= 8 && X0 + LT_W + 8 <= W && Y0 >= 3 && Y0 + LT_H + 3 <= H;
        auto load_items = [&](auto inner_c) {
            constexpr bool IN = decltype(inner_c)::value;
            int hr = tid / LT_G, q = tid - hr * LT_G;
#pragma unroll
            for (int k = 0; k < NI; ++k) {
                const int hrc = min(hr, LT_HR - 1);
                int y = Y0 - 3 + hrc;
                if (!IN) {   // BORDER_REFLECT_101; rows past the needed halo: any row
                    y = y < 0 ? -y : (y >= H ? 2 * H - 2 - y : y);
                    y = min(max(y, 0), H - 1);
                }
                const uint8_t* row = src + __umul24(y, (uint32_t)stride);
                const int xg = X0 - 4 + 4 * q;
                if constexpr (IN) {
                    const uintptr_t a = (uintptr_t)(row + xg);
                    const uint32_t* ab = (const uint32_t*)(a & ~(uintptr_t)3);
                    sh[k] = (uint32_t)(a & 3);
                    d0[k] = ab[0];
                    d1[k] = ab[1];
                } else {
                    // border tiles: four byte loads per group, branch-free, all in flight
                    uint32_t v = 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        int x = xg + j;
                        x = x < 0 ? -x : (x >= W ? 2 * W - 2 - x : x);
                        x = min(max(x, 0), W - 1);   // pixels past the needed halo: any in-row value
                        v |= (uint32_t)row[x] << (8 * j);
                    }
                    d0[k] = v;
                    d1[k] = 0;
                    sh[k] = 0;
                }
                hr += 7;
                q += 18;
                if (q >= LT_G) { q -= LT_G; ++hr; }
            }
        };
        if (inner) load_items(std::true_type{});
        else load_items(std::false_type{});
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const int i = tid + 256 * k;
            if (i < LT_HR * LT_G) lvl[i] = __builtin_amdgcn_alignbyte(d1[k], d0[k], sh[k]);
        }
    } else if (mode == 1) {
        const uint8_t* src = pyr + (size_t)b * g->pyr_bytes + S.off;   // wx0 is a multiple of 4
        if (!stage_dwords_cols<STAGE_MAXK>(src + (size_t)wy0 * S.pitch + wx0, S.pitch, WH,
                                           (WWb + 3) >> 2, (uint32_t*)(win + wcol0), WP / 4, tid))
            stage_dwords<256>(src + (size_t)wy0 * S.pitch + wx0, S.pitch, WH, (WWb + 3) >> 2,
                              (uint32_t*)(win + wcol0), WP / 4, tid);
    } else if (mode == 3) {
        const uint8_t* src = pyr + (size_t)b * g->pyr_bytes + S.off;
        if (!stage_dwords_cols<STAGE_MAXK>(src + (size_t)wy0 * S.pitch + wx0, S.pitch, WH, WP / 4,
                                           (uint32_t*)win, WP / 4, tid))
            stage_dwords<256>(src + (size_t)wy0 * S.pitch + wx0, S.pitch, WH, WP / 4,
                              (uint32_t*)win, WP / 4, tid);
    }
    if (mode == 0) {
    } else if (tid < LT_G) {
        cgrp[tid] = make_uint2(tc.x, tc.y);
        cinf[tid] = tc.z;
        calp[tid] = ta;
        csel[tid] = ts;
    } else if (tid >= 64 && tid < 64 + LT_HR) {
        rinf[tid - 64] = make_uint2(tc.x, tc.y);
    }
    __syncthreads();

    // ---- 2. level l on tile + halo, 4 pixels per item ----
    const uint8_t* src2 = pyr + (size_t)b * g->pyr_bytes + S.off;   // mode 2 only
    // item i = (halo row hr, group q); 256 = 7 * LT_G + 18, advanced without divisions
    const bool full_tile = vw == LT_W && vh == LT_H;   // every halo item is needed
    // mode 3 (generic INTER_LINEAR) on one 4-pixel group: halo row hr, the group's column
    // tables (cg: source columns, ci: flags, al: alphas, sl: v_perm selectors)
    auto item3 = [&](int hr, uint2 cg, uint32_t ci, uint4 al, uint4 sl, auto fast_c) -> uint32_t {
        constexpr bool FASTP = decltype(fast_c)::value;   // simple group, all four pixels SSE2
        uint32_t out = 0;
        const uint2 ri = rinf[hr];
        const int xs[4] = {(int)(cg.x & 0xFFFF), (int)(cg.x >> 16), (int)(cg.y & 0xFFFF),
                           (int)(cg.y >> 16)};
        const uint32_t als[4] = {al.x, al.y, al.z, al.w};
        const int r0 = (int)(ri.x & 0xFFFF), r1 = (int)(ri.x >> 16);
        const int b0 = (int)(int16_t)(ri.y & 0xFFFF), b1 = (int)(int16_t)(ri.y >> 16);
        const uint8_t* w0 = win + __umul24(r0, WP);
        const uint8_t* w1 = win + __umul24(r1, WP);
        if (FASTP || (ci & 0x200u)) {
            // branch-free: v_perm gathers each pixel's two taps as u16s, v_dot2 applies
            // the alphas (HResizeLinear), then VResizeLinear (SSE2 or scalar form)
            const uint32_t sels[4] = {sl.x, sl.y, sl.z, sl.w};
            const int base = xs[0] & ~3, o0 = xs[0] & 3;
            const uint32_t* d0p = (const uint32_t*)(w0 + base);
            const uint32_t* d1p = (const uint32_t*)(w1 + base);
            const uint32_t a0 = d0p[0], a1 = d0p[1], a2 = d0p[2];
            const uint32_t c0 = d1p[0], c1 = d1p[1], c2 = d1p[2];
            // 8-byte windows starting at the group's first tap column (span <= 7)
            const uint32_t wa0 = __builtin_amdgcn_alignbyte(a1, a0, o0);
            const uint32_t wa1 = __builtin_amdgcn_alignbyte(a2, a1, o0);
            const uint32_t wc0 = __builtin_amdgcn_alignbyte(c1, c0, o0);
            const uint32_t wc1 = __builtin_amdgcn_alignbyte(c2, c1, o0);
            // h <= 255*2048, betas in [0, 2048]: the SSE2 clamps never bind; 24-bit
            // multiplies (full rate): h < 2^19, b <= 2048.  Groups whose 4 pixels all
            // take the SSE2 form (all but the right edge) skip the scalar form.
            const bool all_simd = FASTP || ((ci >> 1) & 0x55u) == 0x55u;
            auto hsum = [&](int j, int& h0, int& h1) {
                const uint32_t p0 = __builtin_amdgcn_perm(wa1, wa0, sels[j]);
                const uint32_t p1 = __builtin_amdgcn_perm(wc1, wc0, sels[j]);
                const us2 al = __builtin_bit_cast(us2, als[j]);
                h0 = (int)__builtin_amdgcn_udot2(__builtin_bit_cast(us2, p0), al, 0u, false);
                h1 = (int)__builtin_amdgcn_udot2(__builtin_bit_cast(us2, p1), al, 0u, false);
            };
            // hsum returns H = 16 h (the table alphas are scaled by 16), so
            // ((h >> 4) * b) >> 16 = mulhi_u24(H & ~0xFF, b << 8): one v_and and one
            // v_mul_hi_u32_u24 per term.  No saturation: alphas and betas each sum to
            // 2048, so the two terms are <= (255*2048 >> 4) * 2048 >> 16 = 1020 and
            // the value <= 255.
            const uint32_t bs0 = (uint32_t)b0 << 8, bs1 = (uint32_t)b1 << 8;
            auto mulhi24 = [](uint32_t x, uint32_t y) {
                return (uint32_t)(((uint64_t)(x & 0xFFFFFFu) * (y & 0xFFFFFFu)) >> 32);
            };
            auto vsimd = [&](int H0, int H1) {
                return (int)((mulhi24((uint32_t)H0 & ~0xFFu, bs0) +
                              mulhi24((uint32_t)H1 & ~0xFFu, bs1) + 2u) >> 2);
            };
            if (all_simd) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    int h0, h1;
                    hsum(j, h0, h1);
                    out |= (uint32_t)vsimd(h0, h1) << (8 * j);
                }
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    int h0, h1;
                    hsum(j, h0, h1);
                    const int vs = vsimd(h0, h1);
                    h0 >>= 4;
                    h1 >>= 4;
                    const int vc = min((int)((__umul24(h0, b0) + __umul24(h1, b1) + (1u << 21)) >> 22), 255);
                    out |= (uint32_t)(((ci >> (2 * j + 1)) & 1u) ? vs : vc) << (8 * j);
                }
            }
        } else {   // reflected border group: bytes one by one
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int sxj = xs[j];
                const int f = (int)(ci >> (2 * j)) & 3;
                int h0, h1;
                if (f & 1) {
                    const int aa = (int)(int16_t)(als[j] & 0xFFFF), ab = (int)(int16_t)(als[j] >> 16);
                    h0 = w0[sxj] * aa + w0[sxj + 1] * ab;
                    h1 = w1[sxj] * aa + w1[sxj + 1] * ab;
                } else {
                    h0 = w0[sxj] * 2048;
                    h1 = w1[sxj] * 2048;
                }
                out |= (uint32_t)vresize(h0, h1, b0, b1, (f & 2) != 0) << (8 * j);
            }
        }
        return out;
    };
    auto level_item = [&](int hr, int q, bool all) {
        const int y = Y0 - 3 + hr, xg = X0 - 4 + 4 * q;
        uint32_t out = 0;
        if (all || (y >= ny0 && y <= ny1 && xg + 3 >= nx0 && xg <= nx1)) {
            const uint2 cg = cgrp[q];
            const uint32_t ci = cinf[q];
            const uint2 ri = rinf[hr];
            const int xs[4] = {(int)(cg.x & 0xFFFF), (int)(cg.x >> 16), (int)(cg.y & 0xFFFF),
                               (int)(cg.y >> 16)};
            if (mode == 3) {
                out = item3(hr, cg, ci, calp[q], csel[q], std::false_type{});
            } else if (mode == 2) {
                const int yr = (int)ri.x;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint8_t* s0 = src2 + (size_t)(2 * yr) * S.pitch + 2 * xs[j];
                    out |= (uint32_t)((s0[0] + s0[1] + s0[S.pitch] + s0[S.pitch + 1] + 2) >> 2) << (8 * j);
                }
            } else {
                const uint8_t* wr = win + __umul24(ri.x & 0xFFFF, WP);
                if (ci & 0x100u) {
                    out = *(const uint32_t*)(wr + xs[0]);
                } else {
                    out = (uint32_t)wr[xs[0]] | ((uint32_t)wr[xs[1]] << 8) |
                          ((uint32_t)wr[xs[2]] << 16) | ((uint32_t)wr[xs[3]] << 24);
                }
            }
        }
        lvl[hr * LT_G + q] = out;
    };
    if (!direct && mode == 3 && full_tile) {
        // thread t < 7 LT_G keeps column group q = t % LT_G for halo rows t / LT_G + 7k: the
        // group's tables are read once, not once per item
        if (tid < 7 * LT_G) {
            const int rs = (int)(__umul24((uint32_t)tid, 1928u) >> 16);   // tid / 34, tid < 256
            const int q = tid - rs * LT_G;
            const uint2 cg = cgrp[q];
            const uint32_t ci = cinf[q];
            const uint4 al = calp[q], sl = csel[q];
            // interior tiles: every group of the wave is simple and SSE2-only, so the wave takes
            // the branch-free form with no per-item exec-mask branches
            const bool fast = (ci & 0x200u) && ((ci >> 1) & 0x55u) == 0x55u;
            if (__all(fast)) {
#pragma unroll
                for (int k = 0; k < (LT_HR + 6) / 7; ++k) {
                    const int hr = rs + 7 * k;
                    if (hr < LT_HR) lvl[hr * LT_G + q] = item3(hr, cg, ci, al, sl, std::true_type{});
                }
            } else {
#pragma unroll
                for (int k = 0; k < (LT_HR + 6) / 7; ++k) {
                    const int hr = rs + 7 * k;
                    if (hr < LT_HR) lvl[hr * LT_G + q] = item3(hr, cg, ci, al, sl, std::false_type{});
                }
            }
        }
    } else
    if (!direct) {
        int hr = tid / LT_G, q = tid - hr * LT_G;
        if (full_tile) {
            constexpr int KF = (LT_HR * LT_G) / 256, RF = (LT_HR * LT_G) % 256;
#pragma unroll
            for (int k = 0; k < KF; ++k) {
                level_item(hr, q, true);
                hr += 7;
                q += 18;
                if (q >= LT_G) { q -= LT_G; ++hr; }
            }
            if (tid < RF) level_item(hr, q, true);
        } else {
            for (int i = tid; i < LT_HR * LT_G;
                 i += 256, hr += 7, q += 18, (q >= LT_G ? (q -= LT_G, ++hr) : 0))
                level_item(hr, q, false);
        }
    }
    __syncthreads();

    uint8_t* dlev = pyr + (size_t)b * g->pyr_bytes + L.off;
    uint8_t* dblur = blur + (size_t)b * g->pyr_bytes + L.off;
    const int k0 = g->taps[0], k1 = g->taps[1], k2 = g->taps[2], k3 = g->taps[3];
    const int k4 = g->taps[4], k5 = g->taps[5], k6 = g->taps[6];
    const BlurTaps tp = {(uint32_t)k0 | (uint32_t)k1 << 8 | (uint32_t)k2 << 16 | (uint32_t)k3 << 24,
                         (uint32_t)k4 | (uint32_t)k5 << 8 | (uint32_t)k6 << 16,
                         (uint32_t)k4 * 0x10001u, (uint32_t)k5 * 0x10001u, (uint32_t)k6 * 0x10001u,
                         (uint32_t)k3};
    // full tiles (all but the right / bottom edge) run the fixed-trip-count form
    const bool full = vw == LT_W && vh == LT_H;
    float* rowsf = (float*)rows;
    if (full) tile_out_rows_f<true>(lvl, rowsf, tid, vw, vh, dlev, X0, Y0, L.pitch, tp);
    else tile_out_rows_f<false>(lvl, rowsf, tid, vw, vh, dlev, X0, Y0, L.pitch, tp);
    __syncthreads();
    if (full) tile_columns_f<true>(rowsf, tid, vw, vh, dblur, X0, Y0, L.pitch, L.h, L.bsimd_end, tp);
    else tile_columns_f<false>(rowsf, tid, vw, vh, dblur, X0, Y0, L.pitch, L.h, L.bsimd_end, tp);
}

// ---- k_level_strip: level l and its blur by column strips, one row per step ----
// A wave owns two half-strips (lanes 0-31 / 32-63) of SW_PX output pixels each and walks
// them down STRIP rows (+3 halo rows above and below).  Per step, row y: every lane computes
// its 4-pixel group of level l at row y (source bytes loaded STRIP_PF steps ahead), writes
// it, takes its neighbours' groups with DPP wave shifts and forms the row sums of the
// blur; the last 7 rows' sums stay in registers, so the blurred row y - 3 is one
// symmetric column sum.  No LDS, no barriers: the loads of later rows are in flight while
// the wave computes.  The arithmetic is item3's (resize, mode 3) and tile_out_rows_f /
// tile_columns_f's (blur), bit for bit.
#define STRIP_PF 2   // mode 3: rows of source loads in flight ahead of the row being computed
#define STRIP_ST_POLICY 0   // cache-policy bits of the strip walk stores: nt (2) 1.99 ms, sc1 (16) 1.88 ms vs 1.71 ms
#define STRIP_LEV rlev
#define STRIP_HREUSE 1   // mode 3: reuse the previous step's HResize of a shared source row
#define STRIP_HMASK 1   // mode 3, SSE2 waves: horizontal sums masked once per source row
// One workgroup per strip row (its snw <= 8 waves side by side) with an s_barrier every
// STRIP_SYNC* blocks of 7 steps (0: 4-wave workgroups, no barrier): the waves of a strip row
// then store each row within a few steps of each other, so the 128-byte lines split between
// two waves' 120-pixel runs are merged in L2 before they are written back (without it one
// write-back per part: level 0 wrote 1.24x its bytes, levels 1-7 1.10x).
#define STRIP_SYNC0 0  // level 0
#define STRIP_SYNC3 2  // INTER_LINEAR levels
#define STRIP_SYNC_LEVELS 0xFFFF  // bit l: level l may take strip-row workgroups
#define STRIP_NS3 2  // mode 3: load slots (1, 2 or 3; PF <= NS)
#define STRIP_NS0 7  // mode 0: load slots (1, 2 or 7)
#define STRIP_PF0 6  // mode 0: rows in flight (<= STRIP_NS0)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v3u __attribute__((ext_vector_type(3)));
template <typename F, int... K>
__device__ __forceinline__ void unroll_seq(F&& f, std::integer_sequence<int, K...>) {
    (f(std::integral_constant<int, K>{}), ...);
}
#define STRIP_WPE0 6
#define STRIP_WPE3 5
// One wave's strip of level `level` of image b (wave wv of the image's snw x sns strip waves).
// MODE 0: level 0 from the caller's images (copied into the pyramid as it is blurred);
// MODE 4: level 0 already in the pyramid (written there by the H2D copy or the caller, see
// orbx_batch_input_view): blurred only, the level itself is not stored again;
// MODE 3: an INTER_LINEAR level from the level above.
template <int MODE>
__device__ __forceinline__ void level_strip_wave(const Geometry* __restrict__ g,
                                                 const uint8_t* __restrict__ ltab,
                                                 const uint8_t* __restrict__ in0,
                                                 const uint8_t* __restrict__ in1, int split,
                                                 size_t stride, size_t bstride,
                                                 uint8_t* __restrict__ pyr,
                                                 uint8_t* __restrict__ blur, int level, int sth,
                                                 int sync, int wv, int b, uint32_t* sbl) {
    static_assert(MODE == 0 || MODE == 3 || MODE == 4, "strip kernel: level 0 or INTER_LINEAR levels");
    constexpr bool L0 = MODE != 3;         // level 0: an 8-bit image in, no resize
    const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
    const LevelGeom& L = g->lv[level];
    const int sns = (L.h + sth - 1) / sth;        // strip rows of this call's height
    if (wv >= L.snw * sns) return;                // whole waves only
    const int swx = wv % L.snw, sy = wv / L.snw;
    const int hs = 2 * swx + half;
    const bool hvalid = hs < L.snh;
    const int hsc = min(hs, L.snh - 1);
    const int W = L.w, H = L.h, pitch = L.pitch;
    const int x = hsc * SW_PX - 4 + 4 * l32;      // this lane's group
    const int Y0 = sy * sth, vh = min(sth, H - Y0);
    const bool out_lane = hvalid && l32 >= 1 && l32 <= SW_OUT && x < W;
    const StripLane* T = (const StripLane*)(ltab + L.stab) + hsc * 32 + l32;
    const uint4 t0 = *(const uint4*)T;
    const uint4 al = *(const uint4*)T->alp;
    const uint4 ps = *(const uint4*)T->psel;
    const uint4* RT = (const uint4*)(ltab + L.srow) + Y0;   // step i <-> row y = Y0 - 3 + i
    const int n = vh + 6;

    // Addresses are a wave-uniform row base (SGPRs) + a lane offset that is constant over the
    // walk, so loads and stores take the saddr forms and a step spends no VALU on 64-bit
    // address arithmetic.
    const uint8_t* src;   // level 0: the image (a row's loads start 4 bytes before the row)
    size_t spitch;
    if (MODE == 4) {
        src = pyr + (size_t)b * g->pyr_bytes + L.off;
        spitch = (size_t)pitch;
    } else if (MODE == 0) {
        src = b < split ? in0 + (size_t)b * bstride : in1 + (size_t)(b - split) * bstride;
        spitch = stride;
    } else {
        const LevelGeom& S = g->lv[level - 1];
        src = pyr + (size_t)b * g->pyr_bytes + S.off;
        spitch = (size_t)S.pitch;
    }
    // mode 3: the source level as a buffer (no range clamp: the row tables keep every read
    // inside the level's rows and their padding, as the flat loads did)
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, 0x7FFFFFFF, 0x00020000);
    const uint32_t o0 = t0.x & 3u;         // mode 3: first tap's byte offset in its dword
    const uint32_t boff = t0.x & ~3u;      // mode 3: lane offset of the aligned dwords
    const uint32_t xoff4 = t0.x + 4u;      // mode 0: lane offset of its first byte

    // per-wave forms: every needed lane SSE2 in the vertical resize / the blur's columns
    const bool lane_rsimd = ((t0.y >> 1) & 0x55u) == 0x55u;
    const bool wave_rsimd = __all(!hvalid || lane_rsimd);
    const bool wave_bsimd = __all(!out_lane || x + 4 <= L.bsimd_end);

    // row sums of the blur (exact integers as floats), last 7 rows
    const BlurTaps tp = {(uint32_t)g->taps[0] | (uint32_t)g->taps[1] << 8 | (uint32_t)g->taps[2] << 16 |
                             (uint32_t)g->taps[3] << 24,
                         (uint32_t)g->taps[4] | (uint32_t)g->taps[5] << 8 | (uint32_t)g->taps[6] << 16,
                         0u, 0u, 0u, (uint32_t)g->taps[3]};
    const float inv = 1.0f / 65536.0f;
    const float f3 = (float)g->taps[3] * inv, f4 = (float)g->taps[4] * inv,
                f5 = (float)g->taps[5] * inv, f6 = (float)g->taps[6] * inv;
    // row-pass tap words for pixel j of the group over the dwords left / own / right (byte b
    // of a dword is the pixel at its position b)
    const uint32_t k0 = g->taps[0], k1 = g->taps[1], k2 = g->taps[2], k3 = g->taps[3],
                   k4 = g->taps[4], k5 = g->taps[5], k6 = g->taps[6];
    const uint32_t W00 = k0 << 8 | k1 << 16 | k2 << 24, W01 = k3 | k4 << 8 | k5 << 16 | k6 << 24;
    const uint32_t W10 = k0 << 16 | k1 << 24, W11 = k2 | k3 << 8 | k4 << 16 | k5 << 24, W12 = k6;
    const uint32_t W20 = k0 << 24, W21 = k1 | k2 << 8 | k3 << 16 | k4 << 24, W22 = k5 | k6 << 8;
    (void)W00; (void)W01; (void)W10; (void)W11; (void)W12; (void)W20; (void)W21; (void)W22;

    // the strip's row table entry of step i: a wave-uniform address, so a scalar load
    auto row_info = [&](int i) { return RT[i]; };
    // load slots (a ring of NS; step i consumes slot i mod NS, then refills it with row i+PF
    // ... PF <= NS): mode 0 two dwords of the input row + the perm selector for the row's
    // alignment, mode 3 three dwords of each of the two source rows + the row's betas
    constexpr int NS = L0 ? STRIP_NS0 : STRIP_NS3;
    constexpr int PF = L0 ? STRIP_PF0 : STRIP_PF;
    static_assert(PF <= NS && (NS == 1 || NS == 2 || NS == 3 || NS == 7), "slot ring");
    uint32_t A[NS][3], C[NS][3], RB[NS];
    // mode 3: the source rows' byte offsets of each slot, and the last step's horizontal sums
    // of its second source row (HResize of a row is the same for every output row that
    // reads it: 4 of 5 steps at scale 1.2 take the previous step's second row as their first)
    uint32_t RAo[NS], RCo[NS], HCp[4] = {0u, 0u, 0u, 0u};
    uint32_t prevRC = 0xFFFFFFFFu;
    auto issue = [&](int slot, int i) {
        const int ic = min(i, n - 1);
        const uint4 ri = row_info(ic);
        if (L0) {
            // offsets relative to row - 4 (unsigned); the pointers formed are the load
            // addresses themselves: the aligned dwords holding the group's bytes, which start
            // before the tensor only when its first row does not start on a dword
            const uint8_t* rowp = src + (size_t)(ri.x & 0xFFFFu) * spitch;
            const uint32_t rlo = (uint32_t)(uintptr_t)rowp - 4u;
            const uint32_t o = (rlo + xoff4) & 3u;
            const uint32_t aoff = xoff4 - o;
            // the last dword holding a byte of the row (no read past the image)
            const uint32_t last = ((rlo + 4u + (uint32_t)(W - 1)) & ~3u) - rlo;
            A[slot][0] = *(const uint32_t*)(rowp + aoff - 4);
            A[slot][1] = *(const uint32_t*)(rowp + min(aoff + 4u, last) - 4);
            // t0.z + o in every byte (no carries: bytes <= 4 + 3): o replicated by one v_perm
            A[slot][2] = t0.z + __builtin_amdgcn_perm(0u, o, 0u);
        } else {
            // buffer loads: the source level in the descriptor, the row's byte offset in
            // soffset (scalar) and the lane's in voffset, so a load costs no 64-bit address add
            // (two per step with the flat dwordx3 loads the compiler merged the dwords into)
            const v3u a3 = __builtin_bit_cast(v3u, __builtin_amdgcn_raw_buffer_load_b96(rsrc, boff, ri.x, 0));
            const v3u c3 = __builtin_bit_cast(v3u, __builtin_amdgcn_raw_buffer_load_b96(rsrc, boff, ri.y, 0));
            A[slot][0] = a3.x; A[slot][1] = a3.y; A[slot][2] = a3.z;
            C[slot][0] = c3.x; C[slot][1] = c3.y; C[slot][2] = c3.z;
            RB[slot] = ri.z;
            RAo[slot] = ri.x;
            RCo[slot] = ri.y;
        }
    };
    auto mulhi24 = [](uint32_t a, uint32_t c) {
        return (uint32_t)(((uint64_t)(a & 0xFFFFFFu) * (c & 0xFFFFFFu)) >> 32);
    };
    // this lane's group of level l from load slot `slot`
    auto level_group = [&](int slot, auto simd_c) -> uint32_t {
        if (L0) return __builtin_amdgcn_perm(A[slot][1], A[slot][0], A[slot][2]);
        constexpr bool SIMD = decltype(simd_c)::value;
        const uint32_t rb = RB[slot];
        const int b0 = (int)(int16_t)(rb & 0xFFFF), b1 = (int)(int16_t)(rb >> 16);
        const uint32_t bs0 = (uint32_t)b0 << 8, bs1 = (uint32_t)b1 << 8;
        const uint32_t sels[4] = {ps.x, ps.y, ps.z, ps.w};
        const uint32_t als[4] = {al.x, al.y, al.z, al.w};
        // HResizeLinear of one source row (3 aligned dwords) for this lane's 4 pixels
        auto hrow = [&](const uint32_t* D, uint32_t* hs) {
            const uint32_t w0 = __builtin_amdgcn_alignbyte(D[1], D[0], o0);
            const uint32_t w1 = __builtin_amdgcn_alignbyte(D[2], D[1], o0);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                hs[j] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, __builtin_amdgcn_perm(w1, w0, sels[j])),
                                               __builtin_bit_cast(us2, als[j]), 0u, false);
                // SSE2 form: the row's sums enter the vertical pass as (sum >> 4) << 8, masked
                // once per source row here (a reused row is not masked again)
                if (SIMD && STRIP_HMASK) hs[j] &= ~0xFFu;
            }
        };
        uint32_t hA[4], hC[4];
        if (RAo[slot] == prevRC) {   // wave-uniform
#pragma unroll
            for (int j = 0; j < 4; ++j) hA[j] = HCp[j];
        } else {
            hrow(A[slot], hA);
        }
        hrow(C[slot], hC);
#pragma unroll
        for (int j = 0; j < 4; ++j) HCp[j] = hC[j];
        prevRC = RCo[slot];
        uint32_t out = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            int h0 = (int)hA[j];
            int h1 = (int)hC[j];
            const uint32_t hm = (SIMD && STRIP_HMASK) ? ~0u : ~0xFFu;
            const int vs = (int)((mulhi24((uint32_t)h0 & hm, bs0) +
                                  mulhi24((uint32_t)h1 & hm, bs1) + 2u) >> 2);
            if (SIMD) {
                out |= (uint32_t)vs << (8 * j);
            } else {
                h0 >>= 4;
                h1 >>= 4;
                const int vc = min((int)((__umul24(h0, b0) + __umul24(h1, b1) + (1u << 21)) >> 22), 255);
                out |= (uint32_t)(((t0.y >> (2 * j + 1)) & 1u) ? vs : vc) << (8 * j);
            }
        }
        return out;
    };
    float4 R[7];
    // Stores without branches (a branch per store would cost the walk its counted vmcnt
    // waits): row r's group as one dword (the image's last, partial group spills into the
    // row's >= 4 bytes of padding, pitch >= w + 4); lanes or steps with nothing to write
    // store into the padding dword of the level's row 0.
    uint8_t* const lev0 = pyr + (size_t)b * g->pyr_bytes + L.off;
    uint8_t* const blr0 = blur + (size_t)b * g->pyr_bytes + L.off;
    // buffer stores: a lane or step with nothing to write gets an offset past num_records,
    // which the hardware drops (no branch, no write)
    const int nrec = pitch * H;
    const __amdgpu_buffer_rsrc_t rlev = __builtin_amdgcn_make_buffer_rsrc(lev0, 0, nrec, 0x00020000);
    // the blurred level in 16x4 tiles (blur_off), whole bands
    const __amdgpu_buffer_rsrc_t rblr = __builtin_amdgcn_make_buffer_rsrc(blr0, 0, pitch * ((H + 3) & ~3), 0x00020000);
    // the row's byte offset rides in soffset (scalar), the lane's column in voffset: in range
    // or not whether or not the hardware adds soffset into its range check
    const uint32_t lane_off = out_lane ? (uint32_t)x : 0x80000000u;
    auto store_row = [&](const __amdgpu_buffer_rsrc_t& rs, int r, bool ok, uint32_t v) {
        __builtin_amdgcn_raw_buffer_store_b32(v, rs, ok ? lane_off : 0x80000000u, ok ? r * pitch : 0, STRIP_ST_POLICY);
    };
    // Blurred rows go through the wave's 4 LDS rows (64 dwords each: the wave's 240 output
    // pixels, halo lanes into dwords 60-63); after every 4th row the band leaves as whole
    // tiles: lane t + 15 j (< 60) stores tile t's row j, 16 bytes, so one store instruction
    // writes the wave's 15 tiles (15 whole sectors; row by row, a half-wave's 120 bytes
    // touched 2-3 sectors per row).  Wave strips are 240 pixels = 15 tiles wide.
    const int sbl_dw = (l32 >= 1 && l32 <= SW_OUT) ? SW_OUT * half + l32 - 1 : 60;
    const int ft = lane % 15, fj = lane / 15;
    const int ftx = 15 * (wv % L.snw) + ft;
    const uint32_t fl_off = (lane < 60 && 16 * ftx < W) ? (uint32_t)(64 * ftx + 16 * fj) : 0x80000000u;
    // step i (k = i mod U: the load slot k mod NS, the row-sum register k mod 7)
    // ALL: every step of this block stores both rows (no per-step store predicates)
    auto step = [&](auto k_c, int i, auto rsimd_c, auto bsimd_c, auto all_c) __attribute__((always_inline)) {
        constexpr int k = decltype(k_c)::value;
        constexpr bool ALL = decltype(all_c)::value;
        constexpr bool BSIMD = decltype(bsimd_c)::value;
        // keep each step's memory operations in its step: the scheduler would otherwise sink
        // the prefetch loads toward their use (shorter live ranges), shortening the prefetch
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t v = level_group(k % NS, rsimd_c);
        issue((k + PF) % NS, i + PF);
        if constexpr (MODE != 4) store_row(STRIP_LEV, Y0 + i - 3, ALL || (i >= 3 && i < vh + 3), v);
        // row sums: the groups left and right of this lane's
        const uint32_t d0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, true);  // wave_shr:1 (bound_ctrl: lane 0 reads 0)
        const uint32_t d2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, true);  // wave_shl:1
        float4 o;
        // taps shifted onto the three dwords (10 v_dot4, no v_alignbyte)
        auto dot4 = [](uint32_t a, uint32_t w, uint32_t c) { return __builtin_amdgcn_udot4(a, w, c, false); };
        o.x = (float)dot4(d0, W00, dot4(v, W01, 0u));
        o.y = (float)dot4(d0, W10, dot4(v, W11, dot4(d2, W12, 0u)));
        o.z = (float)dot4(d0, W20, dot4(v, W21, dot4(d2, W22, 0u)));
        o.w = (float)dot4(v, tp.tapA, dot4(d2, tp.tapB, 0u));
        R[k % 7] = o;
        {
            // blurred row y - 3 from the row sums of steps i-6 .. i (every lane computes it;
            // only output lanes of steps 6 .. n-1 store it)
            // two pixels per packed-f32 op (v_pk_add / v_pk_mul / v_pk_fma: per element the
            // same IEEE operations as the scalar form)
            auto r = [&](int t) -> const float4& { return R[(k - t + 14) % 7]; };
            float S[4];
#pragma unroll
            for (int hp = 0; hp < 2; ++hp) {
                auto c = [&](int t) {
                    const float4& q = r(t);
                    return hp == 0 ? f2v{q.x, q.y} : f2v{q.z, q.w};
                };
                const f2v F6 = {f6, f6}, F5 = {f5, f5}, F4 = {f4, f4}, F3 = {f3, f3};
                f2v a = (c(6) + c(0)) * F6;
                a = __builtin_elementwise_fma(c(5) + c(1), F5, a);
                a = __builtin_elementwise_fma(c(4) + c(2), F4, a);
                a = __builtin_elementwise_fma(c(3), F3, a);
                S[2 * hp] = a.x;
                S[2 * hp + 1] = a.y;
            }
            uint32_t packed = 0;
            if (BSIMD) {
#pragma unroll
                for (int j = 0; j < 4; ++j) packed = __builtin_amdgcn_cvt_pk_u8_f32(S[j], j, packed);
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t Si = (uint32_t)(S[j] * 65536.0f);
                    const bool simd = x + j < L.bsimd_end;
                    const uint32_t val = (Si + (simd ? 32767u + ((Si >> 16) & 1u) : 32768u)) >> 16;
                    packed |= min(val, 255u) << (8 * j);
                }
            }
            const int slot = (i + 2) & 3;                // row Y0 + i - 6 (Y0 % 4 == 0)
            sbl[slot * 64 + sbl_dw] = packed;
            if (slot == 3) {   // wave-uniform
                // rows Y0 + i - 9 .. Y0 + i - 6 complete (LDS operations of a wave run in order)
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                // read as the u32 it was written as (a vector-typed read would let the
                // compiler treat the row stores as dead under type-based alias analysis)
                const uint32_t* fp = (const uint32_t*)__builtin_assume_aligned(sbl + 64 * fj + 4 * ft, 16);
                const v4u q = {fp[0], fp[1], fp[2], fp[3]};
                const bool ok = ALL || (i >= 9 && i - 9 < vh);
                __builtin_amdgcn_raw_buffer_store_b128(q, rblr, ok ? fl_off : 0x80000000u,
                                                       ok ? (Y0 + i - 9) * pitch : 0, STRIP_ST_POLICY);
                // wait states before a VALU may overwrite the store's data VGPRs: the 16-byte
                // store reads them after issue, and the compiler inserts none when soffset is
                // an SGPR (measured: lanes 12-15 of each 16 stored the next step's v_perm); the
                // operand keeps them allocated to the stored value until then (without it the
                // scheduler may still put a VALU write of them between the store and the nop:
                // a second band store measured wrong tiles at random, r6zb)
                __asm__ volatile("s_nop 4" ::"v"(q));
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            }
        }
    };
    constexpr int U = NS == 7 ? 7 : 7 * NS;   // steps per block: a multiple of NS and of 7
    auto walk = [&](auto rsimd_c, auto bsimd_c) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            issue(i % NS, i);
            // the same memory-op sequence as a block's last steps (two stores after each
            // issue), so the loop header sees one pending-load state from both edges
            if constexpr (MODE != 4) store_row(STRIP_LEV, 0, false, 0u);
        }
        // whole blocks of U steps (no per-step exits: steps past n load clamped rows and
        // store nothing but the last band's rows past the level, into its padding band)
        // sync > 0 only when a workgroup is one strip row (every wave takes the same steps)
        int nblk = 0;
        auto block = [&](int i0, auto all_c) __attribute__((always_inline)) {
            if (sync > 0) {
                if (nblk % sync == 0) __builtin_amdgcn_s_barrier();
                ++nblk;
            }
            unroll_seq([&](auto k_c) { step(k_c, i0 + decltype(k_c)::value, rsimd_c, bsimd_c, all_c); },
                       std::make_integer_sequence<int, U>{});
        };
        int i0 = 0;
        // the first block (the 6 halo steps), then the blocks that store every step (a copy
        // without the store predicates), then the rest
        static_assert(U >= 6, "the first block holds the halo steps");
        block(0, std::false_type{});
        for (i0 = U; i0 + U <= vh + 3; i0 += U) block(i0, std::true_type{});
        const int nend = ((vh + 3) & ~3) + 6;   // >= n: the last band's flush step < nend
        for (; i0 < nend; i0 += U) block(i0, std::false_type{});
    };
    // two forms only (code size): interior waves, and right-edge waves with per-pixel forms
    if ((L0 || wave_rsimd) && wave_bsimd) walk(std::true_type{}, std::true_type{});
    else walk(std::false_type{}, std::false_type{});
}

template <int MODE>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(MODE != 3 ? STRIP_WPE0 : STRIP_WPE3))) void k_level_strip(const Geometry* __restrict__ g,
                                                     const uint8_t* __restrict__ ltab,
                                                     const uint8_t* __restrict__ in0,
                                                     const uint8_t* __restrict__ in1, int split,
                                                     size_t stride, size_t bstride,
                                                     uint8_t* __restrict__ pyr,
                                                     uint8_t* __restrict__ blur, int level,
                                                     int sth, int sync) {
    int bx, b;
    xcd_block(bx, b);
    // wave of this image; readfirstlane makes it (and the strip row, the row counters and the
    // row addresses derived from it) scalar for the compiler, not per-lane VALU work
    const int wv = bx * (int)(blockDim.x >> 6) + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    __shared__ __attribute__((aligned(16))) uint32_t sbl[8][4 * 64];   // per wave: 4 blurred rows
    level_strip_wave<MODE>(g, ltab, in0, in1, split, stride, bstride, pyr, blur, level, sth, sync,
                           wv, b, sbl[threadIdx.x >> 6]);
}

// ---- k_pyr_chain: every level of a small batch in one launch ----
// A lone frame's pyramid as per-level launches is a chain of eight kernels of a few
// microseconds each, the GPU mostly idle.  Here one workgroup per (tile, image) computes its
// tile of every level with no grid-wide dependency: level 0's footprint is staged from the
// pyramid into LDS, and each level l >= 1 is computed over its footprint (host-built,
// ChainRect: the owned rectangle + blur halo + what the next level's footprint reads) from
// level l - 1's footprint in the other LDS buffer, so the tiles overlap (recomputed halos)
// instead of waiting for each other.  The owned pixels of each level and their blur go to HBM.
// Arithmetic per pixel: HResizeLinear + VResizeLinear(Vec) (vresize, as k_level's scalar
// border path) and RowFilter<uchar,int> + SymmColumnFilter in the exact integer form of
// tile_columns (S < 2^24, SSE2 pixels round half to even) -- src/ORBextractor.cc:1129-1154,
// :1107-1108.
#define CHAIN_NT 1024
__device__ __forceinline__ int reflect101_fast(int p, int len) {
    return (unsigned)p < (unsigned)len ? p : reflect101_i(p, len);
}

// (x * y) >> 32 of two 24-bit values: one v_mul_hi_u32_u24
__device__ __forceinline__ uint32_t mulhi_u24(uint32_t x, uint32_t y) {
    return (uint32_t)(((uint64_t)(x & 0xFFFFFFu) * (y & 0xFFFFFFu)) >> 32);
}

// bit j: pixel x0 + j (clamped to x1) takes the SSE2 vertical form (x < rsimd_end)
__device__ __forceinline__ uint32_t x_simd_bits(int x0, int x1, int rsimd_end) {
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) m |= (min(x0 + j, x1) < rsimd_end ? 1u : 0u) << j;
    return m;
}

// i / d for the item loops (d >= 1, i < 2^26): one v_mul_hi_u32 by m = ceil(2^32 / d)
struct Div {
    uint32_t m, d;
    // floor((2^32 - 1) / d) + 1 == ceil(2^32 / d) for every d >= 2 (a 32-bit division)
    __device__ explicit Div(int dd) : m(dd > 1 ? 0xFFFFFFFFu / (uint32_t)dd + 1u : 0u), d((uint32_t)dd) {}
    __device__ int operator()(int i) const { return d > 1 ? (int)__umulhi((uint32_t)i, m) : i; }
};

// Reflected columns of a footprint that touches the image's left / right edge, written into
// its rows' pads (x = -1..-3 <- 1..3, x = W..W+2 <- W-2..W-4: BORDER_REFLECT_101), so that the
// blur's row pass reads every group as an interior one.  Returns whether it wrote anything (the
// caller then needs a barrier before the row pass); uniform over the workgroup.
template <int NT>
__device__ __forceinline__ bool chain_fill(const ChainRect& c, const LevelGeom& Lv, uint8_t* buf,
                                           int P, int tid) {
    const int W = Lv.w, fh = c.fy1 - c.fy0 + 1;
    const bool left = c.fx0 == 0, right = c.fx1 == W - 1;
    if (!left && !right) return false;
    for (int i = tid; i < 2 * fh; i += NT) {
        const int r = i >> 1;
        uint8_t* row = buf + r * P + 4 - c.fx0;   // row[x] = pixel x
        if ((i & 1) == 0 && left) {
            row[-1] = row[min(1, W - 1)];
            row[-2] = row[reflect101_fast(-2, W)];
            row[-3] = row[reflect101_fast(-3, W)];
        } else if ((i & 1) == 1 && right) {
            row[W] = row[reflect101_fast(W, W)];
            row[W + 1] = row[reflect101_fast(W + 1, W)];
            row[W + 2] = row[reflect101_fast(W + 2, W)];
        }
    }
    return true;
}

// Row pass of the blur of level l's owned rectangle (rows oy0 - 3 .. oy1 + 2, reflected) from
// its footprint in LDS (src: padded rows, chain_pitch P) into rsum (int row sums, RW = 4 ng per
// row): three aligned dwords per 4-pixel group (bytes xg - 4 .. xg + 7, the left pad and
// chain_fill's reflected columns included), the sums as v_dot4 on shifted words, as
// tile_out_rows.
template <int NT>
__device__ __forceinline__ void chain_rows(const ChainRect& c, const LevelGeom& Lv, const uint8_t* src,
                                           int P, int* rsum, const Geometry* g, int tid) {
    const int ow = c.ox1 - c.ox0, oh = c.oy1 - c.oy0;
    if (ow <= 0 || oh <= 0) return;
    const int ng = (ow + 3) >> 2, RW = 4 * ng;
    const int H = Lv.h;
    const uint32_t tapA = (uint32_t)g->taps[0] | (uint32_t)g->taps[1] << 8 | (uint32_t)g->taps[2] << 16 |
                          (uint32_t)g->taps[3] << 24;
    const uint32_t tapB = (uint32_t)g->taps[4] | (uint32_t)g->taps[5] << 8 | (uint32_t)g->taps[6] << 16;
    const Div dv(ng);
    for (int i = tid; i < (oh + 6) * ng; i += NT) {
        const int rr = dv(i), q = i - rr * ng;
        const int ry = reflect101_fast(c.oy0 - 3 + rr, H) - c.fy0;
        const int xg = c.ox0 + 4 * q;
        const uint32_t* sw = (const uint32_t*)(src + ry * P + (xg - c.fx0));   // x = xg - 4 ..
        const uint32_t d0 = sw[0], d1 = sw[1], d2 = sw[2];
        int4 o;
        o.x = (int)__builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d1, d0, 1), tapA,
                  __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d2, d1, 1), tapB, 0u, false), false);
        o.y = (int)__builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d1, d0, 2), tapA,
                  __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d2, d1, 2), tapB, 0u, false), false);
        o.z = (int)__builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d1, d0, 3), tapA,
                  __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d2, d1, 3), tapB, 0u, false), false);
        o.w = (int)__builtin_amdgcn_udot4(d1, tapA, __builtin_amdgcn_udot4(d2, tapB, 0u, false), false);
        *(int4*)(rsum + rr * RW + 4 * q) = o;
    }
}

// Column pass of the blur of level l's owned rectangle from rsum, stored to the blurred
// pyramid: SymmColumnFilter in the exact integer form of tile_columns (S < 2^24, SSE2 pixels
// round half to even).
template <int NT>
__device__ __forceinline__ void chain_cols(const ChainRect& c, const LevelGeom& Lv, const int* rsum,
                                           uint8_t* dblur, const Geometry* g, int tid) {
    const int ow = c.ox1 - c.ox0, oh = c.oy1 - c.oy0;
    if (ow <= 0 || oh <= 0) return;
    const int ng = (ow + 3) >> 2, RW = 4 * ng;
    const uint32_t t3 = (uint32_t)g->taps[3], t4 = (uint32_t)g->taps[4];
    const uint32_t t5 = (uint32_t)g->taps[5], t6 = (uint32_t)g->taps[6];
    const Div dv(ng);
    for (int i = tid; i < oh * ng; i += NT) {
        const int rr = dv(i), q = i - rr * ng;
        const int y = c.oy0 + rr, xg = c.ox0 + 4 * q;
        int4 v[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) v[k] = *(const int4*)(rsum + (rr + k) * RW + 4 * q);
        uint32_t packed = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            auto e = [&](int k) { return (uint32_t)((const int*)&v[k])[j]; };
            const uint32_t S = t3 * e(3) + t4 * (e(2) + e(4)) + t5 * (e(1) + e(5)) + t6 * (e(0) + e(6));
            const bool simd = xg + j < Lv.bsimd_end;
            const uint32_t val = (S + (simd ? 32767u + ((S >> 16) & 1u) : 32768u)) >> 16;
            packed |= min(val, 255u) << (8 * j);
        }
        uint8_t* d = dblur + blur_off(xg, y, Lv.pitch, Lv.h);
        if (xg + 4 <= c.ox1) *(uint32_t*)d = packed;
        else
            for (int j = 0; xg + j < c.ox1; ++j) d[j] = (uint8_t)(packed >> (8 * j));
    }
}


template <int NT>
__global__ __launch_bounds__(NT) void k_pyr_chain(const Geometry* __restrict__ g,
                                                  const uint8_t* __restrict__ ltab,
                                                  const int16_t* __restrict__ rtab,
                                                  uint8_t* __restrict__ pyr,
                                                  uint8_t* __restrict__ blur) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tile = blockIdx.x, b = blockIdx.y;
    const int tid = threadIdx.x;
    const int L = g->nlevels;
    // LDS buffers by arithmetic on smem (a pointer picked from an array loses the LDS address
    // space: every access becomes a flat one)
    const int cbuf = g->chain_buf;
    int* rsum = (int*)(smem + 2 * cbuf);
    uint32_t* tabs = (uint32_t*)(smem + 2 * cbuf + g->chain_rs);
    uint8_t* pyr_b = pyr + (size_t)b * g->pyr_bytes;
    uint8_t* blr_b = blur + (size_t)b * g->pyr_bytes;
    // the tile's rectangles, table offsets (host-built) and the level geometry in LDS: the
    // table phase reads them per lane, and from memory each read would be a round trip
    __shared__ ChainRect CR[ORBX_MAX_LEVELS];
    __shared__ int toffs[2 * (ORBX_MAX_LEVELS + 1)];
    __shared__ LevelGeom LG[ORBX_MAX_LEVELS];
    const ChainRect* gCR = (const ChainRect*)(ltab + g->chain_tab) + (size_t)tile * L;
    if (tid < L) CR[tid] = gCR[tid];
    if (tid < 2 * (L + 1)) toffs[tid] = ((const int*)(ltab + g->chain_toffs))[(size_t)tile * 2 * (L + 1) + tid];
    {
        constexpr int NDW = (int)(sizeof(LevelGeom) / 4);
        for (int i = tid; i < L * NDW; i += NT) ((int*)LG)[i] = ((const int*)g->lv)[i];
    }
    // 1. level 0's footprint, in the same round trip (aligned dwords: fx0 is a multiple of 4,
    //    rows have >= 4 bytes of slack); every load in flight before the first LDS store
    const ChainRect c0 = gCR[0];
    const int fw0 = c0.fx1 - c0.fx0 + 1, fh0 = c0.fy1 - c0.fy0 + 1, P0 = chain_pitch(fw0);
    const int ndw = fw0 > 0 ? (fw0 + 3) >> 2 : 0, nst = ndw * fh0;
    const Div dv0(ndw > 0 ? ndw : 1);
    const uint8_t* s0 = pyr_b + g->lv[0].off + (size_t)c0.fy0 * g->lv[0].pitch + c0.fx0;
    const int pitch0 = g->lv[0].pitch;
    constexpr int SK = 8;
    uint32_t sv[SK];
#pragma unroll
    for (int u = 0; u < SK; ++u) {
        const int i = min(tid + u * NT, nst - 1), r = dv0(max(i, 0)), q = max(i, 0) - r * ndw;
        sv[u] = i >= 0 ? *(const uint32_t*)(s0 + (size_t)r * pitch0 + 4 * q) : 0u;
    }
    __syncthreads();
    // 2. every level's column / row tables, while the staged words are stored.  Per level
    //    (chain_level_words, from word tw[l]): per column group of 4 pixels a base word
    //    (aligned source byte | its offset o0 << 16 | 1 << 20 when all 4 pixels take the SSE2
    //    vertical form), 4 v_perm selectors (each pixel's two taps as u16s from the 8 bytes
    //    at base + o0) and 4 alpha pairs x 16 ((2048, 0) right of xmax: HResizeLinear's
    //    S[sx] * 2048); per row the two source rows | << 16 and the betas.  Entries: one per
    //    group, then one per row (te[l]).
    const int* te = toffs;
    const int* tw = toffs + (L + 1);
    const int ntab = te[L];
    for (int i = tid; i < ntab; i += NT) {
        int l = 1;
        while (i >= te[l + 1]) ++l;   // the level of entry i
        const ChainRect c = CR[l], cs = CR[l - 1];
        const LevelGeom& Ld = LG[l];
        const LevelGeom& Ls = LG[l - 1];
        const int16_t* xofs = rtab + Ld.rtab_off;
        const int16_t* alpha = xofs + Ld.w;
        const int16_t* yofs = alpha + 2 * Ld.w;
        const int16_t* beta = yofs + Ld.h;
        const int ng = (c.fx1 - c.fx0 + 4) >> 2;
        const int k = i - te[l];
        uint32_t* tl = tabs + tw[l];
        uint32_t* cbase = tl;
        uint32_t* csel = tl + ((ng + 3) & ~3);
        uint32_t* cal = csel + 4 * ng;
        if (k < ng) {
            int sx[4];
            uint32_t al[4];
            bool all_simd = true;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int x = min(c.fx0 + 4 * k + j, (int)c.fx1);
                sx[j] = (int)xofs[x] - cs.fx0;
                al[j] = x < Ld.xmax ? ((uint32_t)(uint16_t)alpha[2 * x] | ((uint32_t)(uint16_t)alpha[2 * x + 1] << 16))
                                    : 2048u;
                al[j] = ((al[j] & 0xFFFFu) << 4) | (((al[j] >> 16) << 4) << 16);
                all_simd = all_simd && x < Ld.rsimd_end;
            }
            const int base = sx[0] & ~3, o0 = sx[0] & 3;
            cbase[k] = (uint32_t)base | ((uint32_t)o0 << 16) | (all_simd ? (1u << 20) : 0u) |
                       ((uint32_t)(((x_simd_bits(c.fx0 + 4 * k, (int)c.fx1, Ld.rsimd_end)))) << 21);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int kk = min(max(sx[j] - sx[0], 0), 6);
                csel[4 * k + j] = (uint32_t)kk | (0x0Cu << 8) | ((uint32_t)(kk + 1) << 16) | (0x0Cu << 24);
                cal[4 * k + j] = al[j];
            }
        } else {
            const int y = min(c.fy0 + (k - ng), (int)c.fy1);
            const int sy = yofs[y];
            const int r0 = min(max(sy, 0), Ls.h - 1) - cs.fy0, r1 = min(max(sy + 1, 0), Ls.h - 1) - cs.fy0;
            ((uint2*)(cal + 4 * ng))[k - ng] =
                make_uint2((uint32_t)r0 | ((uint32_t)r1 << 16),
                           (uint32_t)(uint16_t)beta[2 * y] | ((uint32_t)(uint16_t)beta[2 * y + 1] << 16));
        }
    }
#pragma unroll
    for (int u = 0; u < SK; ++u) {
        const int i = tid + u * NT;
        if (i < nst) {
            const int r = dv0(i), q = i - r * ndw;
            ((uint32_t*)(smem + r * P0))[q + 1] = sv[u];   // after the row's 4-byte pad
        }
    }
    for (int i = tid + SK * NT; i < nst; i += NT) {   // footprints beyond SK * NT words
        const int r = dv0(i), q = i - r * ndw;
        ((uint32_t*)(smem + r * P0))[q + 1] = *(const uint32_t*)(s0 + (size_t)r * pitch0 + 4 * q);
    }
    __syncthreads();
    // 3. level 0's blur rows; then per level l >= 1: the previous level's blur columns beside
    //    this level's resize (they share no LDS), then this level's blur rows
    if (chain_fill<NT>(c0, LG[0], smem, P0, tid)) __syncthreads();
    chain_rows<NT>(c0, LG[0], smem, P0, rsum, g, tid);
    __syncthreads();
    int lr = 0;   // the level whose row sums are in rsum (-1: none)
    ChainRect cp = c0;
    for (int l = 1; l < L; ++l) {
        chain_cols<NT>(cp, LG[lr], rsum, blr_b + LG[lr].off, g, tid);
        lr = -1;
        const ChainRect cd = CR[l];
        const LevelGeom& Ld = LG[l];
        const int fw = cd.fx1 - cd.fx0 + 1, fh = cd.fy1 - cd.fy0 + 1;
        if (fw <= 0) break;   // empty footprint: no deeper level of this tile needs anything
        const int Ps = chain_pitch(cp.fx1 - cp.fx0 + 1), Pd = chain_pitch(fw);
        const uint8_t* src = smem + ((l - 1) & 1) * cbuf;
        uint8_t* dst = smem + (l & 1) * cbuf;
        const int ng = (fw + 3) >> 2;
        const uint32_t* cbase = tabs + tw[l];
        const uint4* csel = (const uint4*)(cbase + ((ng + 3) & ~3));
        const uint4* cal = csel + ng;
        const uint2* rowt = (const uint2*)(cal + ng);
        uint8_t* dlev = pyr_b + Ld.off;
        // a thread keeps one column group q (its tables read once per level) and takes the rows
        // r0, r0 + R, ... (R = NT / ng rows at a time), two per trip.  Per row and group: three
        // aligned dwords of each source row realigned to the group's first tap (v_alignbyte),
        // each pixel's two taps as u16s by one v_perm and HResizeLinear as one v_dot2 with the
        // 16x alphas (H = 16 h, exact), as k_level's item3; VResizeLinearVec_32s8u as
        // v_and + v_mul_hi_u32_u24 per term, or the scalar form past the SSE2 loop's end
        const int R = NT / ng;
        const Div dq(ng);
        const int r0 = dq(tid), q = tid - r0 * ng;
        if (r0 < R) {
            const uint32_t bw = cbase[q];
            const int base = (int)(bw & 0xFFFFu), o0 = (int)((bw >> 16) & 3u);
            const bool all_simd = (bw >> 20) & 1u;
            const uint32_t simd_bits = bw >> 21;
            const uint4 sl4 = csel[q], al4 = cal[q];
            const uint32_t sels[4] = {sl4.x, sl4.y, sl4.z, sl4.w}, als[4] = {al4.x, al4.y, al4.z, al4.w};
            const int xg = cd.fx0 + 4 * q;
            const bool own_x = xg >= cd.ox0 && xg < cd.ox1;
            constexpr int RU = 2;
            for (int rb = r0; rb < fh; rb += RU * R) {
                uint2 rt[RU];
                uint32_t w[RU][2][3];
#pragma unroll
                for (int u = 0; u < RU; ++u) rt[u] = rowt[min(rb + u * R, fh - 1)];
#pragma unroll
                for (int u = 0; u < RU; ++u) {
                    const uint32_t* a = (const uint32_t*)(src + (int)(rt[u].x & 0xFFFFu) * Ps + 4 + base);
                    const uint32_t* c2 = (const uint32_t*)(src + (int)(rt[u].x >> 16) * Ps + 4 + base);
                    w[u][0][0] = a[0]; w[u][0][1] = a[1]; w[u][0][2] = a[2];
                    w[u][1][0] = c2[0]; w[u][1][1] = c2[1]; w[u][1][2] = c2[2];
                }
#pragma unroll
                for (int u = 0; u < RU; ++u) {
                    const int r = rb + u * R;
                    if (r >= fh) break;
                    const uint32_t wa0 = __builtin_amdgcn_alignbyte(w[u][0][1], w[u][0][0], o0);
                    const uint32_t wa1 = __builtin_amdgcn_alignbyte(w[u][0][2], w[u][0][1], o0);
                    const uint32_t wc0 = __builtin_amdgcn_alignbyte(w[u][1][1], w[u][1][0], o0);
                    const uint32_t wc1 = __builtin_amdgcn_alignbyte(w[u][1][2], w[u][1][1], o0);
                    const int b0 = (int)(rt[u].y & 0xFFFFu), b1 = (int)(rt[u].y >> 16);
                    const uint32_t bs0 = (uint32_t)b0 << 8, bs1 = (uint32_t)b1 << 8;
                    uint32_t out = 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const us2 al = __builtin_bit_cast(us2, als[j]);
                        const uint32_t H0 = __builtin_amdgcn_udot2(
                            __builtin_bit_cast(us2, __builtin_amdgcn_perm(wa1, wa0, sels[j])), al, 0u, false);
                        const uint32_t H1 = __builtin_amdgcn_udot2(
                            __builtin_bit_cast(us2, __builtin_amdgcn_perm(wc1, wc0, sels[j])), al, 0u, false);
                        // SSE2 form: ((h >> 4) * b) >> 16 = mulhi_u24((16 h) & ~0xFF, b << 8); the
                        // two terms are <= 1020 together, so no saturation (see item3)
                        uint32_t v = (mulhi_u24(H0 & ~0xFFu, bs0) +
                                      mulhi_u24(H1 & ~0xFFu, bs1) + 2u) >> 2;
                        if (!all_simd && !((simd_bits >> j) & 1u))
                            v = min((uint32_t)((__umul24(H0 >> 4, (uint32_t)b0) + __umul24(H1 >> 4, (uint32_t)b1) +
                                                (1u << 21)) >> 22), 255u);
                        out |= v << (8 * j);
                    }
                    *(uint32_t*)(dst + r * Pd + 4 + 4 * q) = out;
                    const int y = cd.fy0 + r;
                    if (own_x && y >= cd.oy0 && y < cd.oy1) {
                        uint8_t* d = dlev + (size_t)y * Ld.pitch + xg;
                        if (xg + 4 <= cd.ox1) *(uint32_t*)d = out;
                        else
                            for (int j = 0; xg + j < cd.ox1; ++j) d[j] = (uint8_t)(out >> (8 * j));
                    }
                }
            }
        }
        __syncthreads();
        if (chain_fill<NT>(cd, Ld, dst, Pd, tid)) __syncthreads();
        chain_rows<NT>(cd, Ld, dst, Pd, rsum, g, tid);
        __syncthreads();
        lr = l;
        cp = cd;
    }
    if (lr >= 0) chain_cols<NT>(cp, LG[lr], rsum, blr_b + LG[lr].off, g, tid);
}

hipError_t launch_pyr_chain(const ExtractLaunch& a, hipStream_t st) {
    const Geometry& G = *a.hg;
    KernelTimer dummy;
    KernelTimer& T = a.timer ? *a.timer : dummy;
    ORBX_TIMED_LAUNCH(T, K_LEVEL, k_pyr_chain<CHAIN_NT>, dim3(G.chain_gx * G.chain_gy, a.batch),
                      dim3(CHAIN_NT), (size_t)G.chain_lds, st, a.dg, a.ltab, a.rtab, a.pyr, a.blur);
    return hipGetLastError();
}

size_t level_lds_bytes(int ltw, int lth, int win_cap) {
    (void)ltw;
    (void)lth;
    auto r = [](size_t v) { return (v + 15) & ~(size_t)15; };
    const size_t tables = r(LT_G * 8) + r(LT_G * 4) + r(LT_G * 16) + r(LT_G * 16) + r(LT_HR * 8);
    const size_t phase12 = tables + r((size_t)win_cap + 16);
    const size_t phase34 = r((size_t)LT_HR * LT_W * 4);
    return r((size_t)LT_HR * LT_G * 4) + (phase12 > phase34 ? phase12 : phase34) + r(64);
}

static int level_mode(const LevelGeom& L, int l) {
    return l == 0 ? 0 : (L.copy ? 1 : (L.area2 ? 2 : 3));
}

typedef void (*LevelKernel)(const Geometry*, const uint8_t*, const uint8_t*, const uint8_t*, int,
                            size_t, size_t, uint8_t*, uint8_t*, int);
static LevelKernel level_kernel(int mode) {
    switch (mode) {
        case 0: return k_level<0>;
        case 1: return k_level<1>;
        case 2: return k_level<2>;
        default: return k_level<3>;
    }
}

// levels [l_begin, l_end) (launch_extract may fork a side branch in between)
hipError_t launch_levels(const ExtractLaunch& a, hipStream_t st, int l_begin, int l_end) {
    const Geometry& G = *a.hg;
    KernelTimer dummy;
    KernelTimer& T = a.timer ? *a.timer : dummy;
    for (int l = l_begin; l < l_end && l < G.nlevels; ++l) {
        const LevelGeom& L = G.lv[l];
        const int mode = level_mode(L, l);
        if (L.strip) {
            const int sth = a.sth[l], sns = (L.h + sth - 1) / sth;
            const int sync = L.snw <= 8 && ((STRIP_SYNC_LEVELS >> l) & 1) ? (mode == 3 ? STRIP_SYNC3 : STRIP_SYNC0) : 0;
            ORBX_TIMED_LAUNCH(T, K_LEVEL,
                              mode == 3 ? k_level_strip<3> : (a.in_place ? k_level_strip<4> : k_level_strip<0>),
                              sync > 0 ? dim3(sns, a.batch) : dim3((L.snw * sns + 3) / 4, a.batch),
                              dim3(sync > 0 ? 64 * L.snw : 256), 0, st, a.dg,
                              a.ltab, a.d_imgs, a.d_imgs2, a.split, a.stride, a.batch_stride,
                              a.pyr, a.blur, l, sth, sync);
        } else if (l == 0 && a.in_place) {
            // the tiled level-0 kernel reading the pyramid's own level 0 (its level stores
            // write back the bytes already there)
            ORBX_TIMED_LAUNCH(T, K_LEVEL, level_kernel(0), dim3(L.ntx * L.nty, a.batch), dim3(256),
                              a.level_lds, st, a.dg, a.ltab, (const uint8_t*)(a.pyr + L.off),
                              (const uint8_t*)(a.pyr + L.off), a.batch, (size_t)L.pitch,
                              (size_t)G.pyr_bytes, a.pyr, a.blur, l);
        } else {
            ORBX_TIMED_LAUNCH(T, K_LEVEL, level_kernel(mode), dim3(L.ntx * L.nty, a.batch), dim3(256),
                              a.level_lds, st, a.dg, a.ltab, a.d_imgs, a.d_imgs2, a.split,
                              a.stride, a.batch_stride, a.pyr, a.blur, l);
        }
        if (l == 0) T.alias(K_LEVEL0);
    }
    return hipGetLastError();
}


hipError_t prepare_level(size_t lds) {
    hipError_t e = hipSuccess;
    for (int m = 0; m < 4 && e == hipSuccess; ++m)
        e = hipFuncSetAttribute((const void*)level_kernel(m),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void*)k_pyr_chain<CHAIN_NT>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    return e;
}

}  // namespace orbx
