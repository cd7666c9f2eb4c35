// orbx_extract.hip — the ORB extractor as gfx950 kernels, batched over B images.
//
// Replaces ORB_SLAM2::ORBextractor::operator() (src/ORBextractor.cc:1065-1127).  Stages:
//   k_level        level l from l-1 + its 7x7 Gaussian (orbx_pyramid.hip; :1129-1154, :1108)
//   k_fast         FAST-9 + cell-local NMS per 30px cell         (ComputeKeyPointsOctTree :801-850)
//   k_octree       quadtree distribution, one workgroup/level    (DistributeOctTree :539-765)
//   k_orient_desc  IC angle + rBRIEF + level-major assembly      (:872-874, :77-147, :1097-1126)
// Every kernel is integer work except three float formulas that the reference evaluates in
// float (fastAtan2, the BRIEF rotation, the blur's SSE2 column pass); the library is built
// with -ffp-contract=off so each of those is a separately rounded v_mul/v_add, as on x86.
#include <hip/hip_runtime.h>

#include <mutex>
#include <type_traits>
#include <stdint.h>

#include "orbx_device.h"
#include "orbx_internal.h"
#include "orbx_math.h"
#include "orbx_kernels.h"

namespace orbx {

__constant__ __attribute__((aligned(4))) int8_t c_pattern[1024] = {
#include "orbx_pattern.inc"
};

// The same score with both polarities in the halves of one packed-f16 register, so every
// run min / max is one v_pk_minimum3 / v_pk_maximum3 for dark and bright together (40 of
// them instead of 80).  A circle pixel n enters as the f16 whose bits are n (a subnormal:
// f16 order = integer order, and the f16 modes keep subnormals), the low half negated:
// y = (-n, n).  Then low = max_arcs min_9 (-n) = -(min_arcs max_9 n) and high =
// max_arcs min_9 n, read back as the low 10 bits of each half (n <= 255, no rounding
// anywhere: min / max only select).  dark = v - min max n, bright = max min n - v.
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f16x2 arc_y(const uint8_t* p) {
    const _Float16 f = __builtin_bit_cast(_Float16, (unsigned short)*p);
    return f16x2{-f, f};   // folded into neg_lo / op_sel_hi source modifiers
}
__device__ __forceinline__ int fast_arc_score_pk(const uint8_t* roi, int cols, int r, int c) {
    const uint8_t* p = roi + r * cols + c;
    const int v = p[0];
    f16x2 y[16];
    y[0] = arc_y(p + 3 * cols);       y[1] = arc_y(p + 3 * cols + 1);
    y[2] = arc_y(p + 2 * cols + 2);   y[3] = arc_y(p + cols + 3);
    y[4] = arc_y(p + 3);              y[5] = arc_y(p - cols + 3);
    y[6] = arc_y(p - 2 * cols + 2);   y[7] = arc_y(p - 3 * cols + 1);
    y[8] = arc_y(p - 3 * cols);       y[9] = arc_y(p - 3 * cols - 1);
    y[10] = arc_y(p - 2 * cols - 2);  y[11] = arc_y(p - cols - 3);
    y[12] = arc_y(p - 3);             y[13] = arc_y(p + cols - 3);
    y[14] = arc_y(p + 2 * cols - 2);  y[15] = arc_y(p + 3 * cols - 1);
#define PMN3(a, b, c) __builtin_elementwise_minimum(__builtin_elementwise_minimum(a, b), c)
#define PMX3(a, b, c) __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c)
    f16x2 m3[16], m9[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) m3[i] = PMN3(y[i], y[(i + 1) & 15], y[(i + 2) & 15]);
#pragma unroll
    for (int i = 0; i < 16; ++i) m9[i] = PMN3(m3[i], m3[(i + 3) & 15], m3[(i + 6) & 15]);
    f16x2 b = PMX3(m9[0], m9[1], m9[2]);
#pragma unroll
    for (int i = 3; i < 15; i += 2) b = PMX3(b, m9[i], m9[i + 1]);
    b = __builtin_elementwise_maximum(b, m9[15]);
#undef PMN3
#undef PMX3
    const uint32_t bits = __builtin_bit_cast(uint32_t, b);
    return max(v - (int)(bits & 0x3FFu), (int)((bits >> 16) & 0x3FFu) - v);
}

// Keypoint tests at both thresholds on the M map in one read of the 3x3 neighbourhood.
__device__ __forceinline__ void fast_nms_kp2(const uint8_t* mb, int mw, int rr, int cc, int t_hi,
                                             int t_lo, bool& k_hi, bool& k_lo, int& score) {
    const uint8_t* p = mb + (rr + 1) * mw + (cc + 1);
    const int m = p[0], s = m - 1;
    score = s;
    const int q0 = p[-mw - 1], q1 = p[-mw], q2 = p[-mw + 1], q3 = p[-1], q4 = p[1];
    const int q5 = p[mw - 1], q6 = p[mw], q7 = p[mw + 1];
    // a neighbour q suppresses at threshold t when q > t and q - 1 >= s, i.e. q >= m: the
    // candidates (q >= m) are the same for both thresholds, and one suppresses at t iff the
    // largest of them exceeds t
    int supp = 0;
#define ORBX_NB(q) supp = max(supp, (q) >= m ? (q) : 0);
    ORBX_NB(q0) ORBX_NB(q1) ORBX_NB(q2) ORBX_NB(q3) ORBX_NB(q4) ORBX_NB(q5) ORBX_NB(q6) ORBX_NB(q7)
#undef ORBX_NB
    const bool base = s > 0;
    k_hi = base && m > t_hi && supp <= t_hi;
    k_lo = base && m > t_lo && supp <= t_lo;
}

#define FAST_PF 6      // prefetched ROI dwords per lane (larger ROIs are staged directly)
                     // 2.304 -> 2.288 ms per step one-stream (r4e A/B, B=512)
#define FAST_WPE 6     // minimum waves per SIMD requested from the register allocator (80 VGPRs)
#define OCT_NT 128         // k_octree threads per list (64 / 128 / 256 / 512) at large batches.
                           // Round 5, 512 pairs (r5v2 / r5v3): 128 threads 0.306 ms one-stream
                           // against 0.265 for 256, but the scheduled step is 1 % faster
                           // (128.5-128.9 k vs 127.2-127.5 k pairs/s): the smaller workgroups
                           // pack beside the pyramid and FAST launches; 64 threads 0.398 ms
#define OCT_NT_SMALL 256   // ... when batch * levels <= 256; one stereo pair: 128 0.112, 256 0.081,
                           // 1024 0.101 ms
#define OD_SPATIAL_MIN_BATCH 16   // ... for batches of at least this many images
#define OD_SP_XS 5     // ... columns of 32 pixels
#define OD_SP_YS 5     // ... in bands of 32 rows.  r5d, 512 pairs: k_orient_desc 1.094 ms in
                       // list order, 1.054 / 1.068 / 1.098 ms for bands of 32 / 64 / 128 rows
                       // (k_octree +0.007 ms for the order)
#define OD_WPE 5       // at most 96 VGPRs: five waves per SIMD (6: spills)
__device__ __forceinline__ void lds_order() { __asm__ volatile("" ::: "memory"); }

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// Pixels s_abs and s_abs+1 of a byte run held in dwords A[0..3] as two zero-extended u16s
// (one v_perm: selector bytes s, 0x0C (= 0x00), s+1, 0x0C over the dword pair).
__device__ __forceinline__ u16x2 pair_u16(const uint32_t* A, int s_abs) {
    const int k = s_abs >> 2, s = s_abs & 3;
    const uint32_t sel = (uint32_t)s | 0x0C00u | (uint32_t)(s + 1) << 16 | 0x0C000000u;
    return __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(A[k + 1], A[k], sel));
}

// Pixels s_abs and s_abs+2 as two zero-extended u16s (one v_perm).  A v_and for the pairs
// that start a dword measured slower (r5c: 77 VGPRs, 1.176 vs 1.165 ms).
__device__ __forceinline__ uint32_t pair_u16_stride2(const uint32_t* A, int s_abs) {
    const int k = s_abs >> 2, s = s_abs & 3;
    const uint32_t sel = (uint32_t)s | 0x0C00u | (uint32_t)(s + 2) << 16 | 0x0C000000u;
    return __builtin_amdgcn_perm(A[k + 1], A[k], sel);
}

// Bit positions of pixels 0..3 in the compass4_fr flag word.
#define CMP_B0 14
#define CMP_B1 15
#define CMP_B2 30
#define CMP_B3 31

// The compass pre-test below on full-rate 32-bit adds and logic only.  With two pixels per
// dword as u16 halves (pixels j and j+2) and K = (0x4000 - t - 1) in each half:
//   n > v + t  <=>  bit 14 of n + (K - v)       n < v - t  <=>  bit 14 of (K + v) - n
// (every half stays inside (0, 0x8000), so no carry or borrow crosses a half), and "two
// neighbouring compass pixels beyond t on one side" is (b0 | b8) & (b4 | b12) on those bits.
// Returns the flags of pixels 0..3 at bits CMP_B0..CMP_B3 (all other bits zero).
template <int XO>
__device__ __forceinline__ uint32_t compass4_fr(const uint8_t* roi0, int rp, int R, int gx, uint32_t K) {
    // R * rp as a 24-bit multiply (v_mul_lo_u32 is a quarter-rate instruction)
    const uint8_t* row = roi0 + __umul24((uint32_t)R, (uint32_t)rp);
    const uint32_t* rc = (const uint32_t*)row + gx;
    const uint32_t* rd = (const uint32_t*)(row + 3 * rp) + gx;
    const uint32_t* ru = (const uint32_t*)(row - 3 * rp) + gx;
    constexpr int KC = (XO + 9) >> 2;
    constexpr int K0 = (XO + 3) >> 2, K1 = (XO + 6) >> 2;
    uint32_t C[5], D[5], U[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        C[k] = k <= KC ? rc[k] : 0u;
        D[k] = (k >= K0 && k <= K1) ? rd[k] : 0u;
        U[k] = (k >= K0 && k <= K1) ? ru[k] : 0u;
    }
    uint32_t F[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int o = XO + 3 + h;                   // byte of pixel h (centre row): pixels h, h+2
        const uint32_t V = pair_u16_stride2(C, o);
        const uint32_t N12 = pair_u16_stride2(C, o - 3), N4 = pair_u16_stride2(C, o + 3);
        const uint32_t N0 = pair_u16_stride2(D, o), N8 = pair_u16_stride2(U, o);
        const uint32_t A = K - V, B = K + V;
        const uint32_t bright = ((N0 + A) | (N8 + A)) & ((N4 + A) | (N12 + A));
        const uint32_t dark = ((B - N0) | (B - N8)) & ((B - N4) | (B - N12));
        F[h] = (bright | dark) & 0x40004000u;       // bits 14 (pixel h), 30 (pixel h + 2)
    }
    return F[0] | (F[1] << 1);
}

// One pixel pair of the compass test (u16 halves as in compass4_fr) with the pairs folded
// first: (b0 | b8) & (b4 | b12) for "brighter than v + t" is min(max(n0, n8), max(n4, n12))
// > v + t, and the darker side is max(min(n0, n8), min(n4, n12)) < v - t, so six packed u16
// min / max and one add or subtract per side replace eight adds and six logic ops (r5c,
// 512 pairs: k_fast 1.218 -> 1.165 ms one-stream, 128.8 k -> 130.2 k pairs/s).
__device__ __forceinline__ uint32_t compass_pair_mm(uint32_t V, uint32_t N0, uint32_t N4,
                                                    uint32_t N8, uint32_t N12, uint32_t K) {
    const u16x2 a0 = __builtin_bit_cast(u16x2, N0), a4 = __builtin_bit_cast(u16x2, N4);
    const u16x2 a8 = __builtin_bit_cast(u16x2, N8), a12 = __builtin_bit_cast(u16x2, N12);
    const uint32_t mb = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(
        __builtin_elementwise_max(a0, a8), __builtin_elementwise_max(a4, a12)));
    const uint32_t md = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(
        __builtin_elementwise_min(a0, a8), __builtin_elementwise_min(a4, a12)));
    return ((mb + (K - V)) | ((K + V) - md)) & 0x40004000u;
}

// The compass pre-test of 16 adjacent pixels (detection columns 16g .. 16g+15 of ROI row R),
// the arithmetic of compass4_fr on four 4-pixel groups.  The centre row's 8 dwords and the
// +-3 rows' 6 are read with 16-byte LDS loads (the ROI rows are 16-byte aligned).  Returns
// bit i = pixel 16g + i passes.
template <int XO>
__device__ __forceinline__ uint32_t compass16_fr(const uint8_t* roi0, int rp, int R, int g, uint32_t K) {
    const uint8_t* row = roi0 + __umul24((uint32_t)R, (uint32_t)rp);
    const uint4* rc = (const uint4*)row + g;
    const uint4* rd = (const uint4*)(row + 3 * rp) + g;
    const uint4* ru = (const uint4*)(row - 3 * rp) + g;
    const uint4 c0 = rc[0], c1 = rc[1], d0 = rd[0], u0 = ru[0];
    const uint2 d1 = *(const uint2*)(rd + 1), u1 = *(const uint2*)(ru + 1);
    const uint32_t C[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    const uint32_t D[6] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y};
    const uint32_t U[6] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y};
    uint32_t mask = 0;
#pragma unroll
    for (int h4 = 0; h4 < 4; ++h4) {
        uint32_t F[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int o = XO + 3 + 4 * h4 + h;      // byte of pixel 4 h4 + h (centre row)
            const uint32_t V = pair_u16_stride2(C, o);
            const uint32_t N12 = pair_u16_stride2(C, o - 3), N4 = pair_u16_stride2(C, o + 3);
            const uint32_t N0 = pair_u16_stride2(D, o), N8 = pair_u16_stride2(U, o);
            F[h] = compass_pair_mm(V, N0, N4, N8, N12, K);
        }
        const uint32_t f = F[0] | (F[1] << 1);       // bits 14, 15, 30, 31: pixels 0..3
        mask |= (((f >> 14) & 3u) | ((f >> 28) & 12u)) << (4 * h4);
    }
    return mask;
}

// Inclusive prefix sum over the wave (DPP row shifts, then the row broadcasts).
__device__ __forceinline__ int wave_incl_scan_dpp(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);   // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);   // row_bcast:31
    return v;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FAST_WPE))) void k_fast(const Geometry* __restrict__ g,
                                              const CellDesc* __restrict__ cells,
                                              const uint8_t* __restrict__ pyr,
                                              int* __restrict__ ccnt,
                                              uint32_t* __restrict__ cand,
                                              int c_begin, int c_end, int nc) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // XCD block order: an XCD walks a contiguous range of (image, cell block), so the ROI
    // borders shared with the neighbouring cells (left / right and the next cell row) hit its L2
    int bx, b;
    xcd_block(bx, b);
    // one wave owns nc (FAST_NC, or fewer for a small batch: fast_cells_per_wave) consecutive
    // cells; no block-level barriers: waves are independent.  Cells [c_begin, c_end) of every
    // image (a launch may cover a range of levels)
    const int c_first = __builtin_amdgcn_readfirstlane(c_begin + (bx * 4 + wid) * nc);
    if (c_first >= c_end) return;
    const int ncw = min(nc, c_end - c_first);
    const int roi_cap = (g->max_roi_bytes + 15) & ~15, mb_cap = (g->max_mbuf_bytes + 15) & ~15;
    const int cl_cap = (g->max_cell_px * 2 + 15) & ~15;
    // one buffer: the corners found so far, then the current pass's survivor list (scored in
    // place: a corner is written at or below the entry it was read from)
    uint8_t* roi0 = smem + wid * (roi_cap + mb_cap + 64 * 2 + cl_cap);
    uint8_t* mb = roi0 + roi_cap;
    int16_t* list = (int16_t*)(mb + mb_cap);
    int16_t* corners = list;
    const uint8_t* pyr_b = pyr + (size_t)b * g->pyr_bytes;

    // ROI of a cell as aligned dwords, dense rows of ndw dwords: LDS dword t = lane + 64j
    // ROI of a cell as a 2-D lane grid: lane (r = lane / 16, col = lane % 16) holds ROI dword
    // col of rows r, r + 4, .., so an element costs one 24-bit multiply-add of address and no
    // divisions (columns >= ndw idle)
    uint32_t pf[FAST_PF2D];
    const int lr2 = lane >> 4, lc2 = lane & 15;
    auto prefetch = [&](const CellDesc& c) -> bool {
        const int ndw = ((c.ini_x & 3) + c.cols + 3) >> 2;
        if (ndw > 16 || c.rows > 4 * FAST_PF2D || c.rows <= 6 || c.cols <= 6) return false;
        const LevelGeom& L = g->lv[c.level];
        // every lane reads its 10 rows unclamped (rows past the ROI land in the LDS buffer's
        // spare rows; the pyramid buffer has FAST_PF2D * 4 rows of slack after the last
        // image): a wave-uniform row base per load plus one lane offset, no per-load VALU
        const uint8_t* src = pyr_b + L.off + (size_t)c.ini_y * L.pitch + (c.ini_x & ~3);
        const uint32_t lane_off = __umul24((uint32_t)lr2, (uint32_t)L.pitch) + 4u * (uint32_t)min(lc2, ndw - 1);
        // buffer loads: the ROI base in the descriptor and row j's offset in soffset (scalar),
        // so a load costs no 64-bit address add (10 per cell with flat loads)
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
        for (int j = 0; j < FAST_PF2D; ++j)
            pf[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, lane_off, (uint32_t)(4 * j) * (uint32_t)L.pitch, 0);
        return true;
    };
    CellDesc cn = cells[c_first];
    bool have = prefetch(cn);
    // The wave's cells' candidates are written back to back from its first cell's slot (the
    // slots of consecutive cells are contiguous, and a cell writes at most its capacity), so
    // the octree reads about one cache line per wave instead of one per cell: a cell's run
    // starts `delta` words before its own slot, ccnt = count | delta << 16
    const uint32_t wslot = (uint32_t)cn.slot;
    uint32_t wpos = 0;
    for (int k = 0; k < ncw; ++k) {
        const int ci = c_first + k;
        const CellDesc c = cn;
        const bool pre = have;
        const int rows = c.rows, cols = c.cols, dh = rows - 6, dw = cols - 6;
        int* cnt_out = ccnt + (size_t)b * g->n_cells + ci;
        const int xo = c.ini_x & 3;
        const int ndw = (xo + cols + 3) >> 2;
        const int lp = fast_lpitch(ndw, dw);   // LDS row pitch of the ROI, dwords
        const int rp = lp * 4;
        if (dh > 0 && dw > 0) {
            if (pre) {
                if (lc2 < ndw) {
                    uint32_t* l = (uint32_t*)roi0 + lr2 * lp + lc2;
#pragma unroll
                    for (int j = 0; j < FAST_PF2D; ++j)
                        l[4 * j * lp] = pf[j];
                }
            } else {
                const LevelGeom& L = g->lv[c.level];
                stage_dwords<64>(pyr_b + L.off + (size_t)c.ini_y * L.pitch + (c.ini_x & ~3),
                                 L.pitch, rows, ndw, (uint32_t*)roi0, lp, lane);
            }
        }
        if (k + 1 < ncw) {   // the next cell's ROI loads stay in flight during this cell
            cn = cells[ci + 1];
            have = prefetch(cn);
        }
        if (dh <= 0 || dw <= 0) {
            if (lane == 0) *cnt_out = 0;
            continue;
        }
        const uint8_t* roi = roi0 + xo;
        const int mw = dw + 2;
        // zero the score map 16 bytes per lane (mb is 16-byte aligned, mb_cap a multiple of 16)
        for (int i = lane; i < ((dh + 2) * mw + 15) >> 4; i += 64) ((uint4*)mb)[i] = make_uint4(0u, 0u, 0u, 0u);
        lds_order();
        const int gsh = ((dw + 3) >> 2) <= 8 ? 3 : 4;
        [[maybe_unused]] const int rpp = 64 >> gsh;
        const int sub = lane >> gsh, gx = lane & ((1 << gsh) - 1);
        const uint32_t colmask4 = (1u << min(max(dw - 4 * gx, 0), 4)) - 1u;
        const uint32_t colmask = ((colmask4 & 3u) << CMP_B0) | ((colmask4 & 12u) << (CMP_B2 - 2));
        [[maybe_unused]] constexpr int PB[4] = {CMP_B0, CMP_B1, CMP_B2, CMP_B3};
        // 16 pixels per lane: lpr lanes per detection row, 64 / lpr rows per pass; one pass
        // is one block of the survivor list
        const int lsh = dw > 32 ? 2 : 1;
        const int rpp16 = 64 >> lsh;
        const int sub16 = lane >> lsh, g16 = lane & ((1 << lsh) - 1);
        const int rem16 = dw - 16 * g16;
        const uint32_t colmask16 = rem16 >= 16 ? 0xFFFFu : (rem16 > 0 ? (1u << rem16) - 1u : 0u);
        const int rows_blk = rpp16;
        (void)colmask; (void)sub; (void)gx;
        uint32_t* slot = cand + (size_t)b * g->cand_words + wslot + wpos;
        const int t_ini = g->ini_th, t_min = g->min_th;
        int base = 0;
        // Two passes: the cell is first detected at iniThFAST alone (compass test, arc scores
        // and NMS at that threshold); only a cell with no keypoint there is detected again at
        // minThFAST (:830-837).
        for (int pass = 0; pass < 2; ++pass) {
        const int tq = pass == 0 ? t_ini : t_min;
        const uint32_t KT = (uint32_t)(0x4000 - tq - 1) * 0x10001u;
        // 1. compass pre-test at tq, 4 pixels per lane: 2^gsh lanes per detection row (groups
        //    of 4 columns), 64 >> gsh rows per pass, so lane order then pixel order within a
        //    lane is raster order.
        int ncorner = 0;
        for (int rb = 0; rb < dh; rb += rows_blk) {
            int nlist = 0;
            {
                const int rr = rb + sub16;
                const int R = min(rr, dh - 1) + 3;
                uint32_t f;
                switch (xo) {
                    case 0: f = compass16_fr<0>(roi0, rp, R, g16, KT); break;
                    case 1: f = compass16_fr<1>(roi0, rp, R, g16, KT); break;
                    case 2: f = compass16_fr<2>(roi0, rp, R, g16, KT); break;
                    default: f = compass16_fr<3>(roi0, rp, R, g16, KT); break;
                }
                f &= rr < dh ? colmask16 : 0u;
                // ordered compaction: lanes are in raster order, bits within a lane too
                const int cnt = __builtin_popcount(f);
                const int incl = wave_incl_scan_dpp(cnt);
                int pos = incl - cnt;
                const int e0 = (rr << 6) | (16 * g16);
                int16_t* pl = list + ncorner;
                while (f) {
                    pl[pos++] = (int16_t)(e0 + __builtin_ctz(f));
                    f &= f - 1u;
                }
                nlist = __builtin_amdgcn_readlane(incl, 63);
            }
            lds_order();
            // 2. full arc score for the survivors only (dense across lanes); those above the
            //    lower threshold are appended to the corner list, keeping raster order
            const int lb = ncorner;
            for (int j0 = 0; j0 < nlist; j0 += 64) {
                const int j = j0 + lane;
                int pe = 0, m = 0;
                if (j < nlist) {
                    pe = list[lb + j];
                    const int rr = pe >> 6, cc = pe & 63;
                    m = fast_arc_score_pk(roi, rp, rr + 3, cc + 3);
                    mb[(rr + 1) * mw + cc + 1] = (uint8_t)max(m, 0);
                }
                const bool corner = j < nlist && m > tq;
                const uint64_t cm = __ballot(corner);
                if (corner) corners[ncorner + lanes_below(cm)] = (int16_t)pe;
                ncorner += __popcll(cm);
            }
            lds_order();
        }
        // 3. cell-local NMS at iniThFAST, or at minThFAST when the cell has no keypoint at
        //    iniThFAST (:833-837); 4. ordered compaction (raster order, as cv::FAST emits).
        const int th_hi = tq, th_lo = tq;
        if (ncorner <= 64) {
            int sc = 0, pe = 0;
            bool k_hi = false, k_lo = false;
            if (lane < ncorner) {
                pe = corners[lane];
                fast_nms_kp2(mb, mw, pe >> 6, pe & 63, th_hi, th_lo, k_hi, k_lo, sc);
            }
            const uint64_t mh = __ballot(k_hi);
            const bool kk = mh ? k_hi : k_lo;
            const uint64_t m = mh ? mh : __ballot(k_lo);
            if (kk) {
                const int idx = lanes_below(m);
                const int x = c.ini_x + (pe & 63) + 3 - ORBX_MIN_BORDER;
                const int y = c.ini_y + (pe >> 6) + 3 - ORBX_MIN_BORDER;
                if (idx < c.cap) slot[idx] = pack_cand(x, y, sc);
            }
            base = __popcll(m);
        } else {
            bool found = false;
            for (int j0 = 0; j0 < ncorner && !found; j0 += 64) {
                const int j = j0 + lane;
                int sc = 0;
                bool k_hi = false, k_lo = false;
                if (j < ncorner) {
                    const int pe = corners[j];
                    fast_nms_kp2(mb, mw, pe >> 6, pe & 63, th_hi, th_lo, k_hi, k_lo, sc);
                }
                found = __ballot(k_hi) != 0;
            }
            for (int j0 = 0; j0 < ncorner; j0 += 64) {
                const int j = j0 + lane;
                int sc = 0, pe = 0;
                bool k_hi = false, k_lo = false;
                if (j < ncorner) {
                    pe = corners[j];
                    fast_nms_kp2(mb, mw, pe >> 6, pe & 63, th_hi, th_lo, k_hi, k_lo, sc);
                }
                const bool kk = found ? k_hi : k_lo;
                const uint64_t m = __ballot(kk);
                if (kk) {
                    const int idx = base + lanes_below(m);
                    const int x = c.ini_x + (pe & 63) + 3 - ORBX_MIN_BORDER;
                    const int y = c.ini_y + (pe >> 6) + 3 - ORBX_MIN_BORDER;
                    if (idx < c.cap) slot[idx] = pack_cand(x, y, sc);
                }
                base += __popcll(m);
            }
        }
        if (base > 0) break;   // wave-uniform: keypoints at this pass's threshold
        lds_order();
        }
        const int nout = min(base, c.cap);
        if (lane == 0) *cnt_out = nout | (int)(((uint32_t)c.slot - (wslot + wpos)) << 16);
        wpos += (uint32_t)nout;
        lds_order();
    }
}

size_t fast_lds_bytes(const Geometry& G) {
    const int roi_cap = (G.max_roi_bytes + 15) & ~15, mb_cap = (G.max_mbuf_bytes + 15) & ~15;
    const int cl_cap = (G.max_cell_px * 2 + 15) & ~15;
    return (size_t)4 * (roi_cap + mb_cap + 64 * 2 + cl_cap);
}

// ----------------------------------------------------------------------------------------
// DistributeOctTree — one workgroup per (image, level).
//
// The reference keeps a std::list of nodes, each owning a vector of keypoints.  Its output
// depends only on (a) the rectangles of the final nodes, (b) their list order, and (c) in
// each node the first max-response keypoint in candidate order.  This kernel keeps the
// list as arrays (double-buffered per round) and gives every candidate the index of its
// node; a round of splits is one pass over the candidates (quadrant + LDS atomic counts)
// and one pass over the nodes (prefix sums place the children exactly where push_front
// would put them: children of the last expanded node first, n4..n1).  Phase 2's
// sort by (size, node) uses the push sequence number as the tie-break.
// ----------------------------------------------------------------------------------------
struct NodeArrays {
    int16_t *x0, *y0, *x1, *y1;
    int32_t *cnt, *seq;
};

struct OctreeSmem {
    NodeArrays A, B;
    int32_t* cc;      // child counts: [NCAP][4] u32, or [NCAP][2] u16 pairs (see octree_level)
    int16_t* cpos;    // [NCAP][4] new position of each child
    int16_t* npos;    // [NCAP] new position of a surviving node
    int16_t* pord;    // [NCAP] processing order in a phase-2 round (-1: not processed)
    int32_t* pre;     // [NCAP] scratch prefix (children before)
    int32_t* pre2;    // [NCAP] scratch prefix (survivors before)
    uint64_t* sortb;  // [NCAP_POW2]
    int* tmp;         // [224] scan scratch + scalars, then the phase-2 bucket arrays
    int ncap;
};

__device__ __forceinline__ void split_lines(int x0, int y0, int x1, int y1, int& sx, int& sy) {
    const int halfX = (int)ceilf((float)(x1 - x0) / 2.0f);
    const int halfY = (int)ceilf((float)(y1 - y0) / 2.0f);
    sx = x0 + halfX;
    sy = y0 + halfY;
}

__device__ __forceinline__ void child_rect(int q, int x0, int y0, int x1, int y1, int sx, int sy,
                                           int& cx0, int& cy0, int& cx1, int& cy1) {
    cx0 = (q & 1) ? sx : x0;
    cx1 = (q & 1) ? x1 : sx;
    cy0 = (q & 2) ? sy : y0;
    cy1 = (q & 2) ? y1 : sy;
}

// Chunked exclusive scan over n items (n may exceed 256).  f(i) gives the value; g(i, excl)
// consumes the exclusive prefix.  Returns the total.  All threads must call.
// Exclusive scan of f over [0, n), gcb(i, prefix) per element.  Up to NT elements: one block
// scan, element i on thread i.  Beyond: each thread scans a contiguous run of ceil(n / NT)
// elements (f evaluated twice per element, so f must not read what gcb writes), one block scan
// of the runs' sums, and a closing barrier (a thread's gcb writes are not the elements a
// thread-strided loop after the scan reads): 3 barriers for any n, where a scan per NT-chunk
// took 2 per chunk (16 for a 2000-node list).
template <int NT, class F, class G>
__device__ __forceinline__ int chunked_scan(int n, int* tmp, F f, G gcb) {
    if (n <= NT) {
        const int i = threadIdx.x;
        const int v = (i < n) ? f(i) : 0;
        int tot;
        const int ex = block_excl_scan<NT / 64>(v, tmp, tot);
        if (i < n) gcb(i, ex);
        return tot;
    }
    const int E = (n + NT - 1) / NT;
    const int i0 = min((int)threadIdx.x * E, n), i1 = min(i0 + E, n);
    int s = 0;
    for (int i = i0; i < i1; ++i) s += f(i);
    int tot;
    int ex = block_excl_scan<NT / 64>(s, tmp, tot);
    for (int i = i0; i < i1; ++i) {
        const int v = f(i);
        gcb(i, ex);
        ex += v;
    }
    __syncthreads();
    return tot;
}


// knode[k]: candidate k's node (< NCAP <= 8192: 13 bits); between a round's quadrant pass and
// its remap pass bits 13-14 also hold the candidate's quadrant in a node being split.
template <int NT, bool KEYS_LDS, bool PACKED>
__device__ void octree_level(const Geometry* __restrict__ g, const LevelGeom& L, int b,
                             int level, int ncand, uint32_t* kdata, int16_t* knode,
                             OctreeSmem& sm, int* __restrict__ ocnt, uint32_t* __restrict__ okp,
                             uint16_t* __restrict__ operm) {
    const int tid = threadIdx.x;
    // child counts per node: PACKED (large batches, candidates in LDS: ncand <= KCAP <= 8192)
    // two 16-bit counts per dword ([NCAP][2]: half the LDS, so a 1500-candidate level-0 list
    // fits the 40 KB budget); else [NCAP][4] dwords (small batches, whose budget is large and
    // whose lone lists are a serial chain the unpacking would lengthen; and the global-scratch
    // path, where a node may hold more than 65535 keys)
    static_assert(KEYS_LDS || !PACKED, "packed counts need ncand <= KCAP");
    uint32_t* const ccw = (uint32_t*)sm.cc;
    auto cc_zero = [&](int n) {
        if (PACKED) {
            ccw[n * 2] = 0u; ccw[n * 2 + 1] = 0u;
        } else {
            ccw[n * 4] = 0u; ccw[n * 4 + 1] = 0u; ccw[n * 4 + 2] = 0u; ccw[n * 4 + 3] = 0u;
        }
    };
    auto cc_add = [&](int n, int q) {
        if (PACKED) atomicAdd(&ccw[n * 2 + (q >> 1)], 1u << (16 * (q & 1)));
        else atomicAdd(&ccw[n * 4 + q], 1u);
    };
    auto cc_get = [&](int n, int q) -> int {
        if (PACKED) return (int)((ccw[n * 2 + (q >> 1)] >> (16 * (q & 1))) & 0xFFFFu);
        return (int)ccw[n * 4 + q];
    };
    const int N = L.nfeat;
    int* tmp = sm.tmp;
    const int nIni = L.n_ini;
    const float hX = L.hx;
    const int Hh = L.h - 2 * ORBX_MIN_BORDER;

    // ---- roots (src/ORBextractor.cc:552-587) ----
    for (int i = tid; i < nIni; i += NT) cc_zero(i);
    __syncthreads();
    for (int k = tid; k < ncand; k += NT) {
        const int x = cand_x(kdata[k]);
        int r = (int)((float)x / hX);
        r = min(r, nIni - 1);
        knode[k] = (int16_t)r;
        cc_add(r, 0);
    }
    __syncthreads();
    int S = chunked_scan<NT>(
        nIni, tmp, [&](int i) { return cc_get(i, 0) > 0 ? 1 : 0; },
        [&](int i, int ex) {
            const int c = cc_get(i, 0);
            if (c > 0) {
                sm.A.x0[ex] = (int16_t)(int)(hX * (float)i);
                sm.A.x1[ex] = (int16_t)(int)(hX * (float)(i + 1));
                sm.A.y0[ex] = 0;
                sm.A.y1[ex] = (int16_t)Hh;
                sm.A.cnt[ex] = c;
                sm.A.seq[ex] = 0;
            }
            sm.npos[i] = (int16_t)ex;
        });
    __syncthreads();
    for (int k = tid; k < ncand; k += NT) knode[k] = sm.npos[knode[k]];
    __syncthreads();

    int seq_base = 1;
    bool phase2 = false;
    NodeArrays cur = sm.A, nxt = sm.B;
    for (int guard = 0; guard < 100000; ++guard) {
        const int prevS = S;
        // ---- split every multi-key node: quadrant of each of its keys ----
        for (int i = tid; i < S; i += NT) {
            cc_zero(i);
            sm.pord[i] = -1;
            // a multi-key node's split lines, once per node (cpos is free until the node pass)
            if (cur.cnt[i] > 1) {
                int sx, sy;
                split_lines(cur.x0[i], cur.y0[i], cur.x1[i], cur.y1[i], sx, sy);
                sm.cpos[i * 4] = (int16_t)sx;
                sm.cpos[i * 4 + 1] = (int16_t)sy;
            }
        }
        __syncthreads();
        // four candidates per thread per trip: their dependent LDS reads (node, then its size
        // and split lines) overlap instead of running one chain after another
        for (int k0 = tid; k0 < ncand; k0 += 4 * NT) {
            int n[4], c[4];
            uint32_t kd[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = min(k0 + u * NT, ncand - 1);
                n[u] = knode[k];
                kd[u] = kdata[k];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) c[u] = cur.cnt[n[u]];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = k0 + u * NT;
                if (k < ncand && c[u] > 1) {
                    const int sx = sm.cpos[n[u] * 4], sy = sm.cpos[n[u] * 4 + 1];
                    const int x = cand_x(kd[u]), y = cand_y(kd[u]);
                    const int q = (x < sx) ? (y < sy ? 0 : 2) : (y < sy ? 1 : 3);
                    knode[k] = (int16_t)(n[u] | q << 13);
                    cc_add(n[u], q);
                }
            }
        }
        __syncthreads();
        auto nonempty = [&](int n) {
            return (cc_get(n, 0) > 0) + (cc_get(n, 1) > 0) + (cc_get(n, 2) > 0) + (cc_get(n, 3) > 0);
        };
        auto multi = [&](int n) {
            return (cc_get(n, 0) > 1) + (cc_get(n, 1) > 1) + (cc_get(n, 2) > 1) + (cc_get(n, 3) > 1);
        };
        int Ctot, Stot, nToExpand = 0;
        if (!phase2) {
            // ---- phase 1 (src/ORBextractor.cc:608-667): expand every multi-key node ----
            if (S < 512) {
                // one scan of packed (children | survivor << 11 | multi-key children << 20):
                // every field's total stays below its width while S < 512 (children and
                // multi-key children <= 4 S < 2048 < 4096, survivors < 512).  The thread that
                // scans node i also writes it below, so no barrier is needed in between.
                const uint32_t tot = (uint32_t)chunked_scan<NT>(
                    S, tmp,
                    [&](int i) {
                        return cur.cnt[i] > 1 ? (int)((uint32_t)nonempty(i) | ((uint32_t)multi(i) << 20))
                                              : (int)(1u << 11);
                    },
                    [&](int i, int ex) {
                        sm.pord[i] = cur.cnt[i] > 1 ? (int16_t)i : (int16_t)-1;
                        sm.pre[i] = (int)((uint32_t)ex & 0x7FFu);
                        sm.pre2[i] = (int)(((uint32_t)ex >> 11) & 0x1FFu);
                    });
                Ctot = (int)(tot & 0x7FFu);
                Stot = (int)((tot >> 11) & 0x1FFu);
                nToExpand = (int)(tot >> 20);
            } else {
            for (int i = tid; i < S; i += NT) sm.pord[i] = cur.cnt[i] > 1 ? (int16_t)i : (int16_t)-1;
            __syncthreads();
            Ctot = chunked_scan<NT>(
                S, tmp, [&](int i) { return sm.pord[i] >= 0 ? nonempty(i) : 0; },
                [&](int i, int ex) { sm.pre[i] = ex; });
            Stot = chunked_scan<NT>(
                S, tmp, [&](int i) { return sm.pord[i] >= 0 ? 0 : 1; },
                [&](int i, int ex) { sm.pre2[i] = ex; });
            // nToExpand: children with more than one key
            int e = 0;
            for (int i = tid; i < S; i += NT) e += sm.pord[i] >= 0 ? multi(i) : 0;
            nToExpand = block_sum<NT / 64>(e, tmp);
            }
            for (int i = tid; i < S; i += NT) {
                if (sm.pord[i] >= 0) {
                    const int c = nonempty(i);
                    const int start = Ctot - sm.pre[i] - c;
                    int sx, sy;
                    const int x0 = cur.x0[i], y0 = cur.y0[i], x1 = cur.x1[i], y1 = cur.y1[i];
                    split_lines(x0, y0, x1, y1, sx, sy);
                    int rank_asc = 0;
                    for (int q = 0; q < 4; ++q) {
                        const int cq = cc_get(i, q);
                        if (cq > 0) {
                            const int pos = start + (c - 1 - rank_asc);   // n4..n1 from the front
                            int cx0, cy0, cx1, cy1;
                            child_rect(q, x0, y0, x1, y1, sx, sy, cx0, cy0, cx1, cy1);
                            nxt.x0[pos] = (int16_t)cx0; nxt.y0[pos] = (int16_t)cy0;
                            nxt.x1[pos] = (int16_t)cx1; nxt.y1[pos] = (int16_t)cy1;
                            nxt.cnt[pos] = cq;
                            nxt.seq[pos] = seq_base + sm.pre[i] + rank_asc;
                            sm.cpos[i * 4 + q] = (int16_t)pos;
                            ++rank_asc;
                        }
                    }
                } else {
                    const int pos = Ctot + sm.pre2[i];
                    nxt.x0[pos] = cur.x0[i]; nxt.y0[pos] = cur.y0[i];
                    nxt.x1[pos] = cur.x1[i]; nxt.y1[pos] = cur.y1[i];
                    nxt.cnt[pos] = cur.cnt[i]; nxt.seq[pos] = cur.seq[i];
                    sm.npos[i] = (int16_t)pos;
                }
            }
        } else {
            // ---- phase 2 (src/ORBextractor.cc:675-740): split largest (size, seq) first ----
            const int nV = chunked_scan<NT>(
                S, tmp, [&](int i) { return cur.cnt[i] > 1 ? 1 : 0; },
                [&](int i, int ex) {
                    if (cur.cnt[i] > 1)
                        sm.sortb[ex] = ((uint64_t)cur.cnt[i] << 40) |
                                       ((uint64_t)(uint32_t)cur.seq[i] << 16) | (uint64_t)i;
                });
            __syncthreads();
            if (nV <= sm.ncap && sm.ncap >= NT) {
                // bucket sort, descending: keys go to buckets by size (min(cnt, 63), larger
                // sizes first), a stable counting sort.  In phase 2 no root is expandable (phase 1's first
                // round split them all), and every other node's seq falls strictly with its
                // position in the list (children go to the front with the highest seqs, and the
                // survivors keep their order), so sortb, built in list order, is already in
                // descending (seq, node) order inside every size: placing the keys of a bucket
                // in sortb order IS the descending (size, seq) order.  Only bucket 63 (sizes
                // >= 63, several sizes) still ranks by comparison.
                int* hist = tmp + 32;     // [64] keys per bucket
                int* start = tmp + 96;    // [64] first position of each bucket
                int* fill = tmp + 160;    // [64] fill cursor / running count
                uint64_t* stage = (uint64_t*)sm.cpos;   // free until the node pass below
                auto bucket = [](uint64_t k) { return min((int)(k >> 40), 63); };
                for (int i = tid; i < 64; i += NT) { hist[i] = 0; fill[i] = 0; }
                constexpr int NW = NT / 64;
                int* wc = sm.pre;         // [NW][64] keys per (wave, bucket) of one chunk
                for (int i = tid; i < NW * 64; i += NT) wc[i] = 0;
                __syncthreads();
                for (int j = tid; j < nV; j += NT) atomicAdd(&hist[bucket(sm.sortb[j])], 1);
                __syncthreads();
                if (tid < 64) {   // one wave: exclusive scan from bucket 63 down
                    const int v = hist[63 - tid];
                    start[63 - tid] = wave_incl_scan(v) - v;
                }
                __syncthreads();
                {
                    const int wid = tid >> 6, lane = tid & 63;
                    for (int c0 = 0; c0 < nV; c0 += NT) {
                        const int j = c0 + tid;
                        const bool valid = j < nV;
                        const uint64_t k = valid ? sm.sortb[j] : 0;
                        const int bk = valid ? bucket(k) : -1;
                        // rank among this wave's lanes of the same bucket, one ballot per
                        // distinct bucket in the wave
                        int rank = 0;
                        uint64_t rem = __ballot(valid);
                        while (rem) {
                            const int b0 = __builtin_amdgcn_readlane(bk, (int)__builtin_ctzll(rem));
                            const uint64_t m = __ballot(bk == b0);
                            if (bk == b0) rank = lanes_below(m);
                            if (lane == 0) wc[wid * 64 + b0] = (int)__popcll(m);
                            rem &= ~m;
                        }
                        __syncthreads();
                        if (valid) {
                            int off = fill[bk] + rank;
                            for (int w = 0; w < wid; ++w) off += wc[w * 64 + bk];
                            stage[start[bk] + off] = k;
                        }
                        __syncthreads();
                        if (tid < 64) {
                            int t = 0;
                            for (int w = 0; w < NW; ++w) { t += wc[w * 64 + tid]; wc[w * 64 + tid] = 0; }
                            fill[tid] += t;
                        }
                        __syncthreads();
                    }
                }
                for (int q = tid; q < nV; q += NT) {
                    const uint64_t k = stage[q];
                    if (bucket(k) < 63) {
                        sm.sortb[q] = k;
                    } else {
                        const int s0 = start[63], s1 = s0 + hist[63];
                        int rank = 0;
                        for (int t = s0; t < s1; ++t) rank += stage[t] > k ? 1 : 0;
                        sm.sortb[s0 + rank] = k;
                    }
                }
            } else
            if (nV <= 4 * NT) {
                // rank sort, descending: a key's position is the number of larger keys (keys
                // are unique: they end in the node index); two barriers instead of bitonic's
                // log^2 stages
                uint64_t key[4];
                int rank[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int i = tid + NT * u;
                    key[u] = i < nV ? sm.sortb[i] : 0;
                    rank[u] = 0;
                }
                for (int j = 0; j < nV; ++j) {
                    const uint64_t kj = sm.sortb[j];
#pragma unroll
                    for (int u = 0; u < 4; ++u) rank[u] += kj > key[u] ? 1 : 0;
                }
                __syncthreads();
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (tid + NT * u < nV) sm.sortb[rank[u]] = key[u];
            } else {
                int P = 1;
                while (P < nV) P <<= 1;
                for (int i = nV + tid; i < P; i += NT) sm.sortb[i] = 0;
                __syncthreads();
                for (int k2 = 2; k2 <= P; k2 <<= 1) {
                    for (int j = k2 >> 1; j > 0; j >>= 1) {
                        for (int i = tid; i < P; i += NT) {
                            const int ixj = i ^ j;
                            if (ixj > i) {
                                const uint64_t a = sm.sortb[i], c = sm.sortb[ixj];
                                const bool desc = (i & k2) == 0;
                                if (desc ? (a < c) : (a > c)) { sm.sortb[i] = c; sm.sortb[ixj] = a; }
                            }
                        }
                        __syncthreads();
                    }
                }
            }
            // running size after processing j (descending order); stop once >= N.  The running
            // size only grows, so J is the first j past N: one atomic per wave (its first lane
            // past N), and no chunk after the one that holds J
            if (tid == 0) tmp[24] = nV - 1;   // past the scan's NT / 64 partials
            __syncthreads();
            // the same scan gives every scanned node its processing position and its
            // children-before prefix (nonempty = delta + 1, so the prefix is the deltas' + j);
            // the nodes of J's chunk past J are marked unprocessed again below
            int c_last = 0;
            {
                int carry = 0;
                for (int c0 = 0; c0 < nV; c0 += NT) {
                    const int j = c0 + tid;
                    const int n = j < nV ? (int)(sm.sortb[j] & 0xFFFF) : 0;
                    const int delta = j < nV ? nonempty(n) - 1 : 0;
                    int tot;
                    const int ex = block_excl_scan<NT / 64>(delta, tmp, tot);
                    if (j < nV) {
                        sm.pre[n] = carry + ex + j;
                        sm.pord[n] = (int16_t)j;
                    }
                    const uint64_t past = __ballot(j < nV && S + carry + ex + delta >= N);
                    if (past && (threadIdx.x & 63) == (int)__builtin_ctzll(past)) atomicMin(&tmp[24], j);
                    carry += tot;
                    c_last = c0;
                    if (S + carry >= N) break;   // block-uniform
                }
            }
            __syncthreads();
            const int J = tmp[24];
            {
                const int j = c_last + tid;
                if (j > J && j < nV) sm.pord[(int)(sm.sortb[j] & 0xFFFF)] = (int16_t)-1;
            }
            if (J >= 0) {   // nV = 0: nothing expandable, J = -1
                const int nJ = (int)(sm.sortb[J] & 0xFFFF);
                Ctot = sm.pre[nJ] + nonempty(nJ);
            } else {
                Ctot = 0;
            }
            __syncthreads();
            Stot = chunked_scan<NT>(
                S, tmp, [&](int i) { return sm.pord[i] >= 0 ? 0 : 1; },
                [&](int i, int ex) { sm.pre2[i] = ex; });
            for (int i = tid; i < S; i += NT) {
                if (sm.pord[i] >= 0) {
                    const int c = nonempty(i);
                    const int start = Ctot - sm.pre[i] - c;
                    int sx, sy;
                    const int x0 = cur.x0[i], y0 = cur.y0[i], x1 = cur.x1[i], y1 = cur.y1[i];
                    split_lines(x0, y0, x1, y1, sx, sy);
                    int rank_asc = 0;
                    for (int q = 0; q < 4; ++q) {
                        const int cq = cc_get(i, q);
                        if (cq > 0) {
                            const int pos = start + (c - 1 - rank_asc);
                            int cx0, cy0, cx1, cy1;
                            child_rect(q, x0, y0, x1, y1, sx, sy, cx0, cy0, cx1, cy1);
                            nxt.x0[pos] = (int16_t)cx0; nxt.y0[pos] = (int16_t)cy0;
                            nxt.x1[pos] = (int16_t)cx1; nxt.y1[pos] = (int16_t)cy1;
                            nxt.cnt[pos] = cq;
                            nxt.seq[pos] = seq_base + sm.pre[i] + rank_asc;
                            sm.cpos[i * 4 + q] = (int16_t)pos;
                            ++rank_asc;
                        }
                    }
                } else {
                    const int pos = Ctot + sm.pre2[i];
                    nxt.x0[pos] = cur.x0[i]; nxt.y0[pos] = cur.y0[i];
                    nxt.x1[pos] = cur.x1[i]; nxt.y1[pos] = cur.y1[i];
                    nxt.cnt[pos] = cur.cnt[i]; nxt.seq[pos] = cur.seq[i];
                    sm.npos[i] = (int16_t)pos;
                }
            }
        }
        __syncthreads();
        for (int k0 = tid; k0 < ncand; k0 += 4 * NT) {   // four chains per trip, as above
            int n[4], q[4], o[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = min(k0 + u * NT, ncand - 1);
                const int kn = knode[k];
                n[u] = kn & 0x1FFF;
                q[u] = (kn >> 13) & 3;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) o[u] = sm.pord[n[u]];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = k0 + u * NT;
                const int t = o[u] >= 0 ? sm.cpos[n[u] * 4 + q[u]] : sm.npos[n[u]];
                if (k < ncand) knode[k] = (int16_t)t;
            }
        }
        __syncthreads();
        NodeArrays t2 = cur; cur = nxt; nxt = t2;
        S = Ctot + Stot;
        seq_base += Ctot;
        if (S >= N || S == prevS) break;
        if (!phase2 && S + nToExpand * 3 > N) phase2 = true;
    }

    // ---- retain the best keypoint of each node (src/ORBextractor.cc:743-762) ----
    uint32_t* best = (uint32_t*)sm.cc;
    // k_orient_desc's processing order (operm): the keypoints by bands of 2^OD_SP_YS rows,
    // each band by columns of 2^OD_SP_XS pixels, so the keypoints a workgroup takes together
    // are neighbours and their patch lines are shared in L1 / L2.  Inside a bucket the order
    // is that of LDS atomics (not deterministic, and it needs not be: every keypoint's angle
    // and descriptor are computed on their own and written at their list index).
    // (taller bands while the buckets would not fit the node arrays' scratch)
    const int sp_cols = (L.w + (1 << OD_SP_XS) - 1) >> OD_SP_XS;
    int sp_ys = OD_SP_YS;
    while (sp_ys < 12 && sp_cols * ((L.h + (1 << sp_ys) - 1) >> sp_ys) > sm.ncap) ++sp_ys;
    const int sp_nb = sp_cols * ((L.h + (1 << sp_ys) - 1) >> sp_ys);
    const bool spatial = operm != nullptr && sp_nb <= sm.ncap;
    int* sp_hist = sm.pre;
    if (spatial)
        for (int i = tid; i < sp_nb; i += NT) sp_hist[i] = 0;
    for (int i = tid; i < S; i += NT) best[i] = 0;
    __syncthreads();
    for (int k = tid; k < ncand; k += NT)
        atomicMax(&best[knode[k]], ((uint32_t)cand_s(kdata[k]) << 24) | (uint32_t)(0xFFFFFF - k));
    __syncthreads();
    uint32_t* out = okp + (size_t)b * g->out_words + L.out_off;
    uint16_t* perm = operm != nullptr ? operm + (size_t)b * g->out_words + L.out_off : nullptr;
    for (int i = tid; i < S; i += NT) {
        const uint32_t w = kdata[0xFFFFFF - (best[i] & 0xFFFFFF)];
        out[i] = w;
        if (spatial) {   // bucket << 16 | rank in the bucket, over the consumed best entry
            const int bk = (cand_y(w) >> sp_ys) * sp_cols + (cand_x(w) >> OD_SP_XS);
            best[i] = (uint32_t)bk << 16 | (uint32_t)atomicAdd(&sp_hist[bk], 1);
        } else if (operm != nullptr) {
            perm[i] = (uint16_t)i;
        }
    }
    if (tid == 0) ocnt[b * g->nlevels + level] = S;
    if (spatial) {
        __syncthreads();
        int* sp_start = sm.pre2;
        chunked_scan<NT>(sp_nb, sm.tmp, [&](int c) { return sp_hist[c]; },
                         [&](int c, int ex) { sp_start[c] = ex; });
        __syncthreads();
        for (int i = tid; i < S; i += NT) {
            const uint32_t kr = best[i];
            perm[sp_start[kr >> 16] + (kr & 0xFFFFu)] = (uint16_t)i;
        }
    }
}

template <int NT>
__global__ __launch_bounds__(NT) void k_octree(const Geometry* __restrict__ g,
                                                const CellDesc* __restrict__ cells,
                                                const int* __restrict__ ccnt,
                                                const uint32_t* __restrict__ cand,
                                                int* __restrict__ ocnt, uint32_t* __restrict__ okp,
                                                uint16_t* __restrict__ operm,
                                                uint8_t* __restrict__ kscratch,
                                                long long kscratch_per_image, int NCAP, int KCAP,
                                                int level_base, int packed) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    // one launch for all levels, the (long) level-0 lists dispatched first
    const int lin = blockIdx.y * gridDim.x + blockIdx.x;
    const int lrel = lin / gridDim.y, b = lin - lrel * gridDim.y, tid = threadIdx.x;
    const int level = level_base + lrel;
    const LevelGeom& L = g->lv[level];
    // carve LDS
    uint8_t* p = smem;
    auto take = [&](size_t bytes) { uint8_t* r = p; p += (bytes + 15) & ~(size_t)15; return r; };
    OctreeSmem sm;
    int NP2 = 1;
    while (NP2 < NCAP) NP2 <<= 1;
    sm.tmp = (int*)take(224 * sizeof(int));
    sm.ncap = NCAP;
    sm.sortb = (uint64_t*)take((size_t)NP2 * 8);
    sm.A.x0 = (int16_t*)take(NCAP * 2); sm.A.y0 = (int16_t*)take(NCAP * 2);
    sm.A.x1 = (int16_t*)take(NCAP * 2); sm.A.y1 = (int16_t*)take(NCAP * 2);
    sm.A.cnt = (int32_t*)take(NCAP * 4); sm.A.seq = (int32_t*)take(NCAP * 4);
    sm.B.x0 = (int16_t*)take(NCAP * 2); sm.B.y0 = (int16_t*)take(NCAP * 2);
    sm.B.x1 = (int16_t*)take(NCAP * 2); sm.B.y1 = (int16_t*)take(NCAP * 2);
    sm.B.cnt = (int32_t*)take(NCAP * 4); sm.B.seq = (int32_t*)take(NCAP * 4);
    sm.cpos = (int16_t*)take((size_t)NCAP * 8);
    sm.npos = (int16_t*)take(NCAP * 2);
    sm.pord = (int16_t*)take(NCAP * 2);
    sm.pre = (int32_t*)take(NCAP * 4);
    sm.pre2 = (int32_t*)take(NCAP * 4);
    // the child counts last but the candidate arrays: the LDS path's counts ([NCAP][2] packed
    // or [NCAP][4]), then its candidates; the global-scratch path's [NCAP][4] counts run on
    // over the (unused) candidate arrays (octree_lds_bytes sizes both)
    sm.cc = (int32_t*)take((size_t)NCAP * (packed ? 8 : 16));
    uint32_t* l_kdata = (uint32_t*)take((size_t)KCAP * 4);
    int16_t* l_knode = (int16_t*)take((size_t)KCAP * 2);

    // count the level's candidates
    const int* cc = ccnt + (size_t)b * g->n_cells + L.cell_begin;
    int part = 0;
    for (int c = tid; c < L.ncells; c += NT) part += cc[c] & 0xFFFF;
    const int ncand = block_sum<NT / 64>(part, sm.tmp);
    if (ncand == 0 || L.n_ini < 1 || L.nfeat <= 0) {
        if (tid == 0) ocnt[b * g->nlevels + level] = 0;
        return;
    }
    const bool in_lds = ncand <= KCAP;
    uint8_t* gs = kscratch + (size_t)b * kscratch_per_image;
    // global fallback region of this level: [kdata u32][knode i16]
    long long lvl_off = 0;
    for (int l = 0; l < level; ++l) lvl_off += (long long)g->lv[l].cand_cap * 8;
    // gather candidates in cell order (cell-major, raster inside a cell)
    const uint32_t* cbase = cand + (size_t)b * g->cand_words;
    const CellDesc* lc = cells + L.cell_begin;
    // the candidate arrays are LDS or global scratch by a runtime test; each branch passes its
    // own pointers (a pointer selected between the two is generic: every access a flat one)
    auto gather_and_split = [&](uint32_t* kdata, int16_t* knode, auto keys_lds_c, auto packed_c) {
    // two adjacent cells per thread, their offsets from one scan of the pairs' sums, and the
    // first 8 candidates of both cells loaded at once (addresses clamped into each cell's
    // slot, so no load is guarded): a level of up to 2 NT cells costs one memory round trip
    // for cells of up to 8 candidates
    {
        int carry = 0;
        for (int c0 = 0; c0 < L.ncells; c0 += 2 * NT) {
            const int ca = c0 + 2 * tid, cb = ca + 1;
            // ccnt = count | (words the cell's run starts before its slot) << 16 (k_fast)
            const int wa = ca < L.ncells ? cc[ca] : 0, wb = cb < L.ncells ? cc[cb] : 0;
            const int na = wa & 0xFFFF, nb = wb & 0xFFFF;
            int tot;
            const int exa = carry + block_excl_scan<NT / 64>(na + nb, sm.tmp, tot);
            const int exb = exa + na;
            carry += tot;
            const uint32_t* sa = cbase + (na > 0 ? lc[ca].slot - (wa >> 16) : 0);
            const uint32_t* sb = cbase + (nb > 0 ? lc[cb].slot - (wb >> 16) : 0);
            for (int e0 = 0; e0 < max(na, nb); e0 += 8) {
                uint32_t va[8], vb[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    va[j] = sa[max(min(e0 + j, na - 1), 0)];
                    vb[j] = sb[max(min(e0 + j, nb - 1), 0)];
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    if (e0 + j < na) kdata[exa + e0 + j] = va[j];
                    if (e0 + j < nb) kdata[exb + e0 + j] = vb[j];
                }
            }
        }
    }
    __syncthreads();
    octree_level<NT, decltype(keys_lds_c)::value, decltype(packed_c)::value>(g, L, b, level, ncand, kdata, knode, sm, ocnt, okp, operm);
    };
    if (in_lds && packed)
        gather_and_split(l_kdata, l_knode, std::true_type{}, std::true_type{});
    else if (in_lds)
        gather_and_split(l_kdata, l_knode, std::true_type{}, std::false_type{});
    else
        gather_and_split((uint32_t*)(gs + lvl_off), (int16_t*)(gs + lvl_off + (long long)L.cand_cap * 4),
                         std::false_type{}, std::false_type{});
}

// ----------------------------------------------------------------------------------------
// Orientation + rBRIEF + assembly: one wave per OD_NK keypoints of one level, in three phases.
//   1. IC_Angle moments, two keypoints at a time (one per half-wave, 32 lanes each) from the
//      31x31 raw patch staged in LDS; the next pair's patch loads are in flight meanwhile.
//      Keypoint k's two sums end up in lane k.
//   2. fastAtan2 and glibc cosf/sinf once for all OD_NK keypoints (lane k: keypoint k): the
//      per-keypoint float / double work is issued once per wave, not once per pair.  Lane k
//      also writes keypoint k's record.
//   3. rBRIEF, two keypoints at a time from the 37x37 blurred patch, same pipelining.
// The per-lane patch offsets are the same for every keypoint of the level, computed once.
// ----------------------------------------------------------------------------------------
static_assert(OD_NK >= 2 && OD_NK <= 64, "keypoints per wave");
// Raw patch (row-major pyramid): 12-byte chunks, three per row (x-15..x+15 from a dword-aligned
// base is <= 34 bytes), into 48-byte LDS rows (16-byte aligned: a lane reads its row's 9
// dwords as two 16-byte reads and one dword).
#define OD_RAW_W 12
#define OD_RAW_CH 3                                // chunks per raw row
#define OD_RAW_RP 48                               // LDS bytes per raw patch row
#define OD_RL4 ((31 * OD_RAW_CH + 31) / 32)        // loads per lane per raw patch (3)
// Blurred patch (16x4-pixel tiled pyramid, blur_off): x-18..x+18 spans 3 or 4 tile columns,
// y-18..y+18 10 tile bands; staged as 10 bands x 4 tile columns x 4 rows of 16-byte chunks
// (one tile row each) into a row-major 40 x 64-byte LDS patch.  A 32-lane load covers two
// bands' 4 tiles (8 whole 64-byte sectors); with 3 tile columns the 4th column's lanes read
// the 3rd's addresses again (no extra sectors).  Row-major, the 37 rows touched ~55 sectors.
#define OD_BLR_W 16
#define OD_BLR_RP 64                               // LDS bytes per blurred patch row
#define OD_BLR_ROWS 40
#define OD_BL4 (OD_BLR_ROWS * 4 / 32)              // loads per lane per blurred patch (5)
#define OD_PATCH_B (OD_BLR_ROWS * OD_BLR_RP > 31 * OD_RAW_RP ? OD_BLR_ROWS * OD_BLR_RP : 31 * OD_RAW_RP)
#define OD_PATCH_DW ((OD_PATCH_B + 15) / 16 * 4)   // dwords per half-wave, 16-byte multiple

// Patch staging chunks of W bytes: buffer load and the store of chunk t at byte W t of the
// half-wave's LDS patch (rows are OD_*_CH chunks apart, so chunk t = row * CH + c).
template <int W> struct od_chunk;
template <> struct od_chunk<8> { typedef uint32_t type __attribute__((ext_vector_type(2))); };
template <> struct od_chunk<12> { typedef uint32_t type __attribute__((ext_vector_type(3))); };
template <> struct od_chunk<16> { typedef uint32_t type __attribute__((ext_vector_type(4))); };
template <int W>
__device__ __forceinline__ typename od_chunk<W>::type od_load(__amdgpu_buffer_rsrc_t r, uint32_t off,
                                                             uint32_t soff = 0) {
    typedef typename od_chunk<W>::type T;
    if constexpr (W == 8) return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(r, off, soff, 0));
    else if constexpr (W == 12) return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b96(r, off, soff, 0));
    else return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b128(r, off, soff, 0));
}
template <int W>
__device__ __forceinline__ void od_store(uint32_t* P, int t, typename od_chunk<W>::type v) {
    uint32_t* d = P + (W / 4) * t;
    if constexpr (W == 8) { typedef uint32_t T2 __attribute__((ext_vector_type(2))); *(T2*)d = v; }
    else if constexpr (W == 12) { d[0] = v.x; d[1] = v.y; d[2] = v.z; }
    else { typedef uint32_t T4 __attribute__((ext_vector_type(4))); *(T4*)d = v; }
}

// Sums over each half-wave (lanes 0-31 / 32-63) as two scalars.
__device__ __forceinline__ void half_sums_dpp(int v, int& lo, int& hi) {
    v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
    v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
    v += __builtin_amdgcn_update_dpp(0, v, 0x124, 0xF, 0xF, false);   // row_ror:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false);   // row_ror:8
    lo = __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16);
    hi = __builtin_amdgcn_readlane(v, 32) + __builtin_amdgcn_readlane(v, 48);
}

__device__ __forceinline__ float readlane_f(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OD_WPE))) void k_orient_desc(
    const Geometry* __restrict__ g, const uint8_t* __restrict__ pyr,
    const uint8_t* __restrict__ blur, const int* __restrict__ ocnt,
    const uint32_t* __restrict__ okp, const uint16_t* __restrict__ operm,
    float* __restrict__ kps, uint8_t* __restrict__ desc, int* __restrict__ nkp, int blk_base,
    int nkp_blk) {
    __shared__ __attribute__((aligned(16))) uint32_t patch[4][2][OD_PATCH_DW];
    // the rBRIEF pattern as floats, pair q = (x1, x2, y1, y2): one 16-byte LDS read per pair
    // and lane instead of a global load and four conversions (which the register budget
    // re-issued for every keypoint pair)
    __shared__ __attribute__((aligned(16))) float spat[256][4];
    {
        const int pw = ((const int*)c_pattern)[threadIdx.x];   // x1, y1, x2, y2 as int8
        *(float4*)spat[threadIdx.x] = float4{(float)(int8_t)pw, (float)(int8_t)(pw >> 16),
                                             (float)(int8_t)(pw >> 8), (float)(pw >> 24)};
        __syncthreads();
    }
    int blk, b;
    xcd_block(blk, b);
    blk += blk_base;   // a launch may cover a range of the blocks (launch_extract's side branch)
    // the wave index as a scalar: the keypoint range, trip counts and pair loop below are then
    // wave-uniform to the compiler (scalar loop control, no exec-mask loop)
    const int wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const int half = lane >> 5, l32 = lane & 31;
    int level = 0;
    while (level + 1 < g->nlevels && blk >= g->orient_block_begin[level + 1]) ++level;
    const int i0 = ((blk - g->orient_block_begin[level]) * 4 + wid) * OD_NK;
    const int* oc = ocnt + b * g->nlevels;
    if (blk == nkp_blk && wid == 0 && lane == 0) {   // every level's count is final here
        int tot = 0;
        for (int l = 0; l < g->nlevels; ++l) tot += oc[l];
        nkp[b] = tot;
    }
    const int n = __builtin_amdgcn_readfirstlane(oc[level]);   // wave-uniform trip counts
    if (i0 >= n) return;
    const int nk = min(OD_NK, n - i0);
    int off = 0;
    for (int l = 0; l < level; ++l) off += oc[l];
    const LevelGeom& L = g->lv[level];
    const int pitch = L.pitch;
    // every keypoint word of the wave in one load: lane k holds keypoint k (processing
    // position i0 + k, list index oi)
    const int oi = operm != nullptr ? operm[(size_t)b * g->out_words + L.out_off + i0 + min(lane, nk - 1)]
                                    : i0 + min(lane, nk - 1);
    const uint32_t cw = okp[(size_t)b * g->out_words + L.out_off + oi];

    const uint8_t* pyr_l = pyr + b * g->pyr_bytes + L.off;
    const uint8_t* blr_l = blur + b * g->pyr_bytes + L.off;
    // per-lane offsets of the raw patch's 12-byte chunks relative to the patch base: chunk
    // t = l32 + 32 j is row t / 3, bytes 12 (t % 3) .. +12 of it; in LDS it lands at 12 t
    uint32_t sor4[OD_RL4];
#pragma unroll
    for (int k = 0; k < OD_RL4; ++k) {
        const int t = min(l32 + 32 * k, 31 * OD_RAW_CH - 1), row = t / OD_RAW_CH;
        sor4[k] = __umul24(row, pitch) + OD_RAW_W * (t - OD_RAW_CH * row);
    }
    // blurred patch: chunk c = l32 + 32 j is tile band c / 16, tile column (c / 4) % 4 (the
    // same for every j), tile row c % 4; relative to the patch's first tile it sits at
    // band * 4 pitch + column * 64 + row * 16, in LDS at patch row 4 band + row, byte 16 column
    const int btc = (l32 >> 2) & 3;
    const uint32_t sob0 = (uint32_t)(__umul24(l32 >> 4, 4 * pitch) + 64 * btc + 16 * (l32 & 3));
    const int bls0 = ((l32 >> 4) * 16 + (l32 & 3) * 4 + btc);   // LDS chunk index, j = 0
    // keypoint of this half-wave in pair p: k = 2p + half (clamped: a lone last keypoint is
    // computed by both halves, the upper half's results are not used)
    auto kp_word = [&](int p) {
        const int k0 = min(2 * p, nk - 1), k1 = min(2 * p + 1, nk - 1);
        const uint32_t c0 = (uint32_t)__builtin_amdgcn_readlane((int)cw, k0);
        const uint32_t c1 = (uint32_t)__builtin_amdgcn_readlane((int)cw, k1);
        return half ? c1 : c0;
    };
    // the keypoint whose patch a load of pair p reads (diagnostic builds 7 / 8 only: the
    // wave's first keypoint for every pair / the pair's first keypoint for both halves)
    auto ld_word = [&](int p) {
        return kp_word(p);
    };
    uint32_t* P = patch[wid][half];
    const int npair = (nk + 1) >> 1;
    // buffer loads: one 32-bit offset add per load instead of a 64-bit address
    const __amdgpu_buffer_rsrc_t rblr = __builtin_amdgcn_make_buffer_rsrc((void*)blr_l, 0, 0x7FFFFFFF, 0x00020000);
    // a raw chunk reads up to 14 bytes past the patch row: the row's padding or the next row of
    // the same buffer (patch rows end at least one row before the level's last)
    const __amdgpu_buffer_rsrc_t rraw = __builtin_amdgcn_make_buffer_rsrc((void*)pyr_l, 0, 0x7FFFFFFF, 0x00020000);
    typedef od_chunk<OD_RAW_W>::type raw_t;
    typedef od_chunk<OD_BLR_W>::type blr_t;
    raw_t vr[OD_RL4];
    blr_t v[OD_BL4];
    auto issue_raw = [&](int p) {
        const uint32_t c = ld_word(p);
        const int x = cand_x(c) + ORBX_MIN_BORDER, y = cand_y(c) + ORBX_MIN_BORDER;
        const uint32_t vo = __umul24((uint32_t)(y - 15), (uint32_t)pitch) + (uint32_t)((x - 15) & ~3);
#pragma unroll
        for (int j = 0; j < OD_RL4; ++j) vr[j] = od_load<OD_RAW_W>(rraw, vo + sor4[j]);
    };
    auto issue_blr = [&](int p) {
        const uint32_t c = ld_word(p);
        const int x = cand_x(c) + ORBX_MIN_BORDER, y = cand_y(c) + ORBX_MIN_BORDER;
        // first tile: band (y - 18) / 4, column (x - 18) / 16; the 4th column only when
        // x + 18 reaches it
        const int tx0 = (x - 18) >> 4;
        const bool c4 = ((x + 18) >> 4) - tx0 == 3;
        uint32_t vo = __umul24((uint32_t)(y - 18) & ~3u, (uint32_t)pitch) + 64u * (uint32_t)tx0 + sob0;
        vo -= (!c4 && btc == 3) ? 64u : 0u;
#pragma unroll
        for (int j = 0; j < OD_BL4; ++j) v[j] = od_load<OD_BLR_W>(rblr, vo, (uint32_t)j * 8u * (uint32_t)pitch);
    };

    // ---- 1. IC_Angle moments (src/ORBextractor.cc:77-104), exact integers in any order: lane
    //      l32 < 31 takes patch row v = l32 - 15 of its half's keypoint.  With the row's pixels
    //      realigned so that byte k of dword d is column u = 4d + k - 15, the circle's columns
    //      |u| <= umax[|v|] are byte masks per dword, fixed per lane: with the pixels masked,
    //      the row sum S is Σ_d dot4(pixels, 1) and Σ (u + 15) I is Σ_d dot4(pixels, 4d + k),
    //      so m_10 = that - 15 S and m_01 = v S.
    const int vrow = l32 - 15;
    uint32_t wM[8];   // the circle's bytes of dword d as 0xFF
    {
        // bit c of cm: column c = u + 15 inside the circle on this row (lane 31: none)
        const int um = l32 < 31 ? g->umax[vrow < 0 ? -vrow : vrow] : -1;
        const uint32_t cm = um < 0 ? 0u : ((2u << (15 + um)) - 1u) & ~((1u << (15 - um)) - 1u);
#pragma unroll
        for (int d = 0; d < 8; ++d) {
            // the 4 bits of dword d as bytes 0 / 1 (bit k lands at bit 8k: no carries)
            const uint32_t m = (((cm >> (4 * d)) & 0xFu) * 0x204081u) & 0x01010101u;
            wM[d] = (m << 8) - m;
        }
    }
    // raw chunk j of this lane: patch row t / 3, bytes 12 (t % 3) of it, at that place in the
    // LDS row
    int lds_raw[OD_RL4];
#pragma unroll
    for (int j = 0; j < OD_RL4; ++j) {
        const int t = l32 + 32 * j, row = t / OD_RAW_CH;
        lds_raw[j] = row * (OD_RAW_RP / 4) + 3 * (t - OD_RAW_CH * row);
    }
    const uint32_t* rrow = P + min(l32, 30) * (OD_RAW_RP / 4);   // this lane's patch row
    int mk10 = 0, mk01 = 0;                   // lane k: keypoint k's moments
    issue_raw(0);
    // one pair; the last pair (peeled: its loads are the blurred patch's, so no loop-carried
    // load registers are copied, and no wait for them, at the loop's back edge)
    auto moments_pair = [&](int p, auto last_c) __attribute__((always_inline)) {
        const int x = cand_x(kp_word(p)) + ORBX_MIN_BORDER;
#pragma unroll
        for (int j = 0; j < OD_RL4; ++j) {
            const int t = l32 + 32 * j;
            if (t < 31 * OD_RAW_CH) {
                uint32_t* d = P + lds_raw[j];
                d[0] = vr[j].x;
                d[1] = vr[j].y;
                d[2] = vr[j].z;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if constexpr (!decltype(last_c)::value) issue_raw(p + 1);   // next pair's patches in flight
        else issue_blr(0);                     // phase 3's first patches in flight
        // the row's 9 dwords; the keypoint sits at byte 15 + a of the staged row
        const uint4 q0 = *(const uint4*)rrow, q1 = *(const uint4*)(rrow + 4);
        const uint32_t D[9] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, rrow[8]};
        const uint32_t a = (uint32_t)(x - 15) & 3u;
        uint32_t S = 0, A = 0;
#pragma unroll
        for (int d = 0; d < 8; ++d) {
            const uint32_t px = __builtin_amdgcn_alignbyte(D[d + 1], D[d], a) & wM[d];
            S = __builtin_amdgcn_udot4(px, 0x01010101u, S, false);
            A = __builtin_amdgcn_udot4(px, 0x03020100u + 0x04040404u * (uint32_t)d, A, false);
        }
        const int m10 = __mul24(-15, (int)S) + (int)A, m01 = __mul24(vrow, (int)S);
        int a10, b10, a01, b01;
        half_sums_dpp(m10, a10, b10);
        half_sums_dpp(m01, a01, b01);
        mk10 = lane == 2 * p ? a10 : (lane == 2 * p + 1 ? b10 : mk10);
        mk01 = lane == 2 * p ? a01 : (lane == 2 * p + 1 ? b01 : mk01);
    };
    for (int p = 0; p + 1 < npair; ++p) moments_pair(p, std::false_type{});
    moments_pair(npair - 1, std::true_type{});

    // ---- 2. angle, cos / sin (src/ORBextractor.cc:103, 113) and the keypoint record ----
    const float angle = cv_fast_atan2((float)mk01, (float)mk10);
    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    const float ang = angle * factorPI;
    const float ca_l = glibc_cosf(ang), sb_l = glibc_sinf(ang);
    if (lane < nk) {
        const size_t o = (size_t)b * g->kp_cap + off + oi;
        const int x = cand_x(cw) + ORBX_MIN_BORDER, y = cand_y(cw) + ORBX_MIN_BORDER;
        float* kp = kps + o * 7;
        const float sc = L.scale;
        kp[0] = level ? (float)x * sc : (float)x;
        kp[1] = level ? (float)y * sc : (float)y;
        kp[2] = (float)L.patch_size;
        kp[3] = angle;
        kp[4] = (float)cand_s(cw);
        ((int*)kp)[5] = level;
        ((int*)kp)[6] = -1;
    }

    // ---- 3. computeOrbDescriptor (src/ORBextractor.cc:108-147) on the blurred level ----
    // this lane's 8 rBRIEF pairs are q = 32w + l32 (spat); a pair's two points side by side,
    // so each product / sum below is one packed-f32 op for both (per element the same IEEE
    // operations as the scalar form)
    typedef float f2 __attribute__((ext_vector_type(2)));
    const uint8_t* blr = (const uint8_t*)P;   // [OD_BLR_ROWS][OD_BLR_RP]
    auto brief_pair = [&](int p, auto last_c) __attribute__((always_inline)) {
        const int x = cand_x(kp_word(p)) + ORBX_MIN_BORDER;
        const int k0 = min(2 * p, nk - 1), k1 = min(2 * p + 1, nk - 1);
        const float ca0 = readlane_f(ca_l, k0), ca1 = readlane_f(ca_l, k1);
        const float sb0 = readlane_f(sb_l, k0), sb1 = readlane_f(sb_l, k1);
        const float ca = half ? ca1 : ca0, sb = half ? sb1 : sb0;
        const int y = cand_y(kp_word(p)) + ORBX_MIN_BORDER;
#pragma unroll
        for (int j = 0; j < OD_BL4; ++j) od_store<OD_BLR_W>(P, bls0 + 32 * j, v[j]);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if constexpr (!decltype(last_c)::value) issue_blr(p + 1);
        // the keypoint in the staged patch: its first tile starts at ((x - 18) & ~15,
        // (y - 18) & ~3)
        const uint8_t* bc = blr + (18 + ((y - 18) & 3)) * OD_BLR_RP + (x - ((x - 18) & ~15));
        // cvRound (:118-120) by the round-to-nearest-even of a float add: for |v| < 2^22,
        // v + 1.5*2^23 holds rint(v) in its low mantissa bits, so its bit pattern is
        // 0x4B400000 + rint(v).  Shifted by log2(OD_BLR_RP) in 32 bits that is a constant +
        // rint(row) * OD_BLR_RP, so one v_lshl_add gives the patch offset up to a constant
        // folded into the base.
        static_assert(OD_BLR_RP == 64, "row offset as a shift by 6");
        const f2 MAGIC = {12582912.0f, 12582912.0f};
        // (the constant is folded into a wrapping u32 offset from the patch start, not into
        // the pointer: a pointer that far outside the LDS object is undefined behaviour, which
        // the compiler may turn into a constant descriptor)
        const uint32_t bko = (uint32_t)(bc - blr) - ((0x4B400000u << 6) + 0x4B400000u);
        const f2 CA = {ca, ca}, SB = {sb, sb};
        uint32_t words[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            // row x*b + y*a and column x*a - y*b of both points (:118-120)
            const float4 pq = *(const float4*)spat[32 * w + l32];
            const f2 PX = {pq.x, pq.y}, PY = {pq.z, pq.w};
            const f2 R = (PX * SB + PY * CA) + MAGIC;
            const f2 C = (PX * CA - PY * SB) + MAGIC;
            const float rx = R.x, ry = R.y, cx = C.x, cy = C.y;
            const uint32_t i0 = (__builtin_bit_cast(uint32_t, rx) << 6) + __builtin_bit_cast(uint32_t, cx) + bko;
            const uint32_t i1 = (__builtin_bit_cast(uint32_t, ry) << 6) + __builtin_bit_cast(uint32_t, cy) + bko;
            const int t0 = blr[i0];
            const int t1 = blr[i1];
            const uint64_t m = __ballot(t0 < t1);
            words[w] = half ? (uint32_t)(m >> 32) : (uint32_t)m;
        }
        const int k = 2 * p + half;
        const int oi0 = __builtin_amdgcn_readlane(oi, k0), oi1 = __builtin_amdgcn_readlane(oi, k1);
        if (k < nk && l32 < 8) {
            const size_t o = (size_t)b * g->kp_cap + off + (half ? oi1 : oi0);
            uint32_t wv = words[0];
#pragma unroll
            for (int w = 1; w < 8; ++w) wv = l32 == w ? words[w] : wv;
            *(uint32_t*)(desc + o * 32 + l32 * 4) = wv;
        }
    };
    for (int p = 0; p + 1 < npair; ++p) brief_pair(p, std::false_type{});
    brief_pair(npair - 1, std::true_type{});
}

// ----------------------------------------------------------------------------------------
// launch sequence
// ----------------------------------------------------------------------------------------
hipError_t launch_extract(const ExtractLaunch& a, hipStream_t st) {
    const Geometry& G = *a.hg;
    KernelTimer dummy;
    KernelTimer& T = a.timer ? *a.timer : dummy;
    const int nt = (long long)a.batch * G.nlevels <= 256 ? OCT_NT_SMALL : OCT_NT;
    // the spatial orientation order pays on large batches only (its L1 / L2 reuse); a lone
    // frame keeps the list order and skips the octree's bucket pass (operm = null)
    uint16_t* const operm = a.batch >= OD_SPATIAL_MIN_BATCH ? a.operm : nullptr;
    auto fast = [&](int c0, int c1, hipStream_t s) {
        if (c1 <= c0) return;
        const int nc = a.fast_nc;
        ORBX_TIMED_LAUNCH(T, K_FAST, k_fast, dim3((c1 - c0 + 4 * nc - 1) / (4 * nc), a.batch),
                          dim3(256), fast_lds_bytes(G), s, a.dg, a.cells, (const uint8_t*)a.pyr,
                          a.ccnt, a.cand, c0, c1, nc);
    };
    // threads per list: OCT_NT, or OCT_NT_SMALL while the batch's lists fit one round on the
    // CUs (each list is a serial chain of rounds with a few barriers each)
    auto oct = [&](dim3 grid, size_t lds, int ncap, int kcap, int level_base, hipStream_t s) {
#define ORBX_OCT_LAUNCH(N)                                                                   \
        ORBX_TIMED_LAUNCH(T, K_OCTREE, k_octree<N>, grid, dim3(N), lds, s, a.dg, a.cells,     \
                          (const int*)a.ccnt, (const uint32_t*)a.cand, a.ocnt, a.okp,         \
                          operm, a.kscratch, a.kscratch_per_image, ncap, kcap, level_base,   \
                          a.oct_small ? 0 : 1)
        if (nt == 64) ORBX_OCT_LAUNCH(64);
        else if (nt == 128) ORBX_OCT_LAUNCH(128);
        else if (nt == 512) ORBX_OCT_LAUNCH(512);
        else ORBX_OCT_LAUNCH(256);
#undef ORBX_OCT_LAUNCH
    };
    auto orient = [&](int blk0, int nblk, int nkp_blk, hipStream_t s) {
        ORBX_TIMED_LAUNCH(T, K_ORIENT, k_orient_desc, dim3(nblk, a.batch), dim3(256), 0, s, a.dg,
                          (const uint8_t*)a.pyr, (const uint8_t*)a.blur, (const int*)a.ocnt,
                          (const uint32_t*)a.okp, (const uint16_t*)operm, a.kps, a.desc, a.nkp,
                          blk0, nkp_blk);
    };
    // Side branch: the first FAST_SIDE_LV levels' FAST (FAST_SIDE 2: + their octree, 3: + their
    // orientation / descriptors) run on the handle's side stream, forked (event) before level
    // FAST_SIDE_AT's launch and joined back before the main stream's orientation launch, so
    // they fill the SIMDs the latency-bound small levels leave idle.  Level 0's FAST reads only
    // the input slot; every other part needs its level (and its blur) launched before the fork.
    const int nside = a.side_lv < G.nlevels - 1 ? a.side_lv : G.nlevels - 1;
    const int mode = a.side_mode;
    // a small batch's octree lists (a few workgroups on the whole chip) take the large LDS
    // budget: every level's candidates stay in LDS instead of the global scratch
    const size_t oct_lds = a.oct_small ? a.octree_lds_small : a.octree_lds;
    const int oct_kcap = a.oct_small ? a.kcap_small : a.kcap;
    const bool side = mode > 0 && a.side && a.ev_fork && a.ev_join && nside >= 1;
    const int c_l1 = side ? G.lv[nside].cell_begin : G.n_cells;
    const bool side_od = side && mode >= 3 && G.orient_block_begin[nside] < G.orient_blocks;
    const int min_fork = (nside == 1 && a.in_place && !side_od) ? 0 : nside;
    const int fork_at = a.side_at < min_fork ? min_fork : a.side_at;
    const int ob0 = side_od ? G.orient_block_begin[nside] : 0;   // first block of the main launch
    // mode 4: level 0's own launch (the blur of the input slot, which only the level-0
    // descriptors read) moves to the side branch too, so the main chain starts with level 1
    // (resized from the input slot itself); needs the images in place
    const bool side_l0 = side_od && mode >= 4 && a.in_place;
    const int main0 = side_l0 ? 1 : 0;
    const int fork_main = fork_at > main0 ? fork_at : main0;
    // the host pyramid copy takes the side stream when the side branch does not
    const bool pyr_fork = a.pyr_host && !side && a.side && a.ev_fork && a.ev_join;
    hipError_t err = hipSuccess;
    if (side) {
        err = launch_levels(a, st, main0, fork_main);
        if (err != hipSuccess) return err;
        if ((err = hipEventRecord(a.ev_fork, st)) != hipSuccess) return err;
        if ((err = hipStreamWaitEvent(a.side, a.ev_fork, 0)) != hipSuccess) return err;
        if (side_l0 && (err = launch_levels(a, a.side, 0, 1)) != hipSuccess) return err;
        fast(0, c_l1, a.side);
        if (mode >= 2) oct(dim3(nside, a.batch), oct_lds, a.ncap, oct_kcap, 0, a.side);
        if (side_od) orient(0, ob0, -1, a.side);
        if ((err = hipEventRecord(a.ev_join, a.side)) != hipSuccess) return err;
        err = launch_levels(a, st, fork_main, G.nlevels);
        if (err != hipSuccess) return err;
        fast(c_l1, G.n_cells, st);
        if (mode >= 2) oct(dim3(G.nlevels - nside, a.batch), oct_lds, a.ncap, oct_kcap, nside, st);
        if ((err = hipStreamWaitEvent(st, a.ev_join, 0)) != hipSuccess) return err;
        if (mode < 2) oct(dim3(G.nlevels, a.batch), oct_lds, a.ncap, oct_kcap, 0, st);
    } else {
        err = a.chain ? launch_pyr_chain(a, st) : launch_levels(a, st, 0, G.nlevels);
        if (err != hipSuccess) return err;
        if (pyr_fork) {   // the pyramid's DMA to the host beside the kernels below
            if ((err = hipEventRecord(a.ev_fork, st)) != hipSuccess ||
                (err = hipStreamWaitEvent(a.side, a.ev_fork, 0)) != hipSuccess ||
                (err = hipMemcpyAsync(a.pyr_host, a.pyr, a.pyr_host_bytes, hipMemcpyDeviceToHost,
                                      a.side)) != hipSuccess ||
                (err = hipEventRecord(a.ev_join, a.side)) != hipSuccess)
                return err;
        }
        fast(0, G.n_cells, st);
        oct(dim3(G.nlevels, a.batch), oct_lds, a.ncap, oct_kcap, 0, st);
    }
    orient(ob0, G.orient_blocks - ob0, ob0, st);
    if (pyr_fork) {
        if ((err = hipStreamWaitEvent(st, a.ev_join, 0)) != hipSuccess) return err;
    } else if (a.pyr_host &&
               (err = hipMemcpyAsync(a.pyr_host, a.pyr, a.pyr_host_bytes, hipMemcpyDeviceToHost,
                                     st)) != hipSuccess) {
        return err;
    }
    return hipGetLastError();
}

size_t octree_lds_bytes(int ncap, int kcap, bool packed) {
    auto r = [](size_t b) { return (b + 15) & ~(size_t)15; };
    int np2 = 1;
    while (np2 < ncap) np2 <<= 1;
    size_t s = r(224 * 4) + r((size_t)np2 * 8);
    s += 2 * (4 * r((size_t)ncap * 2) + 2 * r((size_t)ncap * 4));
    s += r((size_t)ncap * 8) + 2 * r((size_t)ncap * 2) + 2 * r((size_t)ncap * 4);
    // the LDS path's packed counts + candidates, or the global path's wide counts
    const size_t lds_path = r((size_t)ncap * (packed ? 8 : 16)) + r((size_t)kcap * 4) + r((size_t)kcap * 2);
    const size_t glb_path = r((size_t)ncap * 16);
    return s + (lds_path > glb_path ? lds_path : glb_path);
}

}  // namespace orbx

namespace orbx {
hipError_t prepare_stereo(size_t lds);
hipError_t prepare_level(size_t lds);
// Dynamic LDS above 64 KiB needs the per-kernel opt-in (gfx950 has 160 KiB per CU).
// hipFuncSetAttribute acts on the current device, so the sizes already set are kept per device
// (the caller has made the handle's device current) and only ever raised (to the largest size
// any handle on that device needs), under a lock: handles on several host threads may prepare
// concurrently.
hipError_t prepare_kernels(size_t octree_lds, size_t stereo_lds, size_t level_lds,
                           size_t fast_lds) {
    static std::mutex mu;
    static size_t have_dev[ORBX_MAX_DEVICES][4] = {};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= ORBX_MAX_DEVICES) return hipErrorInvalidDevice;
    std::lock_guard<std::mutex> lk(mu);
    size_t* have = have_dev[dev];
    if (octree_lds > have[0]) {
        for (const void* k : {(const void*)k_octree<256>, (const void*)k_octree<64>,
                              (const void*)k_octree<128>, (const void*)k_octree<512>})
            if (e == hipSuccess)
                e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)octree_lds);
        if (e == hipSuccess) have[0] = octree_lds;
    }
    if (e == hipSuccess && fast_lds > have[1]) {
        e = hipFuncSetAttribute((const void*)k_fast, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)fast_lds);
        if (e == hipSuccess) have[1] = fast_lds;
    }
    if (e == hipSuccess && level_lds > have[2]) {
        e = prepare_level(level_lds);
        if (e == hipSuccess) have[2] = level_lds;
    }
    if (e == hipSuccess && stereo_lds > have[3]) {
        e = prepare_stereo(stereo_lds);
        if (e == hipSuccess) have[3] = stereo_lds;
    }
    return e;
}
}  // namespace orbx
