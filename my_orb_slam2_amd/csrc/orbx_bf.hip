// orbx_bf.hip — brute-force Hamming top-2 over a descriptor database (SURVEY §8(b)
// orbx_hamming_bf_top2; §8(e) C4 "per-rank top-2, then an all-gather and a merge").
//
// Semantics: the best / second-best loop every ORBmatcher search runs over its candidates
// (src/ORBmatcher.cc:232-256: bestDist1 = bestDist2 = 256, `dist < bestDist1` moves the best
// to second, else `dist < bestDist2`), with the candidates = every database row in order.
// For query i: best = the FIRST row at the least distance below 256 (-1 if none), second =
// the second least distance of the multiset {256, 256} ∪ {distances} (so it equals the best
// on a tie).  A distance of 256 (every bit differs) never becomes the best, as in the loop.
//
//   k_bf_top2   lane = query (its 8 dwords in VGPRs), a workgroup = 4 waves = 256 queries
//               against one chunk of database rows read by scalar loads (wave-uniform rows,
//               XOR operands straight from SGPRs).  Per row and lane: 8 v_xor + 8 v_bcnt
//               (accumulating) + key = dist << 23 | row-in-chunk, then the top-2 update as one
//               v_min_u32 + one v_med3_u32 on keys (the key order is (distance, row), i.e.
//               the first row wins a tie).  Partial top-2 per (chunk, query) to global.
//   k_bf_merge  folds the chunks' partials in chunk order (= row order): best = the earlier
//               chunk's on equal distance, second = the second least of the two pairs' union
//               (8 threads per query over contiguous chunk ranges, then those 8 in order).
// Issue bound: 8 x 2.3 + 8 x 4.4 + 3 x 4.2 ≈ 66 cycles per 64 distances per SIMD, i.e.
// ≈2.4·10^12 distances/s over 1024 SIMDs at 2.4 GHz (profiles/r01_valu_issue_rates.txt).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "orbx_device.h"
#include "orbx_kernels.h"
#include "orbx_match_kernels.h"

namespace orbx {

namespace {

#define BF_BLK 256     // rows per packed block (128 pairs: the pair index fits 7 bits)

constexpr uint32_t BF_NONE = 256u << 23;       // (distance 256, row 0): the loop's initial value
constexpr int BF_ROW_BITS = 23;                 // rows per chunk < 2^23

__device__ __forceinline__ uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc) {
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}

static_assert(BF_ROW_BITS == 23, "the key's shift is written out in k_bf_top2");

__global__ __launch_bounds__(256) void k_bf_top2(const uint32_t* __restrict__ q, int nq,
                                                  const uint32_t* __restrict__ db, long long ndb,
                                                  int chunk, int nqpad, uint2* __restrict__ part) {
    int bx, c;
    xcd_block(bx, c);                  // the query blocks of one chunk share an XCD's L2
    const int qi = bx * 256 + (int)threadIdx.x;
    const int qc = min(qi, nq - 1);
    uint32_t a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = q[(size_t)qc * 8 + k];
    const long long r0 = (long long)c * chunk;
    const int n = (int)min((long long)chunk, ndb - r0);
    const uint32_t* __restrict__ p = db + r0 * 8;
    uint32_t b1 = BF_NONE, b2 = BF_NONE;
    // per row: 8 v_xor (SGPR operands) + 8 accumulating v_bcnt + one v_lshl_or for the key
    // (written out: the compiler otherwise splits the popcount chain into trees of v_add3 and
    // builds the key with two 4-cycle ops) + v_med3 / v_min for the top-2
    auto row = [&](const uint32_t* r, int e) {
        uint32_t d = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) d = bcnt_acc(a[k] ^ r[k], d);
        uint32_t key;
        asm("v_lshl_or_b32 %0, %1, 23, %2" : "=v"(key) : "v"(d), "s"(e));
        b2 = med3_u32(b1, b2, key);
        b1 = min(b1, key);
    };
    // groups of BF_G rows in two register sets (ping-pong, no copies): the scalar loads
    // (s_load_dwordx8 per row) of one set are in flight while the other set is computed, so
    // the wait for them (scalar loads retire out of order: lgkmcnt(0)) comes a group later
    constexpr int BF_G = 4;
    int e = 0;
    auto load = [&](uint32_t (&g)[BF_G][8], int e0) {
#pragma unroll
        for (int j = 0; j < BF_G; ++j)
#pragma unroll
            for (int k = 0; k < 8; ++k) g[j][k] = p[(size_t)(e0 + j) * 8 + k];
    };
    // Blocks of BF_BLK rows with the top-2 kept as packed 16-bit keys: rows e0 + 2i (low half)
    // and e0 + 2i + 1 (high half) get the key (distance << 7 | i), built by two v_lshl_or per
    // row pair; the top-2 update is three v_pk_min/max_u16 per pair (second = max(best,
    // min(second, key)) for a sorted pair) instead of v_lshl_or + v_med3 + v_min per row.
    // Each half orders its keys by (distance, row), so at the block's end its best and second
    // are inserted into the 32-bit (distance << 23 | row) top-2 with their real rows: the
    // result is the per-row loop's (first row wins a tie).
    auto pair = [&](const uint32_t* ra, const uint32_t* rb, uint32_t pp, uint32_t& h1,
                    uint32_t& h2) {
        uint32_t da = 0, db = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) da = bcnt_acc(a[k] ^ ra[k], da);
#pragma unroll
        for (int k = 0; k < 8; ++k) db = bcnt_acc(a[k] ^ rb[k], db);
        uint32_t x, w;
        asm("v_lshl_or_b32 %0, %1, 7, %2" : "=v"(x) : "v"(da), "s"(pp));
        asm("v_lshl_or_b32 %0, %1, 23, %2" : "=v"(w) : "v"(db), "v"(x));
        uint32_t m;
        asm("v_pk_min_u16 %0, %1, %2" : "=v"(m) : "v"(h2), "v"(w));
        asm("v_pk_max_u16 %0, %1, %2" : "=v"(h2) : "v"(h1), "v"(m));
        asm("v_pk_min_u16 %0, %1, %2" : "=v"(h1) : "v"(h1), "v"(w));
    };
    auto ins = [&](uint32_t key) {
        b2 = med3_u32(b1, b2, key);
        b1 = min(b1, key);
    };
    auto fold = [&](uint32_t h1, uint32_t h2, int e0) {
        // half key k = d << 7 | i of row e0 + 2i (+1 for the high half)
        auto full = [&](uint32_t k, int odd) {
            return ((k >> 7) << BF_ROW_BITS) | (uint32_t)(e0 + 2 * (int)(k & 127u) + odd);
        };
        ins(full(h1 & 0xFFFFu, 0));
        ins(full(h2 & 0xFFFFu, 0));
        ins(full(h1 >> 16, 1));
        ins(full(h2 >> 16, 1));
    };
    constexpr uint32_t H_NONE = (256u << 7) * 0x10001u;   // (256, pair 0) in both halves
    for (; e + BF_BLK <= n; e += BF_BLK) {
        uint32_t h1 = H_NONE, h2 = H_NONE;
        uint32_t A[BF_G][8], B[BF_G][8];
        load(A, e);
        int o = 0;
        for (; o + 2 * BF_G < BF_BLK; o += 2 * BF_G) {
            load(B, e + o + BF_G);
            pair(A[0], A[1], (uint32_t)(o / 2) * 0x10001u, h1, h2);
            pair(A[2], A[3], (uint32_t)(o / 2 + 1) * 0x10001u, h1, h2);
            load(A, e + o + 2 * BF_G);
            pair(B[0], B[1], (uint32_t)(o / 2 + 2) * 0x10001u, h1, h2);
            pair(B[2], B[3], (uint32_t)(o / 2 + 3) * 0x10001u, h1, h2);
        }
        load(B, e + o + BF_G);
        pair(A[0], A[1], (uint32_t)(o / 2) * 0x10001u, h1, h2);
        pair(A[2], A[3], (uint32_t)(o / 2 + 1) * 0x10001u, h1, h2);
        pair(B[0], B[1], (uint32_t)(o / 2 + 2) * 0x10001u, h1, h2);
        pair(B[2], B[3], (uint32_t)(o / 2 + 3) * 0x10001u, h1, h2);
        fold(h1, h2, e);
    }
    for (; e < n; ++e) row(p + (size_t)e * 8, e);
    if (qi < nq) part[(size_t)c * nqpad + qi] = make_uint2(b1, b2);
}

// ---- k_bf_mfma: the distances on the matrix cores ----
// Every bit maps to a signed byte, database row: bit 1 -> +1, 0 -> -1; query: bit 1 -> -64,
// 0 -> +64.  The dot product of a row with a query is then +64 per differing bit and -64 per
// equal bit: 64 (2 popcount(a ^ b) - 256) = 128 dist - 16384, exactly, in int32.
// v_mfma_i32_32x32x32_i8 forms 32 rows x 32 queries of it per 8 instructions (K = 256 =
// 8 x 32) at the i8 matrix rate.  Started from C = 16384 + m (m = the row's index in a
// 128-row superblock), an accumulator IS the 16-bit key dist << 7 | m, so a distance costs
// three full-rate 16-bit min / max ops of the top-2 update and nothing else (k_bf_top2: 8 v_xor
// + 8 v_bcnt + the key).  Issue-bound on the MFMAs and that update, not on HBM (32 B per row
// per query block).
//   workgroup: 4 waves x 64 queries (two 32-query tiles per wave, their signed bytes held in
//   registers for the whole chunk) against the chunk's rows in blocks of 32: the block's 1 KB
//   is read once (a dword per thread), expanded to signed bytes in the A-fragment order, staged
//   in LDS (double-buffered, one barrier per block) and read by every wave (ds_read_b128 per
//   step).  A fragment element j of lane l (r = l & 31, h = l >> 5) at step s is bit
//   32 s + 16 h + j of row r, and the B fragment's element j of lane l is the same bit of
//   query r: the sum pairs equal bits whatever k the hardware gives element j, as long as A
//   and B share it (the parity tests check every distance-derived output).
//   Accumulator register i of lane l holds (row (i & 3) + 8 (i >> 2) + 4 h of the block,
//   query r).  A superblock's 16-bit top-2 is folded into the chunk's 32-bit (dist << 23 |
//   row) top-2, the k_bf_top2 key, and the same partials go to k_bf_merge.
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// 16 bits -> 16 bytes: ((nibble * 0x00204081) & 0x01010101) spreads a nibble's bits to the
// bytes' low bits (t); rows: byte = t ? 0x01 : 0xFF via a packed 16-bit multiply by 0xFE (no
// carries: every byte of t is 0 or 1) and a NOT; queries: byte = t ? 0xC0 : 0x40 (t << 7)
template <bool QUERY>
__device__ __forceinline__ v4i expand16(uint32_t bits, uint32_t fe) {
    v4i r;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        const uint32_t t = (((bits >> (4 * n)) & 15u) * 0x00204081u) & 0x01010101u;
        if (QUERY) {
            r[n] = (int)((t << 7) ^ 0x40404040u);
        } else {
            uint32_t m;
            asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(m) : "v"(t), "v"(fe));
            r[n] = (int)~m;
        }
    }
    return r;
}

__device__ __forceinline__ uint32_t min_u16(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_min_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ uint32_t max_u16(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_max_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// BF_MFMA_WAVES waves x 64 queries per workgroup: 1024 queries, so a 1000-descriptor query
// frame reads each database row once (4 workgroups of 256 queries read it 4 times: PMC traffic
// 4.0x the rows' bytes, profiles/r06_pmc_fetch_bf.csv); the first 256 threads stage a block
constexpr int BF_MFMA_WAVES = 16;
constexpr int BF_MFMA_Q = 64 * BF_MFMA_WAVES;
__global__ __launch_bounds__(64 * BF_MFMA_WAVES) void k_bf_mfma(const uint32_t* __restrict__ q, int nq,
                                                  const uint32_t* __restrict__ db, long long ndb,
                                                  int chunk, int nqpad, uint2* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) v4i frag[2][8 * 64];   // [buffer][step * 64 + lane]
    int bx, c;
    xcd_block(bx, c);
    const int tid = (int)threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r = lane & 31;
    const bool stager = tid < 256;
    const long long r0 = (long long)c * chunk;
    const int n = (int)min((long long)chunk, ndb - r0);
    const uint32_t* __restrict__ p = db + r0 * 8;
    uint32_t fe = 0x00FE00FEu;
    asm volatile("" : "+v"(fe));   // a register operand for v_pk_mul_lo_u16
    // the wave's two query tiles as B fragments: query r of tile t, bits 32 s + 16 h ..
    v4i bq[2][8];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int qi = min(bx * BF_MFMA_Q + w * 64 + t * 32 + r, nq - 1);
#pragma unroll
        for (int s = 0; s < 8; ++s) bq[t][s] = expand16<true>(q[(size_t)qi * 8 + s] >> (16 * h), fe);
    }
    // a stager's share of a block: dword (tid & 7) of row (tid >> 3)
    const int lr = (tid >> 3) & 31, ls = tid & 7;
    auto stage = [&](int buf, uint32_t v) {
        frag[buf][ls * 64 + lr] = expand16<false>(v & 0xFFFFu, fe);
        frag[buf][ls * 64 + 32 + lr] = expand16<false>(v >> 16, fe);
    };
    auto fetch = [&](int e0) { return p[(size_t)min(e0 + lr, n - 1) * 8 + ls]; };
    // accumulator starts of the lane's 16 rows of a block at superblock offset 0
    uint32_t kinit[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) kinit[i] = 16384u + (uint32_t)((i & 3) + 8 * (i >> 2) + 4 * h);
    uint32_t b1[2] = {BF_NONE, BF_NONE}, b2[2] = {BF_NONE, BF_NONE};
    uint32_t l1[2] = {0xFFFFu, 0xFFFFu}, l2[2] = {0xFFFFu, 0xFFFFu};
    const int nblk = (n + 31) / 32;
    // the superblock's 16-bit top-2 -> the chunk's (dist << 23 | row) top-2
    auto fold = [&](int esb) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const uint32_t o1 = l1[t] == 0xFFFFu ? 0xFFFFFFFFu
                                                : ((l1[t] >> 7) << 23) + (uint32_t)esb + (l1[t] & 127u);
            const uint32_t o2 = l2[t] == 0xFFFFu ? 0xFFFFFFFFu
                                                : ((l2[t] >> 7) << 23) + (uint32_t)esb + (l2[t] & 127u);
            b2[t] = min(max(b1[t], o1), min(b2[t], o2));
            b1[t] = min(b1[t], o1);
            l1[t] = l2[t] = 0xFFFFu;
        }
    };
    if (nblk > 0 && stager) stage(0, fetch(0));
    __syncthreads();
    for (int blk = 0; blk < nblk; ++blk) {
        const int buf = blk & 1, e0 = blk * 32, j = blk & 3;
        const uint32_t nxt = (stager && blk + 1 < nblk) ? fetch(e0 + 32) : 0u;   // in flight meanwhile
        v16i acc[2];
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[0][i] = acc[1][i] = (int)(kinit[i] + 32u * (uint32_t)j);
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const v4i a = frag[buf][s * 64 + lane];
#pragma unroll
            for (int t = 0; t < 2; ++t)
                acc[t] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bq[t][s], acc[t], 0, 0, 0);
        }
        if (e0 + 32 <= n) {
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const uint32_t key = (uint32_t)acc[t][i];
                    l2[t] = min_u16(l2[t], max_u16(l1[t], key));
                    l1[t] = min_u16(l1[t], key);
                }
        } else {   // the chunk's last, partial block: rows past n dropped
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const bool ok = e0 + (i & 3) + 8 * (i >> 2) + 4 * h < n;
                    const uint32_t key = ok ? (uint32_t)acc[t][i] : 0xFFFFu;
                    l2[t] = min_u16(l2[t], max_u16(l1[t], key));
                    l1[t] = min_u16(l1[t], key);
                }
        }
        if (j == 3 || blk + 1 == nblk) fold(e0 - 32 * j);
        if (stager && blk + 1 < nblk) stage(buf ^ 1, nxt);
        __syncthreads();
    }
    // the two half-waves hold the same queries' other 16 rows of every block: fold them
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const uint32_t o1 = (uint32_t)__shfl_xor((int)b1[t], 32), o2 = (uint32_t)__shfl_xor((int)b2[t], 32);
        b2[t] = min(max(b1[t], o1), min(b2[t], o2));
        b1[t] = min(b1[t], o1);
        const int qi = bx * BF_MFMA_Q + w * 64 + t * 32 + r;
        if (h == 0 && qi < nq) part[(size_t)c * nqpad + qi] = make_uint2(b1[t], b2[t]);
    }
}

// 32 queries per workgroup, 8 threads per query: thread slice s folds the contiguous chunk
// range [s*L, (s+1)*L) in order, then slice 0 folds the 8 slice results in order (the fold is
// associative: (earlier, later) -> best of the earlier on a tie).
__global__ __launch_bounds__(256) void k_bf_merge(const uint2* __restrict__ part, int nq,
                                                   int nqpad, int nchunks, int chunk,
                                                   long long idx_base, int32_t* __restrict__ best_idx,
                                                   int32_t* __restrict__ best_dist,
                                                   int32_t* __restrict__ second_dist) {
    __shared__ uint32_t sd1[8][32], sd2[8][32];
    __shared__ long long srow[8][32];
    const int ql = (int)threadIdx.x & 31, sl = (int)threadIdx.x >> 5;
    const int qi = blockIdx.x * 32 + ql;
    const int L = (nchunks + 7) / 8;
    const int c0 = sl * L, c1 = min(nchunks, c0 + L);
    uint32_t d1 = 256, d2 = 256;
    long long row = -1;
    if (qi < nq) {
        // eight partials loaded together, then folded in order (branch-free)
        for (int cb = c0; cb < c1; cb += 8) {
            uint2 k[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) k[j] = part[(size_t)min(cb + j, c1 - 1) * nqpad + qi];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (cb + j >= c1) k[j] = make_uint2(BF_NONE, BF_NONE);   // past the range
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t e1 = k[j].x >> BF_ROW_BITS, e2 = k[j].y >> BF_ROW_BITS;
                // second = second least of {d1, d2} ∪ {e1, e2} (both pairs sorted)
                d2 = min(max(d1, e1), min(d2, e2));
                const bool take = e1 < d1;     // strict: the earlier chunk keeps a tie
                d1 = take ? e1 : d1;
                row = take ? (long long)(cb + j) * chunk + (k[j].x & ((1u << BF_ROW_BITS) - 1)) : row;
            }
        }
    }
    sd1[sl][ql] = d1;
    sd2[sl][ql] = d2;
    srow[sl][ql] = row;
    __syncthreads();
    if (sl != 0 || qi >= nq) return;
    for (int t = 1; t < 8; ++t) {
        const uint32_t e1 = sd1[t][ql], e2 = sd2[t][ql];
        d2 = min(max(d1, e1), min(d2, e2));
        if (e1 < d1) {
            d1 = e1;
            row = srow[t][ql];
        }
    }
    best_idx[qi] = row < 0 ? -1 : (int32_t)(idx_base + row);
    best_dist[qi] = (int32_t)d1;
    second_dist[qi] = (int32_t)d2;
}

}  // namespace

// Rows per chunk: enough chunks that the (query block, chunk) grid gives every CU several
// workgroups, rounded so the grid fills the 8 XCDs evenly.
int bf_chunk_rows(long long ndb, int nq, int ncu, int kernel) {
    const int qb = kernel == ORBX_BF_VALU ? (nq + 255) / 256 : (nq + BF_MFMA_Q - 1) / BF_MFMA_Q;
    long long target = (long long)std::max(ncu, 1) * 8 / qb;          // chunks wanted
    if (target < 8) target = 8;
    long long rows = (ndb + target - 1) / target;
    rows = ((rows + 63) / 64) * 64;
    if (rows < 256) rows = 256;
    if (rows > (1ll << BF_ROW_BITS) - 64) rows = (1ll << BF_ROW_BITS) - 64;
    return (int)rows;
}

size_t bf_partial_bytes(long long ndb, int nq, int chunk) {
    const long long nchunks = (ndb + chunk - 1) / chunk;
    const int nqpad = ((nq + BF_MFMA_Q - 1) / BF_MFMA_Q) * BF_MFMA_Q;
    return (size_t)nchunks * (size_t)nqpad * sizeof(uint2);
}

const char* bf_kernel_name(int kernel) {
    return kernel == ORBX_BF_MFMA ? "k_bf_mfma" : kernel == ORBX_BF_VALU ? "k_bf_top2" : nullptr;
}

hipError_t launch_bf_top2(const BfLaunch& a, hipStream_t st, KernelTimer* timer) {
    if (a.nq <= 0) return hipSuccess;
    // the partials' query stride: a multiple of both kernels' queries per workgroup
    const int nqpad = ((a.nq + BF_MFMA_Q - 1) / BF_MFMA_Q) * BF_MFMA_Q;
    const long long nchunks = a.ndb > 0 ? (a.ndb + a.chunk - 1) / a.chunk : 0;
    if (nchunks > INT32_MAX / 2) return hipErrorInvalidValue;
    hipEvent_t e = timer ? timer->start(st) : nullptr;
    if (nchunks > 0 && a.kernel == ORBX_BF_VALU)
        hipLaunchKernelGGL(k_bf_top2, dim3(nqpad / 256, (unsigned)nchunks), dim3(256), 0, st,
                           (const uint32_t*)a.q, a.nq, (const uint32_t*)a.db, a.ndb, a.chunk,
                           nqpad, (uint2*)a.part);
    else if (nchunks > 0)
        hipLaunchKernelGGL(k_bf_mfma, dim3(nqpad / BF_MFMA_Q, (unsigned)nchunks),
                           dim3(BF_MFMA_Q), 0, st, (const uint32_t*)a.q, a.nq,
                           (const uint32_t*)a.db, a.ndb, a.chunk, nqpad, (uint2*)a.part);
    hipLaunchKernelGGL(k_bf_merge, dim3((a.nq + 31) / 32), dim3(256), 0, st, (const uint2*)a.part,
                       a.nq, nqpad, (int)nchunks, a.chunk, a.idx_base, a.best_idx, a.best_dist,
                       a.second_dist);
    if (timer) timer->stop(ORBX_MK_BF, e, st);
    return hipGetLastError();
}

}  // namespace orbx
