// orbx_stereo.hip — Frame::ComputeStereoMatches (src/Frame.cc:496-686) as one gfx950
// workgroup (1024 threads) per stereo pair, batched over pairs.
//
//   1. right keypoints bucketed by (octave, image row) (LDS counting sort) and their
//      descriptors staged in LDS; the reference's vRowIndices lists are recovered exactly by
//      testing each bucketed keypoint's [floor(y-2s), ceil(y+2s)] band over the rows of the
//      three octaves a left keypoint may match, and its "first candidate wins" rule becomes a
//      lexicographic (distance, right index) minimum, so bucket order is free;
//   2. one lane per left keypoint: band / octave / disparity-range filters + 256-bit Hamming
//      from LDS (v_xor + v_bcnt); if the best distance is < 75 the same lane runs the 11x11
//      SAD at 11 shifts on the unblurred pyramids (rows read as aligned dwords, realigned
//      with v_alignbyte; exact integer sums), the parabola fit and the depth, with the
//      reference's float formulas;
//   3. median of the accepted SADs by a two-pass LDS radix select and the 2.1*median cut.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orbx_device.h"
#include "orbx_internal.h"
#include "orbx_kernels.h"

namespace orbx {

#define ST_THREADS 1024
#define ST_WAVES (ST_THREADS / 64)
// split path: the last workgroup of a pair to finish runs the median cut; the split path's
// stores of uRight / depth / SADs are write-through (sc1), so that workgroup reads them from
// memory and overwrites them with no fence between
template <class T>
__device__ __forceinline__ void split_store(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int byte_of(const uint32_t* w, int k) {   // k compile-time
    return (int)((w[k >> 2] >> (8 * (k & 3))) & 255u);
}

__device__ void median_cut(int nv, const int* vsad, const int16_t* vidx, int* hist, int* tmp,
                           float* uR, float* dep, int* nvalid, int b);

// LPK lanes per left keypoint: 1 for large batches (one lane runs a keypoint's search and SAD);
// 8 for small ones, where the launch has few keypoints per lane and a keypoint's serial chain
// is the latency: the lanes split its candidates and its SAD window's rows and combine by
// lane shuffles (the candidates' minimum is order-free, the SAD sums are exact integers).
template <int LPK>
__global__ __launch_bounds__(ST_THREADS) void k_stereo(const Geometry* __restrict__ g,
                                                       const float* __restrict__ kpsL,
                                                       const uint8_t* __restrict__ descL,
                                                       const int* __restrict__ nkpL,
                                                       const uint8_t* __restrict__ pyrL,
                                                       const float* __restrict__ kpsR,
                                                       const uint8_t* __restrict__ descR,
                                                       const int* __restrict__ nkpR,
                                                       const uint8_t* __restrict__ pyrR,
                                                       float mbf, float mb,
                                                       float* __restrict__ uRight,
                                                       float* __restrict__ depth,
                                                       int* __restrict__ nvalid, int nsplit,
                                                       int* __restrict__ scnt,
                                                       int* __restrict__ ssad,
                                                       int16_t* __restrict__ sidx) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    // nsplit > 1 (small batches): workgroup s of pair b takes the s-th slice of its left
    // keypoints and appends the accepted SADs to global scratch; k_stereo_cut then takes the
    // median over the whole pair
    const int b = blockIdx.x / nsplit, slice = blockIdx.x - b * nsplit, tid = threadIdx.x;
    const int KC = g->kp_cap;
    const int H = g->lv[0].h;
    uint8_t* p = smem;
    auto take = [&](size_t bytes) { uint8_t* r = p; p += (bytes + 15) & ~(size_t)15; return r; };
    int* tmp = (int*)take(32 * 4);
    // (octave, row) buckets, or row buckets alone (stereo_ob = 1) when the octave buckets
    // would not fit in LDS beside the descriptors
    const int OB = g->stereo_ob, NB = OB * H;
    uint4* rdesc = (uint4*)take((size_t)KC * 32);   // in bucket order
    // bucket k: counts, then (scan) its start, then (fill) its end = the start of bucket k+1
    int* bend = (int*)take((size_t)NB * 4);
    // per right keypoint, in bucket order: (uR bits, rmin | rmax << 16, oct | iR << 16)
    uint3* rrec = (uint3*)take((size_t)KC * 12);
    int* vsad = (int*)take((size_t)KC * 4);
    int16_t* vidx = (int16_t*)take((size_t)KC * 2);
    int* hist = (int*)take(256 * 4);

    const int NL = min(max(nkpL[b], 0), KC), NR = min(max(nkpR[b], 0), KC);
    const float* kL = kpsL + (size_t)b * KC * 7;
    const float* kR = kpsR + (size_t)b * KC * 7;
    float* uR = uRight + (size_t)b * KC;
    float* dep = depth + (size_t)b * KC;
    for (int i = tid; i < NB; i += ST_THREADS) bend[i] = 0;
    if (tid == 0) tmp[16] = 0;
    __syncthreads();

    // 1. right keypoints -> (octave, row) buckets (src/Frame.cc:516-531): counts, a scan, then
    //    each keypoint's record and descriptor written at its bucket position.  A left
    //    keypoint of level l only matches octaves l-1 .. l+1 (:561-563), and a right keypoint
    //    of octave o lists itself in the rows within 2*scale[o] of its own (:522-530), so the
    //    search reads three bucket windows instead of every octave's keypoints in its rows
    auto rkey = [&](int iR) {
        const int o = OB == 1 ? 0 : min(max(((const int*)kR)[iR * 7 + 5], 0), g->nlevels - 1);
        return o * H + min(max((int)kR[iR * 7 + 1], 0), H - 1);
    };
    for (int iR = tid; iR < NR; iR += ST_THREADS) atomicAdd(&bend[rkey(iR)], 1);
    __syncthreads();
    {
        int carry = 0;
        for (int c0 = 0; c0 < NB; c0 += ST_THREADS) {
            const int i = c0 + tid;
            const int v = i < NB ? bend[i] : 0;
            int tot;
            const int ex = block_excl_scan<ST_WAVES>(v, tmp, tot);
            if (i < NB) bend[i] = carry + ex;
            carry += tot;
        }
    }
    __syncthreads();
    {
        const uint4* src = (const uint4*)(descR + (size_t)b * KC * 32);
        for (int iR = tid; iR < NR; iR += ST_THREADS) {
            const uint4 d0 = src[2 * iR], d1 = src[2 * iR + 1];
            const float kx = kR[iR * 7 + 0], ky = kR[iR * 7 + 1];
            const int oct = ((const int*)kR)[iR * 7 + 5];
            const float r = 2.0f * g->lv[oct].scale;
            const int mx = (int)ceilf(ky + r), mn = (int)floorf(ky - r);
            const int pos = atomicAdd(&bend[rkey(iR)], 1);
            rrec[pos] = make_uint3(__float_as_uint(kx),
                                   (uint32_t)(uint16_t)mn | ((uint32_t)(uint16_t)mx << 16),
                                   (uint32_t)oct | ((uint32_t)iR << 16));
            rdesc[2 * pos] = d0;
            rdesc[2 * pos + 1] = d1;
        }
    }
    __syncthreads();

    // 2. per left keypoint: descriptor search (src/Frame.cc:542-587) + SAD (:591-667)
    const float maxD = mbf / mb;   // minZ = mb, maxD = mbf/minZ (Frame.cc:534-536)
    const float minD = 0;
    const int chunk = (NL + nsplit - 1) / nsplit;
    const int iL0 = slice * chunk, iL1 = min(NL, iL0 + chunk);
    const int sub = tid % LPK;   // this lane's share of its keypoint (control flow is per group)
    for (int iL = iL0 + tid / LPK; iL < iL1; iL += ST_THREADS / LPK) {
        if (nsplit > 1) {
            if (sub == 0) {
                split_store(uR + iL, -1.0f);
                split_store(dep + iL, -1.0f);
            }
        } else {
            uR[iL] = -1.0f;
            dep[iL] = -1.0f;
        }
        const float uL = kL[iL * 7 + 0], vL = kL[iL * 7 + 1];
        const int levelL = ((const int*)kL)[iL * 7 + 5];
        const int row = (int)vL;
        const float minU = uL - maxD, maxU = uL - minD;
        if (maxU < 0 || row >= H) continue;
        uint4 dl0, dl1;
        {
            const uint4* q = (const uint4*)(descL + ((size_t)b * KC + iL) * 32);
            dl0 = q[0];
            dl1 = q[1];
        }
        int best = 100, bestR = -1;   // ORBmatcher::TH_HIGH, strict '<': first minimum wins
        int bestE = -1;
        // octaves levelL-1 .. levelL+1: a right keypoint of octave o whose band
        // [floor(y - 2s), ceil(y + 2s)] holds `row` has int(y) within ceil(2s) + 1 rows of it
        // (one group of every octave when OB = 1: the window of the largest scale, octaves
        // tested per candidate)
        const int o0 = max(levelL - 1, 0), o1 = min(levelL + 1, g->nlevels - 1);
        for (int o = OB == 1 ? 0 : o0; o <= (OB == 1 ? 0 : o1); ++o) {
            const int win = g->lv[OB == 1 ? o1 : o].stereo_win;
            const int r0 = max(row - win, 0), r1 = min(row + win, H - 1);
            const int k0 = o * H + r0;
            const int e1 = bend[o * H + r1];
            for (int e = (k0 > 0 ? bend[k0 - 1] : 0) + sub; e < e1; e += LPK) {
                const uint3 rc = rrec[e];
                const int mn = (int)(int16_t)(rc.y & 0xFFFF), mx = (int)(int16_t)(rc.y >> 16);
                if (mn > row || mx < row) continue;
                const int oc = (int)(rc.z & 0xFFFF);
                if (oc < levelL - 1 || oc > levelL + 1) continue;
                const float u = __uint_as_float(rc.x);
                if (u >= minU && u <= maxU) {
                    const int iR = (int)(rc.z >> 16);
                    const uint4 a = rdesc[2 * e], c = rdesc[2 * e + 1];
                    const int dist = __popc(dl0.x ^ a.x) + __popc(dl0.y ^ a.y) + __popc(dl0.z ^ a.z) +
                                     __popc(dl0.w ^ a.w) + __popc(dl1.x ^ c.x) + __popc(dl1.y ^ c.y) +
                                     __popc(dl1.z ^ c.z) + __popc(dl1.w ^ c.w);
                    if (dist < best || (dist == best && bestR >= 0 && iR < bestR)) {
                        best = dist;
                        bestR = iR;
                        bestE = e;
                    }
                }
            }
        }
        if (LPK > 1) {   // the group's minimum of (distance, right index)
#pragma unroll
            for (int m = 1; m < LPK; m <<= 1) {
                const int b2 = __shfl_xor(best, m, LPK), r2 = __shfl_xor(bestR, m, LPK);
                const int e2 = __shfl_xor(bestE, m, LPK);
                if (r2 >= 0 && (bestR < 0 || b2 < best || (b2 == best && r2 < bestR))) {
                    best = b2;
                    bestR = r2;
                    bestE = e2;
                }
            }
        }
        if (bestR < 0 || best >= 75) continue;   // thOrbDist = (TH_HIGH + TH_LOW) / 2

        // ---- sliding-window SAD on the unblurred level of the left keypoint ----
        const LevelGeom& LV = g->lv[levelL];
        const float uR0 = __uint_as_float(rrec[bestE].x);
        const float sf = LV.inv_scale;
        const float scaleduL = roundf(uL * sf);
        const float scaledvL = roundf(vL * sf);
        const float scaleduR0 = roundf(uR0 * sf);
        const int w = 5, L5 = 5;
        const float iniu = scaleduR0 + L5 - w;
        const float endu = scaleduR0 + L5 + w + 1;
        if (iniu < 0 || endu >= LV.w) continue;
        const int pitch = LV.pitch;
        const uint8_t* PL = pyrL + (size_t)b * g->pyr_bytes + LV.off;
        const uint8_t* PR = pyrR + (size_t)b * g->pyr_bytes + LV.off;
        const int yl = (int)scaledvL, xl = (int)scaleduL, xr = (int)scaleduR0;
        int acc[11];
        if constexpr (LPK == 1) {
            int accl[11];   // its own array: declared outside, `acc` made this path spill
            uint32_t E[11];
            // all 11 row pairs of the window are loaded before any is used (one memory latency
            // per keypoint instead of one per row): left x-5..x+5 (4 dwords), right x-10..x+10
            // (7 dwords), realigned with v_alignbyte
            const uint32_t* pl0 = (const uint32_t*)(PL + (size_t)(yl - w) * pitch + ((xl - w) & ~3));
            const uint32_t* pr0 = (const uint32_t*)(PR + (size_t)(yl - w) * pitch + ((xr - L5 - w) & ~3));
            const int shl = (xl - w) & 3, shr = (xr - L5 - w) & 3;
            const int pdw = pitch >> 2;   // rows are 64-byte aligned
            uint32_t lraw[11][4], rraw[11][7];
#pragma unroll
            for (int r = 0; r < 11; ++r) {
#pragma unroll
                for (int i = 0; i < 4; ++i) lraw[r][i] = pl0[r * pdw + i];
#pragma unroll
                for (int i = 0; i < 7; ++i) rraw[r][i] = pr0[r * pdw + i];
            }
            auto lrow = [&](int r, uint32_t (&o)[3]) {
#pragma unroll
                for (int i = 0; i < 3; ++i) o[i] = __builtin_amdgcn_alignbyte(lraw[r][i + 1], lraw[r][i], shl);
            };
            auto rrow = [&](int r, uint32_t (&o)[6]) {
#pragma unroll
                for (int i = 0; i < 6; ++i) o[i] = __builtin_amdgcn_alignbyte(rraw[r][i + 1], rraw[r][i], shr);
            };
            int cL, cR[11];
            {
                uint32_t lc[3], rc[6];
                lrow(w, lc);
                rrow(w, rc);
                cL = byte_of(lc, 5);
#pragma unroll
                for (int k = 0; k < 11; ++k) cR[k] = byte_of(rc, k + 5);
            }
            // sum_x |(l_x - cL) - (r_{k+x} - cR_k)| = sum_x |(l_x + 256) - (r_{k+x} + 256 + cL - cR_k)|
            // with every operand in [0, 1023]: v_sad_u16 takes two pixels per instruction (pixel
            // pairs packed as u16 halves by v_perm), the 11th pixel one v_sad_u32-style |a - b|
#pragma unroll
            for (int k = 0; k < 11; ++k) {
                accl[k] = 0;
                E[k] = (uint32_t)(256 + cL - cR[k]) * 0x10001u;
            }
            auto pair_sel = [](int s0) {   // bytes s0, s0 + 1 of an 8-byte (hi:lo) pair as u16s
                return (uint32_t)(s0 & 7) | 0x0C00u | (uint32_t)((s0 + 1) & 7) << 16 | 0x0C000000u;
            };
#pragma unroll
            for (int r = 0; r < 11; ++r) {
                uint32_t lw[3], rw[6];
                lrow(r, lw);
                rrow(r, rw);
                uint32_t LP[5];
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    const int b0 = 2 * j;   // bytes b0, b0 + 1 of lw
                    LP[j] = __builtin_amdgcn_perm(lw[(b0 >> 2) + 1 < 3 ? (b0 >> 2) + 1 : 2], lw[b0 >> 2],
                                                  pair_sel(b0 & 3)) + 0x01000100u;
                }
                const int l10 = byte_of(lw, 10) + 256;
                // right pixel pairs starting at every byte 0..19: RP[m] = (r_m, r_{m+1})
                uint32_t RP[20];
#pragma unroll
                for (int m = 0; m < 20; ++m)
                    RP[m] = __builtin_amdgcn_perm(rw[(m >> 2) + 1 < 6 ? (m >> 2) + 1 : 5], rw[m >> 2],
                                                  pair_sel(m & 3));
#pragma unroll
                for (int k = 0; k < 11; ++k) {
                    uint32_t a = (uint32_t)accl[k];
#pragma unroll
                    for (int j = 0; j < 5; ++j) a = __builtin_amdgcn_sad_u16(LP[j], RP[k + 2 * j] + E[k], a);
                    const int d = l10 - (byte_of(rw, k + 10) + (int)(E[k] & 0xFFFFu));
                    accl[k] = (int)a + (d < 0 ? -d : d);
                }
            }
#pragma unroll
            for (int k = 0; k < 11; ++k) acc[k] = accl[k];
        } else {
            const int pdw = pitch >> 2;   // rows are 64-byte aligned
            const int shl = (xl - w) & 3, shr = (xr - L5 - w) & 3;
            const uint32_t* pl0 = (const uint32_t*)(PL + (size_t)(yl - w) * pitch + ((xl - w) & ~3));
            const uint32_t* pr0 = (const uint32_t*)(PR + (size_t)(yl - w) * pitch + ((xr - L5 - w) & ~3));
            auto align_l = [&](const uint32_t (&raw)[4], uint32_t (&o)[3]) {
#pragma unroll
                for (int i = 0; i < 3; ++i) o[i] = __builtin_amdgcn_alignbyte(raw[i + 1], raw[i], shl);
            };
            auto align_r = [&](const uint32_t (&raw)[7], uint32_t (&o)[6]) {
#pragma unroll
                for (int i = 0; i < 6; ++i) o[i] = __builtin_amdgcn_alignbyte(raw[i + 1], raw[i], shr);
            };
            // sum_x |(l_x - cL) - (r_{k+x} - cR_k)| = sum_x |(l_x + 256) - (r_{k+x} + 256 + cL - cR_k)|
            // with every operand in [0, 1023]: v_sad_u16 takes two pixels per instruction (pixel
            // pairs packed as u16 halves by v_perm), the 11th pixel one v_sad_u32-style |a - b|
            uint32_t E[11];
            auto pair_sel = [](int s0) {   // bytes s0, s0 + 1 of an 8-byte (hi:lo) pair as u16s
                return (uint32_t)(s0 & 7) | 0x0C00u | (uint32_t)((s0 + 1) & 7) << 16 | 0x0C000000u;
            };
            auto centre = [&](const uint32_t (&lc)[3], const uint32_t (&rc)[6]) {
                const int cL = byte_of(lc, 5);
#pragma unroll
                for (int k = 0; k < 11; ++k) {
                    acc[k] = 0;
                    E[k] = (uint32_t)(256 + cL - byte_of(rc, k + 5)) * 0x10001u;
                }
            };
            auto sad_row = [&](const uint32_t (&lw)[3], const uint32_t (&rw)[6]) {
                uint32_t LP[5];
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    const int b0 = 2 * j;   // bytes b0, b0 + 1 of lw
                    LP[j] = __builtin_amdgcn_perm(lw[(b0 >> 2) + 1 < 3 ? (b0 >> 2) + 1 : 2], lw[b0 >> 2],
                                                  pair_sel(b0 & 3)) + 0x01000100u;
                }
                const int l10 = byte_of(lw, 10) + 256;
                // right pixel pairs starting at every byte 0..19: RP[m] = (r_m, r_{m+1})
                uint32_t RP[20];
#pragma unroll
                for (int m = 0; m < 20; ++m)
                    RP[m] = __builtin_amdgcn_perm(rw[(m >> 2) + 1 < 6 ? (m >> 2) + 1 : 5], rw[m >> 2],
                                                  pair_sel(m & 3));
#pragma unroll
                for (int k = 0; k < 11; ++k) {
                    uint32_t a = (uint32_t)acc[k];
#pragma unroll
                    for (int j = 0; j < 5; ++j) a = __builtin_amdgcn_sad_u16(LP[j], RP[k + 2 * j] + E[k], a);
                    const int d = l10 - (byte_of(rw, k + 10) + (int)(E[k] & 0xFFFFu));
                    acc[k] = (int)a + (d < 0 ? -d : d);
                }
            };
            // lane `sub` of the group takes rows sub, sub + LPK, ... (and reads the centre row
            // for the offsets); the group's row sums are added by shuffles
            constexpr int RPL = (11 + LPK - 1) / LPK;
            uint32_t lraw[RPL + 1][4], rraw[RPL + 1][7];
#pragma unroll
            for (int t = 0; t <= RPL; ++t) {
                const int r = t == RPL ? w : min(sub + LPK * t, 10);
#pragma unroll
                for (int i = 0; i < 4; ++i) lraw[t][i] = pl0[r * pdw + i];
#pragma unroll
                for (int i = 0; i < 7; ++i) rraw[t][i] = pr0[r * pdw + i];
            }
            {
                uint32_t lc[3], rc[6];
                align_l(lraw[RPL], lc);
                align_r(rraw[RPL], rc);
                centre(lc, rc);
            }
#pragma unroll
            for (int t = 0; t < RPL; ++t) {
                if (sub + LPK * t < 11) {
                    uint32_t lw[3], rw[6];
                    align_l(lraw[t], lw);
                    align_r(rraw[t], rw);
                    sad_row(lw, rw);
                }
            }
#pragma unroll
            for (int k = 0; k < 11; ++k)
#pragma unroll
                for (int m = 1; m < LPK; m <<= 1) acc[k] += __shfl_xor(acc[k], m, LPK);
        }
        int bestDist = 0x7FFFFFFF;
        int bestinc = 0;
#pragma unroll
        for (int k = 0; k < 11; ++k) {
            const float dist = (float)acc[k];
            if (dist < (float)bestDist) {
                bestDist = (int)dist;
                bestinc = k - L5;
            }
        }
        if (bestinc == -L5 || bestinc == L5) continue;
        float d1 = 0.f, d2 = 0.f, d3 = 0.f;
#pragma unroll
        for (int k = 1; k < 10; ++k) {
            if (k - L5 == bestinc) {
                d1 = (float)acc[k - 1];
                d2 = (float)acc[k];
                d3 = (float)acc[k + 1];
            }
        }
        const float deltaR = (d1 - d3) / (2.0f * (d1 + d3 - 2.0f * d2));
        if (deltaR < -1 || deltaR > 1) continue;
        float bestuR = LV.scale * ((float)scaleduR0 + (float)bestinc + deltaR);
        float disparity = (uL - bestuR);
        if (disparity >= minD && disparity < maxD) {
            if (disparity <= 0) {
                disparity = (float)0.01;
                bestuR = (float)((double)uL - 0.01);
            }
            if (sub != 0) {
            } else if (nsplit == 1) {
                dep[iL] = mbf / disparity;
                uR[iL] = bestuR;
                const int pos = atomicAdd(&tmp[16], 1);
                vsad[pos] = bestDist;
                vidx[pos] = (int16_t)iL;
            } else {
                split_store(dep + iL, mbf / disparity);
                split_store(uR + iL, bestuR);
                // a pair has at most KC accepted SADs; the guard keeps a corrupted counter from
                // writing past the pair's slots
                const int pos = atomicAdd(&scnt[b], 1);
                if (pos < KC) {
                    split_store(ssad + (size_t)b * KC + pos, bestDist);
                    split_store(sidx + (size_t)b * KC + pos, (int16_t)iL);
                }
            }
        }
    }
    if (nsplit > 1) {
        // the pair's last workgroup to finish takes the median: every wave's write-through
        // stores complete, then the workgroup's arrival is one agent-scope acq_rel add (its
        // release orders this workgroup's stores, ordered before it by the barrier, ahead of
        // the arrival; its acquire makes every earlier arrival's stores visible to the last
        // workgroup, whose barrier passes that on to its other waves); the last one reads the
        // pair's SADs by write-through loads into LDS
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0)
            tmp[17] = __hip_atomic_fetch_add(&scnt[256 + b], 1, __ATOMIC_ACQ_REL,
                                             __HIP_MEMORY_SCOPE_AGENT) == nsplit - 1;
        __syncthreads();
        if (!tmp[17]) return;
        const int nv = min(__hip_atomic_load(&scnt[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), KC);
        for (int j = tid; j < nv; j += ST_THREADS) {
            vsad[j] = __hip_atomic_load(ssad + (size_t)b * KC + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            vidx[j] = __hip_atomic_load(sidx + (size_t)b * KC + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (tid == 0) {
            scnt[b] = 0;
            scnt[256 + b] = 0;
        }
        median_cut(nv, vsad, vidx, hist, tmp, uR, dep, nvalid, b);
        return;
    }
    __syncthreads();
    median_cut(tmp[16], vsad, vidx, hist, tmp, uR, dep, nvalid, b);
}

// 3. median and outlier cut (src/Frame.cc:672-685) over the nv accepted SADs of pair b; the
//    median value depends only on the multiset of SADs, so the append order is free.
__device__ void median_cut(int nv, const int* vsad, const int16_t* vidx, int* hist, int* tmp,
                           float* uR, float* dep, int* nvalid, int b) {
    const int tid = threadIdx.x;
    if (nv == 0) {
        if (tid == 0 && nvalid) nvalid[b] = 0;
        return;
    }
    const int kth = nv / 2;
    if (tid < 256) hist[tid] = 0;
    __syncthreads();
    for (int j = tid; j < nv; j += ST_THREADS) atomicAdd(&hist[vsad[j] >> 8], 1);
    __syncthreads();
    if (tid == 0) {
        int acc = 0, bin = 0;
        for (; bin < 256; ++bin) {
            if (acc + hist[bin] > kth) break;
            acc += hist[bin];
        }
        tmp[18] = bin;
        tmp[19] = kth - acc;
    }
    __syncthreads();
    const int hb = tmp[18];
    if (tid < 256) hist[tid] = 0;
    __syncthreads();
    for (int j = tid; j < nv; j += ST_THREADS)
        if ((vsad[j] >> 8) == hb) atomicAdd(&hist[vsad[j] & 255], 1);
    __syncthreads();
    if (tid == 0) {
        int acc = 0, bin = 0;
        const int k2 = tmp[19];
        for (; bin < 256; ++bin) {
            if (acc + hist[bin] > k2) break;
            acc += hist[bin];
        }
        tmp[20] = (hb << 8) | bin;
    }
    __syncthreads();
    const float median = (float)tmp[20];
    const float thDist = 1.5f * 1.4f * median;
    int dropped = 0;
    for (int j = tid; j < nv; j += ST_THREADS) {
        if (!((float)vsad[j] < thDist)) {
            uR[vidx[j]] = -1;
            dep[vidx[j]] = -1;
            ++dropped;
        }
    }
    dropped = block_sum<ST_WAVES>(dropped, tmp);
    if (tid == 0 && nvalid) nvalid[b] = nv - dropped;
}

size_t stereo_lds_bytes(int kp_cap, int height, int ob) {
    auto r = [](size_t v) { return (v + 15) & ~(size_t)15; };
    size_t s = r(32 * 4) + r((size_t)kp_cap * 32) + r((size_t)ob * height * 4);
    s += r((size_t)kp_cap * 12);
    s += r((size_t)kp_cap * 4) + r((size_t)kp_cap * 2) + r(256 * 4);
    return s;
}

// Small batches (at most ST_LPK_BATCH pairs): ST_LPK lanes per left keypoint, ST_LPK_SPLIT
// workgroups per pair (every keypoint of a 2000-keypoint image in flight at once).  One pair
// (r4p, r4w): 1 lane 47.8 us, 2 x 8 workgroups 37.3, 4 x 8 33.9, 4 x 16 30.7, 8 x 16 30.5.
#define ST_LPK 8
#define ST_LPK_SPLIT 16
#define ST_LPK_BATCH 32

hipError_t prepare_stereo(size_t lds) {
    hipError_t e = hipFuncSetAttribute((const void*)k_stereo<1>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void*)k_stereo<ST_LPK>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    return e;
}

// Workgroups per pair: up to ST_SPLIT while the launch has at most 256 workgroups (one per
// pair would leave most CUs idle and run two left keypoints per thread in series).  One
// stereo pair: k_stereo 0.089 ms unsplit, 0.058 split in 2, 0.050 in 4; 64 pairs: 0.107 /
// 0.080 / 0.070 ms; 512 pairs are not split.
#define ST_SPLIT 4
static bool stereo_lpk(int batch) { return ST_LPK > 1 && batch <= ST_LPK_BATCH; }
int stereo_split(int batch) {
    int ns = stereo_lpk(batch) ? ST_LPK_SPLIT : ST_SPLIT;
    while (ns > 1 && batch * ns > 256) ns >>= 1;
    return ns;
}

hipError_t launch_stereo(const StereoLaunch& a, hipStream_t st) {
    // timed by the kernel's own dispatch (ORBX_TIMED_LAUNCH)
    KernelTimer* T = a.timer && a.timer->on ? a.timer : nullptr;
    hipEvent_t e0 = T ? T->get() : nullptr, e1 = T ? T->get() : nullptr;
    if (!e0 || !e1) e0 = e1 = nullptr;
    const int ns = stereo_split(a.batch);
    hipExtLaunchKernelGGL(stereo_lpk(a.batch) ? k_stereo<ST_LPK> : k_stereo<1>,
                          dim3(a.batch * ns), dim3(ST_THREADS), (uint32_t)a.lds, st, e0,
                          e1, 0u, a.dg, a.kpsL, a.descL, a.nkpL, a.pyrL,
                          a.kpsR, a.descR, a.nkpR, a.pyrR, a.mbf, a.mb, a.uR, a.depth, a.nvalid,
                          ns, a.scnt, a.ssad, a.sidx);
    if (e0 && e1) T->pending.push_back(KernelTimer::Rec{K_STEREO, e0, e1});
    return hipGetLastError();
}

}  // namespace orbx
