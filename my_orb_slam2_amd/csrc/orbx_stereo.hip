// orbx_stereo.hip — Frame::ComputeStereoMatches (src/Frame.cc:496-686) as one gfx950
// workgroup per stereo pair, batched over pairs.
//
//   1. right keypoints bucketed by image row (LDS counting sort); the reference's
//      vRowIndices lists are recovered exactly by testing each bucketed keypoint's
//      [floor(y-2s), ceil(y+2s)] band, and the reference's "first candidate wins" rule
//      becomes a lexicographic (distance, right index) minimum, so bucket order is free;
//   2. one thread per left keypoint: band / octave / disparity-range filters + 256-bit
//      Hamming (v_xor + v_bcnt), best < 75 goes to the SAD stage;
//   3. one wave per match: 11x11 SAD at 11 shifts on the unblurred pyramids (exact integer
//      sums, lanes own window pixels), parabola fit, depth — float formulas as the reference;
//   4. median of the accepted SADs by a two-pass LDS radix select and the 2.1*median cut.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orbx_device.h"
#include "orbx_internal.h"
#include "orbx_kernels.h"

namespace orbx {

__device__ __forceinline__ int hamming256(const uint32_t a[8], const uint8_t* bptr) {
    const uint4* q = (const uint4*)bptr;
    const uint4 b0 = q[0], b1 = q[1];
    return __popc(a[0] ^ b0.x) + __popc(a[1] ^ b0.y) + __popc(a[2] ^ b0.z) + __popc(a[3] ^ b0.w) +
           __popc(a[4] ^ b1.x) + __popc(a[5] ^ b1.y) + __popc(a[6] ^ b1.z) + __popc(a[7] ^ b1.w);
}

__global__ __launch_bounds__(256) void k_stereo(const Geometry* __restrict__ g,
                                                const float* __restrict__ kpsL,
                                                const uint8_t* __restrict__ descL,
                                                const int* __restrict__ nkpL,
                                                const uint8_t* __restrict__ pyrL,
                                                const float* __restrict__ kpsR,
                                                const uint8_t* __restrict__ descR,
                                                const int* __restrict__ nkpR,
                                                const uint8_t* __restrict__ pyrR, float mbf,
                                                float mb, float* __restrict__ uRight,
                                                float* __restrict__ depth,
                                                int* __restrict__ nvalid) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int b = blockIdx.x, tid = threadIdx.x;
    const int wid = tid >> 6, lane = tid & 63;
    const int KC = g->kp_cap;
    const int H = g->lv[0].h;
    uint8_t* p = smem;
    auto take = [&](size_t bytes) { uint8_t* r = p; p += (bytes + 15) & ~(size_t)15; return r; };
    int* tmp = (int*)take(32 * 4);
    int* rowstart = (int*)take((size_t)(H + 1) * 4);
    int* cursor = (int*)take((size_t)(H + 1) * 4);
    int16_t* bucket = (int16_t*)take((size_t)KC * 2);
    float* rx = (float*)take((size_t)KC * 4);
    int16_t* rmin = (int16_t*)take((size_t)KC * 2);
    int16_t* rmax = (int16_t*)take((size_t)KC * 2);
    int16_t* rrow = (int16_t*)take((size_t)KC * 2);
    int8_t* roct = (int8_t*)take((size_t)KC);
    int* mlist = (int*)take((size_t)KC * 4);     // (iL << 16) | iR
    int* vsad = (int*)take((size_t)KC * 4);
    int16_t* vidx = (int16_t*)take((size_t)KC * 2);
    int* hist = (int*)take(256 * 4);

    const int NL = min(max(nkpL[b], 0), KC), NR = min(max(nkpR[b], 0), KC);
    const float* kL = kpsL + (size_t)b * KC * 7;
    const float* kR = kpsR + (size_t)b * KC * 7;
    float* uR = uRight + (size_t)b * KC;
    float* dep = depth + (size_t)b * KC;
    for (int i = tid; i < NL; i += 256) { uR[i] = -1.0f; dep[i] = -1.0f; }
    for (int i = tid; i <= H; i += 256) rowstart[i] = 0;
    if (tid == 0) { tmp[16] = 0; tmp[17] = 0; }
    __syncthreads();

    // 1. right keypoints -> rows (src/Frame.cc:516-531)
    for (int iR = tid; iR < NR; iR += 256) {
        const float ky = kR[iR * 7 + 1];
        const int oct = ((const int*)kR)[iR * 7 + 5];
        const float r = 2.0f * g->lv[oct].scale;
        rmax[iR] = (int16_t)(int)ceilf(ky + r);
        rmin[iR] = (int16_t)(int)floorf(ky - r);
        rx[iR] = kR[iR * 7 + 0];
        roct[iR] = (int8_t)oct;
        const int row = min(max((int)ky, 0), H - 1);
        rrow[iR] = (int16_t)row;
        atomicAdd(&rowstart[row], 1);
    }
    __syncthreads();
    {
        int carry = 0;
        for (int c0 = 0; c0 < H + 1; c0 += 256) {
            const int i = c0 + tid;
            const int v = i < H + 1 ? rowstart[i] : 0;
            int tot;
            const int ex = block_excl_scan(v, tmp, tot);
            if (i < H + 1) { rowstart[i] = carry + ex; cursor[i] = carry + ex; }
            carry += tot;
        }
    }
    __syncthreads();
    for (int iR = tid; iR < NR; iR += 256) {
        const int pos = atomicAdd(&cursor[rrow[iR]], 1);
        bucket[pos] = (int16_t)iR;
    }
    __syncthreads();

    // 2. descriptor search per left keypoint (src/Frame.cc:542-587)
    const float maxD = mbf / mb;   // minZ = mb, maxD = mbf/minZ (Frame.cc:534-536)
    const float minD = 0;
    for (int iL = tid; iL < NL; iL += 256) {
        const float uL = kL[iL * 7 + 0], vL = kL[iL * 7 + 1];
        const int levelL = ((const int*)kL)[iL * 7 + 5];
        const int row = (int)vL;
        const float minU = uL - maxD, maxU = uL - minD;
        if (maxU < 0 || row >= H) continue;
        uint32_t dl[8];
        {
            const uint4* q = (const uint4*)(descL + ((size_t)b * KC + iL) * 32);
            const uint4 a0 = q[0], a1 = q[1];
            dl[0] = a0.x; dl[1] = a0.y; dl[2] = a0.z; dl[3] = a0.w;
            dl[4] = a1.x; dl[5] = a1.y; dl[6] = a1.z; dl[7] = a1.w;
        }
        int best = 100, bestR = -1;   // ORBmatcher::TH_HIGH, strict '<': first minimum wins
        const int r0 = max(row - g->stereo_win, 0), r1 = min(row + g->stereo_win, H - 1);
        for (int e = rowstart[r0]; e < rowstart[r1 + 1]; ++e) {
            const int iR = bucket[e];
            if (rmin[iR] > row || rmax[iR] < row) continue;
            const int o = roct[iR];
            if (o < levelL - 1 || o > levelL + 1) continue;
            const float u = rx[iR];
            if (u >= minU && u <= maxU) {
                const int dist = hamming256(dl, descR + ((size_t)b * KC + iR) * 32);
                if (dist < best || (dist == best && bestR >= 0 && iR < bestR)) {
                    best = dist;
                    bestR = iR;
                }
            }
        }
        if (bestR >= 0 && best < 75) {   // thOrbDist = (TH_HIGH + TH_LOW) / 2
            const int pos = atomicAdd(&tmp[16], 1);
            mlist[pos] = (iL << 16) | bestR;
        }
    }
    __syncthreads();

    // 3. SAD refinement, one wave per match (src/Frame.cc:591-667)
    const int nm = tmp[16];
    for (int m = wid; m < nm; m += 4) {
        const int iL = mlist[m] >> 16, iR = mlist[m] & 0xFFFF;
        const float uL = kL[iL * 7 + 0], vL = kL[iL * 7 + 1];
        const int oct = ((const int*)kL)[iL * 7 + 5];
        const LevelGeom& LV = g->lv[oct];
        const float uR0 = rx[iR];
        const float sf = LV.inv_scale;
        const float scaleduL = roundf(uL * sf);
        const float scaledvL = roundf(vL * sf);
        const float scaleduR0 = roundf(uR0 * sf);
        const int w = 5, L5 = 5;
        const float iniu = scaleduR0 + L5 - w;
        const float endu = scaleduR0 + L5 + w + 1;
        if (iniu < 0 || endu >= LV.w) continue;   // wave-uniform
        const int pitch = LV.pitch;
        const uint8_t* PL = pyrL + (size_t)b * g->pyr_bytes + LV.off;
        const uint8_t* PR = pyrR + (size_t)b * g->pyr_bytes + LV.off;
        const int yl = (int)scaledvL, xl = (int)scaleduL, xr = (int)scaleduR0;
        const int cL = PL[(size_t)yl * pitch + xl];
        int acc[11];
#pragma unroll
        for (int k = 0; k < 11; ++k) acc[k] = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int pix = lane + 64 * h;
            if (pix < 121) {
                const int yy = pix / 11 - w, xx = pix % 11 - w;
                const int il = PL[(size_t)(yl + yy) * pitch + xl + xx] - cL;
                const uint8_t* rowR = PR + (size_t)(yl + yy) * pitch + xr + xx;
                const uint8_t* ctrR = PR + (size_t)yl * pitch + xr;
#pragma unroll
                for (int k = 0; k < 11; ++k) {
                    const int ir = rowR[k - L5] - ctrR[k - L5];
                    const int d = il - ir;
                    acc[k] += d < 0 ? -d : d;
                }
            }
        }
#pragma unroll
        for (int k = 0; k < 11; ++k) acc[k] = wave_sum(acc[k]);
        if (lane == 0) {
            int bestDist = 0x7FFFFFFF;
            int bestinc = 0;
            for (int k = 0; k < 11; ++k) {
                const float dist = (float)acc[k];
                if (dist < (float)bestDist) {
                    bestDist = (int)dist;
                    bestinc = k - L5;
                }
            }
            if (bestinc != -L5 && bestinc != L5) {
                const float dist1 = (float)acc[L5 + bestinc - 1];
                const float dist2 = (float)acc[L5 + bestinc];
                const float dist3 = (float)acc[L5 + bestinc + 1];
                const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
                if (!(deltaR < -1 || deltaR > 1)) {
                    float bestuR = LV.scale * ((float)scaleduR0 + (float)bestinc + deltaR);
                    float disparity = (uL - bestuR);
                    if (disparity >= minD && disparity < maxD) {
                        if (disparity <= 0) {
                            disparity = (float)0.01;
                            bestuR = (float)((double)uL - 0.01);
                        }
                        dep[iL] = mbf / disparity;
                        uR[iL] = bestuR;
                        const int pos = atomicAdd(&tmp[17], 1);
                        vsad[pos] = bestDist;
                        vidx[pos] = (int16_t)iL;
                    }
                }
            }
        }
    }
    __syncthreads();

    // 4. median and outlier cut (src/Frame.cc:672-685)
    const int nv = tmp[17];
    if (nv == 0) {
        if (tid == 0 && nvalid) nvalid[b] = 0;
        return;
    }
    const int kth = nv / 2;
    hist[tid] = 0;
    __syncthreads();
    for (int j = tid; j < nv; j += 256) atomicAdd(&hist[vsad[j] >> 8], 1);
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
    hist[tid] = 0;
    __syncthreads();
    for (int j = tid; j < nv; j += 256)
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
        tmp[21] = 0;
    }
    __syncthreads();
    const float median = (float)tmp[20];
    const float thDist = 1.5f * 1.4f * median;
    int dropped = 0;
    for (int j = tid; j < nv; j += 256) {
        if (!((float)vsad[j] < thDist)) {
            uR[vidx[j]] = -1;
            dep[vidx[j]] = -1;
            ++dropped;
        }
    }
    dropped = block_sum(dropped, tmp);
    if (tid == 0 && nvalid) nvalid[b] = nv - dropped;
}

size_t stereo_lds_bytes(int kp_cap, int height) {
    auto r = [](size_t v) { return (v + 15) & ~(size_t)15; };
    size_t s = r(32 * 4) + 2 * r((size_t)(height + 1) * 4);
    s += r((size_t)kp_cap * 2) + r((size_t)kp_cap * 4) + 3 * r((size_t)kp_cap * 2) + r(kp_cap);
    s += r((size_t)kp_cap * 4) * 2 + r((size_t)kp_cap * 2) + r(256 * 4);
    return s;
}

hipError_t prepare_stereo(size_t lds) {
    return hipFuncSetAttribute((const void*)k_stereo, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)lds);
}

hipError_t launch_stereo(const StereoLaunch& a, hipStream_t st) {
    hipEvent_t e = a.timer ? a.timer->start(st) : nullptr;
    hipLaunchKernelGGL(k_stereo, dim3(a.batch), dim3(256), a.lds, st, a.dg, a.kpsL, a.descL,
                       a.nkpL, a.pyrL, a.kpsR, a.descR, a.nkpR, a.pyrR, a.mbf, a.mb, a.uR,
                       a.depth, a.nvalid);
    if (a.timer) a.timer->stop(K_STEREO, e, st);
    return hipGetLastError();
}

}  // namespace orbx
