// orbx_match.hip — gfx950 kernels of the descriptor matchers (src/ORBmatcher.cc).
//
// The matchers are integer/bit work (XOR + v_bcnt over 256-bit descriptors) with a greedy,
// order-dependent claim step.  The kernels keep the reference's exact selection semantics
// while moving the distance work off the sequential chain:
//   k_bow            one workgroup per (keyframe, frame) job, walking the shared FeatureVector
//                    nodes: static best / second of every A feature (one thread each, B side
//                    in LDS), then an in-order replay of the greedy claims that re-scans only
//                    the A features whose static pair meets a claim.
//   k_triangulate    one workgroup per keyframe pair, one wave per KF1 node; every idx1 is
//                    independent (vbMatched2 is never set, :722), so each is a wave-min over
//                    (distance, reversed position) keys = the reference's last-wins ties.
//   k_proj_search    one wave per projected MapPoint: the grid window is a set of contiguous
//                    CSR spans (one per grid column), scanned 64 candidates at a time; yields
//                    the static top-2 (or the final answer for the claim-free modes).
//   k_proj_resolve   one wave replays the greedy claims in MapPoint order; a query whose
//                    static best/second are still unclaimed is decided from them (exact:
//                    the dynamic candidate set is a subset), otherwise the wave re-scans
//                    its window against the claim state in LDS.
//   k_proj_finish    rotation-consistency filter (ComputeThreeMaxima) and count.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <climits>

#include "orbx_device.h"
#include "orbx_kernels.h"
#include "orbx_match_kernels.h"

namespace orbx {
namespace {

constexpr int TH_HIGH = 100, TH_LOW = 50, HISTO = 30;
constexpr uint32_t INF = 0xFFFFFFFFu;

struct Desc {
    uint32_t w[8];
};

__device__ __forceinline__ Desc load_desc(const uint8_t* base, long long i) {
    const uint4* p = (const uint4*)(base + 32 * i);
    const uint4 a = p[0], b = p[1];
    return Desc{{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}};
}

// ORBmatcher::DescriptorDistance (:1715-1731): popcount of the XOR, 8 words, as a chain
// of accumulating v_bcnt_u32_b32 (the compiler otherwise sums 8 counts with 3 v_add3).
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc) {
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}

// median of three (one v_med3_u32; a 2-input v_min / v_max costs the same issue slot)
__device__ __forceinline__ uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

__device__ __forceinline__ int hamming(const Desc& a, const Desc& b) {
    uint32_t d = __popc(a.w[0] ^ b.w[0]);
#pragma unroll
    for (int k = 1; k < 8; ++k) d = bcnt_acc(a.w[k] ^ b.w[k], d);
    return (int)d;
}

// Wave-wide unsigned min, uniform result: DPP within rows of 16, then 4 readlanes.
// Must be called with all 64 lanes active.
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, true));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, true));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x124, 0xF, 0xF, true));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x128, 0xF, 0xF, true));
    const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
    const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)v, 32);
    const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
    return min(min(a, b), min(c, d));
}

// Rotation bin of the matchers (e.g. :269-275): float difference, +360 when negative,
// round(rot * (1.0f/30)) half away from zero, 30 -> 0.
__device__ __forceinline__ int rot_bin(float a1, float a2) {
    const float factor = 1.0f / HISTO;
    float rot = a1 - a2;
    if (rot < 0.0f) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == HISTO) bin = 0;
    return bin;
}

// ComputeThreeMaxima (:1669-1710) on 30 counts.  Returns the kept bins.
struct Top3 {
    int i1, i2, i3;
    __device__ bool keeps(int b) const { return b == i1 || b == i2 || b == i3; }
};

__device__ __forceinline__ Top3 three_maxima(const int* h) {
    int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
    for (int i = 0; i < HISTO; i++) {
        const int s = h[i];
        const bool g1 = s > max1, g2 = !g1 && s > max2, g3 = !g1 && !g2 && s > max3;
        // branch-free form of the reference's if / else-if chain
        max3 = g1 || g2 ? max2 : (g3 ? s : max3);
        ind3 = g1 || g2 ? ind2 : (g3 ? i : ind3);
        max2 = g1 ? max1 : (g2 ? s : max2);
        ind2 = g1 ? ind1 : (g2 ? i : ind2);
        max1 = g1 ? s : max1;
        ind1 = g1 ? i : ind1;
    }
    if (max2 < 0.1f * (float)max1) {
        ind2 = -1; ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
        ind3 = -1;
    }
    return {ind1, ind2, ind3};
}

// float -> int as the x86-64 reference converts (int)floor(v): cvttss2si yields INT_MIN for
// NaN and out-of-range values (the GPU's v_cvt_i32_f32 saturates instead).
__device__ __forceinline__ int x86_int(float f) {
    return (f >= -2147483648.0f && f < 2147483648.0f) ? (int)f : INT_MIN;
}

// ---------------------------------------------------------------------------------------
// SearchByBoW (:182-319 and :563-696)
// ---------------------------------------------------------------------------------------

// One workgroup (4 waves) per (keyframe, frame) job.  A B feature belongs to exactly one
// FeatureVector node, so the greedy claims of different nodes never interact and each
// shared node is an independent problem:
//   1. the node's B descriptors (and a per-position key suffix: the position, or INF for a
//      feature the reference skips statically) are staged in LDS;
//   2. every A feature of the node gets its STATIC best and second key (distance << 20 |
//      position) over all of them, one thread per A feature scanning the LDS copy (broadcast
//      reads, no reductions);
//   3. wave 0 replays the reference's loop over the A features in order, 64 at a time.  The
//      claimed set only grows, so an A feature whose static best and second are both still
//      unclaimed at its turn has exactly those as its dynamic best and second: it is decided
//      without looking at the candidates again.  Only an A feature whose static pair meets a
//      claim is re-scanned (all 64 lanes, against the claim bitmap).  Within a chunk, the
//      lanes before the first one that claims or conflicts are decided together.
// BLDS = false reads the B descriptors from global memory (nodes too large for LDS).
#define BOW_R 4   // A features per thread in the static pass
#define BOW_T 256 // threads per job
template <bool BLDS>
__global__ __launch_bounds__(BOW_T) void k_bow(BowLaunch g) {
    extern __shared__ __attribute__((aligned(16))) int lds[];
    const int job = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int ka = g.a_fixed ? 0 : job, kb = g.b_fixed ? 0 : job;
    const int fa0 = g.A.feat_off[ka], nA = g.A.feat_off[ka + 1] - fa0;
    const int fb0 = g.B.feat_off[kb], nBt = g.B.feat_off[kb + 1] - fb0;
    const int nOut = g.kf_kf ? nA : nBt;
    int32_t* out = g.out + (size_t)job * g.out_stride;
    if (nA < 0 || nBt < 0 || nA > g.A.max_feat || nBt > g.B.max_feat || nOut > g.out_stride) {
        for (int i = tid; i < g.out_stride; i += BOW_T) out[i] = -1;
        if (tid == 0) {
            g.nmatches[job] = 0;
            atomicOr(g.err, 1);
        }
        return;
    }
    const int amax = g.A.max_feat, bmax = g.B.max_feat;
    const int smax = g.kf_kf ? amax : bmax;
    // LDS carve (bow_lds_bytes): B descriptors first (16-byte aligned)
    uint4* bdesc = (uint4*)lds;                                    // [bmax][2] (BLDS)
    uint32_t* pkey = (uint32_t*)(lds + (BLDS ? 8 * bmax : 0));     // [bmax]
    uint32_t* top1 = pkey + bmax;                                  // [amax]
    uint32_t* top2 = top1 + amax;                                  // [amax]
    int* state = (int*)(top2 + amax);                              // [smax] match | bin << 24
    uint32_t* claimed = (uint32_t*)(state + smax);                 // [(bmax + 31) / 32] per node
    int* hist = (int*)(claimed + (bmax + 31) / 32);                // [32] + 8 scan scratch
    for (int i = tid; i < nOut; i += BOW_T) state[i] = -1;
    if (tid < 32) hist[tid] = 0;

    const bool kfkf = g.kf_kf != 0;
    const int na0 = g.A.node_off[ka], na1 = g.A.node_off[ka + 1];
    int bn = g.B.node_off[kb];
    const int bn1 = g.B.node_off[kb + 1];
    for (int ga = na0; ga < na1; ++ga) {
        // Lock-step FeatureVector walk (:205-295): both maps ascending, so the shared nodes
        // are found by advancing the B cursor to the first id >= the A id.
        const uint32_t id = g.A.node_id[ga];
        while (bn < bn1 && g.B.node_id[bn] < id) ++bn;
        if (bn >= bn1) break;
        if (g.B.node_id[bn] != id) continue;
        const int a0 = g.A.node_feat_off[ga], nAn = g.A.node_feat_off[ga + 1] - a0;
        const int b0 = g.B.node_feat_off[bn], nB = g.B.node_feat_off[bn + 1] - b0;
        ++bn;
        if (nB <= 0 || nAn <= 0) continue;
        __syncthreads();   // the previous node's readers are done with the LDS arrays
        // ---- 1. stage the node's B side ----
        for (int p = tid; p < nB; p += BOW_T) {
            const int f = g.B.node_feat[b0 + p];
            const bool in = (unsigned)f < (unsigned)nBt;
            const int fc = in ? f : 0;
            // :240 skips claimed frame features only; KF-KF also needs a valid MapPoint (:633)
            const bool ok = in && (!kfkf || g.B.flag[fb0 + fc]);
            pkey[p] = ok ? (uint32_t)p : INF;
            if (BLDS) {
                const uint4* s = (const uint4*)(g.B.desc + 32 * ((size_t)fb0 + fc));
                bdesc[2 * p] = s[0];
                bdesc[2 * p + 1] = s[1];
            }
        }
        for (int i = tid; i < (nB + 31) / 32; i += BOW_T) claimed[i] = 0u;
        __syncthreads();
        // ---- 2. static best / second of every A feature of the node: BOW_R rows per
        //      thread (rows i, i + 256, ...), so one LDS read of a B descriptor feeds BOW_R
        //      distances ----
        for (int i0 = tid; i0 < nAn; i0 += BOW_T * BOW_R) {
            Desc ad[BOW_R];
            bool vl[BOW_R];
            uint32_t k1[BOW_R], k2[BOW_R];
            bool any = false;
#pragma unroll
            for (int r = 0; r < BOW_R; ++r) {
                const int i = i0 + BOW_T * r;
                const int fa = i < nAn ? g.A.node_feat[a0 + i] : -1;
                vl[r] = (unsigned)fa < (unsigned)nA && g.A.flag[fa0 + max(fa, 0)];
                ad[r] = load_desc(g.A.desc, (long long)fa0 + (vl[r] ? fa : 0));
                k1[r] = INF;
                k2[r] = INF;
                any |= vl[r];
            }
            if (any) {
                for (int p = 0; p < nB; ++p) {
                    Desc bd;
                    if (BLDS) {
                        const uint4 u0 = bdesc[2 * p], u1 = bdesc[2 * p + 1];
                        bd = Desc{{u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w}};
                    } else {
                        const int f = g.B.node_feat[b0 + p];
                        bd = load_desc(g.B.desc, (long long)fb0 + ((unsigned)f < (unsigned)nBt ? f : 0));
                    }
                    const uint32_t pk = pkey[p];
#pragma unroll
                    for (int r = 0; r < BOW_R; ++r) {
                        const uint32_t key = ((uint32_t)hamming(ad[r], bd) << 20) | pk;
                        k2[r] = med3_u32(k1[r], k2[r], key);   // k1 <= k2: the new second
                        k1[r] = min(k1[r], key);
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < BOW_R; ++r) {
                const int i = i0 + BOW_T * r;
                if (i < nAn) {
                    top1[i] = vl[r] ? k1[r] : INF - 1;   // INF - 1: A feature skipped (:224-228 / :599-603)
                    top2[i] = k2[r];
                }
            }
        }
        __syncthreads();
        // ---- 3. greedy replay in A order (wave 0) ----
        if (wid == 0) {
            auto is_claimed = [&](uint32_t k) {
                const uint32_t p = k & 0xFFFFFu;
                return k < INF - 1 && ((claimed[p >> 5] >> (p & 31)) & 1u);
            };
            auto pass = [&](int d1, int d2) {
                return (kfkf ? d1 < TH_LOW : d1 <= TH_LOW) && (float)d1 < g.ratio * (float)d2;
            };
            for (int c0 = 0; c0 < nAn; c0 += 64) {
                const int i = c0 + lane;
                const bool inr = i < nAn;
                const uint32_t k1 = inr ? top1[i] : INF - 1, k2 = inr ? top2[i] : INF;
                const bool vl = k1 != INF - 1;
                const int fa = inr ? g.A.node_feat[a0 + i] : 0;
                const int d1 = k1 == INF ? 256 : (int)(k1 >> 20);
                const int d2 = k2 == INF ? 256 : min((int)(k2 >> 20), 256);
                const bool sacc = vl && pass(d1, d2);
                int start = 0;
                while (true) {
                    const bool conflict = vl && (is_claimed(k1) || is_claimed(k2));
                    const uint64_t ev = __ballot((conflict || sacc) && lane >= start);
                    if (!ev) break;
                    const int t = __builtin_ctzll(ev);
                    const bool tconf = (__ballot(conflict) >> t) & 1u;
                    uint32_t m1;
                    bool tacc;
                    if (tconf) {
                        // dynamic best / second over the unclaimed candidates
                        const int fat = __builtin_amdgcn_readlane(fa, t);
                        const Desc ad = load_desc(g.A.desc, (long long)fa0 + fat);
                        uint32_t q1 = INF, q2 = INF;
                        for (int p = lane; p < nB; p += 64) {
                            Desc bd;
                            if (BLDS) {
                                const uint4 u0 = bdesc[2 * p], u1 = bdesc[2 * p + 1];
                                bd = Desc{{u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w}};
                            } else {
                                const int f = g.B.node_feat[b0 + p];
                                bd = load_desc(g.B.desc, (long long)fb0 + ((unsigned)f < (unsigned)nBt ? f : 0));
                            }
                            const bool cl = (claimed[p >> 5] >> (p & 31)) & 1u;
                            const uint32_t key = cl ? INF : (((uint32_t)hamming(ad, bd) << 20) | pkey[p]);
                            q2 = min(q2, max(q1, key));
                            q1 = min(q1, key);
                        }
                        m1 = wave_min_u32(q1);
                        const uint32_t m2 = wave_min_u32(q1 == m1 ? q2 : q1);
                        const int e1 = m1 == INF ? 256 : (int)(m1 >> 20);
                        const int e2 = m2 == INF ? 256 : min((int)(m2 >> 20), 256);
                        tacc = pass(e1, e2);
                    } else {
                        m1 = (uint32_t)__builtin_amdgcn_readlane((int)k1, t);
                        tacc = true;
                    }
                    if (tacc) {
                        const int pos = (int)(m1 & 0xFFFFFu);
                        if (lane == 0) {
                            claimed[pos >> 5] |= 1u << (pos & 31);
                            const int fbm = g.B.node_feat[b0 + pos];
                            const int fat = __builtin_amdgcn_readlane(fa, t);
                            if (kfkf) state[fat] = fbm;
                            else state[fbm] = fat;
                        }
                        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    }
                    start = t + 1;
                }
            }
        }
    }
    __syncthreads();
    // Rotation consistency (:298-316 / :675-693) and the count.  The histogram only needs
    // the bin of every match, so it is built here from the final state.
    if (g.check_ori) {
        for (int i = tid; i < nOut; i += BOW_T) {
            const int s = state[i];
            if (s >= 0) {
                const int ia = kfkf ? i : s, ib = kfkf ? s : i;
                const int bin = rot_bin(g.A.keys[fa0 + ia].angle, g.B.keys[fb0 + ib].angle);
                state[i] = s | (bin << 24);
                atomicAdd(&hist[bin], 1);
            }
        }
        __syncthreads();
    }
    const Top3 top = g.check_ori ? three_maxima(hist) : Top3{-1, -1, -1};
    int cnt = 0;
    for (int i = tid; i < nOut; i += BOW_T) {
        const int s = state[i];
        int r = -1;
        if (s >= 0) {
            const int bin = s >> 24;
            if (!g.check_ori || top.keeps(bin)) {
                r = s & 0xFFFFFF;
                ++cnt;
            }
        }
        out[i] = r;
    }
    for (int i = nOut + tid; i < g.out_stride; i += BOW_T) out[i] = -1;
    cnt = block_sum<BOW_T / 64>(cnt, hist + 32);
    if (tid == 0) g.nmatches[job] = cnt;
}

// ---------------------------------------------------------------------------------------
// SearchForTriangulation (:702-872) + CheckDistEpipolarLine (:147-167)
// ---------------------------------------------------------------------------------------

__global__ __launch_bounds__(256) void k_triangulate(TriLaunch g) {
    extern __shared__ int lds[];
    int* state = lds;
    int* hist = lds + g.db.max_feat;
    __shared__ int red[4];
    const int job = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int k1 = g.kf1[job], k2 = g.kf2[job];
    const orbx_kf_db& db = g.db;
    const int f10 = db.feat_off[k1], n1 = db.feat_off[k1 + 1] - f10;
    const int f20 = db.feat_off[k2], n2 = db.feat_off[k2 + 1] - f20;
    int32_t* out = g.out + g.job_off[job];
    if (n1 < 0 || n2 < 0 || n1 > db.max_feat || n2 > db.max_feat ||
        g.job_off[job + 1] - g.job_off[job] < n1) {
        if (tid == 0) {
            g.nmatches[job] = 0;
            atomicOr(g.err, 1);
        }
        return;
    }
    for (int i = tid; i < n1; i += 256) state[i] = -1;
    if (tid < 32) hist[tid] = 0;
    __syncthreads();

    float F[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) F[k] = g.F12[9 * job + k];
    const float ex = g.epi[2 * job], ey = g.epi[2 * job + 1];
    // Per shared node, lanes take the KF1 features (one idx1 per lane: every idx1 is
    // independent, :722) and scan the node's KF2 features, staged once per 64 in this wave's
    // LDS slice, in their order: the reference's `dist > bestDist` skip with bestDist updated
    // on acceptance keeps the LAST accepted candidate of the smallest distance (:786-811).
    __shared__ uint4 sBd[4][64][2];
    __shared__ float sBx[4][64], sBy[4][64], sBa[4][64];
    __shared__ int sBf[4][64];   // octave | stereo << 8 | valid << 9 | idx2 << 10
    const int na0 = db.node_off[k1], na1 = db.node_off[k1 + 1];
    const int nb0 = db.node_off[k2], nb1 = db.node_off[k2 + 1];
    // features by node-entry position (contiguous per node) when the database carries the
    // node-order copies, else gathered by feature index
    const bool nord = db.node_keys != nullptr;
    for (int ga = na0 + w; ga < na1; ga += 4) {
        const uint32_t id = db.node_id[ga];
        int lo = nb0, hi = nb1;   // lower_bound
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (db.node_id[mid] < id) lo = mid + 1; else hi = mid;
        }
        if (lo >= nb1 || db.node_id[lo] != id) continue;
        const int a0 = db.node_feat_off[ga], a1 = db.node_feat_off[ga + 1];
        const int b0 = db.node_feat_off[lo], nB = db.node_feat_off[lo + 1] - b0;
        for (int ac = a0; ac < a1; ac += 64) {
            const int ia = ac + lane;
            const int idx1 = ia < a1 ? db.node_feat[ia] : -1;
            bool validA = (unsigned)idx1 < (unsigned)n1;
            const int i1 = validA ? idx1 : 0;
            const long long pa = nord ? (long long)(ia < a1 ? ia : a0) : (long long)f10 + i1;
            validA = validA && !(nord ? db.node_flag[pa] : db.flag[pa]);   // :749
            const float ur1 = nord ? (db.node_u_right ? db.node_u_right[pa] : -1.0f)
                                   : (db.u_right ? db.u_right[pa] : -1.0f);
            const bool bStereo1 = ur1 >= 0;
            if (g.only_stereo && !bStereo1) validA = false;
            const orbx_keypoint kp1 = nord ? db.node_keys[pa] : db.keys[pa];
            // CheckDistEpipolarLine's line coefficients depend on kp1 only.
            const float a = kp1.x * F[0] + kp1.y * F[3] + F[6];
            const float b = kp1.x * F[1] + kp1.y * F[4] + F[7];
            const float c = kp1.x * F[2] + kp1.y * F[5] + F[8];
            const float den = a * a + b * b;
            const Desc d1 = load_desc(nord ? db.node_desc : db.desc, pa);
            int bestDist = TH_LOW, bestIdx2 = -1;
            float bestAng = 0.f;
            for (int bc = 0; bc < nB; bc += 64) {
                const int cnt = min(64, nB - bc);
                if (lane < cnt) {
                    const int idx2 = db.node_feat[b0 + bc + lane];
                    bool ok = (unsigned)idx2 < (unsigned)n2;
                    const int i2 = ok ? idx2 : 0;
                    const long long pb = nord ? (long long)(b0 + bc + lane) : (long long)f20 + i2;
                    ok = ok && !(nord ? db.node_flag[pb] : db.flag[pb]);   // :773
                    const float ur2 = nord ? (db.node_u_right ? db.node_u_right[pb] : -1.0f)
                                           : (db.u_right ? db.u_right[pb] : -1.0f);
                    const bool st2 = ur2 >= 0;
                    if (g.only_stereo && !st2) ok = false;
                    const orbx_keypoint kp2 = nord ? db.node_keys[pb] : db.keys[pb];
                    const uint4* q = (const uint4*)((nord ? db.node_desc : db.desc) + 32 * pb);
                    sBd[w][lane][0] = q[0];
                    sBd[w][lane][1] = q[1];
                    sBx[w][lane] = kp2.x;
                    sBy[w][lane] = kp2.y;
                    sBa[w][lane] = kp2.angle;
                    sBf[w][lane] = min(max(kp2.octave, 0), MATCH_MAX_LEVELS - 1) | (st2 ? 256 : 0) |
                                   (ok ? 512 : 0) | (i2 << 10);
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                for (int p = 0; p < cnt; ++p) {
                    const int fl = sBf[w][p];
                    if (!(fl & 512)) continue;   // uniform: a skipped KF2 feature
                    const uint4 u0 = sBd[w][p][0], u1 = sBd[w][p][1];
                    const Desc d2 = Desc{{u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w}};
                    const int dist = hamming(d1, d2);
                    if (dist > bestDist) continue;   // :786 (bestDist <= TH_LOW)
                    const int o2 = fl & 255;
                    const float x2 = sBx[w][p], y2 = sBy[w][p];
                    if (!bStereo1 && !(fl & 256)) {   // :791-798
                        const float distex = ex - x2;
                        const float distey = ey - y2;
                        if (distex * distex + distey * distey < 100 * g.scale[o2]) continue;
                    }
                    if (den == 0) continue;
                    const float num = a * x2 + b * y2 + c;
                    const float dsqr = num * num / den;
                    if (!((double)dsqr < 3.84 * (double)g.sigma2[o2])) continue;
                    bestDist = dist;
                    bestIdx2 = fl >> 10;
                    bestAng = sBa[w][p];
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            }
            if (validA && bestIdx2 >= 0) {
                int bin = 0;
                if (g.check_ori) {
                    bin = rot_bin(kp1.angle, bestAng);
                    atomicAdd(&hist[bin], 1);
                }
                state[idx1] = bestIdx2 | (bin << 24);
            }
        }
    }
    __syncthreads();
    const Top3 top = g.check_ori ? three_maxima(hist) : Top3{-1, -1, -1};
    int cnt = 0;
    for (int i = tid; i < n1; i += 256) {
        const int s = state[i];
        int r = -1;
        if (s >= 0) {
            const int bin = s >> 24;
            if (!g.check_ori || top.keeps(bin)) {
                r = s & 0xFFFFFF;
                ++cnt;
            }
        }
        out[i] = r;
    }
    const int tot = block_sum<4>(cnt, red);
    if (tid == 0) g.nmatches[job] = tot;
}

// ---------------------------------------------------------------------------------------
// Projection searches (:46-132, :321-434, :879-1156, :1158-1382, :1392-1667, :446-561)
// ---------------------------------------------------------------------------------------

struct ModeInfo {
    bool frame_grid;   // Frame::GetFeaturesInArea with level arguments
    bool init256;      // best (and second) initialised to 256: a distance of 256 never counts
    bool stereo;       // |ur - uRight| > radius rejects (uRight > 0)
    bool kf_level;     // octave in [pred-1, pred] (matcher-side)
    bool fuse;         // reprojection chi2 test (:968-992)
    bool rot;          // rotation-consistency filter
    bool greedy;       // sequential claims
    int th;            // acceptance threshold on the best distance
};

__device__ __forceinline__ ModeInfo mode_info(int mode, int orb_dist) {
    switch (mode) {
        case ORBX_PROJ_FRAME_MAPPOINTS: return {true, true, true, false, false, false, true, TH_HIGH};
        case ORBX_PROJ_KF_SCW:          return {false, true, false, true, false, false, true, TH_LOW};
        case ORBX_PROJ_LAST_FRAME:      return {true, true, true, false, false, true, true, TH_HIGH};
        case ORBX_PROJ_KEYFRAME:        return {true, true, false, false, false, true, true, orb_dist};
        case ORBX_PROJ_FUSE:            return {false, true, false, true, true, false, false, TH_LOW};
        case ORBX_PROJ_FUSE_SCW:        return {false, false, false, true, false, false, false, TH_LOW};
        case ORBX_PROJ_SIM3:            return {false, false, false, true, false, false, false, TH_HIGH};
        default:                        return {true, false, false, false, false, true, true, TH_LOW};
    }
}

struct NoDyn {
    __device__ bool operator()(int, int) const { return true; }
};
struct ClaimDyn {   // claimed features are skipped
    const uint8_t* claimed;
    __device__ bool operator()(int i, int) const { return claimed[i] == 0; }
};
struct InitDyn {    // :485 vMatchedDistance[i2] <= dist skips
    const int* mdist;
    __device__ bool operator()(int i, int d) const { return mdist[i] > d; }
};

constexpr uint32_t POS_MASK = (1u << 23) - 1;

// The target featureset of job j (see ProjLaunch).
__device__ __forceinline__ orbx_featureset job_target(const ProjLaunch& g, int j) {
    orbx_featureset T = g.T;
    if (g.t_off) {
        const int f0 = g.t_off[j];
        T.n = g.t_off[j + 1] - f0;
        T.keys += f0;
        T.desc += 32 * (size_t)f0;
        if (T.u_right) T.u_right += f0;
        T.grid_off += (size_t)j * (T.grid_cols * T.grid_rows + 1);
        T.grid_feat += g.g_off[j];
    }
    return T;
}

__device__ __forceinline__ int job_first_query(const ProjLaunch& g, int j) {
    return g.q_off ? g.q_off[j] : 0;
}
__device__ __forceinline__ int job_end_query(const ProjLaunch& g, int j) {
    return g.q_off ? g.q_off[j + 1] : g.nq;
}
// job of query qi: upper_bound(q_off, qi) - 1
__device__ __forceinline__ int job_of_query(const ProjLaunch& g, int qi) {
    if (!g.q_off) return 0;
    int lo = 0, hi = g.njobs;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (g.q_off[mid] <= qi) lo = mid; else hi = mid;
    }
    return lo;
}

// GetFeaturesInArea + the mode's candidate filters + DescriptorDistance, reduced to the
// first two keys (distance << 23 | grid CSR position) in the reference's visiting order
// (cell column ix, then row iy, then the cell's vector: exactly increasing CSR position).
// A group of G lanes (16: one DPP row, or the whole wave) scans one query's window.
template <int G>
__device__ __forceinline__ uint32_t group_min_u32(uint32_t v) {
    if constexpr (G == 64) {
        return wave_min_u32(v);
    } else {
        static_assert(G == 16, "groups are DPP rows or waves");
        v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, true));
        v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, true));
        v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x124, 0xF, 0xF, true));
        v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x128, 0xF, 0xF, true));
        return v;
    }
}

template <int G, class Dyn, class Sink>
__device__ __forceinline__ void window_scan(const ProjLaunch& g, const orbx_featureset& T,
                                            const ModeInfo& mi, const orbx_proj_query& q,
                                            const Desc& qd, Dyn dyn, Sink& sink) {
    const int lane = lane_id() & (G - 1);
    const float x = q.u, y = q.v, r = q.radius;
    const int nMinCellX = max(0, x86_int(floorf((x - T.min_x - r) * T.grid_inv_w)));
    if (nMinCellX >= T.grid_cols) return;
    const int nMaxCellX = min(T.grid_cols - 1, x86_int(ceilf((x - T.min_x + r) * T.grid_inv_w)));
    if (nMaxCellX < 0) return;
    const int nMinCellY = max(0, x86_int(floorf((y - T.min_y - r) * T.grid_inv_h)));
    if (nMinCellY >= T.grid_rows) return;
    const int nMaxCellY = min(T.grid_rows - 1, x86_int(ceilf((y - T.min_y + r) * T.grid_inv_h)));
    if (nMaxCellY < 0) return;
    const bool checkLevels = mi.frame_grid && ((q.min_level > 0) || (q.max_level >= 0));
    for (int ix = nMinCellX; ix <= nMaxCellX; ++ix) {
        const int p0 = T.grid_off[ix * T.grid_rows + nMinCellY];
        const int p1 = T.grid_off[ix * T.grid_rows + nMaxCellY + 1];
        for (int base = p0; base < p1; base += G) {
            const int p = base + lane;
            if (p >= p1) continue;
            const int i = T.grid_feat[p];
            if ((unsigned)i >= (unsigned)T.n) continue;
            const orbx_keypoint kp = T.keys[i];
            if (checkLevels) {
                if (kp.octave < q.min_level) continue;
                if (q.max_level >= 0 && kp.octave > q.max_level) continue;
            }
            const float distx = kp.x - x, disty = kp.y - y;
            if (!(fabsf(distx) < r && fabsf(disty) < r)) continue;
            if (mi.kf_level && (kp.octave < q.pred_level - 1 || kp.octave > q.pred_level)) continue;
            const float uR = T.u_right ? T.u_right[i] : -1.0f;
            if (mi.stereo && uR > 0) {
                const float er = fabsf(q.ur - uR);
                if (er > r) continue;
            }
            if (mi.fuse) {
                const float is2 = g.inv_sigma2[min(max(kp.octave, 0), MATCH_MAX_LEVELS - 1)];
                const float ex = x - kp.x, ey = y - kp.y;
                if (uR >= 0) {
                    const float er = q.ur - uR;
                    const float e2 = ex * ex + ey * ey + er * er;
                    if ((double)(e2 * is2) > 7.8) continue;
                } else {
                    const float e2 = ex * ex + ey * ey;
                    if ((double)(e2 * is2) > 5.99) continue;
                }
            }
            const int d = hamming(qd, load_desc(T.desc, i));
            if (mi.init256 && d >= 256) continue;
            if (!dyn(i, d)) continue;
            sink((uint32_t)d << 23 | (uint32_t)p);
        }
    }
}

struct Top2Sink {
    uint32_t k1 = INF, k2 = INF;
    __device__ void operator()(uint32_t key) {
        if (key < k1) { k2 = k1; k1 = key; }
        else if (key < k2) { k2 = key; }
    }
};

// The group-wide two smallest keys of the window (INF when absent).
template <int G = 64, class Dyn>
__device__ void window_top2(const ProjLaunch& g, const orbx_featureset& T, const ModeInfo& mi,
                            const orbx_proj_query& q, const Desc& qd, Dyn dyn, uint32_t& o1,
                            uint32_t& o2) {
    Top2Sink t;
    window_scan<G>(g, T, mi, q, qd, dyn, t);
    o1 = group_min_u32<G>(t.k1);
    o2 = group_min_u32<G>(t.k1 == o1 ? t.k2 : t.k1);
}

// Lane-local sorted PROJ_K smallest keys (branch-free insertion).
struct TopKSink {
    uint32_t k[PROJ_K];
    __device__ TopKSink() {
#pragma unroll
        for (int j = 0; j < PROJ_K; ++j) k[j] = INF;
    }
    __device__ void operator()(uint32_t key) {
        uint32_t x = key;
#pragma unroll
        for (int j = 0; j < PROJ_K; ++j) {
            const uint32_t lo = min(k[j], x);
            x = max(k[j], x);
            k[j] = lo;
        }
    }
};

// The group-wide PROJ_K smallest keys: group lane r < count holds the r-th; more = keys
// beyond them.
template <int G, class Dyn>
__device__ void window_topk(const ProjLaunch& g, const orbx_featureset& T, const ModeInfo& mi,
                            const orbx_proj_query& q, const Desc& qd, Dyn dyn, uint32_t& mine,
                            int& count, bool& more) {
    TopKSink t;
    window_scan<G>(g, T, mi, q, qd, dyn, t);
    const int lane = lane_id() & (G - 1);
    mine = INF;
    count = 0;
    more = false;
    for (int r = 0; r < PROJ_K; ++r) {
        const uint32_t m = group_min_u32<G>(t.k[0]);
        if (m == INF) return;
        if (lane == r) mine = m;
        ++count;
        if (t.k[0] == m) {   // keys are unique (CSR position): one lane pops its head
#pragma unroll
            for (int j = 0; j < PROJ_K - 1; ++j) t.k[j] = t.k[j + 1];
            t.k[PROJ_K - 1] = INF;
        }
    }
    more = group_min_u32<G>(t.k[0]) != INF;
}

struct Cand {
    int i, d, lvl, bin;
};

__device__ __forceinline__ Cand decode_key(const orbx_featureset& T, const ModeInfo& mi,
                                           uint32_t k, float qangle) {
    if (k == INF) return {-1, 0, -1, 0};
    const int i = T.grid_feat[k & POS_MASK];
    const orbx_keypoint kp = T.keys[i];
    return {i, (int)(k >> 23), kp.octave, mi.rot ? rot_bin(qangle, kp.angle) : 0};
}

__device__ __forceinline__ int pack_cand(const Cand& c) {
    return c.d | (c.lvl & 0xF) << 9 | c.bin << 13;
}

__global__ __launch_bounds__(256) void k_proj_search(ProjLaunch g) {
    // one 16-lane group (a DPP row) per query, 16 queries per block
    constexpr int G = 16;
    const int qi = blockIdx.x * (256 / G) + (threadIdx.x / G), lane = lane_id() & (G - 1);
    if (qi >= g.nq) return;
    const ModeInfo mi = mode_info(g.mode, g.orb_dist);
    const orbx_proj_query q = g.q[qi];
    if (!(q.radius >= 0)) {
        if (lane == 0) {
            if (mi.greedy && g.mode != PROJ_INIT) g.ncand[qi] = 0;
            else if (mi.greedy) g.top2[qi] = make_int4(-1, -1, 0, 0);
            else g.out[qi] = -1;
        }
        return;
    }
    const Desc qd = load_desc(g.qdesc, qi);
    const int job = job_of_query(g, qi);
    const orbx_featureset T = job_target(g, job);
    uint32_t m1, m2;
    if (mi.greedy && g.mode != PROJ_INIT) {
        // claim modes: the PROJ_K best candidates, sorted, for the replay.  Features claimed
        // before the call are out for every query and are filtered here.
        uint32_t mine;
        int count;
        bool more;
        if (g.claimed_in)
            window_topk<G>(g, T, mi, q, qd, ClaimDyn{g.claimed_in + (g.t_off ? g.t_off[job] : 0)},
                        mine, count, more);
        else
            window_topk<G>(g, T, mi, q, qd, NoDyn{}, mine, count, more);
        if (lane < PROJ_K) {
            const Cand c = decode_key(T, mi, mine, q.angle);
            g.cand[(size_t)qi * PROJ_K + lane] = make_int2(c.i, pack_cand(c));
        }
        if (lane == 0) g.ncand[qi] = more ? PROJ_K + 1 : count;
        return;
    }
    window_top2<G>(g, T, mi, q, qd, NoDyn{}, m1, m2);
    if (lane != 0) return;
    if (mi.greedy) {
        const Cand c1 = decode_key(T, mi, m1, q.angle), c2 = decode_key(T, mi, m2, q.angle);
        g.top2[qi] = make_int4(c1.i, c2.i, pack_cand(c1), pack_cand(c2));
    } else {
        g.out[qi] = (m1 != INF && (int)(m1 >> 23) <= mi.th) ? T.grid_feat[m1 & POS_MASK] : -1;
    }
}

// Claim-mode replays keep an owner word per target feature when it fits in the LDS.
__host__ __device__ inline bool proj_resolve_parallel(int max_t) {
    return 4 * 32 + 5 * (size_t)max_t + 16 <= MATCH_MAX_LDS;
}

// Greedy replay in MapPoint order (one wave per job).
__global__ __launch_bounds__(64) void k_proj_resolve(ProjLaunch g) {
    extern __shared__ int lds[];
    const int lane = lane_id(), job = blockIdx.x;
    const ModeInfo mi = mode_info(g.mode, g.orb_dist);
    const bool init = g.mode == PROJ_INIT;
    const orbx_featureset T = job_target(g, job);
    const int q0 = job_first_query(g, job), q1 = job_end_query(g, job);
    const int nT = T.n, nq = q1 - q0;
    const uint8_t* claimed_in = g.claimed_in ? g.claimed_in + (g.t_off ? g.t_off[job] : 0) : nullptr;
    if (nT > g.max_t) {   // the LDS was sized for max_t: flag the job, no matches
        if (lane == 0) atomicOr(g.err, 1);
        for (int i = q0 + lane; i < q1; i += 64) g.out[i] = -1;
        if (lane < 32) g.hist[32 * job + lane] = 0;
        return;
    }
    int* hist = lds;                         // 32
    const bool par = proj_resolve_parallel(g.max_t);
    int* owner = lds + 32;                   // nT (claim modes, par): earliest acceptor lane
    uint8_t* claimed = (uint8_t*)(lds + 32 + (par ? g.max_t : 0));   // nT (claim modes)
    int* mdist = lds + 32;                   // nT (init): vMatchedDistance
    int* m21 = mdist + nT;                   // nT (init): vnMatches21
    int* m12 = m21 + nT;                     // nq (init): vnMatches12
    if (lane < 32) hist[lane] = 0;
    if (init) {
        for (int i = lane; i < nT; i += 64) { mdist[i] = INT_MAX; m21[i] = -1; }
        for (int i = lane; i < nq; i += 64) m12[i] = -1;
    } else {
        for (int i = lane; i < nT; i += 64) claimed[i] = claimed_in ? (claimed_in[i] != 0) : 0;
        if (par)
            for (int i = lane; i < nT; i += 64) owner[i] = 64;
    }
    __syncthreads();
    for (int qb = 0; qb < nq && !init; qb += 64) {
        // Claim modes, 64 queries at a time.  Lane t holds query t's list of its PROJ_K best
        // candidates (sorted by key, pre-claimed features already out).  Each round every
        // pending lane decides against the current claims; a lane whose best or second is
        // also accepted by an earlier pending lane (owner[] holds the earliest acceptor), or
        // that follows a lane needing a full re-scan, waits for the next round.  The lanes
        // before the first waiting one decide exactly as the sequential loop would, and
        // commit together.  Without the owner array (large targets) one lane per round.
        const int cnt = min(64, nq - qb);
        const int qi = q0 + qb + lane;
        const bool mine = lane < cnt;
        const int nc = mine ? g.ncand[qi] : 0;
        // a query whose MapPoint has no observations leaves its feature unclaimed (:90-92,
        // :1471-1473 test Observations() > 0 of the MapPoint already there)
        // (only FRAME_MAPPOINTS and LAST_FRAME test Observations(); KEYFRAME / KF_SCW skip any
        // matched feature, :1609-1610, :406)
        const bool claims = !(mine && g.qflags && (g.qflags[qi] & ORBX_QF_NO_CLAIM) &&
                              (g.mode == ORBX_PROJ_FRAME_MAPPOINTS || g.mode == ORBX_PROJ_LAST_FRAME));
        const int nv = min(nc, PROJ_K);
        int2 L[PROJ_K];
        {
            const int4* src = (const int4*)(g.cand + (size_t)(mine ? qi : q0) * PROJ_K);
#pragma unroll
            for (int k = 0; k < PROJ_K / 2; ++k) {
                const int4 v = (2 * k < nv) ? src[k] : make_int4(-1, 0, -1, 0);
                L[2 * k] = make_int2(v.x, v.y);
                L[2 * k + 1] = make_int2(v.z, v.w);
            }
        }
        int res = -1, rbin = 0;
        int start = 0;
        while (start < cnt) {
            Cand b = {-1, 0, -1, 0}, c = {-1, 0, -1, 0};
            int nfree = 0;
#pragma unroll
            for (int k = 0; k < PROJ_K; ++k) {
                const bool fr = k < nv && claimed[max(L[k].x, 0)] == 0;
                const Cand x = {L[k].x, L[k].y & 0x1FF, (L[k].y >> 9) & 0xF, (L[k].y >> 13) & 0x1F};
                if (fr && nfree == 0) b = x;
                else if (fr && nfree == 1) c = x;
                nfree += fr;
            }
            const bool act = lane >= start && lane < cnt;
            const bool rescan = act && nfree < 2 && nc > PROJ_K;
            bool acc;
            if (g.mode == ORBX_PROJ_FRAME_MAPPOINTS) {   // :121-124
                const int bestDist = b.i >= 0 ? b.d : 256, bestLevel = b.i >= 0 ? b.lvl : -1;
                const int bestDist2 = c.i >= 0 ? c.d : 256, bestLevel2 = c.i >= 0 ? c.lvl : -1;
                acc = bestDist <= TH_HIGH &&
                      !(bestLevel == bestLevel2 && (float)bestDist > g.ratio * (float)bestDist2);
            } else {
                acc = b.i >= 0 && b.d <= mi.th;
            }
            acc = acc && act && !rescan;
            int f = start + 1;
            if (par) {
                if (acc && claims) atomicMin(&owner[b.i], lane);
                bool wait = rescan && lane > start;
                if (act && lane > start) {
                    if (b.i >= 0 && owner[b.i] < lane) wait = true;
                    if (c.i >= 0 && owner[c.i] < lane) wait = true;
                }
                if (acc && claims) owner[b.i] = 64;
                const uint64_t w = __ballot(wait);
                f = w ? (int)__builtin_ctzll(w) : cnt;
            }
            if ((__ballot(rescan) >> start) & 1) {
                // the first pending query's list ran out: re-scan its window, alone
                const int qs = q0 + qb + start;
                const orbx_proj_query q = g.q[qs];
                const Desc qd = load_desc(g.qdesc, qs);
                uint32_t m1, m2;
                window_top2(g, T, mi, q, qd, ClaimDyn{claimed}, m1, m2);
                const Cand rb = decode_key(T, mi, m1, q.angle), rc = decode_key(T, mi, m2, q.angle);
                bool racc;
                if (g.mode == ORBX_PROJ_FRAME_MAPPOINTS) {
                    const int bestDist = rb.i >= 0 ? rb.d : 256, bestLevel = rb.i >= 0 ? rb.lvl : -1;
                    const int bestDist2 = rc.i >= 0 ? rc.d : 256, bestLevel2 = rc.i >= 0 ? rc.lvl : -1;
                    racc = bestDist <= TH_HIGH &&
                           !(bestLevel == bestLevel2 && (float)bestDist > g.ratio * (float)bestDist2);
                } else {
                    racc = rb.i >= 0 && rb.d <= mi.th;
                }
                if (lane == start) {
                    res = racc ? rb.i : -1;
                    if (racc) {
                        if (claims) claimed[rb.i] = 1;
                        rbin = rb.bin;
                        if (mi.rot && g.check_ori) atomicAdd(&hist[rb.bin], 1);
                    }
                }
                ++start;
                continue;
            }
            if (lane >= start && lane < f) {
                res = acc ? b.i : -1;
                if (acc) {
                    if (claims) claimed[b.i] = 1;
                    rbin = b.bin;
                    if (mi.rot && g.check_ori) atomicAdd(&hist[b.bin], 1);
                }
            }
            start = f;
        }
        if (mine) {
            g.out[qi] = res;
            if (res >= 0) g.out_bin[qi] = (int8_t)rbin;
        }
    }
    for (int qb = 0; qb < nq && init; qb += 64) {
        const int cnt = min(64, nq - qb);
        const int4 s = (lane < cnt) ? g.top2[q0 + qb + lane] : make_int4(-1, -1, 0, 0);
        for (int t = 0; t < cnt; ++t) {
            const int qj = qb + t, qi = q0 + qj;   // job-local / global query index
            Cand b = {__builtin_amdgcn_readlane(s.x, t), 0, -1, 0};
            Cand c = {__builtin_amdgcn_readlane(s.y, t), 0, -1, 0};
            const int w1 = __builtin_amdgcn_readlane(s.z, t), w2 = __builtin_amdgcn_readlane(s.w, t);
            b.d = w1 & 0x1FF; b.lvl = (w1 >> 9) & 0xF; b.bin = (w1 >> 13) & 0x1F;
            c.d = w2 & 0x1FF; c.lvl = (w2 >> 9) & 0xF; c.bin = (w2 >> 13) & 0x1F;
            if (b.i < 0) {
                if (lane == 0 && !init) g.out[qi] = -1;
                continue;   // no static candidate: none under any claim state either
            }
            auto pass = [&](const Cand& x) {
                return init ? (mdist[x.i] > x.d) : (claimed[x.i] == 0);
            };
            const bool fast = pass(b) && (c.i < 0 || pass(c));
            if (!fast) {
                // The static best or second is gone: re-scan the window against the state.
                const orbx_proj_query q = g.q[qi];
                const Desc qd = load_desc(g.qdesc, qi);
                uint32_t m1, m2;
                if (init) window_top2(g, T, mi, q, qd, InitDyn{mdist}, m1, m2);
                else window_top2(g, T, mi, q, qd, ClaimDyn{claimed}, m1, m2);
                b = decode_key(T, mi, m1, q.angle);
                c = decode_key(T, mi, m2, q.angle);
            }
            bool acc;
            if (g.mode == ORBX_PROJ_FRAME_MAPPOINTS) {   // :121-124
                const int bestDist = b.i >= 0 ? b.d : 256, bestLevel = b.i >= 0 ? b.lvl : -1;
                const int bestDist2 = c.i >= 0 ? c.d : 256, bestLevel2 = c.i >= 0 ? c.lvl : -1;
                acc = bestDist <= TH_HIGH &&
                      !(bestLevel == bestLevel2 && (float)bestDist > g.ratio * (float)bestDist2);
            } else if (init) {                           // :500-502
                const int bestDist = b.i >= 0 ? b.d : INT_MAX;
                const int bestDist2 = c.i >= 0 ? c.d : INT_MAX;
                acc = bestDist <= TH_LOW && (float)bestDist < (float)bestDist2 * g.ratio;
            } else {
                acc = b.i >= 0 && b.d <= mi.th;
            }
            if (lane == 0) {
                if (init) {
                    if (acc) {   // :504-512 (re-assignment)
                        const int prev = m21[b.i];
                        if (prev >= 0) m12[prev] = -1;
                        m12[qj] = b.i;
                        m21[b.i] = qj;
                        mdist[b.i] = b.d;
                        g.out_bin[qi] = (int8_t)b.bin;
                        if (g.check_ori) hist[b.bin] += 1;
                    }
                } else {
                    g.out[qi] = acc ? b.i : -1;
                    if (acc) {
                        claimed[b.i] = 1;
                        g.out_bin[qi] = (int8_t)b.bin;
                        if (mi.rot && g.check_ori) hist[b.bin] += 1;
                    }
                }
            }
        }
    }
    __syncthreads();
    if (init)
        for (int i = lane; i < nq; i += 64) g.out[q0 + i] = m12[i];
    if (lane < 32) g.hist[32 * job + lane] = hist[lane];
}

__global__ __launch_bounds__(256) void k_proj_finish(ProjLaunch g) {
    __shared__ int red[4];
    __shared__ int h[32];
    const int tid = threadIdx.x;
    const ModeInfo mi = mode_info(g.mode, g.orb_dist);
    const bool filt = mi.rot && g.check_ori && !g.prefilter;
    const int job = blockIdx.x;
    const int q0 = job_first_query(g, job), q1 = job_end_query(g, job);
    if (tid < 32) h[tid] = filt ? g.hist[32 * job + tid] : 0;
    __syncthreads();
    const Top3 top = filt ? three_maxima(h) : Top3{-1, -1, -1};
    int cnt = 0;
    for (int i = q0 + tid; i < q1; i += 256) {
        int r = g.out[i];
        if (r >= 0 && filt) {
            const int bin = g.out_bin[i];
            if (!top.keeps(bin)) {
                r = -1;
                g.out[i] = -1;
            }
        }
        cnt += r >= 0;
    }
    const int tot = block_sum<4>(cnt, red);
    if (tid == 0) g.nmatches[job] = tot;
}

// ---------------------------------------------------------------------------------------
// MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:252-313)
// ---------------------------------------------------------------------------------------
// One wave per map point: its N descriptors are staged in LDS, lane i computes row i of the
// distance matrix into LDS (u16), finds the row's median vDists[(N-1)/2] by a binary search
// over distance values (9 counting passes), and a wave-min over (median << 16 | i) keeps the
// first row with the least median.
__global__ __launch_bounds__(64) void k_distinctive(const uint8_t* __restrict__ desc,
                                                    const int32_t* __restrict__ off, int np,
                                                    int32_t* __restrict__ best, int* err) {
    extern __shared__ uint32_t dl[];   // [MAXOBS][8] descriptors, then [64][MAXOBS+1] u16 rows
    constexpr int MAXN = ORBX_MAX_OBSERVATIONS;
    uint16_t* rows = (uint16_t*)(dl + MAXN * 8);
    const int p = blockIdx.x, lane = threadIdx.x;
    if (p >= np) return;
    const int o0 = off[p], N = off[p + 1] - o0;
    if (N <= 0 || N > MAXN) {
        if (lane == 0) {
            best[p] = -1;
            if (N > MAXN) atomicOr(err, 1);
        }
        return;
    }
    for (int t = lane; t < N * 8; t += 64)
        dl[t] = ((const uint32_t*)(desc + 32 * (size_t)o0))[t];
    __syncthreads();
    const int k = (N - 1) >> 1;   // vDists[0.5*(N-1)]
    uint32_t bestkey = INF;
    uint16_t* row = rows + lane * (MAXN + 1);
    for (int i0 = 0; i0 < N; i0 += 64) {
        const int i = i0 + lane;
        const bool has = i < N;
        const int ic = has ? i : N - 1;
        Desc di;
#pragma unroll
        for (int w = 0; w < 8; ++w) di.w[w] = dl[ic * 8 + w];
        for (int j = 0; j < N; ++j) {
            Desc dj;
#pragma unroll
            for (int w = 0; w < 8; ++w) dj.w[w] = dl[j * 8 + w];
            row[j] = (uint16_t)hamming(di, dj);
        }
        int lo = 0, hi = 256;   // smallest v with #(row <= v) >= k + 1
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            int cnt = 0;
            for (int j = 0; j < N; ++j) cnt += row[j] <= mid;
            if (cnt >= k + 1) hi = mid; else lo = mid + 1;
        }
        const uint32_t key = has ? ((uint32_t)lo << 16 | (uint32_t)i) : INF;
        bestkey = min(bestkey, wave_min_u32(key));
    }
    if (lane == 0) best[p] = (int)(bestkey & 0xFFFFu);
}

}  // namespace

hipError_t launch_distinctive(const uint8_t* desc, const int32_t* off, int np, int32_t* best,
                              int* err, hipStream_t st) {
    if (np <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_distinctive, dim3(np), dim3(64), distinctive_lds_bytes(), st, desc, off,
                       np, best, err);
    return hipGetLastError();
}

size_t distinctive_lds_bytes() {
    return (size_t)ORBX_MAX_OBSERVATIONS * 32 + 64 * (ORBX_MAX_OBSERVATIONS + 1) * 2;
}

bool proj_mode_greedy(int mode) {
    return mode == ORBX_PROJ_FRAME_MAPPOINTS || mode == ORBX_PROJ_KF_SCW ||
           mode == ORBX_PROJ_LAST_FRAME || mode == ORBX_PROJ_KEYFRAME || mode == PROJ_INIT;
}

static size_t bow_lds_raw(const BowLaunch& a, bool blds) {
    const size_t am = (size_t)a.A.max_feat, bm = (size_t)a.B.max_feat;
    const size_t sm = a.kf_kf ? am : bm;
    return (blds ? 32 * bm : 0) + 4 * bm + 8 * am + 4 * sm + 4 * ((bm + 31) / 32) + 4 * 40;
}

static bool bow_blds(const BowLaunch& a) { return bow_lds_raw(a, true) <= MATCH_MAX_LDS; }

size_t bow_lds_bytes(const BowLaunch& a) { return bow_lds_raw(a, bow_blds(a)); }

hipError_t launch_bow(const BowLaunch& a, hipStream_t st) {
    if (a.njobs <= 0) return hipSuccess;
    const size_t lds = bow_lds_bytes(a);
    if (lds > MATCH_MAX_LDS) return hipErrorInvalidValue;
    if (bow_blds(a))
        hipLaunchKernelGGL(k_bow<true>, dim3(a.njobs), dim3(BOW_T), lds, st, a);
    else
        hipLaunchKernelGGL(k_bow<false>, dim3(a.njobs), dim3(BOW_T), lds, st, a);
    return hipGetLastError();
}

size_t tri_lds_bytes(int max_feat) { return 4 * ((size_t)max_feat + 32); }

// orbx_kf_db_node_order: one workgroup per keyframe, one thread per node entry of it
__global__ __launch_bounds__(256) void k_node_order(orbx_kf_db db, int n, orbx_keypoint* keys,
                                                     uint8_t* desc, float* ur, uint8_t* flag) {
    const int k = blockIdx.x;
    const int f0 = db.feat_off[k], nf = db.feat_off[k + 1] - f0;
    const int p0 = db.node_feat_off[db.node_off[k]], p1 = min(db.node_feat_off[db.node_off[k + 1]], n);
    for (int p = p0 + (int)threadIdx.x; p < p1; p += 256) {
        const int i = db.node_feat[p];
        const bool ok = (unsigned)i < (unsigned)nf;
        const long long f = (long long)f0 + (ok ? i : 0);
        orbx_keypoint kp = db.keys[f];
        const uint4* s = (const uint4*)(db.desc + 32 * f);
        uint4 d0 = s[0], d1 = s[1];
        if (!ok) {
            kp = orbx_keypoint{};
            d0 = d1 = make_uint4(0u, 0u, 0u, 0u);
        }
        keys[p] = kp;
        ((uint4*)(desc + 32 * (long long)p))[0] = d0;
        ((uint4*)(desc + 32 * (long long)p))[1] = d1;
        if (ur) ur[p] = ok && db.u_right ? db.u_right[f] : -1.0f;
        flag[p] = ok ? db.flag[f] : (uint8_t)1;
    }
}

hipError_t launch_node_order(const orbx_kf_db& db, int n, orbx_keypoint* keys, uint8_t* desc,
                             float* ur, uint8_t* flag, hipStream_t st) {
    if (db.nkf <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_node_order, dim3(db.nkf), dim3(256), 0, st, db, n, keys, desc, ur, flag);
    return hipGetLastError();
}

hipError_t launch_triangulate(const TriLaunch& a, hipStream_t st) {
    if (a.njobs <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_triangulate, dim3(a.njobs), dim3(256), tri_lds_bytes(a.db.max_feat), st, a);
    return hipGetLastError();
}

size_t proj_resolve_lds_bytes(int mode, int n_target, int nq) {
    if (mode == PROJ_INIT) return 4 * (32 + 2 * (size_t)n_target + (size_t)nq);
    return 4 * 32 + (proj_resolve_parallel(n_target) ? 5 : 1) * (size_t)n_target + 16;
}

hipError_t launch_proj(const ProjLaunch& a, hipStream_t st, KernelTimer* timer) {
    if (a.nq <= 0) return hipSuccess;
    hipEvent_t e = timer ? timer->start(st) : nullptr;
    hipLaunchKernelGGL(k_proj_search, dim3((a.nq + 15) / 16), dim3(256), 0, st, a);
    if (timer) timer->stop(ORBX_MK_PROJ_SEARCH, e, st);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return err;
    if (proj_mode_greedy(a.mode)) {
        e = timer ? timer->start(st) : nullptr;
        // LDS per job: the largest target, and (init) the largest query list = nq bound
        hipLaunchKernelGGL(k_proj_resolve, dim3(a.njobs), dim3(64),
                           proj_resolve_lds_bytes(a.mode, a.max_t, a.nq), st, a);
        if (timer) timer->stop(ORBX_MK_PROJ_RESOLVE, e, st);
        err = hipGetLastError();
        if (err != hipSuccess) return err;
    }
    hipLaunchKernelGGL(k_proj_finish, dim3(a.njobs), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t prepare_match_kernels() {
    const int lds = (int)MATCH_MAX_LDS;
    hipError_t e;
    if ((e = hipFuncSetAttribute((const void*)k_bow<true>, hipFuncAttributeMaxDynamicSharedMemorySize, lds)) != hipSuccess) return e;
    if ((e = hipFuncSetAttribute((const void*)k_bow<false>, hipFuncAttributeMaxDynamicSharedMemorySize, lds)) != hipSuccess) return e;
    if ((e = hipFuncSetAttribute((const void*)k_triangulate, hipFuncAttributeMaxDynamicSharedMemorySize, (int)TRI_MAX_LDS)) != hipSuccess) return e;
    if ((e = hipFuncSetAttribute((const void*)k_distinctive, hipFuncAttributeMaxDynamicSharedMemorySize, lds)) != hipSuccess) return e;
    return hipFuncSetAttribute((const void*)k_proj_resolve, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
}

}  // namespace orbx
