// orbx_kfdb.hip — ORB_SLAM2::KeyFrameDatabase (src/KeyFrameDatabase.cc) resident in HBM
// (include/orbx_kfdb.h).
//
// Layout (slot = add order, which is every inverted-file list's order, :40-46):
//   words / vals   the BowVectors of all slots, concatenated (u32 word ids ascending per slot,
//                  f64 weights): slot s owns [off[s], off[s+1])
//   alive[s]       0 once erased (:48-67)
//   cov[s][K]      GetBestCovisibilityKeyFrames(K) of slot s (slots, -1 padded)
//   state[s]       mRelocScore, persistent across queries as on the reference's KeyFrame
//
// A detect call is two launches on the database's stream:
//   k_kfdb_scan    one wave per slot: the query's words in LDS, a binary search per slot word
//                  gives the number of shared words (mnRelocWords / mnLoopWords: a keyframe
//                  appears once per word it holds in the inverted file), the L1 score of
//                  DBoW2 (terms summed in ascending word order, L1Scoring::score's double sum,
//                  ScoringObject.cpp:23-67) and the query position of the first shared word.
//                  The reference meets keyframe s first at that word, in slot order among
//                  keyframes meeting it first there: (first, s) orders lKFsSharingWords.
//   k_kfdb_select  one workgroup: maxCommonWords, the 0.8 filter, the covisibility
//                  accumulation per listed slot (independent), bestAccScore, the 0.75
//                  retention, and the de-duplicated list in lKFsSharingWords order (a bitonic
//                  sort of the retained (first, slot) keys in LDS); the relocalisation query
//                  then stores its scores as the slots' mRelocScore.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/orbx_kfdb.h"
#include "orbx_device.h"
#include "orbx_host.h"

using namespace orbx;

namespace {

constexpr int SEL_THREADS = 1024;
constexpr int SEL_WAVES = SEL_THREADS / 64;
constexpr int RCAP = 8192;        // retained candidates sorted in LDS
constexpr int QMAX = 8192;        // query words (LDS)
constexpr int EXCL_MAX = 8192;    // connected keyframes of a loop query (LDS)
constexpr int KMAX = 64;          // covisibles per slot

// ---- scan ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_kfdb_scan(const uint32_t* __restrict__ qword,
                                                   const double* __restrict__ qval, int nq,
                                                   int nslots, const int32_t* __restrict__ off,
                                                   const uint8_t* __restrict__ alive,
                                                   const uint32_t* __restrict__ word,
                                                   const double* __restrict__ val,
                                                   int32_t* __restrict__ common,
                                                   float* __restrict__ score,
                                                   int32_t* __restrict__ first) {
    extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
    uint32_t* qw = (uint32_t*)sm;
    double* qv = (double*)(sm + ((4 * (size_t)nq + 15) & ~(size_t)15));
    double* term = qv + nq + 64 * (threadIdx.x >> 6);   // 64 per wave
    for (int i = threadIdx.x; i < nq; i += 256) {
        qw[i] = qword[i];
        qv[i] = qval[i];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int s = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (s >= nslots) return;
    int cnt = 0, fst = INT_MAX;
    double acc = 0;
    if (alive[s]) {
        const int o0 = off[s], o1 = off[s + 1];
        for (int base = o0; base < o1; base += 64) {
            const int p = base + lane;
            double t = 0;
            bool hit = false;
            int lo = 0;
            if (p < o1) {
                const uint32_t w = word[p];
                int hi = nq;   // lower_bound of w in the query's words
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (qw[mid] < w) lo = mid + 1; else hi = mid;
                }
                if (lo < nq && qw[lo] == w) {
                    const double vi = qv[lo], wi = val[p];
                    t = fabs(vi - wi) - fabs(vi) - fabs(wi);
                    hit = true;
                }
            }
            const uint64_t m = __ballot(hit);
            if (m == 0) continue;
            // the slot's words ascend, so the first hit of the first chunk with one is the
            // smallest shared word: its query position
            if (fst == INT_MAX) fst = __shfl(lo, __builtin_ctzll(m), 64);
            cnt += __popcll(m);
            term[lane] = t;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (lane == 0) {
                uint64_t mm = m;
                while (mm) {   // L1Scoring::score's sequential sum, ascending words
                    const int j = __builtin_ctzll(mm);
                    mm &= mm - 1;
                    acc += term[j];
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    if (lane == 0) {
        common[s] = cnt;
        score[s] = (float)(-acc / 2.0);   // float si = mpVoc->score(...)
        first[s] = cnt ? fst : INT_MAX;
    }
}

// ---- select ----------------------------------------------------------------------------------
__device__ __forceinline__ int block_max(int v, int* tmp) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) tmp[threadIdx.x >> 6] = v;
    __syncthreads();
    int r = tmp[0];
#pragma unroll
    for (int w = 1; w < SEL_WAVES; ++w) r = max(r, tmp[w]);
    __syncthreads();
    return r;
}

__device__ __forceinline__ float block_maxf(float v, float* tmp) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) tmp[threadIdx.x >> 6] = v;
    __syncthreads();
    float r = tmp[0];
#pragma unroll
    for (int w = 1; w < SEL_WAVES; ++w) r = fmaxf(r, tmp[w]);
    __syncthreads();
    return r;
}

// out: [0] candidate count (or -1: more retained entries than RCAP), [1 ..] slots
__global__ __launch_bounds__(SEL_THREADS) void k_kfdb_select(
    int loop, int nslots, int K, const uint8_t* __restrict__ alive,
    const int32_t* __restrict__ cov, const int32_t* __restrict__ common,
    const float* __restrict__ score, const int32_t* __restrict__ first,
    float* __restrict__ state, const int32_t* __restrict__ excl, int nexcl, float min_score,
    float* __restrict__ acc_s, int32_t* __restrict__ best_s, int32_t* __restrict__ firstpos,
    int32_t* __restrict__ out, int cap) {
    __shared__ int itmp[SEL_WAVES + 1];
    __shared__ float ftmp[SEL_WAVES];
    __shared__ uint64_t key[RCAP];
    __shared__ int32_t bval[RCAP];
    __shared__ int32_t ex[EXCL_MAX];
    const int tid = threadIdx.x;
    for (int i = tid; i < nexcl; i += SEL_THREADS) ex[i] = excl[i];
    __syncthreads();
    // GetConnectedKeyFrames() membership: a binary search in the sorted list
    auto excluded = [&](int s) {
        int lo = 0, hi = nexcl;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (ex[mid] < s) lo = mid + 1; else hi = mid;
        }
        return lo < nexcl && ex[lo] == s;
    };
    // in lKFsSharingWords: shares a word (erased slots are in no inverted-file list, their
    // common count is 0) and, for a loop query, is not connected to the query keyframe
    auto shares = [&](int s) { return common[s] > 0 && (!loop || !excluded(s)); };

    // maxCommonWords (:120-125 / :251-257)
    int mx = 0;
    for (int s = tid; s < nslots; s += SEL_THREADS)
        if (shares(s)) mx = max(mx, common[s]);
    mx = block_max(mx, itmp);
    if (mx == 0) {   // lKFsSharingWords empty
        if (tid == 0) out[0] = 0;
        return;
    }
    const int minC = (int)((float)mx * 0.8f);   // int minCommonWords = maxCommonWords*0.8f

    // lScoreAndMatch and the covisibility accumulation (:133-184 / :266-314), one listed slot
    // per thread (each is independent: it reads only this query's scan and the stored state)
    float bmax = loop ? min_score : 0.0f;
    int nlisted = 0;
    for (int s = tid; s < nslots; s += SEL_THREADS) {
        float a = -1.0f;
        int bk = -1;
        if (shares(s) && common[s] > minC && (!loop || score[s] >= min_score)) {
            const float sc = score[s];
            float bestScore = sc;
            a = sc;
            bk = s;
            for (int j = 0; j < K; ++j) {
                const int nb = cov[(size_t)s * K + j];
                if (nb < 0) break;
                if (nb >= nslots || !alive[nb]) continue;
                float v;
                if (loop) {   // mnLoopQuery == id && mnLoopWords > minCommonWords
                    if (!(common[nb] > minC && !excluded(nb))) continue;
                    v = score[nb];
                } else {      // mnRelocQuery == id: shares a word with the frame
                    if (common[nb] <= 0) continue;
                    v = common[nb] > minC ? score[nb] : state[nb];   // mRelocScore
                }
                a += v;
                if (v > bestScore) {
                    bk = nb;
                    bestScore = v;
                }
            }
            bmax = fmaxf(bmax, a);
            ++nlisted;
        }
        acc_s[s] = a;
        best_s[s] = bk;
    }
    nlisted = block_sum<SEL_WAVES>(nlisted, itmp);
    bmax = block_maxf(bmax, ftmp);
    if (nlisted == 0) {   // lScoreAndMatch empty
        if (tid == 0) out[0] = 0;
    } else {
        const float thr = 0.75f * bmax;   // minScoreToRetain
        // retained entries, compacted in slot order, then sorted by (first, slot)
        int R = 0;
        for (int c0 = 0; c0 < nslots; c0 += SEL_THREADS) {
            const int s = c0 + tid;
            const bool keep = s < nslots && best_s[s] >= 0 && acc_s[s] > thr;
            int tot;
            const int pos = R + block_excl_scan<SEL_WAVES>(keep ? 1 : 0, itmp, tot);
            if (keep && pos < RCAP) {
                key[pos] = ((uint64_t)(uint32_t)first[s] << 32) | (uint32_t)s;
                bval[pos] = best_s[s];
            }
            R += tot;
        }
        if (R > RCAP) {
            if (tid == 0) out[0] = -1;
        } else {
            int P2 = 1;
            while (P2 < R) P2 <<= 1;
            for (int i = R + tid; i < P2; i += SEL_THREADS) {
                key[i] = ~0ull;
                bval[i] = -1;
            }
            __syncthreads();
            for (int k = 2; k <= P2; k <<= 1)
                for (int j = k >> 1; j > 0; j >>= 1) {
                    for (int i = tid; i < P2; i += SEL_THREADS) {
                        const int p = i ^ j;
                        if (p > i) {
                            const bool up = (i & k) == 0;
                            const uint64_t a = key[i], b = key[p];
                            if ((a > b) == up) {
                                key[i] = b;
                                key[p] = a;
                                const int t = bval[i];
                                bval[i] = bval[p];
                                bval[p] = t;
                            }
                        }
                    }
                    __syncthreads();
                }
            // spAlreadyAddedKF: the first occurrence of each pBestKF in list order
            for (int i = tid; i < R; i += SEL_THREADS) atomicMin(&firstpos[bval[i]], i);
            __syncthreads();
            int n = 0;
            for (int c0 = 0; c0 < R; c0 += SEL_THREADS) {
                const int i = c0 + tid;
                const bool keep = i < R && __hip_atomic_load(&firstpos[bval[i]], __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT) == i;
                int tot;
                const int pos = n + block_excl_scan<SEL_WAVES>(keep ? 1 : 0, itmp, tot);
                if (keep && pos < cap) out[1 + pos] = bval[i];
                n += tot;
            }
            __syncthreads();
            for (int i = tid; i < R; i += SEL_THREADS) firstpos[bval[i]] = INT_MAX;
            if (tid == 0) out[0] = n;
        }
    }
    // the relocalisation query leaves its scores on the keyframes (pKFi->mRelocScore = si for
    // every keyframe past the 0.8 filter, :274); every read of the old state is done
    __syncthreads();
    if (!loop)
        for (int s = tid; s < nslots; s += SEL_THREADS)
            if (common[s] > minC) state[s] = score[s];
}

size_t scan_lds(int nq) { return ((4 * (size_t)nq + 15) & ~(size_t)15) + 8 * (size_t)nq + 8 * 256; }

}  // namespace

struct orbx_kfdb {
    orbx_kfdb_params prm;
    hipStream_t stream = nullptr;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    mutable std::mutex mu;   // const queries (orbx_kfdb_size) lock it too
    // host mirror of the resident database
    std::vector<uint32_t> words;
    std::vector<double> vals;
    std::vector<int32_t> off{0};
    std::vector<uint8_t> alive;
    std::vector<int32_t> cov;
    // uploaded prefixes / dirty ranges
    size_t up_entries = 0, up_slots = 0;
    bool alive_dirty = false;
    int cov_lo = INT_MAX, cov_hi = -1;
    size_t dev_entries = 0, dev_slots = 0;   // device capacities
    DevBuf d_words, d_vals, d_off, d_alive, d_cov, d_state, d_common, d_score, d_first, d_acc,
        d_best, d_firstpos, d_q, d_out;
    std::vector<uint8_t> stage;
    double t_scan = 0, t_select = 0;
};

namespace {

// Brings the device copy up to date with the host mirror (on the database's stream).
orbx_status sync_device(orbx_kfdb* db) {
    hipStream_t st = db->stream;
    const size_t S = db->alive.size(), E = db->words.size();
    const int K = db->prm.covisibles;
    if (S > db->dev_slots || E > db->dev_entries) {
        // grow to twice the need and upload everything; the new slots' state starts at 0
        const size_t nS = std::max<size_t>(2 * S, 1024), nE = std::max<size_t>(2 * E, 65536);
        if (!HIPOK(hipStreamSynchronize(st))) return ORBX_ERR_DEVICE;
        DevBuf old_state;
        std::swap(old_state, db->d_state);
        const size_t keep = db->dev_slots;
        if (!db->d_words.ensure(4 * nE) || !db->d_vals.ensure(8 * nE) ||
            !db->d_off.ensure(4 * (nS + 1)) || !db->d_alive.ensure(nS) ||
            !db->d_cov.ensure(4 * nS * K) || !db->d_state.ensure(4 * nS) ||
            !db->d_common.ensure(4 * nS) || !db->d_score.ensure(4 * nS) ||
            !db->d_first.ensure(4 * nS) || !db->d_acc.ensure(4 * nS) || !db->d_best.ensure(4 * nS) ||
            !db->d_firstpos.ensure(4 * nS))
            return ORBX_ERR_DEVICE;
        if (!HIPOK(hipMemsetAsync(db->d_state.p, 0, 4 * nS, st)) ||
            (keep && old_state.p &&
             !HIPOK(hipMemcpyAsync(db->d_state.p, old_state.p, 4 * std::min(keep, S),
                                   hipMemcpyDeviceToDevice, st))) ||
            !HIPOK(hipMemsetAsync(db->d_firstpos.p, 0x7F, 4 * nS, st)) ||
            !HIPOK(hipStreamSynchronize(st)))
            return ORBX_ERR_DEVICE;
        old_state.release();
        db->dev_slots = nS;
        db->dev_entries = nE;
        db->up_entries = db->up_slots = 0;
        db->alive_dirty = true;
        db->cov_lo = 0;
        db->cov_hi = (int)S - 1;
    }
    if (E > db->up_entries) {
        const size_t a = db->up_entries;
        if (!HIPOK(hipMemcpyAsync(db->d_words.as<uint32_t>() + a, db->words.data() + a, 4 * (E - a),
                                  hipMemcpyHostToDevice, st)) ||
            !HIPOK(hipMemcpyAsync(db->d_vals.as<double>() + a, db->vals.data() + a, 8 * (E - a),
                                  hipMemcpyHostToDevice, st)))
            return ORBX_ERR_DEVICE;
        db->up_entries = E;
    }
    if (S > db->up_slots || db->up_slots == 0) {
        const size_t a = db->up_slots;
        if (!HIPOK(hipMemcpyAsync(db->d_off.as<int32_t>() + a, db->off.data() + a, 4 * (S + 1 - a),
                                  hipMemcpyHostToDevice, st)))
            return ORBX_ERR_DEVICE;
        db->up_slots = S;
        db->alive_dirty = true;
    }
    if (db->alive_dirty && S) {
        if (!HIPOK(hipMemcpyAsync(db->d_alive.p, db->alive.data(), S, hipMemcpyHostToDevice, st)))
            return ORBX_ERR_DEVICE;
        db->alive_dirty = false;
    }
    if (db->cov_hi >= db->cov_lo) {
        const size_t a = (size_t)db->cov_lo * K, b = (size_t)(db->cov_hi + 1) * K;
        if (!HIPOK(hipMemcpyAsync(db->d_cov.as<int32_t>() + a, db->cov.data() + a, 4 * (b - a),
                                  hipMemcpyHostToDevice, st)))
            return ORBX_ERR_DEVICE;
        db->cov_lo = INT_MAX;
        db->cov_hi = -1;
    }
    return ORBX_OK;
}

bool valid_bow(const uint32_t* w, const double* v, int n) {
    if (n < 0 || (n > 0 && (!w || !v))) return false;
    for (int i = 1; i < n; ++i)
        if (w[i] <= w[i - 1]) return false;
    return true;
}

orbx_status detect(orbx_kfdb* db, bool loop, const uint32_t* qw, const double* qv, int nq,
                   const int32_t* conn, int nc, float min_score, int32_t* cand, int cap,
                   int32_t* ncand) {
    if (!db || !ncand || cap < 0 || (cap > 0 && !cand) || !valid_bow(qw, qv, nq) || nc < 0 ||
        (nc > 0 && !conn))
        return ORBX_ERR_INVALID;
    if (nq > QMAX || nc > EXCL_MAX) return ORBX_ERR_UNSUPPORTED;
    std::lock_guard<std::mutex> lk(db->mu);
    if (!HIPOK(hipSetDevice(db->prm.device))) return ORBX_ERR_DEVICE;
    *ncand = 0;
    const int S = (int)db->alive.size();
    if (S == 0 || nq == 0) return ORBX_OK;   // lKFsSharingWords empty
    orbx_status s = sync_device(db);
    if (s != ORBX_OK) return s;
    hipStream_t st = db->stream;
    // query block: words | values | connected (sorted)
    std::vector<int32_t> ex(conn, conn + nc);
    std::sort(ex.begin(), ex.end());
    ex.erase(std::unique(ex.begin(), ex.end()), ex.end());
    const size_t o_v = ((size_t)4 * nq + 15) & ~(size_t)15, o_x = o_v + 8 * (size_t)nq;
    db->stage.resize(o_x + 4 * ex.size() + 16);
    std::memcpy(db->stage.data(), qw, 4 * (size_t)nq);
    std::memcpy(db->stage.data() + o_v, qv, 8 * (size_t)nq);
    if (!ex.empty()) std::memcpy(db->stage.data() + o_x, ex.data(), 4 * ex.size());
    const int ocap = std::min(cap, S);
    if (!db->d_q.ensure(db->stage.size()) || !db->d_out.ensure(4 * ((size_t)ocap + 2)) ||
        !HIPOK(hipMemcpyAsync(db->d_q.p, db->stage.data(), db->stage.size(), hipMemcpyHostToDevice, st)))
        return ORBX_ERR_DEVICE;
    const uint8_t* q = db->d_q.as<uint8_t>();
    (void)hipEventRecord(db->ev[0], st);
    hipLaunchKernelGGL(k_kfdb_scan, dim3((S + 3) / 4), dim3(256), scan_lds(nq), st,
                       (const uint32_t*)q, (const double*)(q + o_v), nq, S, db->d_off.as<int32_t>(),
                       db->d_alive.as<uint8_t>(), db->d_words.as<uint32_t>(), db->d_vals.as<double>(),
                       db->d_common.as<int32_t>(), db->d_score.as<float>(), db->d_first.as<int32_t>());
    (void)hipEventRecord(db->ev[1], st);
    hipLaunchKernelGGL(k_kfdb_select, dim3(1), dim3(SEL_THREADS), 0, st, loop ? 1 : 0, S,
                       db->prm.covisibles, db->d_alive.as<uint8_t>(), db->d_cov.as<int32_t>(),
                       db->d_common.as<int32_t>(), db->d_score.as<float>(), db->d_first.as<int32_t>(),
                       db->d_state.as<float>(), (const int32_t*)(q + o_x), (int)ex.size(), min_score,
                       db->d_acc.as<float>(), db->d_best.as<int32_t>(), db->d_firstpos.as<int32_t>(),
                       db->d_out.as<int32_t>(), ocap);
    (void)hipEventRecord(db->ev[2], st);
    if (!HIPOK(hipGetLastError())) return ORBX_ERR_DEVICE;
    std::vector<int32_t> res((size_t)ocap + 1);
    if (!HIPOK(hipMemcpyAsync(res.data(), db->d_out.p, 4 * res.size(), hipMemcpyDeviceToHost, st)) ||
        !HIPOK(hipStreamSynchronize(st)))
        return ORBX_ERR_DEVICE;
    float a = 0, b = 0;
    if (hipEventElapsedTime(&a, db->ev[0], db->ev[1]) == hipSuccess &&
        hipEventElapsedTime(&b, db->ev[1], db->ev[2]) == hipSuccess) {
        db->t_scan = a;
        db->t_select = b;
    }
    if (res[0] < 0) return ORBX_ERR_UNSUPPORTED;   // more than RCAP retained entries
    *ncand = res[0];
    std::memcpy(cand, res.data() + 1, 4 * (size_t)std::min(res[0], ocap));
    return res[0] > cap ? ORBX_ERR_CAPACITY : ORBX_OK;
}

}  // namespace

extern "C" {

orbx_status orbx_kfdb_create(const orbx_kfdb_params* params, orbx_kfdb** out) {
    if (!out) return ORBX_ERR_INVALID;
    *out = nullptr;
    orbx_kfdb_params p{10, 0};
    if (params) p = *params;
    if (p.covisibles < 1 || p.covisibles > KMAX || p.device < 0) return ORBX_ERR_INVALID;
    int ndev = 0;
    if (!HIPOK(hipGetDeviceCount(&ndev)) || ndev <= 0) return ORBX_ERR_DEVICE;
    if (p.device >= ndev) return ORBX_ERR_INVALID;
    orbx_kfdb* db = new orbx_kfdb();
    db->prm = p;
    bool ok = HIPOK(hipSetDevice(p.device)) &&
              HIPOK(hipStreamCreateWithFlags(&db->stream, hipStreamNonBlocking));
    for (int i = 0; i < 3 && ok; ++i) ok = HIPOK(hipEventCreate(&db->ev[i]));
    if (ok) {
        // the scan's LDS: query words + weights + 64 terms per wave.  The attribute belongs to
        // the current device (set above), so it is set once per device, not once per process
        static std::mutex amu;
        static bool have[ORBX_MAX_DEVICES] = {};
        std::lock_guard<std::mutex> lk(amu);
        if (p.device >= ORBX_MAX_DEVICES) {
            ok = false;
        } else if (!have[p.device]) {
            ok = HIPOK(hipFuncSetAttribute((const void*)k_kfdb_scan,
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)scan_lds(QMAX)));
            have[p.device] = ok;
        }
    }
    if (!ok) {
        orbx_kfdb_destroy(db);
        return ORBX_ERR_DEVICE;
    }
    *out = db;
    return ORBX_OK;
}

orbx_status orbx_kfdb_destroy(orbx_kfdb* db) {
    if (!db) return ORBX_ERR_INVALID;
    (void)hipSetDevice(db->prm.device);
    if (db->stream) (void)hipStreamSynchronize(db->stream);
    DevBuf* bufs[] = {&db->d_words, &db->d_vals, &db->d_off, &db->d_alive, &db->d_cov,
                      &db->d_state, &db->d_common, &db->d_score, &db->d_first, &db->d_acc,
                      &db->d_best, &db->d_firstpos, &db->d_q, &db->d_out};
    for (DevBuf* b : bufs) b->release();
    for (hipEvent_t e : db->ev)
        if (e) (void)hipEventDestroy(e);
    if (db->stream) (void)hipStreamDestroy(db->stream);
    delete db;
    return ORBX_OK;
}

orbx_status orbx_kfdb_add(orbx_kfdb* db, const uint32_t* words, const double* values, int32_t n,
                          int32_t* slot) {
    if (!db || !valid_bow(words, values, n)) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(db->mu);
    if (db->alive.size() >= (size_t)INT_MAX / 2) return ORBX_ERR_CAPACITY;
    db->words.insert(db->words.end(), words, words + n);
    db->vals.insert(db->vals.end(), values, values + n);
    db->off.push_back((int32_t)db->words.size());
    db->alive.push_back(1);
    db->cov.insert(db->cov.end(), (size_t)db->prm.covisibles, -1);
    if (slot) *slot = (int32_t)db->alive.size() - 1;
    return ORBX_OK;
}

orbx_status orbx_kfdb_erase(orbx_kfdb* db, int32_t slot) {
    if (!db) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(db->mu);
    if (slot < 0 || (size_t)slot >= db->alive.size()) return ORBX_ERR_INVALID;
    db->alive[(size_t)slot] = 0;
    db->alive_dirty = true;
    return ORBX_OK;
}

orbx_status orbx_kfdb_clear(orbx_kfdb* db) {
    if (!db) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(db->mu);
    db->words.clear();
    db->vals.clear();
    db->off.assign(1, 0);
    db->alive.clear();
    db->cov.clear();
    db->up_entries = db->up_slots = 0;
    db->alive_dirty = false;
    db->cov_lo = INT_MAX;
    db->cov_hi = -1;
    // the slots restart: their state must start at 0 again
    if (db->d_state.p) {
        (void)hipSetDevice(db->prm.device);
        if (!HIPOK(hipMemsetAsync(db->d_state.p, 0, db->d_state.n, db->stream)) ||
            !HIPOK(hipStreamSynchronize(db->stream)))
            return ORBX_ERR_DEVICE;
    }
    return ORBX_OK;
}

orbx_status orbx_kfdb_size(const orbx_kfdb* db, int32_t* nslots) {
    if (!db || !nslots) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(db->mu);
    *nslots = (int32_t)db->alive.size();
    return ORBX_OK;
}

orbx_status orbx_kfdb_set_covisibles(orbx_kfdb* db, int32_t slot, const int32_t* neighbours,
                                     int32_t n) {
    if (!db || n < 0 || (n > 0 && !neighbours)) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(db->mu);
    if (slot < 0 || (size_t)slot >= db->alive.size()) return ORBX_ERR_INVALID;
    const int K = db->prm.covisibles;
    // checked before the row is written: an invalid call leaves the host and device rows alike
    for (int j = 0; j < K && j < n; ++j)
        if (neighbours[j] < 0) return ORBX_ERR_INVALID;
    int32_t* row = db->cov.data() + (size_t)slot * K;
    for (int j = 0; j < K; ++j) row[j] = j < n ? neighbours[j] : -1;
    db->cov_lo = std::min(db->cov_lo, slot);
    db->cov_hi = std::max(db->cov_hi, slot);
    return ORBX_OK;
}

orbx_status orbx_kfdb_detect_relocalization(orbx_kfdb* db, const uint32_t* qwords,
                                            const double* qvalues, int32_t nq, int32_t* cand,
                                            int32_t cap, int32_t* ncand) {
    return detect(db, false, qwords, qvalues, nq, nullptr, 0, 0.0f, cand, cap, ncand);
}

orbx_status orbx_kfdb_detect_loop(orbx_kfdb* db, const uint32_t* qwords, const double* qvalues,
                                  int32_t nq, const int32_t* connected, int32_t nc,
                                  float min_score, int32_t* cand, int32_t cap, int32_t* ncand) {
    return detect(db, true, qwords, qvalues, nq, connected, nc, min_score, cand, cap, ncand);
}

orbx_status orbx_kfdb_last_timing(const orbx_kfdb* db, double* scan_ms, double* select_ms) {
    if (!db) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(db->mu);
    if (scan_ms) *scan_ms = db->t_scan;
    if (select_ms) *select_ms = db->t_select;
    return ORBX_OK;
}

}  // extern "C"
