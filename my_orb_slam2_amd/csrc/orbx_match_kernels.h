// orbx_match_kernels.h — launch descriptors of the matcher kernels (orbx_match.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/orbx_match.h"

namespace orbx {

// Internal projection mode after the public ones: SearchForInitialization (:446-561).
constexpr int PROJ_INIT = ORBX_PROJ_MODE_COUNT;
constexpr int PROJ_K = 8;             // candidate list length of the claim-mode replay
constexpr int MATCH_MAX_LEVELS = 16;

// SearchByBoW over jobs: job j pairs keyframe (a_fixed ? 0 : j) of A with keyframe
// (b_fixed ? 0 : j) of B.  kf_kf = 0: SearchByBoW(KeyFrame*, Frame&) (A = keyframe, B = frame,
// outputs indexed by B feature); kf_kf = 1: SearchByBoW(KeyFrame*, KeyFrame*) (outputs indexed
// by A feature).
struct BowLaunch {
    orbx_kf_db A, B;
    int a_fixed, b_fixed, kf_kf, njobs;
    float ratio;
    int check_ori;
    int32_t* out;
    int out_stride;
    int32_t* nmatches;
    int* err;
};

hipError_t launch_node_order(const orbx_kf_db& db, int n, orbx_keypoint* keys, uint8_t* desc,
                             float* ur, uint8_t* flag, hipStream_t st);

struct TriLaunch {
    orbx_kf_db db;
    int njobs;
    const int32_t* kf1;
    const int32_t* kf2;
    const float* F12;
    const float* epi;
    float sigma2[MATCH_MAX_LEVELS];
    float scale[MATCH_MAX_LEVELS];
    int only_stereo, check_ori;
    const int32_t* job_off;
    int32_t* out;
    int32_t* nmatches;
    int* err;
};

// Projection searches (modes of orbx_proj_mode plus PROJ_INIT) over njobs independent jobs
// (frames).  With t_off == nullptr there is one job: target T, queries [0, nq).  Otherwise
// job j's target is T's arrays offset by t_off[j] features (keys/desc/u_right/claimed) and
// g_off[j] grid entries (grid_feat, job-local indices), with its own grid_off block of
// cols*rows+1 entries; its queries are [q_off[j], q_off[j+1]).
struct ProjLaunch {
    int mode;
    orbx_featureset T;           // device pointers
    int njobs;
    const int32_t* t_off;
    const int32_t* g_off;
    const int32_t* q_off;
    int max_t;                   // largest target (LDS sizing of the resolve phase)
    const uint8_t* qdesc;
    const orbx_proj_query* q;
    int nq;
    float inv_sigma2[MATCH_MAX_LEVELS];
    int orb_dist;
    float ratio;
    int check_ori;
    const uint8_t* claimed_in;   // may be null
    const uint8_t* qflags;       // nq ORBX_QF_* per query, may be null
    int prefilter;               // ORBX_PROJ_PREFILTER: no rotation-consistency filter
    int32_t* out;                // nq
    int4* top2;                  // nq (PROJ_INIT: static best and second)
    int2* cand;                  // nq x PROJ_K (claim modes: sorted candidate lists)
    int32_t* ncand;              // nq (list length; PROJ_K + 1 = truncated)
    int8_t* out_bin;             // nq
    int32_t* hist;               // 32 per job
    int32_t* nmatches;           // per job
    int* err;
};

bool proj_mode_greedy(int mode);
hipError_t launch_bow(const BowLaunch& a, hipStream_t st);
size_t bow_lds_bytes(const BowLaunch& a);
hipError_t launch_triangulate(const TriLaunch& a, hipStream_t st);
size_t tri_lds_bytes(int max_feat);
// Phase A (window search, static top-2), B (sequential greedy claims), C (rotation filter
// and count).  launch_proj runs the phases the mode needs; `timer` ids ORBX_MK_*.
struct KernelTimer;
hipError_t launch_proj(const ProjLaunch& a, hipStream_t st, KernelTimer* timer);
size_t proj_resolve_lds_bytes(int mode, int n_target, int nq);
hipError_t prepare_match_kernels();
// Brute-force Hamming top-2 (orbx_bf.hip): q nq x 32, db ndb x 32 (device); part = scratch of
// bf_partial_bytes(ndb, nq, chunk) bytes.
struct BfLaunch {
    const uint8_t* q;
    int nq;
    const uint8_t* db;
    long long ndb;
    long long idx_base;
    int chunk;
    void* part;
    int32_t* best_idx;
    int32_t* best_dist;
    int32_t* second_dist;
    int kernel;            // ORBX_BF_MFMA / ORBX_BF_VALU
};
int bf_chunk_rows(long long ndb, int nq, int ncu, int kernel);
size_t bf_partial_bytes(long long ndb, int nq, int chunk);
struct KernelTimer;
hipError_t launch_bf_top2(const BfLaunch& a, hipStream_t st, KernelTimer* timer);
const char* bf_kernel_name(int kernel);
hipError_t launch_distinctive(const uint8_t* desc, const int32_t* off, int np, int32_t* best,
                              int* err, hipStream_t st);
size_t distinctive_lds_bytes();
// 160 KB of LDS per workgroup on gfx950, minus room for the kernels' static arrays
constexpr size_t MATCH_MAX_LDS = 160 * 1024 - 256;
// k_triangulate also holds 12 KiB of static LDS (one staged KF2 node slice per wave)
constexpr size_t TRI_MAX_LDS = MATCH_MAX_LDS - 16 * 1024;

}  // namespace orbx
