// orbx_kernels.h — host-side launch descriptors of the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stddef.h>
#include <stdint.h>

#include "orbx_internal.h"

#include <vector>

namespace orbx {

// K_LEVEL0 times the level-0 launch alone (it is also part of K_LEVEL, all levels)
enum KernelId { K_LEVEL = 0, K_FAST, K_OCTREE, K_ORIENT, K_STEREO, K_LEVEL0, K_COUNT };

// Optional per-kernel HIP-event timing (orbx_profile_*): the extraction and stereo kernels
// get their events from their own dispatch (ORBX_TIMED_LAUNCH); durations are read back by
// collect().
struct KernelTimer {
    bool on = false;
    std::vector<hipEvent_t> pool;
    size_t used = 0;
    struct Rec { int id; hipEvent_t a, b; };
    std::vector<Rec> pending;
    double ms[K_COUNT] = {0};
    long long n[K_COUNT] = {0};
    hipEvent_t get() {
        if (used == pool.size()) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
            pool.push_back(e);
        }
        return pool[used++];
    }
    hipEvent_t start(hipStream_t st) {
        if (!on) return nullptr;
        hipEvent_t e = get();
        if (e) (void)hipEventRecord(e, st);
        return e;
    }
    void stop(int id, hipEvent_t a, hipStream_t st) {
        if (!on || !a) return;
        hipEvent_t b = get();
        if (!b) return;
        (void)hipEventRecord(b, st);
        pending.push_back(Rec{id, a, b});
        last = b;
    }
    // Start of a kernel launched right after the previous timed one on the same stream: the
    // previous stop event doubles as this start (one marker between two kernels, not two).
    hipEvent_t start_after(hipStream_t st) {
        if (!on) return nullptr;
        return last ? last : start(st);
    }
    hipEvent_t last = nullptr;
    // the last recorded interval counted a second time under `id` (a sub-total)
    void alias(int id) {
        if (!on || pending.empty()) return;
        Rec r = pending.back();
        r.id = id;
        pending.push_back(r);
    }
    void collect() {
        for (auto& r : pending) {
            float t = 0.f;
            if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&t, r.a, r.b) == hipSuccess) {
                ms[r.id] += t;
                n[r.id] += 1;
            }
        }
        pending.clear();
        used = 0;
        last = nullptr;
    }
    void destroy() {
        for (auto e : pool) (void)hipEventDestroy(e);
        pool.clear();
        used = 0;
    }
};

// A kernel launch timed by its own dispatch (hipExtLaunchKernel sets the two events from the
// kernel's start and end, as rocprofv3's kernel trace sees them): with a side branch or another
// batch in flight a kernel may wait for the device after its stream reaches it, and a stream-
// ordered event pair would charge it that wait.  The interval is recorded under ID; untimed
// launches (timing off) are plain launches.
#define ORBX_TIMED_LAUNCH(T, ID, KERNEL, GRID, BLOCK, SHM, ST, ...)                            \
    do {                                                                                      \
        hipEvent_t a_ = (T).on ? (T).get() : nullptr;                                         \
        hipEvent_t z_ = (T).on ? (T).get() : nullptr;                                         \
        if (a_ && z_) {                                                                       \
            hipExtLaunchKernelGGL(KERNEL, GRID, BLOCK, (uint32_t)(SHM), ST, a_, z_, 0u,       \
                                  __VA_ARGS__);                                               \
            (T).pending.push_back(KernelTimer::Rec{ID, a_, z_});                              \
        } else {                                                                              \
            hipLaunchKernelGGL(KERNEL, GRID, BLOCK, SHM, ST, __VA_ARGS__);                    \
        }                                                                                     \
    } while (0)

struct ExtractLaunch {
    const Geometry* hg;        // host copy of the geometry
    const Geometry* dg;        // device copy
    const CellDesc* cells;     // device
    const int16_t* rtab;       // device
    const uint8_t* ltab;       // device: k_level per-tile tables
    const uint8_t* d_imgs;      // images [0, split)
    const uint8_t* d_imgs2;     // images [split, batch) (stereo: right views)
    int split;
    size_t stride, batch_stride;
    int batch;
    size_t level_lds;
    uint8_t* pyr;
    uint8_t* blur;
    int* ccnt;
    uint32_t* cand;
    int* ocnt;
    uint32_t* okp;
    uint16_t* operm;   // [B][out_words] k_orient_desc's processing order (list indices)
    uint8_t* kscratch;
    long long kscratch_per_image;
    int ncap, kcap;          // level 0 (the largest node list)
    size_t octree_lds;
    int ncap1, kcap1;        // levels 1.. (a second launch with a smaller LDS footprint)
    size_t octree_lds1;
    // small batches (a few octree workgroups on the chip): the large LDS budget
    int oct_small = 0, kcap_small = 0;
    size_t octree_lds_small = 0;
    int fast_nc = 4;         // k_fast cells per wave
    float* kps;
    uint8_t* desc;
    int* nkp;
    KernelTimer* timer;
    // k_level_strip output rows per strip of each level for this call's batch (a kernel
    // argument: a batch-size change needs no device-side table update)
    int sth[ORBX_MAX_LEVELS];
    // 1: level 0 of every image is already in the pyramid (d_imgs unused)
    int in_place;
    // the handle's side stream and fork / join events (level-0 branch, launch_extract)
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // the host copy of image 0's pyramid block (mvImagePyramid, orbx_extractor_host_pyramid):
    // pyr_host_bytes from the pyramid into pinned pyr_host, on the side stream beside the
    // FAST / octree / orientation launches (after them when the side branch is in use)
    uint8_t* pyr_host = nullptr;
    size_t pyr_host_bytes = 0;
    // side branch: 0 off, 1 FAST, 2 + octree, 3 + orientation / descriptors of levels
    // [0, side_lv), forked before level side_at's launch
    int side_mode = 0, side_at = 0, side_lv = 1;
    // 1: the whole pyramid as one k_pyr_chain launch (small in-place batches, no side branch)
    int chain = 0;
};


struct StereoLaunch {
    const Geometry* dg;
    int batch;
    const float* kpsL;
    const uint8_t* descL;
    const int* nkpL;
    const uint8_t* pyrL;
    const float* kpsR;
    const uint8_t* descR;
    const int* nkpR;
    const uint8_t* pyrR;
    float mbf, mb;
    float* uR;
    float* depth;
    int* nvalid;
    size_t lds;
    KernelTimer* timer;
    // split path (stereo_split(batch) > 1): per pair an accepted-SAD count (zero on entry,
    // left zero) and kp_cap (SAD, left index) slots
    int* scnt;
    int* ssad;
    int16_t* sidx;
};

hipError_t launch_extract(const ExtractLaunch& a, hipStream_t st);
hipError_t launch_levels(const ExtractLaunch& a, hipStream_t st, int l_begin, int l_end);
hipError_t launch_pyr_chain(const ExtractLaunch& a, hipStream_t st);
size_t level_lds_bytes(int ltw, int lth, int win_cap);
size_t fast_lds_bytes(const Geometry& g);
size_t octree_lds_bytes(int ncap, int kcap, bool packed);
hipError_t launch_stereo(const StereoLaunch& a, hipStream_t st);
int stereo_split(int batch);   // workgroups per pair of a launch_stereo over `batch` pairs
size_t stereo_lds_bytes(int kp_cap, int height, int ob);  // ob: octave bucket groups

}  // namespace orbx
