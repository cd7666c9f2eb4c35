// orbx_capi.hip — the extern "C" boundary (include/orbx.h) over the gfx950 kernels.
//
// Host responsibilities: the ORBextractor constructor tables (src/ORBextractor.cc:410-470),
// the per-image-size geometry (pyramid sizes :1134, FAST cell grid :793-818, octree roots
// :543-545, OpenCV resize coefficient tables), the HBM workspace, and the launch sequence.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <thread>
#include <vector>

#include "../../include/orbx.h"
#include "orbx_internal.h"
#include "orbx_kernels.h"

#ifndef ORBX_SRC_HASH
#define ORBX_SRC_HASH "0000000000000000"   // my_orb_slam2_amd/build.py passes the real one
#endif
// "orbx-src:<hash>" is also how build.py finds the hash in the binary (staleness check)
#define ORBX_VERSION "orbx 0.3.0 (gfx950) orbx-src:" ORBX_SRC_HASH

namespace orbx {
hipError_t prepare_kernels(size_t octree_lds, size_t stereo_lds, size_t level_lds,
                           size_t fast_lds);
}

using namespace orbx;

#include "orbx_host.h"

namespace orbx {
thread_local char g_err[256] = "";
bool hip_ok(hipError_t e, const char* what) {
    if (e == hipSuccess) return true;
    snprintf(g_err, sizeof(g_err), "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
    return false;
}
}  // namespace orbx

// A helper thread that stages the right image of a stereo frame while the calling thread
// stages the left one (orbx_stereo_frame_view): the copy of a cold 0.47 MB image into pinned
// memory is tens of microseconds on one core.
struct OrbxStager {
    std::mutex mu;
    std::condition_variable cv;
    std::function<void()> job;
    bool has_job = false, done = true, stop = false;
    std::thread th;
    OrbxStager() : th([this] { run(); }) {}
    ~OrbxStager() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        th.join();
    }
    void run() {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv.wait(lk, [&] { return has_job || stop; });
            if (stop) return;
            std::function<void()> j = std::move(job);
            has_job = false;
            lk.unlock();
            j();
            lk.lock();
            done = true;
            cv.notify_all();
        }
    }
    void post(std::function<void()> j) {
        std::lock_guard<std::mutex> lk(mu);
        job = std::move(j);
        has_job = true;
        done = false;
        cv.notify_all();
    }
    void wait() {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return done; });
    }
};

struct orbx_extractor {
    orbx_extractor_params prm;
    int device = 0;
    int ncu = 256;                // compute units of the device (strip-height heuristic)
    hipStream_t stream = nullptr;
    // `done` is recorded after the last work issued for this handle (on `done_stream`): a
    // later call on another stream waits for it, and table updates / buffer growth / host
    // fetches wait on it instead of on the whole device
    hipEvent_t done = nullptr;
    hipStream_t done_stream = nullptr;
    bool have_done = false;
    // side branch of launch_extract (level-0 FAST beside the level launches): a stream of its
    // own, forked from and joined back into the call's stream by two events
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    int side_mode = FAST_SIDE, side_at = FAST_SIDE_AT, side_lv = FAST_SIDE_LV;
    bool side_auto = true;   // the built-in default: no side branch below SIDE_MIN_BATCH images
    // orbx_extract's device sequence (H2D, kernels, D2H) as one HIP graph, rebuilt when its
    // key (image size, effective schedule, every buffer address it names) changes
    hipGraphExec_t g1 = nullptr;
    std::vector<const void*> g1key;
    // orbx_stereo_frame_view's sequence (2-D H2D, two-image extraction, stereo, D2H) likewise
    hipGraphExec_t g2 = nullptr;
    std::vector<const void*> g2key;
    // pinned staging of the host-image path (orbx_extract / orbx_stereo_match)
    uint8_t* h_in = nullptr;
    size_t h_in_n = 0;
    uint8_t* h_out = nullptr;
    size_t h_out_n = 0;
    // mvImagePyramid on the host (orbx_extractor_host_pyramid): every orbx_extract(_view) also
    // copies its image's pyramid block here (a pinned block of its own: no other call writes it)
    bool host_pyr = false;
    bool host_pyr_ok = false;   // h_pyr holds the last orbx_extract(_view)'s pyramid
    uint8_t* h_pyr = nullptr;
    size_t h_pyr_n = 0;
    // ORBextractor tables
    std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
    std::vector<int> nfeat;
    int umax[16];
    int taps[7];
    // geometry of the current image size
    bool have_geom = false;
    Geometry hg;
    std::vector<CellDesc> cells;
    std::vector<int16_t> rtab;
    std::vector<uint8_t> ltab;   // k_level per-tile tables (LevelColTab / LevelRowTab)
    int ncap = 0, kcap = 0, ncap1 = 0, kcap1 = 0;
    size_t octree_lds = 0, octree_lds1 = 0, stereo_lds = 0, level_lds = 0;
    int kcap_small = 0;               // small-batch octree: candidates held in LDS
    size_t octree_lds_small = 0;
    int cap_batch = 0;
    DevBuf d_geom, d_cells, d_rtab, d_ltab, d_pyr, d_blur, d_ccnt, d_cand, d_ocnt, d_okp, d_kscr,
        d_kps, d_desc, d_nkp, d_uR, d_dep, d_nv, d_sscr;
    // the extraction outputs as one allocation: [nkp[B] | kps[B][KC] | desc[B][KC][32]]
    // (d_nkp / d_kps / d_desc are views of it): one DMA returns one image's results
    DevBuf d_outs;
    size_t o_stereo = 0;   // offset of the stereo block in d_outs
    long long kscratch_per_image = 0;
    KernelTimer timer;
    // last extraction
    int last_batch = 0;
    bool last_valid = false;
    int last_n = 0;          // keypoints of the last orbx_extract (host image path)
    // images [0, pyr_images) of d_pyr hold the raw pyramids of the last call (mvImagePyramid,
    // orbx_pyramid_level).  A stereo frame (orbx_stereo_frame_view) leaves them only when
    // keep_pyr is set, solo or served alike (orbx_extractor_keep_pyramid)
    int pyr_images = 0;
    uint64_t serial = 0;     // +1 whenever the pyramids change (orbx_extractor_serial)
    bool keep_pyr = false;
    bool fs_user = false;    // counted as a user of its frame server (released with the last)
    std::unique_ptr<OrbxStager> stager;   // created by the first stereo-frame call
    // guards every field above against concurrent calls on one handle (const queries too)
    mutable std::mutex mu;
};

namespace {


inline int cvRound(float v) { return (int)lrintf(v); }
inline int cvRound(double v) { return (int)lrint(v); }
inline int cvFloor(float v) { int i = cvRound(v); float d = (float)(v - i); return i - (d < 0); }
inline int cvCeil(float v) { int i = cvRound(v); float d = (float)(i - v); return i + (d < 0); }
inline short sat_short(float v) {
    int i = cvRound(v);
    return (short)std::min(std::max(i, (int)SHRT_MIN), (int)SHRT_MAX);
}
size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

void compute_tables(orbx_extractor* h) {
    const int L = h->prm.nlevels;
    const double scaleFactor = (double)h->prm.scale_factor;   // ORBextractor::scaleFactor is double
    h->scale.assign(L, 0.f);
    h->sigma2.assign(L, 0.f);
    h->inv_scale.assign(L, 0.f);
    h->inv_sigma2.assign(L, 0.f);
    h->nfeat.assign(L, 0);
    h->scale[0] = 1.0f;
    h->sigma2[0] = 1.0f;
    for (int i = 1; i < L; i++) {
        h->scale[i] = (float)(h->scale[i - 1] * scaleFactor);
        h->sigma2[i] = h->scale[i] * h->scale[i];
    }
    for (int i = 0; i < L; i++) {
        h->inv_scale[i] = 1.0f / h->scale[i];
        h->inv_sigma2[i] = 1.0f / h->sigma2[i];
    }
    const int nfeatures = h->prm.nfeatures;
    float factor = (float)(1.0f / scaleFactor);
    float nDesired = nfeatures * (1 - factor) / (1 - (float)pow((double)factor, (double)L));
    int sum = 0;
    for (int level = 0; level < L - 1; level++) {
        h->nfeat[level] = cvRound(nDesired);
        sum += h->nfeat[level];
        nDesired *= factor;
    }
    h->nfeat[L - 1] = std::max(nfeatures - sum, 0);
    // umax (src/ORBextractor.cc:454-469)
    const int HP = 15;
    int v, v0, vmax = cvFloor((float)(HP * std::sqrt(2.f) / 2 + 1));
    int vmin = cvCeil((float)(HP * std::sqrt(2.f) / 2));
    const double hp2 = HP * HP;
    for (v = 0; v <= vmax; ++v) h->umax[v] = cvRound(std::sqrt(hp2 - v * v));
    for (v = HP, v0 = 0; v >= vmin; --v) {
        while (h->umax[v0] == h->umax[v0 + 1]) ++v0;
        h->umax[v] = v0;
        ++v0;
    }
    // getGaussianKernel(7, 2, CV_32F) -> x256 fixed point (FilterEngine 8U path)
    float cf[7];
    double s2 = -0.5 / (2.0 * 2.0), ksum = 0;
    for (int i = 0; i < 7; ++i) {
        double x = i - 3.0;
        cf[i] = (float)std::exp(s2 * x * x);
        ksum += cf[i];
    }
    ksum = 1. / ksum;
    for (int i = 0; i < 7; ++i) cf[i] = (float)(cf[i] * ksum);
    for (int i = 0; i < 7; ++i) h->taps[i] = cvRound(cf[i] * 256.f);
}

int reflect101_h(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p;
        else p = 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

void reflected_range_h(int lo, int hi, int len, int& mn, int& mx) {
    mn = 1 << 30;
    mx = -1;
    for (int p = lo; p <= hi; ++p) {
        const int r = reflect101_h(p, len);
        mn = std::min(mn, r);
        mx = std::max(mx, r);
    }
}

int vresize_simd_end(int width) {
    int x = 0;
    for (; x <= width - 16; x += 16) {}
    for (; x < width - 4; x += 4) {}
    return x;
}

// Strip height of a level for a batch of nimg images: STRIP_TH rows while the level's strip
// walks give every SIMD of the device (ncu CUs x 4) two waves, else the tallest of 32 / 16 / 8
// rows that does (8 at most).  A strip walk is a serial chain of rows, so a small batch (one
// stereo frame at a time: the tracking thread's case) is latency-bound on the few long walks
// of each level: 8-row strips take one stereo pair's pyramid from 0.218 to 0.082 ms (the
// halo rows cost more work, which only large batches would notice).
static int strip_default(const LevelGeom& lv, int nimg, int ncu) {
    const long long target = 2LL * ncu * 4;
    int th = STRIP_TH;
    while (th > 8 && (long long)lv.snw * ((lv.h + th - 1) / th) * nimg < target) th /= 2;
    return th;
}

// Every strip level's height for a batch of nimg images (a launch argument of k_level_strip,
// so a batch-size change touches no device state).
static void strip_heights(const orbx_extractor* h, int nimg, int* sth) {
    for (int l = 0; l < ORBX_MAX_LEVELS; ++l) sth[l] = STRIP_TH;
    for (int l = 0; l < h->hg.nlevels; ++l) {
        const LevelGeom& lv = h->hg.lv[l];
        if (lv.strip) sth[l] = strip_default(lv, nimg, h->ncu);
    }
}

static int stereo_split_of(int pairs) { return orbx::stereo_split(pairs); }

// Small-batch launch policies.
#define OCT_LDS_SMALL_KB 152   // octree LDS budget for small batches (one workgroup per list)
#define OCT_SMALL_BATCH 16
// images per call up to which the octree takes that budget (one workgroup per CU is still
// every list at once up to 32 images; a frame-server batch of 2-16 images: 46.4 -> 42.0 us
// with 16 instead of 4, r4aa)
#define CHAIN_MAX_BATCH 8      // images per call up to which the pyramid is one k_pyr_chain launch
                               // (r5c16: 16 images lost at K = 8 sessions, 9.5-9.9 k vs 10.2-10.7 k pairs/s)
#define SIDE_MIN_BATCH 16      // images per call from which the default side branch forks

// k_fast cells per wave: FAST_NC (the next cell's ROI loads overlap the current cell) while the
// launch gives every CU two workgroups, fewer for small batches (a wave's cells run in series,
// so one image's FAST is a chain of FAST_NC cells otherwise).
static int fast_cells_per_wave(int ncells, int batch, int ncu) {
    int nc = FAST_NC;
    while (nc > 1 && (long long)ncells * batch / (4 * nc) < 2LL * ncu) nc >>= 1;
    return nc;
}

// Stream captures (extract1_graph) against waits on an event recorded on another stream: the
// runtime refuses hipStreamWaitEvent (hipErrorStreamCaptureIsolation) while the stream the event
// was last recorded on is being captured, even when the record came before the capture began.
// A handle's done event can sit on another handle's stream (orbx_stereo_match records the right
// handle's on the left's), whose thread may be capturing a graph just then (a handle re-captures
// when its pinned blocks grow), so such waits and the captures exclude each other.  Captures
// happen on a handle's first calls and after a regrowth; the waits take the lock shared.
static std::shared_mutex g_capture_mu;

// Orders stream st after all work issued so far for this handle (on whatever stream).
static bool order_after_last(orbx_extractor* h, hipStream_t st) {
    if (h->have_done && h->done_stream != st) {
        std::shared_lock<std::shared_mutex> lk(g_capture_mu);
        return HIPOK(hipStreamWaitEvent(st, h->done, 0));
    }
    return true;
}

// Marks the end of the work just issued for this handle on st.
static bool mark_done(orbx_extractor* h, hipStream_t st) {
    h->done_stream = st;
    h->have_done = true;
    return HIPOK(hipEventRecord(h->done, st));
}

// Waits (host) until the handle's issued work has finished: its tables may then change and
// its buffers grow.  Other streams and handles on the device keep running.
static bool wait_idle(orbx_extractor* h) {
    return !h->have_done || HIPOK(hipEventSynchronize(h->done));
}

// The host wait of the single-image calls (orbx_extract, orbx_stereo_match): polls the handle's
// last event for up to WAIT_SPIN_US (yielding the core between polls) before a blocking wait.
// A blocking wait returns tens of microseconds after the work ends (the thread sleeps); the
// drop-in path waits twice per stereo frame on its critical path.
#define WAIT_SPIN_US 400
static bool wait_done(orbx_extractor* h) {
    const int spin_us = WAIT_SPIN_US;
    if (spin_us > 0) {
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            const hipError_t e = hipEventQuery(h->done);
            if (e == hipSuccess) return true;
            if (e != hipErrorNotReady) return HIPOK(e);
            if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us)) break;
            std::this_thread::yield();
        }
    }
    return HIPOK(hipEventSynchronize(h->done));
}

// Host staging buffer (pinned) of at least n bytes.
static bool ensure_pinned(uint8_t*& p, size_t& cap, size_t n) {
    if (p && cap >= n) return true;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    if (!HIPOK(hipHostMalloc((void**)&p, n, hipHostMallocDefault))) { p = nullptr; return false; }
    cap = n;
    return true;
}

// k_level_strip tables of level l (StripLane per half-strip lane, rows -3 .. h+2); the level
// keeps the tiled kernel (strip = 0) for modes 1 / 2 or when a group's taps do not fit the
// 8-byte window the strip kernel reads
void build_strip_tables(orbx_extractor* h, int l, int mode, const int16_t* xofs,
                        const int16_t* alpha, const int16_t* yofs, const int16_t* beta) {
    Geometry& G = h->hg;
    LevelGeom& lv = G.lv[l];
    lv.strip = 0;
    if (mode != 0 && mode != 3) return;
    const LevelGeom& S = G.lv[l > 0 ? l - 1 : 0];
    lv.snh = (lv.w + SW_PX - 1) / SW_PX;
    lv.snw = (lv.snh + 1) / 2;
    std::vector<StripLane> sl((size_t)lv.snh * 32);
    for (int hs = 0; hs < lv.snh; ++hs)
        for (int q = 0; q < 32; ++q) {
            StripLane& e = sl[(size_t)hs * 32 + q];
            memset(&e, 0, sizeof(e));
            int xr[4];
            const int xg = hs * SW_PX - 4 + 4 * q;
            for (int j = 0; j < 4; ++j)   // groups past every output's halo: any in-row column
                xr[j] = xg > lv.w + 3 ? lv.w - 1 : reflect101_h(xg + j, lv.w);
            if (mode == 0) {
                const int mn = std::min(std::min(xr[0], xr[1]), std::min(xr[2], xr[3]));
                e.base = (uint32_t)mn;
                for (int j = 0; j < 4; ++j) {
                    if (xr[j] - mn > 4) return;   // + the row address's low 2 bits <= 7
                    e.sel |= (uint32_t)(xr[j] - mn) << (8 * j);
                }
            } else {
                int sx[4];
                for (int j = 0; j < 4; ++j) sx[j] = xofs[xr[j]];
                const int mn = std::min(std::min(sx[0], sx[1]), std::min(sx[2], sx[3]));
                e.base = (uint32_t)mn;
                for (int j = 0; j < 4; ++j) {
                    const int k = sx[j] - mn;
                    // taps k, k+1 of the 8 bytes from the first tap column (o0 + 11 < 16 read)
                    if (k > 6) return;
                    e.psel[j] = (uint32_t)k | (0x0Cu << 8) | ((uint32_t)(k + 1) << 16) | (0x0Cu << 24);
                    uint32_t a0 = (uint16_t)alpha[2 * xr[j]], a1 = (uint16_t)alpha[2 * xr[j] + 1];
                    if (xr[j] >= lv.xmax) { a0 = 2048; a1 = 0; }   // HResizeLinear: S[sx] * 2048
                    e.alp[j] = (a0 << 4) | ((a1 << 4) << 16);
                    e.flags |= (uint32_t)((xr[j] < lv.xmax ? 1 : 0) | (xr[j] < lv.rsimd_end ? 2 : 0))
                               << (2 * j);
                }
            }
        }
    std::vector<uint32_t> rt((size_t)4 * (lv.h + 6));
    for (int k = 0; k < lv.h + 6; ++k) {
        const int yr = reflect101_h(k - 3, lv.h);
        if (mode == 0) {
            rt[4 * k] = (uint32_t)yr;
        } else {
            const int sy = yofs[yr];
            const uint32_t r0 = (uint32_t)std::min(std::max(sy, 0), S.h - 1);
            const uint32_t r1 = (uint32_t)std::min(std::max(sy + 1, 0), S.h - 1);
            rt[4 * k] = r0 * (uint32_t)S.pitch;       // byte offsets of the two source rows
            rt[4 * k + 1] = r1 * (uint32_t)S.pitch;
            rt[4 * k + 2] = (uint32_t)(uint16_t)beta[2 * yr] | ((uint32_t)(uint16_t)beta[2 * yr + 1] << 16);
        }
    }
    h->ltab.resize(align_up(h->ltab.size(), 16));
    lv.stab = (int)h->ltab.size();
    h->ltab.insert(h->ltab.end(), (const uint8_t*)sl.data(), (const uint8_t*)(sl.data() + sl.size()));
    h->ltab.resize(align_up(h->ltab.size(), 16));
    lv.srow = (int)h->ltab.size();
    h->ltab.insert(h->ltab.end(), (const uint8_t*)rt.data(), (const uint8_t*)(rt.data() + rt.size()));
    h->ltab.resize(align_up(h->ltab.size(), 16));
    lv.strip = 1;
}

// Per-size geometry.  Returns ORBX_OK or ORBX_ERR_UNSUPPORTED.
// k_pyr_chain tiles (orbx_pyramid.hip): per tile of a gx x gy grid and per level, the owned
// rectangle and the footprint, built from the deepest level up: a level's footprint is its
// owned rectangle + the blur halo, joined with the source rows / columns the next level's
// footprint reads through the resize tables (xofs / yofs of level l + 1, as cv::resize's
// HResizeLinear / VResizeLinear index them).  chain_ok stays 0 (per-level launches) unless
// every level l >= 1 is INTER_LINEAR and the two level buffers + row sums fit the LDS.
static void build_chain(orbx_extractor* h) {
    Geometry& G = h->hg;
    const int L = G.nlevels;
    G.chain_ok = 0;
    G.chain_gx = G.chain_gy = 1;
    G.chain_tab = G.chain_toffs = 0;
    G.chain_buf = G.chain_rs = G.chain_lds = 0;
    for (int l = 1; l < L; ++l) {
        if (G.lv[l].copy || G.lv[l].area2) return;
        // a 4-pixel group's taps must fit the 8 bytes one v_perm pair reads (source span <= 6,
        // i.e. scale factors up to about 2.3; groups start at multiples of 4)
        const int16_t* xofs = h->rtab.data() + G.lv[l].rtab_off;
        for (int x = 0; x < G.lv[l].w; x += 4)
            if (xofs[std::min(x + 3, G.lv[l].w - 1)] - xofs[x] > 5) return;
    }
    const int gx = std::max(1, (G.lv[0].w + CHAIN_TW - 1) / CHAIN_TW);
    const int gy = std::max(1, (G.lv[0].h + CHAIN_TH - 1) / CHAIN_TH);
    std::vector<ChainRect> rects((size_t)gx * gy * L);
    // k_pyr_chain table offsets per tile: [L + 1] entry prefix, then [L + 1] word prefix
    std::vector<int32_t> toffs((size_t)gx * gy * 2 * (L + 1), 0);
    size_t buf = 16, rs = 16, ct = 16;
    for (int ty = 0; ty < gy; ++ty)
        for (int tx = 0; tx < gx; ++tx) {
            size_t tab = 0;   // table entries of the tile's levels 1.. (k_pyr_chain phase 1)
            bool have_next = false;
            int nx0 = 0, nx1 = -1, ny0 = 0, ny1 = -1;   // footprint of level l + 1
            for (int l = L - 1; l >= 0; --l) {
                const LevelGeom& lv = G.lv[l];
                const int W = lv.w, Hh = lv.h;
                const int ox0 = tx == 0 ? 0 : ((int)((long long)tx * W / gx) & ~3);
                const int ox1 = std::max(ox0, tx == gx - 1 ? W : ((int)((long long)(tx + 1) * W / gx) & ~3));
                const int oy0 = (int)((long long)ty * Hh / gy);
                const int oy1 = std::max(oy0, ty == gy - 1 ? Hh : (int)((long long)(ty + 1) * Hh / gy));
                int fx0 = INT_MAX, fx1 = -1, fy0 = INT_MAX, fy1 = -1;
                if (ox1 > ox0 && oy1 > oy0) {
                    fx0 = std::max(ox0 - 3, 0);
                    fx1 = std::min(ox1 + 2, W - 1);
                    fy0 = std::max(oy0 - 3, 0);
                    fy1 = std::min(oy1 + 2, Hh - 1);
                }
                if (have_next) {
                    const LevelGeom& D = G.lv[l + 1];
                    const int16_t* xofs = h->rtab.data() + D.rtab_off;
                    const int16_t* yofs = xofs + 3 * D.w;
                    fx0 = std::min(fx0, std::min(std::max((int)xofs[nx0], 0), W - 1));
                    fx1 = std::max(fx1, std::min((int)xofs[nx1] + 1, W - 1));
                    fy0 = std::min(fy0, std::min(std::max((int)yofs[ny0], 0), Hh - 1));
                    fy1 = std::max(fy1, std::min(std::max((int)yofs[ny1] + 1, 0), Hh - 1));
                }
                ChainRect& c = rects[((size_t)ty * gx + tx) * L + l];
                c.ox0 = (int16_t)ox0;
                c.ox1 = (int16_t)ox1;
                c.oy0 = (int16_t)oy0;
                c.oy1 = (int16_t)oy1;
                if (fx1 < 0) {
                    c.fx0 = c.fy0 = 0;
                    c.fx1 = c.fy1 = -1;
                    have_next = false;
                    continue;
                }
                fx0 &= ~3;
                c.fx0 = (int16_t)fx0;
                c.fx1 = (int16_t)fx1;
                c.fy0 = (int16_t)fy0;
                c.fy1 = (int16_t)fy1;
                have_next = true;
                nx0 = fx0;
                nx1 = fx1;
                ny0 = fy0;
                ny1 = fy1;
                const int fw = fx1 - fx0 + 1;
                buf = std::max(buf, (size_t)chain_pitch(fw) * (fy1 - fy0 + 1) + 16);
                rs = std::max(rs, (size_t)4 * ((ox1 - ox0 + 3) & ~3) * (oy1 - oy0 + 6));
                if (l > 0) tab += chain_level_words((fw + 3) >> 2, fy1 - fy0 + 1);
            }
            ct = std::max(ct, 4 * tab);
            int32_t* te = &toffs[((size_t)ty * gx + tx) * 2 * (L + 1)];
            int32_t* tw = te + (L + 1);
            for (int l = 1; l < L; ++l) {
                const ChainRect& c = rects[((size_t)ty * gx + tx) * L + l];
                const int fw = c.fx1 - c.fx0 + 1, fh = c.fy1 - c.fy0 + 1;
                te[l + 1] = te[l] + (fw > 0 ? ((fw + 3) >> 2) + ((fh + 1) & ~1) : 0);
                tw[l + 1] = tw[l] + (fw > 0 ? chain_level_words((fw + 3) >> 2, fh) : 0);
            }
        }
    auto r16 = [](size_t v) { return (v + 15) & ~(size_t)15; };
    const size_t lds = 2 * r16(buf) + r16(rs) + r16(ct);
    if (lds > 150 * 1024) return;
    G.chain_gx = gx;
    G.chain_gy = gy;
    G.chain_buf = (int)r16(buf);
    G.chain_rs = (int)r16(rs);
    G.chain_lds = (int)lds;
    while (h->ltab.size() % 16) h->ltab.push_back(0);
    G.chain_tab = (int)h->ltab.size();
    h->ltab.insert(h->ltab.end(), (const uint8_t*)rects.data(), (const uint8_t*)(rects.data() + rects.size()));
    while (h->ltab.size() % 16) h->ltab.push_back(0);
    G.chain_toffs = (int)h->ltab.size();
    h->ltab.insert(h->ltab.end(), (const uint8_t*)toffs.data(), (const uint8_t*)(toffs.data() + toffs.size()));
    G.chain_ok = 1;
}

orbx_status build_geometry(orbx_extractor* h, int W, int H) {
    Geometry& G = h->hg;
    memset(&G, 0, sizeof(G));
    // k_level's row pass folds the symmetric Gaussian taps (getGaussianKernel is symmetric)
    for (int i = 0; i < 3; ++i)
        if (h->taps[i] != h->taps[6 - i]) return ORBX_ERR_UNSUPPORTED;
    h->cells.clear();
    h->rtab.clear();
    const int L = h->prm.nlevels;
    G.width = W;
    G.height = H;
    G.nlevels = L;
    G.ini_th = std::min(std::max(h->prm.ini_th_fast, 0), 255);
    G.min_th = std::min(std::max(h->prm.min_th_fast, 0), 255);
    memcpy(G.taps, h->taps, sizeof(G.taps));
    memcpy(G.umax, h->umax, sizeof(G.umax));
    // k_stereo buckets right keypoints by (octave, row); a keypoint of octave o lists itself
    // in the rows of its band [floor(y - 2 scale[o]), ceil(y + 2 scale[o])] (src/Frame.cc:522-530)
    for (int l = 0; l < L; ++l)
        G.lv[l].stereo_win = (int)std::ceil(2.0f * h->scale[l]) + 2;
    long long off = 0, cand = 0;
    int out = 0, blur_tiles = 0, oblocks = 0;
    for (int l = 0; l < L; ++l) {
        LevelGeom& lv = G.lv[l];
        lv.w = cvRound((float)W * h->inv_scale[l]);
        lv.h = cvRound((float)H * h->inv_scale[l]);
        if (lv.w <= 0 || lv.h <= 0) return ORBX_ERR_UNSUPPORTED;
        if (lv.w > 4096 + 32 || lv.h > 4096 + 32) return ORBX_ERR_UNSUPPORTED;   // 12-bit packing
        lv.pitch = (int)align_up(lv.w + 4, 64);   // >= 4 bytes of slack for dword staging
        lv.off = off;
        // whole bands of 4 rows: the blurred pyramid (same offsets) is stored in 16x4 tiles
        off += (long long)align_up((size_t)lv.pitch * align_up((size_t)lv.h, 4), 256);
        lv.scale = h->scale[l];
        lv.inv_scale = h->inv_scale[l];
        lv.nfeat = h->nfeat[l];
        lv.patch_size = (int)(31 * h->scale[l]);
        // FAST cell grid (src/ORBextractor.cc:785-818)
        const int minB = ORBX_MIN_BORDER;
        const int maxBX = lv.w - ORBX_EDGE + 3, maxBY = lv.h - ORBX_EDGE + 3;
        const float width = (float)(maxBX - minB), height = (float)(maxBY - minB);
        const int nCols = (int)(width / 30.f), nRows = (int)(height / 30.f);
        lv.ncols = nCols;
        lv.nrows = nRows;
        lv.cell_begin = (int)h->cells.size();
        lv.cand_off = cand;
        int lcap = 0;
        if (nCols > 0 && nRows > 0) {
            const int wCell = (int)std::ceil(width / nCols);
            const int hCell = (int)std::ceil(height / nRows);
            lv.wcell = wCell;
            lv.hcell = hCell;
            for (int i = 0; i < nRows; i++) {
                const float iniY = (float)(minB + i * hCell);
                float maxY = iniY + hCell + 6;
                if (iniY >= maxBY - 3) continue;
                if (maxY > maxBY) maxY = (float)maxBY;
                for (int j = 0; j < nCols; j++) {
                    const float iniX = (float)(minB + j * wCell);
                    float maxX = iniX + wCell + 6;
                    if (iniX >= maxBX - 6) continue;
                    if (maxX > maxBX) maxX = (float)maxBX;
                    CellDesc c;
                    memset(&c, 0, sizeof(c));
                    c.level = (int16_t)l;
                    c.ini_x = (int16_t)(int)iniX;
                    c.ini_y = (int16_t)(int)iniY;
                    c.cols = (int16_t)((int)maxX - (int)iniX);
                    c.rows = (int16_t)((int)maxY - (int)iniY);
                    const int dh = c.rows - 6, dw = c.cols - 6;
                    c.cap = (dh > 0 && dw > 0) ? ((dw + 1) / 2) * ((dh + 1) / 2) : 0;
                    c.slot = (int32_t)cand;
                    cand += c.cap;
                    lcap += c.cap;
                    // k_fast stages the ROI as aligned dwords: <= cols + 6 bytes per row
                    {
                        const int lpc = std::max((c.cols + 6 + 3) / 4, fast_lpitch((3 + c.cols + 3) / 4, dw));
                        // a prefetched ROI writes all 4 * FAST_PF2D rows
                        const int rows_w = std::max((int)c.rows, 4 * FAST_PF2D);
                        G.max_roi_bytes = std::max(G.max_roi_bytes, rows_w * lpc * 4);
                    }
                    if (dh > 0 && dw > 0) {
                        G.max_mbuf_bytes = std::max(G.max_mbuf_bytes, ((dh + 2) * (dw + 2) + 3) & ~3);
                        G.max_cell_px = std::max(G.max_cell_px, dh * dw);
                    }
                    if (dw > 64 || dh > 511) return ORBX_ERR_UNSUPPORTED;   // k_fast lane mapping
                    h->cells.push_back(c);
                }
            }
        }
        lv.ncells = (int)h->cells.size() - lv.cell_begin;
        lv.cand_cap = lcap;
        G.max_ncand_level = std::max(G.max_ncand_level, lcap);
        // octree roots (src/ORBextractor.cc:543-545)
        lv.n_ini = 0;
        lv.hx = 0.f;
        if (maxBY - minB > 0) {
            const float r = std::round(static_cast<float>(maxBX - minB) / (maxBY - minB));
            if (r >= 1.f && r < 4096.f) {
                lv.n_ini = (int)r;
                lv.hx = static_cast<float>(maxBX - minB) / lv.n_ini;
            }
        }
        lv.out_cap = std::max(std::max(lv.nfeat + 3, 4 * lv.n_ini), 4);
        lv.kp_level_cap = lv.out_cap;
        lv.out_off = out;
        out += lv.out_cap;
        G.max_out_cap = std::max(G.max_out_cap, lv.out_cap);
        G.blur_tile_begin[l] = blur_tiles;
        blur_tiles += ((lv.w + 63) / 64) * ((lv.h + 15) / 16);
        G.orient_block_begin[l] = oblocks;
        oblocks += (lv.out_cap + 4 * OD_NK - 1) / (4 * OD_NK);
        lv.bsimd_end = h->prm.cv_simd ? (lv.w / 4) * 4 : 0;
        // resize tables (cv::resize INTER_LINEAR 8U, imgwarp.cpp)
        lv.copy = lv.area2 = 0;
        lv.rtab_off = 0;
        lv.xmax = lv.w;
        lv.rsimd_end = 0;
        if (l > 0) {
            const LevelGeom& S = G.lv[l - 1];
            const int sw = S.w, sh = S.h, dw = lv.w, dh = lv.h;
            if (sw == dw && sh == dh) {
                lv.copy = 1;
            } else {
                const double inv_sx = (double)dw / sw, inv_sy = (double)dh / sh;
                const double scale_x = 1. / inv_sx, scale_y = 1. / inv_sy;
                const int isx = cvRound(scale_x), isy = cvRound(scale_y);
                const bool area_fast = std::abs(scale_x - isx) < DBL_EPSILON &&
                                       std::abs(scale_y - isy) < DBL_EPSILON;
                if (area_fast && isx == 2 && isy == 2) {
                    lv.area2 = 1;
                } else {
                    lv.rtab_off = (int)h->rtab.size();
                    std::vector<int16_t> xofs(dw), alpha(2 * dw), yofs(dh), beta(2 * dh);
                    int xmax = dw;
                    for (int dx = 0; dx < dw; ++dx) {
                        float fx = (float)((dx + 0.5) * scale_x - 0.5);
                        int sx = cvFloor(fx);
                        fx -= sx;
                        if (sx < 0) { fx = 0, sx = 0; }
                        if (sx + 1 >= sw) {
                            xmax = std::min(xmax, dx);
                            if (sx >= sw - 1) fx = 0, sx = sw - 1;
                        }
                        xofs[dx] = (int16_t)sx;
                        alpha[2 * dx] = sat_short((1.f - fx) * 2048);
                        alpha[2 * dx + 1] = sat_short(fx * 2048);
                    }
                    for (int dy = 0; dy < dh; ++dy) {
                        float fy = (float)((dy + 0.5) * scale_y - 0.5);
                        int sy = cvFloor(fy);
                        fy -= sy;
                        yofs[dy] = (int16_t)sy;
                        beta[2 * dy] = sat_short((1.f - fy) * 2048);
                        beta[2 * dy + 1] = sat_short(fy * 2048);
                    }
                    h->rtab.insert(h->rtab.end(), xofs.begin(), xofs.end());
                    h->rtab.insert(h->rtab.end(), alpha.begin(), alpha.end());
                    h->rtab.insert(h->rtab.end(), yofs.begin(), yofs.end());
                    h->rtab.insert(h->rtab.end(), beta.begin(), beta.end());
                    lv.xmax = xmax;
                    lv.rsimd_end = h->prm.cv_simd ? vresize_simd_end(dw) : 0;
                }
            }
        }
    }
    // k_level tiles (128 x 32): per tile column / row the staged source window and the
    // group / row tables the kernel reads (LevelColTab / LevelRowTab), and the largest window
    G.ltw = LT_W;
    G.lth = LT_H;
    G.win_cap = 16;
    h->ltab.clear();
    for (int l = 0; l < L; ++l) {
        LevelGeom& lv = G.lv[l];
        lv.ntx = (lv.w + G.ltw - 1) / G.ltw;
        lv.nty = (lv.h + G.lth - 1) / G.lth;
        const int mode = l == 0 ? 0 : (lv.copy ? 1 : (lv.area2 ? 2 : 3));
        const LevelGeom& S = G.lv[l > 0 ? l - 1 : 0];
        const int16_t* xofs = h->rtab.data() + lv.rtab_off;
        const int16_t* alpha = xofs + lv.w;
        const int16_t* yofs = alpha + 2 * lv.w;
        const int16_t* beta = yofs + lv.h;
        std::vector<LevelColTab> ct(lv.ntx);
        std::vector<LevelRowTab> rt(lv.nty);
        for (int tx = 0; tx < lv.ntx; ++tx) {
            const int X0 = tx * G.ltw, vw = std::min(G.ltw, lv.w - X0);
            int x0, x1;
            if (mode == 3) {
                int mnx, mxx;
                reflected_range_h(X0 - 3, X0 + vw + 2, lv.w, mnx, mxx);
                x0 = xofs[mnx] & ~3;
                x1 = std::min((int)xofs[mxx] + 1, S.w - 1);
            } else {
                x0 = std::max(X0 - 4, 0);
                x1 = std::min(X0 + G.ltw + 3, lv.w - 1);
            }
            LevelColTab& c = ct[tx];
            memset(&c, 0, sizeof(c));
            c.x0 = x0;
            c.ww = x1 - x0 + 1;
            for (int q = 0; q < LT_G; ++q) {
                int sx[4];
                uint32_t fl = 0, al[4] = {0, 0, 0, 0};
                for (int j = 0; j < 4; ++j) {
                    const int xr = reflect101_h(X0 - 4 + 4 * q + j, lv.w);
                    if (mode == 3) {
                        sx[j] = xofs[xr] - x0;
                        al[j] = (uint32_t)(uint16_t)alpha[2 * xr] |
                                ((uint32_t)(uint16_t)alpha[2 * xr + 1] << 16);
                        fl |= (uint32_t)((xr < lv.xmax ? 1 : 0) | (xr < lv.rsimd_end ? 2 : 0))
                              << (2 * j);
                    } else {
                        sx[j] = (mode == 2) ? xr : xr - (X0 - 4);   // window column (modes 0/1)
                    }
                    // pixels of a group outside the needed halo may reflect anywhere: keep
                    // their (unused) reads inside the window
                    if (mode == 3) sx[j] = std::min(std::max(sx[j], 0), std::max(c.ww - 1, 0));
                    else if (mode != 2) sx[j] = std::min(std::max(sx[j], 0), LT_G * 4 - 1);
                }
                const bool contig = sx[1] == sx[0] + 1 && sx[2] == sx[0] + 2 &&
                                    sx[3] == sx[0] + 3 && (sx[0] & 3) == 0;
                const int o0 = sx[0] & 3;
                (void)o0;
                const bool simple = sx[1] >= sx[0] && sx[2] >= sx[1] && sx[3] >= sx[2] &&
                                    sx[3] - sx[0] <= 6;
                c.cgrp[2 * q] = (uint32_t)sx[0] | ((uint32_t)sx[1] << 16);
                c.cgrp[2 * q + 1] = (uint32_t)sx[2] | ((uint32_t)sx[3] << 16);
                const uint32_t hi = 0;
                for (int j = 0; j < 4; ++j) {
                    // simple groups: pixel j's taps are bytes k, k+1 of the 8 bytes from sx0
                    // (the kernel aligns the window to sx0 with v_alignbyte); v_perm picks
                    // them as u16s
                    const int k = std::min(std::max(sx[j] - sx[0], 0), 6);
                    c.csel[4 * q + j] = (uint32_t)k | (0x0Cu << 8) |
                                        ((uint32_t)(k + 1) << 16) | (0x0Cu << 24);
                    // right of xmax HResizeLinear uses S[sx] * 2048: the same dot product
                    // with alphas (2048, 0)
                    if (mode == 3 && !((fl >> (2 * j)) & 1u)) al[j] = 2048u;
                }
                // simple groups carry 16 x the alphas (<= 32768 still a u16): the kernel's
                // dot product then yields 16 h, whose low byte cleared is (h >> 4) << 8
                if (mode == 3 && simple)
                    for (int j = 0; j < 4; ++j)
                        al[j] = ((al[j] & 0xFFFFu) << 4) | (((al[j] >> 16) << 4) << 16);
                c.cinf[q] = fl | (contig ? 0x100u : 0u) | (simple ? 0x200u : 0u) | hi;
                for (int j = 0; j < 4; ++j) c.calp[4 * q + j] = al[j];
            }
        }
        for (int ty = 0; ty < lv.nty; ++ty) {
            const int Y0 = ty * G.lth, vh = std::min(G.lth, lv.h - Y0);
            int y0, y1;
            if (mode == 3) {
                int mny, mxy;
                reflected_range_h(Y0 - 3, Y0 + vh + 2, lv.h, mny, mxy);
                y0 = std::min(std::max((int)yofs[mny], 0), S.h - 1);
                y1 = std::min(std::max((int)yofs[mxy] + 1, 0), S.h - 1);
            } else {
                y0 = std::max(Y0 - 3, 0);
                y1 = std::min(Y0 + G.lth + 2, lv.h - 1);
            }
            LevelRowTab& r = rt[ty];
            memset(&r, 0, sizeof(r));
            r.y0 = y0;
            r.wh = y1 - y0 + 1;
            for (int k = 0; k < LT_HR; ++k) {
                const int yr = reflect101_h(Y0 - 3 + k, lv.h);
                if (mode == 3) {
                    const int sy = yofs[yr];
                    const uint32_t y0r = (uint32_t)(std::min(std::max(sy, 0), S.h - 1) - y0);
                    const uint32_t y1r = (uint32_t)(std::min(std::max(sy + 1, 0), S.h - 1) - y0);
                    r.rinf[2 * k] = y0r | (y1r << 16);
                    r.rinf[2 * k + 1] = (uint32_t)(uint16_t)beta[2 * yr] |
                                        ((uint32_t)(uint16_t)beta[2 * yr + 1] << 16);
                } else {
                    r.rinf[2 * k] = (uint32_t)(mode == 2 ? yr : yr - y0);
                }
            }
        }
        for (int ty = 0; ty < lv.nty; ++ty)
            for (int tx = 0; tx < lv.ntx; ++tx) {
                int bytes = 0;
                if (mode == 0 || mode == 1) bytes = (G.ltw + 8) * rt[ty].wh;
                else if (mode == 3) bytes = ((ct[tx].ww + 3) & ~3) * rt[ty].wh;
                G.win_cap = std::max(G.win_cap, bytes);
            }
        lv.ctab = (int)h->ltab.size();
        h->ltab.insert(h->ltab.end(), (const uint8_t*)ct.data(),
                       (const uint8_t*)(ct.data() + ct.size()));
        lv.rowtab = (int)h->ltab.size();
        h->ltab.insert(h->ltab.end(), (const uint8_t*)rt.data(),
                       (const uint8_t*)(rt.data() + rt.size()));
        build_strip_tables(h, l, mode, xofs, alpha, yofs, beta);
    }
    build_chain(h);
    h->level_lds = level_lds_bytes(G.ltw, G.lth, G.win_cap);
    if (h->level_lds > 160 * 1024) return ORBX_ERR_UNSUPPORTED;
    G.blur_tile_begin[L] = blur_tiles;
    G.orient_block_begin[L] = oblocks;
    G.blur_tiles = blur_tiles;
    G.orient_blocks = oblocks;
    G.n_cells = (int)h->cells.size();
    G.kp_cap = out;
    G.out_words = out;
    G.pyr_bytes = off;
    G.cand_words = std::max(cand, 1LL);
    if (G.max_roi_bytes == 0) G.max_roi_bytes = 16;
    if (G.max_mbuf_bytes == 0) G.max_mbuf_bytes = 16;
    if (G.max_out_cap > 8192) return ORBX_ERR_UNSUPPORTED;
    h->kscratch_per_image = 0;
    for (int l = 0; l < L; ++l) h->kscratch_per_image += (long long)G.lv[l].cand_cap * 8;
    h->kscratch_per_image = (long long)align_up((size_t)std::max(h->kscratch_per_image, 16LL), 256);
    // octree LDS (all levels in one launch): node arrays for the largest level's list, the
    // candidate arrays in LDS up to the OCT_LDS_KB budget (a level with more candidates keeps
    // them in global scratch)
    int ncand0 = 0, ncand1 = 0, ocmax = 16;
    for (int l = 0; l < L; ++l) {
        int n = 0;
        for (int k = 0; k < G.lv[l].ncells; ++k) n += h->cells[G.lv[l].cell_begin + k].cap;
        if (l == 0) ncand0 = n; else ncand1 = std::max(ncand1, n);
        ocmax = std::max(ocmax, G.lv[l].out_cap);
    }
    {
        h->ncap = (int)align_up((size_t)ocmax, 16);
        int kc = std::min(std::max(std::max(ncand0, ncand1), 64), 8192);
        while (kc > 64 && octree_lds_bytes(h->ncap, kc, true) > OCT_LDS_KB * 1024) kc -= 64;
        h->kcap = kc;
        h->octree_lds = octree_lds_bytes(h->ncap, h->kcap, true);
        h->ncap1 = h->ncap;
        h->kcap1 = h->kcap;
        h->octree_lds1 = h->octree_lds;
    }
    {
        // small batches: the same node arrays, candidates in LDS up to OCT_LDS_SMALL_KB
        int kc = std::min(std::max(std::max(ncand0, ncand1), 64), 8192);
        while (kc > 64 && octree_lds_bytes(h->ncap, kc, false) > OCT_LDS_SMALL_KB * 1024) kc -= 64;
        h->kcap_small = std::max(kc, h->kcap);
        h->octree_lds_small = std::max(octree_lds_bytes(h->ncap, h->kcap_small, false), h->octree_lds);
    }
    G.stereo_ob = G.nlevels;
    h->stereo_lds = stereo_lds_bytes(G.kp_cap, G.lv[0].h, G.stereo_ob);
    if (h->stereo_lds > 160 * 1024) {   // row buckets only (octaves tested per candidate)
        G.stereo_ob = 1;
        h->stereo_lds = stereo_lds_bytes(G.kp_cap, G.lv[0].h, G.stereo_ob);
    }
    if (h->octree_lds > 160 * 1024 || h->stereo_lds > 160 * 1024) return ORBX_ERR_UNSUPPORTED;
    if (G.kp_cap > 32767) return ORBX_ERR_UNSUPPORTED;   // 16-bit keypoint indices in stereo
    return ORBX_OK;
}

orbx_status ensure_workspace(orbx_extractor* h, int W, int H, int batch) {
    if (batch < 1) return ORBX_ERR_INVALID;
    if (!HIPOK(hipSetDevice(h->device))) return ORBX_ERR_DEVICE;
    const bool same = h->have_geom && h->hg.width == W && h->hg.height == H;
    if (!same) {
        // this handle's earlier calls may still read the old tables (on their streams)
        if (!wait_idle(h)) return ORBX_ERR_DEVICE;
        orbx_status s = build_geometry(h, W, H);
        if (s != ORBX_OK) { h->have_geom = false; return s; }
        if (!h->d_geom.ensure(sizeof(Geometry))) return ORBX_ERR_DEVICE;
        if (!h->d_cells.ensure(std::max<size_t>(h->cells.size(), 1) * sizeof(CellDesc))) return ORBX_ERR_DEVICE;
        if (!h->d_rtab.ensure(std::max<size_t>(h->rtab.size(), 1) * 2)) return ORBX_ERR_DEVICE;
        if (!h->d_ltab.ensure(std::max<size_t>(h->ltab.size(), 16))) return ORBX_ERR_DEVICE;
        // uploads on the handle's own (non-blocking) stream: nothing else on the device waits
        hipStream_t st = h->stream;
        if (!HIPOK(hipMemcpyAsync(h->d_ltab.p, h->ltab.data(), h->ltab.size(), hipMemcpyHostToDevice, st)) ||
            !HIPOK(hipMemcpyAsync(h->d_geom.p, &h->hg, sizeof(Geometry), hipMemcpyHostToDevice, st)))
            return ORBX_ERR_DEVICE;
        if (!h->cells.empty() &&
            !HIPOK(hipMemcpyAsync(h->d_cells.p, h->cells.data(), h->cells.size() * sizeof(CellDesc),
                                  hipMemcpyHostToDevice, st)))
            return ORBX_ERR_DEVICE;
        if (!h->rtab.empty() &&
            !HIPOK(hipMemcpyAsync(h->d_rtab.p, h->rtab.data(), h->rtab.size() * 2, hipMemcpyHostToDevice, st)))
            return ORBX_ERR_DEVICE;
        if (!HIPOK(hipStreamSynchronize(st))) return ORBX_ERR_DEVICE;
        if (!HIPOK(prepare_kernels(std::max(h->octree_lds, h->octree_lds_small), h->stereo_lds,
                                   std::max(h->level_lds, (size_t)h->hg.chain_lds), fast_lds_bytes(h->hg))))
            return ORBX_ERR_DEVICE;
        h->have_geom = true;
        h->cap_batch = 0;
    }
    if (batch > h->cap_batch) {
        // growing frees the old buffers: the handle's work in flight must be done
        if (!wait_idle(h)) return ORBX_ERR_DEVICE;
        h->pyr_images = 0;   // the pyramids go with them
        ++h->serial;
        const Geometry& G = h->hg;
        const size_t B = (size_t)batch;
        // k_fast reads up to 4 * FAST_PF2D rows past a cell's ROI
        const size_t pyr_slack = (size_t)4 * FAST_PF2D * G.lv[0].pitch + 256;
        bool ok = h->d_pyr.ensure(B * G.pyr_bytes + pyr_slack) &&
                  h->d_blur.ensure(B * G.pyr_bytes) &&
                  h->d_ccnt.ensure(B * std::max(G.n_cells, 1) * 4) &&
                  h->d_cand.ensure(B * G.cand_words * 4) &&
                  h->d_ocnt.ensure(B * G.nlevels * 4) && h->d_okp.ensure(B * G.out_words * 6) &&
                  h->d_kscr.ensure(B * h->kscratch_per_image);
        const size_t o_kps = align_up(B * 4, 256);
        const size_t o_desc = o_kps + align_up(B * G.kp_cap * sizeof(orbx_keypoint), 256);
        const size_t o_end = o_desc + B * G.kp_cap * 32;
        // then one pair's stereo block [nvalid | uRight[KC] | depth[KC]]
        // (orbx_stereo_frame_view: its outputs come back with the keypoints in one DMA)
        h->o_stereo = align_up(o_end, 256);
        ok = ok && h->d_outs.ensure(h->o_stereo + 256 + 8 * (size_t)G.kp_cap);
        if (!ok) return ORBX_ERR_DEVICE;
        uint8_t* ob = h->d_outs.as<uint8_t>();
        h->d_nkp.view(ob, B * 4);
        h->d_kps.view(ob + o_kps, B * G.kp_cap * sizeof(orbx_keypoint));
        h->d_desc.view(ob + o_desc, B * G.kp_cap * 32);
        h->cap_batch = batch;
    }
    return ORBX_OK;
}

// d_imgs == nullptr: level 0 of every image is already in the pyramid (in place).
// The launch descriptor of one batched extraction (d_imgs == nullptr: level 0 of every image
// is already in the pyramid, in place).
ExtractLaunch extract_launch(orbx_extractor* h, const uint8_t* d_imgs, const uint8_t* d_imgs2,
                             int split, int batch, size_t stride, size_t batch_stride) {
    ExtractLaunch a;
    a.in_place = d_imgs == nullptr;
    if (a.in_place) {
        d_imgs = h->d_pyr.as<uint8_t>();
        d_imgs2 = nullptr;
        stride = (size_t)h->hg.lv[0].pitch;
        batch_stride = (size_t)h->hg.pyr_bytes;
    }
    a.hg = &h->hg;
    a.dg = h->d_geom.as<Geometry>();
    a.cells = h->d_cells.as<CellDesc>();
    a.rtab = h->d_rtab.as<int16_t>();
    a.ltab = h->d_ltab.as<uint8_t>();
    a.d_imgs = d_imgs;
    a.d_imgs2 = d_imgs2 ? d_imgs2 : d_imgs;
    a.split = d_imgs2 ? split : batch;
    a.level_lds = h->level_lds;
    a.stride = stride;
    a.batch_stride = batch_stride;
    a.batch = batch;
    a.pyr = h->d_pyr.as<uint8_t>();
    a.blur = h->d_blur.as<uint8_t>();
    a.ccnt = h->d_ccnt.as<int>();
    a.cand = h->d_cand.as<uint32_t>();
    a.ocnt = h->d_ocnt.as<int>();
    a.okp = h->d_okp.as<uint32_t>();
    a.operm = (uint16_t*)(a.okp + (size_t)batch * h->hg.out_words);
    a.kscratch = h->d_kscr.as<uint8_t>();
    a.kscratch_per_image = h->kscratch_per_image;
    a.ncap = h->ncap;
    a.kcap = h->kcap;
    a.octree_lds = h->octree_lds;
    a.ncap1 = h->ncap1;
    a.kcap1 = h->kcap1;
    a.octree_lds1 = h->octree_lds1;
    a.kcap_small = h->kcap_small;
    a.octree_lds_small = h->octree_lds_small;
    a.oct_small = batch <= OCT_SMALL_BATCH ? 1 : 0;
    a.fast_nc = fast_cells_per_wave(h->hg.n_cells, batch, h->ncu);
    a.kps = h->d_kps.as<float>();
    a.desc = h->d_desc.as<uint8_t>();
    a.nkp = h->d_nkp.as<int>();
    a.timer = &h->timer;
    a.side = h->side;
    a.ev_fork = h->ev_fork;
    a.ev_join = h->ev_join;
    // the default schedule forks the side branch only for batches that can fill the chip: a
    // small batch's kernels are latency chains, and the fork / join events between the two
    // streams cost more than the overlap gives (an explicit orbx_extractor_set_overlap applies
    // at every batch size)
    a.side_mode = (h->side_auto && batch < SIDE_MIN_BATCH) ? 0
                                                                                     : h->side_mode;
    a.side_at = h->side_at;
    a.side_lv = h->side_lv;
    a.chain = (h->hg.chain_ok && a.in_place && a.side_mode == 0 &&
               batch <= CHAIN_MAX_BATCH) ? 1 : 0;
    strip_heights(h, batch, a.sth);
    return a;
}

orbx_status run_extract(orbx_extractor* h, const uint8_t* d_imgs, const uint8_t* d_imgs2,
                        int split, int batch, size_t stride, size_t batch_stride, hipStream_t st) {
    const ExtractLaunch a = extract_launch(h, d_imgs, d_imgs2, split, batch, stride, batch_stride);
    if (!order_after_last(h, st)) return ORBX_ERR_DEVICE;
    if (!HIPOK(launch_extract(a, st)) || !mark_done(h, st)) return ORBX_ERR_DEVICE;
    h->last_batch = batch;
    h->last_valid = true;
    h->pyr_images = h->last_batch;
    ++h->serial;
    h->last_n = -1;   // on the device only (orbx_extract records it once copied back)
    return ORBX_OK;
}

// Batched calls run on exactly the stream the caller names; 0 is the null (legacy default)
// stream, which orders them with the caller's other default-stream work.
hipStream_t pick_stream(orbx_extractor*, void* s) { return (hipStream_t)s; }

// The launch of stereo over pairs (image i of L at offset offL, image i of R at offset offR),
// its scratch allocated: nothing in it allocates or waits, so it can be enqueued in a graph
// capture.  The images' extraction must be issued (not necessarily run) before the launch.
orbx_status stereo_launch_args(orbx_extractor* L, orbx_extractor* R, int batch, int offL,
                               int offR, float mbf, float mb, float* d_uR, float* d_dep,
                               int* d_nv, hipStream_t st, StereoLaunch& a) {
    if (L->hg.width != R->hg.width || L->hg.height != R->hg.height ||
        L->hg.nlevels != R->hg.nlevels || L->hg.kp_cap != R->hg.kp_cap)
        return ORBX_ERR_INVALID;
    const size_t KC = (size_t)L->hg.kp_cap;
    a.dg = L->d_geom.as<Geometry>();
    a.batch = batch;
    a.kpsL = L->d_kps.as<float>() + offL * KC * 7;
    a.descL = L->d_desc.as<uint8_t>() + offL * KC * 32;
    a.nkpL = L->d_nkp.as<int>() + offL;
    a.pyrL = L->d_pyr.as<uint8_t>() + offL * (size_t)L->hg.pyr_bytes;
    a.kpsR = R->d_kps.as<float>() + offR * KC * 7;
    a.descR = R->d_desc.as<uint8_t>() + offR * KC * 32;
    a.nkpR = R->d_nkp.as<int>() + offR;
    a.pyrR = R->d_pyr.as<uint8_t>() + offR * (size_t)R->hg.pyr_bytes;
    a.mbf = mbf;
    a.mb = mb;
    a.uR = d_uR;
    a.depth = d_dep;
    a.nvalid = d_nv;
    a.lds = L->stereo_lds;
    a.timer = &L->timer;
    a.scnt = nullptr;
    a.ssad = nullptr;
    a.sidx = nullptr;
    if (stereo_split(batch) > 1) {
        // split path scratch: counters (zeroed when allocated; the median cut leaves them zero),
        // then per pair kp_cap SADs and left indices
        // (a fixed counter block: one slot per pair of the largest split batch, so a later
        // call with another batch finds its counters zero)
        // (stereo_split(batch) > 1 only for batch <= 128, so 256 counters always suffice)
        // (then 256 done-counters of the fused cut, also zero on entry and left zero)
        const size_t cnt_bytes = 2 * 256 * 4;
        const size_t need = cnt_bytes + (size_t)batch * KC * 6;
        // a reallocation (detected by capacity: the allocator may hand back the same
        // address) starts from zeroed counters
        const size_t cap_before = L->d_sscr.n;
        if (need > cap_before && !wait_idle(L)) return ORBX_ERR_DEVICE;
        if (!L->d_sscr.ensure(need)) return ORBX_ERR_DEVICE;
        if (L->d_sscr.n != cap_before &&
            !HIPOK(hipMemsetAsync(L->d_sscr.p, 0, cnt_bytes, st)))
            return ORBX_ERR_DEVICE;
        uint8_t* base = L->d_sscr.as<uint8_t>();
        a.scnt = (int*)base;
        a.ssad = (int*)(base + cnt_bytes);
        a.sidx = (int16_t*)(base + cnt_bytes + (size_t)batch * KC * 4);
    }
    return ORBX_OK;
}

// Stereo over pairs of the handles' last extractions.
orbx_status run_stereo(orbx_extractor* L, orbx_extractor* R, int batch, int offL, int offR,
                       float mbf, float mb, float* d_uR, float* d_dep, int* d_nv, hipStream_t st) {
    if (!L->last_valid || !R->last_valid) return ORBX_ERR_STATE;
    if (offL + batch > L->last_batch || offR + batch > R->last_batch) return ORBX_ERR_INVALID;
    StereoLaunch a;
    const orbx_status s = stereo_launch_args(L, R, batch, offL, offR, mbf, mb, d_uR, d_dep, d_nv,
                                             st, a);
    if (s != ORBX_OK) return s;
    if (!order_after_last(L, st) || (R != L && !order_after_last(R, st))) return ORBX_ERR_DEVICE;
    if (!HIPOK(launch_stereo(a, st)) || !mark_done(L, st) || (R != L && !mark_done(R, st)))
        return ORBX_ERR_DEVICE;
    return ORBX_OK;
}

}  // namespace

// ---- several sessions' stereo frames as one batch (orbx_stereo_frame_view) -----------------
// Tracking sessions on one device each call orbx_stereo_frame_view on their own handle.  A
// call that finds the device's frame server idle (nothing running, nothing queued) runs on its
// own handle (one graph replay, stereo_frame_solo).  A call that arrives while another runs
// joins the batch being formed: it stages its two images into its slot of the server's pinned
// input block and issues that slot's DMA to the server's device staging on the server's copy
// stream right away (the copy overlaps the running batch).  When the device frees, a waiting
// thread takes the formed batch (up to FS_MAX_FRAMES frames of one image size and camera) and
// replays the server's graph for its size on the server's own handle: the lefts as images
// [0, m), the rights as [m, 2m), one extraction of the 2m images, one stereo launch over the
// m pairs, the outputs back into the pair's pinned output block.  Each waiting thread then
// copies its frame's outputs into its own handle's pinned block.  Two block pairs alternate,
// each with its own server handle: a batch forms in one while the other's runs, and up to
// FS_INFLIGHT batches run at once.  With several sessions the runtime's submission path,
// not the GPU, bounded the rate of one-call frames (14 submissions each).
#define STAGE_THREAD 1
// orbx_stereo_frame_view: the right image staged by a helper thread (0 never, 1 for frames that
// queue for the frame server, 2 always).  Measured (r04_ab_runs.txt, r4i): the helper's wake-up
// costs a lone caller with cache-hot images more (0.239 -> 0.257 ms) than it saves on cold ones
// (0.268 -> 0.259 ms); with 8 sessions it raised 9.4-9.6k to 9.6-9.9k pairs/s.
#define EXTRACT_GRAPH 1   // orbx_extract replays its device sequence from a per-handle graph
// Batches on the device at once (each on its block pair's own server handle): a batch of a
// few frames is a latency-bound chain that leaves most of the GPU idle, so the next one runs
// beside it.
#define FS_INFLIGHT 2
#define FS_MAX_FRAMES 8
#define FRAME_SERVER 1
struct FsReq {
    orbx_extractor* h;            // the caller's handle (its stager)
    int slot = -1, blk = -1;      // its frame in the batch, the block pair of that batch
    orbx_status st = ORBX_OK;
    bool taken = false;           // its batch has a lead (only an untaken frame may lead)
    bool done = false;
};
struct FsLayout {                  // the layout of one server output block
    size_t o_kps = 0, o_desc = 0, o_st = 0, kc = 0;
    int m = 0;
};
struct FsBatch {                   // the size and camera of a batch's frames
    int width = 0, height = 0;
    float mbf = 0.f, mb = 0.f;
    size_t pitch0 = 0, img_bytes = 0;
};
struct FsGraph {
    hipGraphExec_t gx = nullptr;
    std::vector<const void*> key;
};
struct FrameServer {
    std::mutex mu;
    std::condition_variable cv;
    int inflight = 0;              // batches (and lone calls) on the device
    bool pair_busy[2] = {false, false};   // a batch of block pair i is on the device
    orbx_extractor* sh[2] = {nullptr, nullptr};   // the server's handle per block pair
    // the batch being formed: n frames joined, `staged` of them copied into input block blk
    int blk = 0, n = 0, staged = 0;
    FsBatch geo;
    FsReq* req[FS_MAX_FRAMES] = {};
    // block pair i: the input block (frame j's left at 2j, its right at 2j+1, img_bytes each)
    // and the output block of a batch; the next batch forms in the other pair
    uint8_t* hin[2] = {nullptr, nullptr};
    size_t hin_n[2] = {0, 0};
    // each frame's images go on to the device as soon as they are staged, on the copy stream
    // (while the batch before runs), into the device staging block of its pair
    DevBuf dstage[2];
    hipStream_t cst = nullptr;
    hipEvent_t cev[2] = {nullptr, nullptr};   // recorded on cst when a pair's batch is taken
    uint8_t* hout[2] = {nullptr, nullptr};
    size_t hout_n[2] = {0, 0};
    int readers[2] = {0, 0};       // threads still copying out of each output block
    FsLayout lay[2];
    FsGraph graphs[2][FS_MAX_FRAMES + 1];   // per block pair and batch size
    int users = 0;                 // live handles that called orbx_stereo_frame_view
    orbx_frame_server_stats stats{};   // always counted (orbx_frame_server_get_stats)
    // Frees every device / pinned resource (server handles, graphs, staging, streams); the
    // object itself (mutex, condition variable) stays, so references held by callers stay
    // valid.  Only when idle: nothing forming, running or being copied out.
    bool idle() const { return n == 0 && inflight == 0 && readers[0] == 0 && readers[1] == 0; }
    void release_resources() {
        // first drain every copy that may still read or write the pinned / staging blocks: a
        // batch whose event record failed returns without run_served, and its staging copies
        // on cst can still be pending; the server handles' graphs DMA into hout
        if (cst) (void)hipStreamSynchronize(cst);
        for (int b = 0; b < 2; ++b)
            if (sh[b]) {
                (void)wait_idle(sh[b]);
                if (sh[b]->stream) (void)hipStreamSynchronize(sh[b]->stream);
                if (sh[b]->side) (void)hipStreamSynchronize(sh[b]->side);
            }
        for (int b = 0; b < 2; ++b) {
            for (FsGraph& G : graphs[b]) {
                if (G.gx) (void)hipGraphExecDestroy(G.gx);
                G.gx = nullptr;
                G.key.clear();
            }
            if (sh[b]) (void)orbx_extractor_destroy(sh[b]);
            sh[b] = nullptr;
            if (hin[b]) (void)hipHostFree(hin[b]);
            if (hout[b]) (void)hipHostFree(hout[b]);
            hin[b] = hout[b] = nullptr;
            hin_n[b] = hout_n[b] = 0;
            dstage[b].release();
            if (cev[b]) (void)hipEventDestroy(cev[b]);
            cev[b] = nullptr;
            pair_busy[b] = false;
            lay[b] = FsLayout{};
        }
        if (cst) {
            (void)hipStreamSynchronize(cst);
            (void)hipStreamDestroy(cst);
        }
        cst = nullptr;
        blk = n = staged = 0;
        stats.resident = 0;
    }
};

// One server per (device, extractor parameters).  The registry owns them for the life of the
// process; their resources are freed when the last handle that used one is destroyed
// (frame_server_unuse) or on orbx_frame_server_release.
static std::mutex& fs_registry_mu() {
    static std::mutex mu;
    return mu;
}
static FrameServer& frame_server(const orbx_extractor* h) {
    static std::map<std::vector<int>, std::unique_ptr<FrameServer>> servers;
    const orbx_extractor_params& p = h->prm;
    int sf;
    std::memcpy(&sf, &p.scale_factor, 4);
    const std::vector<int> key = {h->device, p.nfeatures, sf, p.nlevels, p.ini_th_fast,
                                  p.min_th_fast, p.cv_simd};
    std::lock_guard<std::mutex> lk(fs_registry_mu());
    std::unique_ptr<FrameServer>& s = servers[key];
    if (!s) s.reset(new FrameServer());
    return *s;
}

// A handle that called orbx_stereo_frame_view counts as a user of its server until destroyed.
static void frame_server_use(orbx_extractor* h, FrameServer& fs) {
    std::lock_guard<std::mutex> hl(h->mu);
    if (h->fs_user) return;
    h->fs_user = true;
    std::lock_guard<std::mutex> lk(fs.mu);
    ++fs.users;
}
void frame_server_unuse(orbx_extractor* h) {
    if (!h->fs_user) return;
    FrameServer& fs = frame_server(h);
    std::lock_guard<std::mutex> lk(fs.mu);
    h->fs_user = false;
    if (--fs.users == 0 && fs.idle()) fs.release_resources();
}

static bool extract1_graph(orbx_extractor* h, const ExtractLaunch& a, hipStream_t st, int width,
                           int height, const std::function<bool(const ExtractLaunch&)>& enqueue,
                           hipGraphExec_t& gx, std::vector<const void*>& gkey,
                           std::vector<const void*> extra);

// One batch of m frames (staged in input block `blk`) on the server's handle, replayed from
// the server's graph for (blk, m): two 2-D DMAs (the lefts, the rights), the extraction of
// the 2m images, the stereo match of the m pairs, two DMAs back into output block blk.
static orbx_status run_served(FrameServer& fs, const orbx_extractor* h0, int m, int blk,
                              const FsBatch& g) {
    if (!fs.sh[blk]) {
        orbx_extractor_params p = h0->prm;
        p.max_batch = 2 * FS_MAX_FRAMES;
        const orbx_status s = orbx_extractor_create(&p, &fs.sh[blk]);
        if (s != ORBX_OK) return s;
    }
    orbx_extractor* S = fs.sh[blk];
    std::lock_guard<std::mutex> lk(S->mu);
    // the workspace for the largest batch: one layout (and graph key) for every m
    orbx_status s = ensure_workspace(S, g.width, g.height, 2 * FS_MAX_FRAMES);
    if (s != ORBX_OK) return s;
    const LevelGeom& L0 = S->hg.lv[0];
    if ((size_t)L0.pitch != g.pitch0) return ORBX_ERR_INVALID;   // the staging layout
    const size_t KC = (size_t)S->hg.kp_cap, pyrb = (size_t)S->hg.pyr_bytes;
    const size_t o_kps = (size_t)((uint8_t*)S->d_kps.p - (uint8_t*)S->d_outs.p);
    const size_t o_desc = (size_t)((uint8_t*)S->d_desc.p - (uint8_t*)S->d_outs.p);
    const size_t o_end = o_desc + 2 * (size_t)m * KC * 32;
    // stereo block: [nvalid[m] | uRight[m][KC] | depth[m][KC]]
    const size_t so_u = align_up(4 * (size_t)m, 256), so_d = so_u + (size_t)m * KC * 4;
    const size_t s_end = so_d + (size_t)m * KC * 4, o_st = align_up(o_end, 256);
    const size_t s_max = align_up(4 * (size_t)FS_MAX_FRAMES, 256) + 8 * FS_MAX_FRAMES * KC;
    const size_t o_max = align_up(o_desc + 2 * (size_t)FS_MAX_FRAMES * KC * 32, 256);
    if (!S->d_uR.ensure(s_max) || !ensure_pinned(fs.hout[blk], fs.hout_n[blk], o_max + s_max))
        return ORBX_ERR_DEVICE;
    hipStream_t st = S->stream;
    if (!order_after_last(S, st)) return ORBX_ERR_DEVICE;
    uint8_t* d_l0 = S->d_pyr.as<uint8_t>() + L0.off;
    uint8_t* dso = S->d_uR.as<uint8_t>();
    const uint8_t* dsg = fs.dstage[blk].as<uint8_t>();
    uint8_t* hout = fs.hout[blk];
    const size_t ib = g.img_bytes;
    const ExtractLaunch a = extract_launch(S, nullptr, nullptr, 2 * m, 2 * m, 0, 0);
    StereoLaunch sa;
    s = stereo_launch_args(S, S, m, 0, m, g.mbf, g.mb, (float*)(dso + so_u),
                           (float*)(dso + so_d), (int*)dso, st, sa);
    if (s != ORBX_OK) return s;
    // frame i's left into image slot i, its right into slot m + i (from the device staging);
    // back: the counts and keypoints of the 2m images, their descriptors, the stereo block
    const size_t kps_end = o_kps + 2 * (size_t)m * KC * sizeof(orbx_keypoint);
    auto enqueue = [&](const ExtractLaunch& ea) {
        return HIPOK(hipMemcpy2DAsync(d_l0, pyrb, dsg, 2 * ib, ib, (size_t)m,
                                      hipMemcpyDeviceToDevice, st)) &&
               HIPOK(hipMemcpy2DAsync(d_l0 + (size_t)m * pyrb, pyrb, dsg + ib, 2 * ib, ib,
                                      (size_t)m, hipMemcpyDeviceToDevice, st)) &&
               HIPOK(launch_extract(ea, st)) && HIPOK(launch_stereo(sa, st)) &&
               HIPOK(hipMemcpyAsync(hout, S->d_outs.p, kps_end, hipMemcpyDeviceToHost, st)) &&
               HIPOK(hipMemcpyAsync(hout + o_desc, S->d_outs.as<uint8_t>() + o_desc,
                                    o_end - o_desc, hipMemcpyDeviceToHost, st)) &&
               HIPOK(hipMemcpyAsync(hout + o_st, dso, s_end, hipMemcpyDeviceToHost, st));
    };
    uint32_t mbf_bits, mb_bits;
    std::memcpy(&mbf_bits, &g.mbf, 4);
    std::memcpy(&mb_bits, &g.mb, 4);
    FsGraph& G = fs.graphs[blk][m];
    const bool graph =
        EXTRACT_GRAPH && !S->timer.on &&
        extract1_graph(S, a, st, g.width, g.height, enqueue, G.gx, G.key,
                       {dsg, hout, S->d_sscr.p, dso, (const void*)(uintptr_t)mbf_bits,
                        (const void*)(uintptr_t)mb_bits, (const void*)(intptr_t)m,
                        (const void*)ib});
    if (!HIPOK(hipStreamWaitEvent(st, fs.cev[blk], 0)) ||   // the frames' copies to the device
        !(graph ? HIPOK(hipGraphLaunch(G.gx, st)) : enqueue(a)) || !mark_done(S, st) ||
        !wait_done(S))
        return ORBX_ERR_DEVICE;
    S->last_batch = 2 * m;
    S->last_valid = true;
    S->pyr_images = 2 * m;
    ++S->serial;
    S->last_n = -1;
    fs.lay[blk] = FsLayout{o_kps, o_desc, o_st, KC, m};
    return ORBX_OK;
}

// The waiting thread's own frame, from the server block into its handle's pinned block.
static orbx_status copy_served(FrameServer& fs, const FsReq& r, const FsBatch& g,
                               orbx_stereo_frame_out* out) {
    const FsLayout& ly = fs.lay[r.blk];
    const uint8_t* ho = fs.hout[r.blk];
    const size_t KC = ly.kc;
    int32_t n[2];
    std::memcpy(&n[0], ho + 4 * (size_t)r.slot, 4);
    std::memcpy(&n[1], ho + 4 * (size_t)(ly.m + r.slot), 4);
    const size_t nl = (size_t)std::max(n[0], 0), nr = (size_t)std::max(n[1], 0);
    orbx_extractor* h = r.h;
    std::lock_guard<std::mutex> lk(h->mu);
    const size_t need = (nl + nr) * (28 + 32) + nl * 8 + 64;
    if (!ensure_pinned(h->h_out, h->h_out_n, need)) return ORBX_ERR_DEVICE;
    uint8_t* o = h->h_out;
    const size_t img[2] = {(size_t)r.slot, (size_t)(ly.m + r.slot)};
    const size_t cnt[2] = {nl, nr};
    for (int v = 0; v < 2; ++v) {
        std::memcpy(o, ho + ly.o_kps + img[v] * KC * 28, cnt[v] * 28);
        out->kps[v] = (const orbx_keypoint*)o;
        o += cnt[v] * 28;
    }
    for (int v = 0; v < 2; ++v) {
        std::memcpy(o, ho + ly.o_desc + img[v] * KC * 32, cnt[v] * 32);
        out->desc[v] = o;
        o += cnt[v] * 32;
    }
    const uint8_t* sb = ho + ly.o_st;
    const size_t so_u = align_up(4 * (size_t)ly.m, 256), so_d = so_u + (size_t)ly.m * KC * 4;
    std::memcpy(&out->n_valid, sb + 4 * (size_t)r.slot, 4);
    std::memcpy(o, sb + so_u + (size_t)r.slot * KC * 4, nl * 4);
    out->u_right = (const float*)o;
    o += nl * 4;
    std::memcpy(o, sb + so_d + (size_t)r.slot * KC * 4, nl * 4);
    out->depth = (const float*)o;
    out->n[0] = n[0];
    out->n[1] = n[1];
    // this handle's own workspace does not hold the frame's keypoints ...
    h->last_valid = false;
    h->pyr_images = 0;
    ++h->serial;
    if (!h->keep_pyr) return ORBX_OK;
    // ... but its pyramids when asked for (orbx_extractor_keep_pyramid): both views' blocks,
    // device to device from the server handle, whose workspace this block pair's next batch
    // does not touch while this thread holds its reader count
    // The frame's keypoints, descriptors and stereo outputs are complete at this point: a
    // failure below leaves the handle in the "no pyramid" state (orbx_pyramid_level returns
    // ORBX_ERR_STATE) and the frame still succeeds.  The handle's workspace is the two-image
    // one its own solo frames run in (the server serves only handles that run solo when it is
    // idle), so sizing it here allocates nothing those would not.
    const orbx_extractor* S = fs.sh[r.blk];
    if (ensure_workspace(h, g.width, g.height, 2) != ORBX_OK) return ORBX_OK;
    const size_t pyrb = (size_t)h->hg.pyr_bytes;
    if (!S || (size_t)S->hg.pyr_bytes != pyrb || S->hg.lv[0].pitch != h->hg.lv[0].pitch)
        return ORBX_OK;
    const uint8_t* src = S->d_pyr.as<uint8_t>();
    uint8_t* dst = h->d_pyr.as<uint8_t>();
    if (!HIPOK(hipSetDevice(h->device)) || !order_after_last(h, h->stream) ||
        !HIPOK(hipMemcpyAsync(dst, src + img[0] * pyrb, pyrb, hipMemcpyDeviceToDevice, h->stream)) ||
        !HIPOK(hipMemcpyAsync(dst + pyrb, src + img[1] * pyrb, pyrb, hipMemcpyDeviceToDevice,
                              h->stream)) ||
        !mark_done(h, h->stream) || !wait_done(h))
        return ORBX_OK;
    h->last_batch = 2;
    h->pyr_images = 2;
    ++h->serial;
    return ORBX_OK;
}

extern "C" {

const char* orbx_version(void) { return ORBX_VERSION; }

const char* orbx_last_error(void) { return g_err; }

const char* orbx_kernel_name(int id) {
    static const char* names[K_COUNT] = {"k_level", "k_fast", "k_octree", "k_orient_desc",
                                         "k_stereo", "k_level0"};
    return (id >= 0 && id < K_COUNT) ? names[id] : "";
}

orbx_status orbx_extractor_set_overlap(orbx_extractor* h, int mode, int fork_level, int levels) {
    if (!h || mode > 4 || (mode > 0 && (fork_level < 0 || levels < 1))) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(h->mu);
    if (mode < 0) {
        h->side_mode = FAST_SIDE;
        h->side_at = FAST_SIDE_AT;
        h->side_lv = FAST_SIDE_LV;
        h->side_auto = true;
    } else {
        h->side_mode = mode;
        h->side_at = fork_level;
        h->side_lv = levels;
        h->side_auto = false;
    }
    return ORBX_OK;
}

orbx_status orbx_extractor_get_overlap(const orbx_extractor* h, int* mode, int* fork_level,
                                       int* levels) {
    if (!h) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(h->mu);
    if (mode) *mode = h->side_mode;
    if (fork_level) *fork_level = h->side_at;
    if (levels) *levels = h->side_lv;
    return ORBX_OK;
}

orbx_status orbx_profile_enable(orbx_extractor* h, int on) {
    if (!h) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(h->mu);
    h->timer.on = on != 0;
    return ORBX_OK;
}

orbx_status orbx_profile_collect(orbx_extractor* h, double* total_ms, int64_t* launches) {
    if (!h) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(h->mu);
    h->timer.collect();
    for (int k = 0; k < K_COUNT; ++k) {
        if (total_ms) total_ms[k] = h->timer.ms[k];
        if (launches) launches[k] = h->timer.n[k];
        h->timer.ms[k] = 0;
        h->timer.n[k] = 0;
    }
    return ORBX_OK;
}

orbx_status orbx_extractor_launch_info(const orbx_extractor* h, int batch, int* strip_rows,
                                       int* stereo_split) {
    if (!h || batch < 1) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(h->mu);
    if (!h->have_geom) return ORBX_ERR_STATE;
    int sth[ORBX_MAX_LEVELS];
    strip_heights(h, batch, sth);
    if (strip_rows)
        for (int l = 0; l < h->hg.nlevels; ++l) strip_rows[l] = h->hg.lv[l].strip ? sth[l] : 0;
    if (stereo_split) *stereo_split = stereo_split_of(std::max(batch / 2, 1));
    return ORBX_OK;
}

orbx_status orbx_device_count(int* n) {
    if (!n) return ORBX_ERR_INVALID;
    int c = 0;
    if (!HIPOK(hipGetDeviceCount(&c))) { *n = 0; return ORBX_ERR_DEVICE; }
    *n = c;
    return ORBX_OK;
}

int orbx_descriptor_distance(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 32; ++i) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return d;
}

static hipError_t create_side_stream(hipStream_t* s) {
    return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

orbx_status orbx_extractor_create(const orbx_extractor_params* p, orbx_extractor** out) {
    if (!p || !out) return ORBX_ERR_INVALID;
    *out = nullptr;
    if (p->nlevels < 1 || p->nlevels > ORBX_MAX_LEVELS || p->nfeatures < 0 ||
        !(p->scale_factor > 0.f) || p->max_batch < 0)
        return ORBX_ERR_INVALID;
    int ndev = 0;
    if (!HIPOK(hipGetDeviceCount(&ndev)) || ndev <= 0) return ORBX_ERR_DEVICE;
    if (p->device < 0 || p->device >= ndev) return ORBX_ERR_INVALID;
    orbx_extractor* h = new orbx_extractor();
    h->prm = *p;
    if (h->prm.max_batch < 1) h->prm.max_batch = 1;
    h->device = p->device;
    compute_tables(h);
    hipDeviceProp_t prop;
    if (!HIPOK(hipSetDevice(h->device)) || !HIPOK(hipGetDeviceProperties(&prop, h->device)) ||
        !HIPOK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking)) ||
        !HIPOK(hipEventCreateWithFlags(&h->done, hipEventDisableTiming)) ||
        !HIPOK(create_side_stream(&h->side)) ||
        !HIPOK(hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming)) ||
        !HIPOK(hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming))) {
        if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
        if (h->side) (void)hipStreamDestroy(h->side);
        if (h->done) (void)hipEventDestroy(h->done);
        if (h->stream) (void)hipStreamDestroy(h->stream);
        delete h;
        return ORBX_ERR_DEVICE;
    }
    h->ncu = std::max(prop.multiProcessorCount, 1);
    *out = h;
    return ORBX_OK;
}

orbx_status orbx_extractor_destroy(orbx_extractor* h) {
    if (!h) return ORBX_ERR_INVALID;
    frame_server_unuse(h);
    (void)hipSetDevice(h->device);
    (void)wait_idle(h);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->h_in) (void)hipHostFree(h->h_in);
    if (h->h_out) (void)hipHostFree(h->h_out);
    if (h->h_pyr) (void)hipHostFree(h->h_pyr);
    DevBuf* bufs[] = {&h->d_geom, &h->d_cells, &h->d_rtab, &h->d_ltab, &h->d_pyr, &h->d_blur,
                      &h->d_ccnt, &h->d_cand, &h->d_ocnt, &h->d_okp, &h->d_kscr, &h->d_kps,
                      &h->d_desc, &h->d_nkp, &h->d_uR, &h->d_dep, &h->d_nv, &h->d_sscr,
                      &h->d_outs};
    for (DevBuf* b : bufs) b->release();
    h->timer.destroy();
    if (h->g1) (void)hipGraphExecDestroy(h->g1);
    if (h->g2) (void)hipGraphExecDestroy(h->g2);
    if (h->side) (void)hipStreamSynchronize(h->side);
    if (h->done) (void)hipEventDestroy(h->done);
    if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
    if (h->ev_join) (void)hipEventDestroy(h->ev_join);
    if (h->side) (void)hipStreamDestroy(h->side);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return ORBX_OK;
}

orbx_status orbx_extractor_tables(const orbx_extractor* h, float* scale, float* inv_scale,
                                  float* sigma2, float* inv_sigma2, int* features_per_level) {
    if (!h) return ORBX_ERR_INVALID;
    for (int i = 0; i < h->prm.nlevels; ++i) {
        if (scale) scale[i] = h->scale[i];
        if (inv_scale) inv_scale[i] = h->inv_scale[i];
        if (sigma2) sigma2[i] = h->sigma2[i];
        if (inv_sigma2) inv_sigma2[i] = h->inv_sigma2[i];
        if (features_per_level) features_per_level[i] = h->nfeat[i];
    }
    return ORBX_OK;
}


// The graph of orbx_extract's device sequence for the handle's current state, captured on st
// when missing or stale.
static bool extract1_graph(orbx_extractor* h, const ExtractLaunch& a, hipStream_t st, int width,
                           int height, const std::function<bool(const ExtractLaunch&)>& enqueue,
                           hipGraphExec_t& gx, std::vector<const void*>& gkey,
                           std::vector<const void*> extra) {
    const DevBuf* bufs[] = {&h->d_geom, &h->d_cells, &h->d_rtab, &h->d_ltab, &h->d_pyr,
                            &h->d_blur, &h->d_ccnt, &h->d_cand, &h->d_ocnt, &h->d_okp,
                            &h->d_kscr, &h->d_outs};
    std::vector<const void*> key = {(const void*)(intptr_t)width, (const void*)(intptr_t)height,
                                    (const void*)(intptr_t)a.side_mode,
                                    (const void*)(intptr_t)a.side_at,
                                    (const void*)(intptr_t)a.side_lv, h->h_in, h->h_out,
                                    // the output block's layout (a regrown buffer may come
                                    // back at the same address)
                                    (const void*)(intptr_t)h->cap_batch,
                                    (const void*)(intptr_t)h->hg.kp_cap};
    for (const DevBuf* b : bufs) key.push_back(b->p);
    key.insert(key.end(), extra.begin(), extra.end());
    if (gx && key == gkey) return true;
    if (gx) {
        (void)hipGraphExecDestroy(gx);
        gx = nullptr;
    }
    hipGraph_t g = nullptr;
    bool ok = false, ended = false;
    {
        std::unique_lock<std::shared_mutex> lk(g_capture_mu);   // see order_after_last
        if (!HIPOK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal))) return false;
        ok = enqueue(a);
        ended = HIPOK(hipStreamEndCapture(st, &g));
    }
    hipGraphExec_t ex = nullptr;
    const bool inst = ok && ended && g && HIPOK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    if (g) (void)hipGraphDestroy(g);
    if (!inst) return false;
    gx = ex;
    gkey = key;
    return true;
}

// orbx_extract's device sequence for one host image, up to the outputs in the handle's pinned
// block (nkp at 0, keypoints at *o_kps, descriptors at *o_desc).  Called with h->mu held.
static orbx_status extract_host(orbx_extractor* h, const uint8_t* img, int width, int height,
                                size_t stride, size_t* o_kps_out, size_t* o_desc_out) {
    orbx_status s = ensure_workspace(h, width, height, 1);
    if (s != ORBX_OK) return s;
    hipStream_t st = h->stream;
    // The image goes through the handle's pinned staging, laid out with the pyramid's row
    // pitch, and one linear DMA writes it straight into pyramid level 0 (mvImagePyramid[0]):
    // the extraction then only blurs it (no device-side copy of the input; a pitched 2-D
    // host copy would run row by row).  Every output comes back in one pinned block: one
    // host wait per call.
    const LevelGeom& L0 = h->hg.lv[0];
    const size_t pitch0 = (size_t)L0.pitch, img_bytes = pitch0 * (size_t)height;
    const size_t KC = (size_t)h->hg.kp_cap;
    // the outputs' device block (batch 1): nkp at 0, keypoints at o_kps, descriptors at o_desc
    const size_t o_kps = (size_t)((uint8_t*)h->d_kps.p - (uint8_t*)h->d_outs.p);
    const size_t o_desc = (size_t)((uint8_t*)h->d_desc.p - (uint8_t*)h->d_outs.p);
    const size_t o_end = o_desc + KC * 32;
    h->host_pyr_ok = false;
    if (!ensure_pinned(h->h_in, h->h_in_n, img_bytes) ||
        !ensure_pinned(h->h_out, h->h_out_n, o_end) ||
        (h->host_pyr && !ensure_pinned(h->h_pyr, h->h_pyr_n, (size_t)h->hg.pyr_bytes)))
        return ORBX_ERR_DEVICE;
    for (int y = 0; y < height; ++y)
        std::memcpy(h->h_in + (size_t)y * pitch0, img + (size_t)y * stride, (size_t)width);
    if (!order_after_last(h, st)) return ORBX_ERR_DEVICE;
    // the device sequence: one linear DMA into level 0, the kernels, one DMA of the outputs
    auto enqueue = [&](const ExtractLaunch& a) {
        return HIPOK(hipMemcpyAsync(h->d_pyr.as<uint8_t>() + L0.off, h->h_in, img_bytes,
                                    hipMemcpyHostToDevice, st)) &&
               HIPOK(launch_extract(a, st)) &&
               HIPOK(hipMemcpyAsync(h->h_out, h->d_outs.p, o_end, hipMemcpyDeviceToHost, st));
    };
    ExtractLaunch a = extract_launch(h, nullptr, nullptr, 1, 1, 0, 0);
    if (h->host_pyr) {
        a.pyr_host = h->h_pyr;
        a.pyr_host_bytes = (size_t)h->hg.pyr_bytes;
    }
    // replayed from a graph (one launch instead of ~15 enqueues: several tracking sessions
    // on one GPU contend for the runtime's per-call work), eagerly when kernels are timed
    const bool graph = EXTRACT_GRAPH && !h->timer.on &&
                       extract1_graph(h, a, st, width, height, enqueue, h->g1, h->g1key,
                                      {(const void*)a.pyr_host});
    if (!(graph ? HIPOK(hipGraphLaunch(h->g1, st)) : enqueue(a)) || !mark_done(h, st) ||
        !wait_done(h))
        return ORBX_ERR_DEVICE;
    h->last_batch = 1;
    h->last_valid = true;
    h->pyr_images = h->last_batch;
    ++h->serial;
    h->host_pyr_ok = h->host_pyr;
    std::memcpy(&h->last_n, h->h_out, 4);
    *o_kps_out = o_kps;
    *o_desc_out = o_desc;
    return ORBX_OK;
}

orbx_status orbx_extract(orbx_extractor* h, const uint8_t* img, int width, int height,
                         size_t stride, orbx_keypoint* kps, int kp_cap, uint8_t* desc,
                         int* n_out) {
    if (!h || !n_out) return ORBX_ERR_INVALID;
    if (width <= 0 || height <= 0 || !img) {   // cv::Mat::empty(): silent return
        *n_out = -1;
        return ORBX_OK;
    }
    if (stride < (size_t)width) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(h->mu);
    size_t o_kps = 0, o_desc = 0;
    const orbx_status s = extract_host(h, img, width, height, stride, &o_kps, &o_desc);
    if (s != ORBX_OK) return s;
    const int n = h->last_n;
    *n_out = n;
    const int m = std::min(n, kp_cap);
    if (m > 0) {
        if (kps) std::memcpy(kps, h->h_out + o_kps, (size_t)m * sizeof(orbx_keypoint));
        if (desc) std::memcpy(desc, h->h_out + o_desc, (size_t)m * 32);
    }
    return n > kp_cap ? ORBX_ERR_CAPACITY : ORBX_OK;
}

orbx_status orbx_extract_view(orbx_extractor* h, const uint8_t* img, int width, int height,
                              size_t stride, const orbx_keypoint** kps, const uint8_t** desc,
                              int* n_out) {
    if (!h || !n_out || !kps || !desc) return ORBX_ERR_INVALID;
    *kps = nullptr;
    *desc = nullptr;
    if (width <= 0 || height <= 0 || !img) {
        *n_out = -1;
        return ORBX_OK;
    }
    if (stride < (size_t)width) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(h->mu);
    size_t o_kps = 0, o_desc = 0;
    const orbx_status s = extract_host(h, img, width, height, stride, &o_kps, &o_desc);
    if (s != ORBX_OK) return s;
    *n_out = h->last_n;
    *kps = (const orbx_keypoint*)(h->h_out + o_kps);
    *desc = h->h_out + o_desc;
    return ORBX_OK;
}

// Both images of a stereo frame into pinned staging at dst, rows at the pyramid's level-0
// pitch, the left at dst and the right at dst + img_bytes.  Called with h->mu held.
static void stage_frame(orbx_extractor* h, uint8_t* dst, size_t pitch0, size_t img_bytes,
                        const uint8_t* left, size_t stride_left, const uint8_t* right,
                        size_t stride_right, int width, int height, bool queued) {
    auto copy = [=](int v) {
        const uint8_t* img = v ? right : left;
        const size_t stride = v ? stride_right : stride_left;
        uint8_t* d = dst + (size_t)v * img_bytes;
        for (int y = 0; y < height; ++y)
            std::memcpy(d + (size_t)y * pitch0, img + (size_t)y * stride, (size_t)width);
    };
    const int stage_thread = STAGE_THREAD;
    if (stage_thread == 2 || (stage_thread == 1 && queued)) {
        if (!h->stager) h->stager.reset(new OrbxStager());
        h->stager->post([=] { copy(1); });
        copy(0);
        h->stager->wait();
    } else {
        copy(0);
        copy(1);
    }
}

// orbx_stereo_frame_view on the caller's own handle (one graph replay).
static orbx_status stereo_frame_solo(orbx_extractor* h, const uint8_t* left, size_t stride_left,
                                     const uint8_t* right, size_t stride_right, int width,
                                     int height, float mbf, float mb,
                                     orbx_stereo_frame_out* out) {
    std::lock_guard<std::mutex> lk(h->mu);
    orbx_status s = ensure_workspace(h, width, height, 2);
    if (s != ORBX_OK) return s;
    hipStream_t st = h->stream;
    const LevelGeom& L0 = h->hg.lv[0];
    const size_t pitch0 = (size_t)L0.pitch, img_bytes = pitch0 * (size_t)height;
    const size_t KC = (size_t)h->hg.kp_cap;
    // outputs of both images: [nkp | kps[.][KC] | desc[.][KC][32]] (the handle's output block,
    // two images of its capacity), the pair's stereo block [nvalid | uRight[KC] | depth[KC]]
    // at o_stereo; one DMA back when the block holds just the two images, else two
    const size_t o_kps = (size_t)((uint8_t*)h->d_kps.p - (uint8_t*)h->d_outs.p);
    const size_t o_desc = (size_t)((uint8_t*)h->d_desc.p - (uint8_t*)h->d_outs.p);
    const size_t o_end = o_desc + 2 * KC * 32;
    const size_t so_u = 256, so_d = so_u + KC * 4, s_end = so_d + KC * 4;
    const size_t o_s = h->o_stereo;
    const bool one_dma = h->cap_batch == 2;
    if (!ensure_pinned(h->h_out, h->h_out_n, o_s + s_end)) return ORBX_ERR_DEVICE;
    if (!ensure_pinned(h->h_in, h->h_in_n, 2 * img_bytes)) return ORBX_ERR_DEVICE;
    stage_frame(h, h->h_in, pitch0, img_bytes, left, stride_left, right, stride_right, width,
                height, false);
    uint8_t* d_l0 = h->d_pyr.as<uint8_t>() + L0.off;   // image 0's level-0 slot
    const size_t pyrb = (size_t)h->hg.pyr_bytes;
    if (!order_after_last(h, st)) return ORBX_ERR_DEVICE;
    uint8_t* dso = h->d_outs.as<uint8_t>() + o_s;
    const ExtractLaunch a = extract_launch(h, nullptr, nullptr, 2, 2, 0, 0);
    StereoLaunch sa;   // pair 0 = (image 0, image 1) of this handle
    s = stereo_launch_args(h, h, 1, 0, 1, mbf, mb, (float*)(dso + so_u), (float*)(dso + so_d),
                           (int*)dso, st, sa);
    if (s != ORBX_OK) return s;
    // the device sequence: both images into their level-0 slots by one 2-D DMA (a row = one
    // image; an image DMA'd ahead of the graph while the other is staged measured the same at
    // one session and slower at eight: one more submission), the two-image extraction, the
    // stereo match, the outputs back
    auto enqueue = [&](const ExtractLaunch& ea) {
        bool ok = HIPOK(hipMemcpy2DAsync(d_l0, pyrb, h->h_in, img_bytes, img_bytes, 2,
                                         hipMemcpyHostToDevice, st)) &&
                  HIPOK(launch_extract(ea, st)) && HIPOK(launch_stereo(sa, st));
        if (one_dma)
            return ok && HIPOK(hipMemcpyAsync(h->h_out, h->d_outs.p, o_s + s_end,
                                              hipMemcpyDeviceToHost, st));
        return ok &&
               HIPOK(hipMemcpyAsync(h->h_out, h->d_outs.p, o_end, hipMemcpyDeviceToHost, st)) &&
               HIPOK(hipMemcpyAsync(h->h_out + o_s, dso, s_end, hipMemcpyDeviceToHost, st));
    };
    uint32_t mbf_bits, mb_bits;
    std::memcpy(&mbf_bits, &mbf, 4);
    std::memcpy(&mb_bits, &mb, 4);
    const bool graph =
        EXTRACT_GRAPH && !h->timer.on &&
        extract1_graph(h, a, st, width, height, enqueue, h->g2, h->g2key,
                       {h->d_sscr.p, (const void*)(uintptr_t)mbf_bits,
                        (const void*)(uintptr_t)mb_bits, (const void*)(uintptr_t)one_dma});
    if (!(graph ? HIPOK(hipGraphLaunch(h->g2, st)) : enqueue(a)) || !mark_done(h, st) ||
        !wait_done(h))
        return ORBX_ERR_DEVICE;
    h->last_batch = 2;
    h->last_valid = true;
    h->pyr_images = h->keep_pyr ? 2 : 0;
    ++h->serial;   // the stereo-frame pyramid contract (keep_pyr)
    h->last_n = -1;   // not the single-image state orbx_stereo_match expects
    const uint8_t* ho = h->h_out;
    std::memcpy(out->n, ho, 8);
    for (int v = 0; v < 2; ++v) {
        out->kps[v] = (const orbx_keypoint*)(ho + o_kps + (size_t)v * KC * sizeof(orbx_keypoint));
        out->desc[v] = ho + o_desc + (size_t)v * KC * 32;
    }
    std::memcpy(&out->n_valid, ho + o_s, 4);
    out->u_right = (const float*)(ho + o_s + so_u);
    out->depth = (const float*)(ho + o_s + so_d);
    return ORBX_OK;
}

orbx_status orbx_stereo_frame_view(orbx_extractor* h, const uint8_t* left, size_t stride_left,
                                   const uint8_t* right, size_t stride_right, int width,
                                   int height, float mbf, float mb, orbx_stereo_frame_out* out) {
    if (!h || !out || !left || !right || width <= 0 || height <= 0 ||
        stride_left < (size_t)width || stride_right < (size_t)width)
        return ORBX_ERR_INVALID;
    if (!FRAME_SERVER)
        return stereo_frame_solo(h, left, stride_left, right, stride_right, width, height, mbf,
                                 mb, out);
    FrameServer& fs = frame_server(h);
    frame_server_use(h, fs);
    const int inflight_max = FS_INFLIGHT;
    std::unique_lock<std::mutex> lk(fs.mu);
    if (fs.inflight == 0 && fs.n == 0) {   // alone on the device: on this handle
        ++fs.inflight;
        fs.stats.solo_calls++;
        lk.unlock();
        const orbx_status s = stereo_frame_solo(h, left, stride_left, right, stride_right, width,
                                                height, mbf, mb, out);
        lk.lock();
        --fs.inflight;
        fs.cv.notify_all();
        return s;
    }
    lk.unlock();
    FsBatch g{width, height, mbf, mb, 0, 0};
    {
        std::lock_guard<std::mutex> hl(h->mu);
        const orbx_status s = ensure_workspace(h, width, height, 1);   // the level-0 pitch
        if (s != ORBX_OK) return s;
        g.pitch0 = (size_t)h->hg.lv[0].pitch;
        g.img_bytes = g.pitch0 * (size_t)height;
    }
    auto same = [](const FsBatch& x, const FsBatch& y) {
        return x.width == y.width && x.height == y.height && x.pitch0 == y.pitch0 &&
               std::memcmp(&x.mbf, &y.mbf, 4) == 0 && std::memcmp(&x.mb, &y.mb, 4) == 0;
    };
    FsReq r{h};
    lk.lock();
    // join the batch being formed (after a full one, or one of another size or camera, goes)
    // (a batch opens in a block pair whose last batch has finished)
    fs.cv.wait(lk, [&] {
        return fs.n == 0 ? !fs.pair_busy[fs.blk] : fs.n < FS_MAX_FRAMES && same(fs.geo, g);
    });
    if (fs.n == 0) {   // open it: its blocks were last used by a batch that has finished
        const size_t bytes = 2 * FS_MAX_FRAMES * g.img_bytes;
        if (!HIPOK(hipSetDevice(h->device)) ||
            (!fs.cst && !HIPOK(hipStreamCreateWithFlags(&fs.cst, hipStreamNonBlocking))) ||
            (!fs.cev[fs.blk] &&
             !HIPOK(hipEventCreateWithFlags(&fs.cev[fs.blk], hipEventDisableTiming))) ||
            !ensure_pinned(fs.hin[fs.blk], fs.hin_n[fs.blk], bytes) ||
            !fs.dstage[fs.blk].ensure(bytes))
            return ORBX_ERR_DEVICE;
        fs.geo = g;
    }
    r.slot = fs.n++;
    r.blk = fs.blk;
    fs.req[r.slot] = &r;
    const size_t fofs = (size_t)r.slot * 2 * g.img_bytes;
    uint8_t* dst = fs.hin[r.blk] + fofs;
    uint8_t* ddst = fs.dstage[r.blk].as<uint8_t>() + fofs;
    lk.unlock();
    bool copied;
    {
        std::lock_guard<std::mutex> hl(h->mu);
        stage_frame(h, dst, g.pitch0, g.img_bytes, left, stride_left, right, stride_right, width,
                    height, true);
        copied = HIPOK(hipSetDevice(h->device)) &&
                 HIPOK(hipMemcpyAsync(ddst, dst, 2 * g.img_bytes, hipMemcpyHostToDevice, fs.cst));
    }
    lk.lock();
    if (!copied) r.st = ORBX_ERR_DEVICE;   // the batch still counts the slot
    ++fs.staged;
    fs.cv.notify_all();
    while (!r.done) {
        // only a frame of the batch being formed leads it (a frame whose batch already has a
        // lead waits for it, instead of leading someone else's batch and holding its reader
        // slot meanwhile)
        if (r.taken || fs.inflight >= inflight_max || fs.n == 0 || fs.staged < fs.n) {
            fs.cv.wait(lk);
            continue;
        }
        // lead: the batch being formed goes, the next one forms in the other block pair
        const int m = fs.n, blk = fs.blk;
        FsReq* take[FS_MAX_FRAMES];
        std::copy(fs.req, fs.req + m, take);
        for (int i = 0; i < m; ++i) take[i]->taken = true;
        // every frame's copy is on the stream by now (each was issued before its `staged`)
        const bool recorded = HIPOK(hipEventRecord(fs.cev[blk], fs.cst));
        const FsBatch bg = fs.geo;
        fs.n = fs.staged = 0;
        fs.blk ^= 1;
        ++fs.inflight;
        fs.pair_busy[blk] = true;
        fs.stats.batches++;
        fs.stats.served_frames += m;
        fs.stats.batches_of_size[m]++;
        fs.stats.batches_per_pair[blk]++;
        fs.stats.peak_inflight = std::max(fs.stats.peak_inflight, fs.inflight);
        fs.stats.resident = 1;
        fs.cv.notify_all();
        fs.cv.wait(lk, [&] { return fs.readers[blk] == 0; });   // two batches ago: copied out
        lk.unlock();
        orbx_status bs = recorded ? run_served(fs, take[0]->h, m, blk, bg) : ORBX_ERR_DEVICE;
        for (int i = 0; i < m; ++i)
            if (take[i]->st != ORBX_OK) bs = take[i]->st;   // a frame's copy failed
        lk.lock();
        for (int i = 0; i < m; ++i) {
            take[i]->st = bs;
            take[i]->done = true;
        }
        if (bs == ORBX_OK) fs.readers[blk] += m;
        --fs.inflight;
        fs.pair_busy[blk] = false;
        fs.cv.notify_all();
    }
    lk.unlock();
    const orbx_status s = r.st == ORBX_OK ? copy_served(fs, r, g, out) : r.st;
    if (r.st == ORBX_OK) {
        lk.lock();
        --fs.readers[r.blk];
        fs.cv.notify_all();
    }
    return s;
}

uint64_t orbx_extractor_serial(const orbx_extractor* h) {
    if (!h) return 0;
    std::lock_guard<std::mutex> lk(h->mu);
    return h->serial;
}

orbx_status orbx_extractor_host_pyramid(orbx_extractor* h, int on) {
    if (!h) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(h->mu);
    h->host_pyr = on != 0;
    if (!h->host_pyr) h->host_pyr_ok = false;
    return ORBX_OK;
}

orbx_status orbx_host_pyramid_view(const orbx_extractor* h, orbx_host_pyramid* out) {
    if (!h || !out) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(h->mu);
    if (!h->host_pyr_ok || !h->have_geom || !h->h_pyr) return ORBX_ERR_STATE;
    std::memset(out, 0, sizeof(*out));
    out->nlevels = h->hg.nlevels;
    for (int l = 0; l < h->hg.nlevels && l < 16; ++l) {
        const LevelGeom& L = h->hg.lv[l];
        out->data[l] = h->h_pyr + L.off;
        out->width[l] = L.w;
        out->height[l] = L.h;
        out->step[l] = (size_t)L.pitch;
    }
    return ORBX_OK;
}

orbx_status orbx_extractor_keep_pyramid(orbx_extractor* h, int on) {
    if (!h) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(h->mu);
    h->keep_pyr = on != 0;
    return ORBX_OK;
}

orbx_status orbx_frame_server_get_stats(const orbx_extractor* h, orbx_frame_server_stats* out,
                                        int reset) {
    if (!h || !out) return ORBX_ERR_INVALID;
    FrameServer& fs = frame_server(h);
    std::lock_guard<std::mutex> lk(fs.mu);
    *out = fs.stats;
    out->users = fs.users;
    if (reset) {
        const int32_t resident = fs.stats.resident;
        fs.stats = orbx_frame_server_stats{};
        fs.stats.resident = resident;
    }
    return ORBX_OK;
}

orbx_status orbx_frame_server_release(const orbx_extractor* h) {
    if (!h) return ORBX_ERR_INVALID;
    FrameServer& fs = frame_server(h);
    std::lock_guard<std::mutex> lk(fs.mu);
    if (!fs.idle()) return ORBX_ERR_STATE;
    fs.release_resources();
    return ORBX_OK;
}

static orbx_status copy_level(orbx_extractor* h, const DevBuf& buf, int index, int level,
                              uint8_t* out, int* width, int* height, bool blurred = false) {
    if (!h) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(h->mu);
    if (level < 0 || level >= h->hg.nlevels || index < 0) return ORBX_ERR_INVALID;
    // the raw pyramid of images [0, pyr_images); the blurred one of a full last call only
    if (index >= h->pyr_images || (blurred && (!h->last_valid || index >= h->last_batch)))
        return ORBX_ERR_STATE;
    const LevelGeom& lv = h->hg.lv[level];
    if (width) *width = lv.w;
    if (height) *height = lv.h;
    if (!out) return ORBX_OK;
    (void)hipSetDevice(h->device);
    const uint8_t* src = buf.as<uint8_t>() + (size_t)index * h->hg.pyr_bytes + lv.off;
    if (blurred) {
        // 16x4 tiles (blur_off): the level's whole bands to the host, then de-tiled
        const size_t bytes = (size_t)lv.pitch * align_up((size_t)lv.h, 4);
        std::vector<uint8_t> tiles(bytes);
        if (!order_after_last(h, h->stream) ||
            !HIPOK(hipMemcpyAsync(tiles.data(), src, bytes, hipMemcpyDeviceToHost, h->stream)) ||
            !HIPOK(hipStreamSynchronize(h->stream)))
            return ORBX_ERR_DEVICE;
        for (int y = 0; y < lv.h; ++y)
            for (int x = 0; x < lv.w; x += 16)
                std::memcpy(out + (size_t)y * lv.w + x, tiles.data() + blur_off(x, y, lv.pitch, lv.h),
                            (size_t)std::min(16, lv.w - x));
        return ORBX_OK;
    }
    if (!order_after_last(h, h->stream) ||
        !HIPOK(hipMemcpy2DAsync(out, lv.w, src, lv.pitch, lv.w, lv.h, hipMemcpyDeviceToHost, h->stream)) ||
        !HIPOK(hipStreamSynchronize(h->stream)))
        return ORBX_ERR_DEVICE;
    return ORBX_OK;
}

orbx_status orbx_pyramid_level(orbx_extractor* h, int index, int level, uint8_t* out, int* width,
                               int* height) {
    if (!h) return ORBX_ERR_INVALID;
    return copy_level(h, h->d_pyr, index, level, out, width, height);
}

orbx_status orbx_blur_level(orbx_extractor* h, int index, int level, uint8_t* out, int* width,
                            int* height) {
    if (!h) return ORBX_ERR_INVALID;
    return copy_level(h, h->d_blur, index, level, out, width, height, true);
}

orbx_status orbx_extractor_prepare(orbx_extractor* h, int width, int height, int batch,
                                   int* kp_cap) {
    if (!h || width <= 0 || height <= 0 || batch < 1) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(h->mu);
    orbx_status s = ensure_workspace(h, width, height, batch);
    if (s == ORBX_OK && kp_cap) *kp_cap = h->hg.kp_cap;
    return s;
}

orbx_status orbx_extract_batch_device(orbx_extractor* h, const uint8_t* d_imgs, int batch,
                                      int width, int height, size_t stride, size_t batch_stride,
                                      void* stream) {
    if (!h || !d_imgs || batch < 1 || width <= 0 || height <= 0 || stride < (size_t)width)
        return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(h->mu);
    orbx_status s = ensure_workspace(h, width, height, batch);
    if (s != ORBX_OK) return s;
    return run_extract(h, d_imgs, nullptr, batch, batch, stride, batch_stride, pick_stream(h, stream));
}

orbx_status orbx_batch_input_view(orbx_extractor* h, int width, int height, int batch,
                                  uint8_t** d_level0, size_t* pitch, size_t* image_stride) {
    if (!h || width <= 0 || height <= 0 || batch < 1 || !d_level0) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(h->mu);
    orbx_status s = ensure_workspace(h, width, height, batch);
    if (s != ORBX_OK) return s;
    *d_level0 = h->d_pyr.as<uint8_t>() + h->hg.lv[0].off;
    if (pitch) *pitch = (size_t)h->hg.lv[0].pitch;
    if (image_stride) *image_stride = (size_t)h->hg.pyr_bytes;
    return ORBX_OK;
}

orbx_status orbx_extract_batch_resident(orbx_extractor* h, int batch, void* stream) {
    if (!h || batch < 1) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(h->mu);
    if (!h->have_geom) return ORBX_ERR_STATE;
    if (batch > h->cap_batch) return ORBX_ERR_INVALID;
    if (!HIPOK(hipSetDevice(h->device))) return ORBX_ERR_DEVICE;
    return run_extract(h, nullptr, nullptr, batch, batch, 0, 0, pick_stream(h, stream));
}

orbx_status orbx_stereo_frames_resident(orbx_extractor* h, int batch, float mbf, float mb,
                                        float* d_uRight, float* d_depth, int32_t* d_nvalid,
                                        void* stream) {
    if (!h || batch < 1 || !d_uRight || !d_depth) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(h->mu);
    if (!h->have_geom) return ORBX_ERR_STATE;
    if (2 * batch > h->cap_batch) return ORBX_ERR_INVALID;
    if (!HIPOK(hipSetDevice(h->device))) return ORBX_ERR_DEVICE;
    hipStream_t st = pick_stream(h, stream);
    orbx_status s = run_extract(h, nullptr, nullptr, 2 * batch, 2 * batch, 0, 0, st);
    if (s != ORBX_OK) return s;
    return run_stereo(h, h, batch, 0, batch, mbf, mb, d_uRight, d_depth, d_nvalid, st);
}

orbx_status orbx_batch_view_get(const orbx_extractor* h, orbx_batch_view* v) {
    if (!h || !v) return ORBX_ERR_STATE;
    // a snapshot under the handle's lock: an extraction running on another thread cannot
    // change the batch size or reallocate the buffers halfway through the copy
    std::lock_guard<std::mutex> lk(h->mu);
    if (!h->last_valid) return ORBX_ERR_STATE;
    memset(v, 0, sizeof(*v));
    v->batch = h->last_batch;
    v->kp_cap = h->hg.kp_cap;
    v->kps = h->d_kps.as<orbx_keypoint>();
    v->desc = h->d_desc.as<uint8_t>();
    v->nkp = h->d_nkp.as<int32_t>();
    v->pyramid = h->d_pyr.as<uint8_t>();
    v->pyr_bytes = (size_t)h->hg.pyr_bytes;
    for (int l = 0; l < h->hg.nlevels && l < 16; ++l) {
        v->level_w[l] = h->hg.lv[l].w;
        v->level_h[l] = h->hg.lv[l].h;
        v->level_pitch[l] = h->hg.lv[l].pitch;
        v->level_off[l] = (size_t)h->hg.lv[l].off;
    }
    return ORBX_OK;
}

orbx_status orbx_batch_fetch(orbx_extractor* h, int first, int count, int32_t* nkp,
                             orbx_keypoint* kps, uint8_t* desc) {
    if (!h || first < 0 || count < 0) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(h->mu);
    if (!h->last_valid || first + count > h->last_batch) return ORBX_ERR_INVALID;
    (void)hipSetDevice(h->device);
    // after the handle's last launches (on whatever stream), on the handle's own stream
    hipStream_t st = h->stream;
    if (!order_after_last(h, st)) return ORBX_ERR_DEVICE;
    const size_t KC = (size_t)h->hg.kp_cap;
    if (nkp && !HIPOK(hipMemcpyAsync(nkp, h->d_nkp.as<int32_t>() + first, (size_t)count * 4,
                                     hipMemcpyDeviceToHost, st)))
        return ORBX_ERR_DEVICE;
    if (kps && !HIPOK(hipMemcpyAsync(kps, h->d_kps.as<orbx_keypoint>() + first * KC,
                                     (size_t)count * KC * sizeof(orbx_keypoint),
                                     hipMemcpyDeviceToHost, st)))
        return ORBX_ERR_DEVICE;
    if (desc && !HIPOK(hipMemcpyAsync(desc, h->d_desc.as<uint8_t>() + first * KC * 32,
                                      (size_t)count * KC * 32, hipMemcpyDeviceToHost, st)))
        return ORBX_ERR_DEVICE;
    return HIPOK(hipStreamSynchronize(st)) ? ORBX_OK : ORBX_ERR_DEVICE;
}

orbx_status orbx_stereo_match(orbx_extractor* left, orbx_extractor* right, float mbf, float mb,
                              float* uRight, float* depth, int n_left, int* n_valid) {
    if (!left || !right || left == right) return ORBX_ERR_INVALID;
    // both handles: the right pyramid is read, so neither may be re-extracted meanwhile
    std::scoped_lock lk(left->mu, right->mu);
    if (!left->last_valid || !right->last_valid || left->last_batch != 1 || right->last_batch != 1)
        return ORBX_ERR_STATE;
    (void)hipSetDevice(left->device);
    const size_t KC = (size_t)left->hg.kp_cap;
    // the results in one device block, copied back by one DMA into one pinned block:
    // [nvalid | uRight[KC] | depth[KC]]; the left keypoint count is the handle's own (its
    // orbx_extract returned it)
    const size_t o_u = 256, o_d = o_u + KC * 4;
    if (!left->d_uR.ensure(o_d + KC * 4)) return ORBX_ERR_DEVICE;
    if (!ensure_pinned(left->h_out, left->h_out_n, o_d + KC * 4)) return ORBX_ERR_DEVICE;
    uint8_t* dso = left->d_uR.as<uint8_t>();
    hipStream_t st = left->stream;
    orbx_status s = run_stereo(left, right, 1, 0, 0, mbf, mb, (float*)(dso + o_u),
                               (float*)(dso + o_d), (int*)dso, st);
    if (s != ORBX_OK) return s;
    uint8_t* ho = left->h_out;
    const bool known = left->last_n >= 0;   // else a batched call of one image set the state
    if (!HIPOK(hipMemcpyAsync(ho, dso, o_d + KC * 4, hipMemcpyDeviceToHost, st)) ||
        (!known && !HIPOK(hipMemcpyAsync(ho + 8, left->d_nkp.p, 4, hipMemcpyDeviceToHost, st))) ||
        !mark_done(left, st) || !wait_done(left))
        return ORBX_ERR_DEVICE;
    int n = left->last_n;
    if (!known) std::memcpy(&n, ho + 8, 4);
    int nv = 0;
    std::memcpy(&nv, ho, 4);
    const int m = std::min(n, n_left);
    if (m > 0) {
        if (uRight) std::memcpy(uRight, ho + o_u, (size_t)m * 4);
        if (depth) std::memcpy(depth, ho + o_d, (size_t)m * 4);
    }
    if (n_valid) *n_valid = nv;
    return n > n_left ? ORBX_ERR_CAPACITY : ORBX_OK;
}

orbx_status orbx_stereo_match_batch_device(orbx_extractor* left, orbx_extractor* right, float mbf,
                                           float mb, float* d_uRight, float* d_depth,
                                           int32_t* d_nvalid, void* stream) {
    if (!left || !right || left == right || !d_uRight || !d_depth) return ORBX_ERR_INVALID;
    std::scoped_lock lk(left->mu, right->mu);
    (void)hipSetDevice(left->device);
    if (left->last_batch != right->last_batch) return ORBX_ERR_INVALID;
    return run_stereo(left, right, left->last_batch, 0, 0, mbf, mb, d_uRight, d_depth, d_nvalid,
                      pick_stream(left, stream));
}

orbx_status orbx_stereo_frames_device(orbx_extractor* h, const uint8_t* d_left,
                                      const uint8_t* d_right, int batch, int width, int height,
                                      size_t stride, size_t batch_stride, float mbf, float mb,
                                      float* d_uRight, float* d_depth, int32_t* d_nvalid,
                                      void* stream) {
    if (!h || !d_left || !d_right || batch < 1 || width <= 0 || height <= 0 ||
        stride < (size_t)width || !d_uRight || !d_depth)
        return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(h->mu);
    orbx_status s = ensure_workspace(h, width, height, 2 * batch);
    if (s != ORBX_OK) return s;
    hipStream_t st = pick_stream(h, stream);
    s = run_extract(h, d_left, d_right, batch, 2 * batch, stride, batch_stride, st);
    if (s != ORBX_OK) return s;
    return run_stereo(h, h, batch, 0, batch, mbf, mb, d_uRight, d_depth, d_nvalid, st);
}

}  // extern "C"
