// orbx_match_capi.hip — the extern "C" matcher boundary (include/orbx_match.h).
//
// Host side: argument validation, packing of the caller's arrays into one staging block
// (one H2D copy per call), the launch sequence on the matcher's stream, and the host-only
// tails of the reference methods (SearchBySim3's agreement check :1363-1379,
// SearchForInitialization's vbPrevMatched update :555-558, the (idx1, idx2) pair list of
// SearchForTriangulation :861-869).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/orbx_match.h"
#include "orbx_host.h"
#include "orbx_kernels.h"
#include "orbx_match_kernels.h"

using namespace orbx;

static_assert((int)ORBX_MK_COUNT <= (int)orbx::K_COUNT, "the matcher timer shares KernelTimer's slots");

struct orbx_matcher {
    orbx_matcher_params prm;
    hipStream_t stream = nullptr;
    int ncu = 256;                     // compute units of the device (BF chunk sizing)
    DevBuf d_in, d_out, d_aux, d_proj, d_bf;
    int* d_err = nullptr;
    std::vector<uint8_t> staging;
    KernelTimer timer;
    std::mutex mu;
    // recorded after the last brute-force launch (its partial-result scratch d_bf is shared by
    // every call): a call on another stream waits for it before reusing the scratch
    hipEvent_t bf_done = nullptr;
    hipStream_t bf_stream = nullptr;
    bool have_bf = false;
    int bf_kernel = ORBX_BF_MFMA;
};

namespace {

constexpr int MAX_FEAT = 32768;        // per featureset (on-chip claim / state arrays)
constexpr int MAX_POS = 1 << 23;       // grid CSR positions in the 32-bit search keys

size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

// Accumulates the caller's arrays into one host block copied to the device at once.
struct Packer {
    std::vector<uint8_t>& h;
    explicit Packer(std::vector<uint8_t>& buf) : h(buf) { h.clear(); }
    size_t reserve(size_t bytes) {
        const size_t off = align256(h.size());
        h.resize(off + std::max<size_t>(bytes, 4), 0);
        return off;
    }
    size_t add(const void* p, size_t bytes) {
        const size_t off = reserve(bytes);
        if (bytes && p) std::memcpy(h.data() + off, p, bytes);
        return off;
    }
    template <class T> T* at(size_t off) { return (T*)(h.data() + off); }
};

bool valid_nodes(const orbx_featureset* f) {
    if (f->n_nodes < 0) return false;
    if (f->n_nodes == 0) return true;
    if (!f->node_id || !f->node_off || !f->node_feat) return false;
    for (int j = 0; j < f->n_nodes; ++j) {
        if (f->node_off[j + 1] < f->node_off[j]) return false;
        if (j > 0 && f->node_id[j] <= f->node_id[j - 1]) return false;
    }
    if (f->node_off[0] < 0) return false;
    for (int k = f->node_off[0]; k < f->node_off[f->n_nodes]; ++k)
        if (f->node_feat[k] < 0 || f->node_feat[k] >= f->n) return false;
    return true;
}

bool valid_grid(const orbx_featureset* f) {
    if (f->grid_cols <= 0 || f->grid_rows <= 0 || !f->grid_off) return false;
    const long long cells = (long long)f->grid_cols * f->grid_rows;
    if (cells > (1 << 20) || f->grid_off[0] != 0) return false;
    for (long long c = 0; c < cells; ++c)
        if (f->grid_off[c + 1] < f->grid_off[c]) return false;
    const int tot = f->grid_off[cells];
    if (tot > MAX_POS || (tot > 0 && !f->grid_feat)) return false;
    for (int k = 0; k < tot; ++k)
        if (f->grid_feat[k] < 0 || f->grid_feat[k] >= f->n) return false;
    return true;
}

bool valid_feat(const orbx_featureset* f, bool nodes, bool grid) {
    if (!f || f->n < 0 || f->n > MAX_FEAT) return false;
    if (f->n > 0 && (!f->keys || !f->desc)) return false;
    if (nodes && !valid_nodes(f)) return false;
    if (grid && !valid_grid(f)) return false;
    return true;
}

// A keyframe database built from host featuresets (device offsets inside the staging block).
struct DbOffsets {
    size_t feat_off, keys, desc, u_right, flag, node_off, node_id, node_feat_off, node_feat;
    int nkf, max_feat;
};

DbOffsets pack_db(Packer& P, const orbx_featureset* const* fs, const uint8_t* const* flags,
                  int nkf) {
    DbOffsets o{};
    o.nkf = nkf;
    int nf = 0, nn = 0, nnf = 0;
    for (int k = 0; k < nkf; ++k) {
        nf += fs[k]->n;
        nn += fs[k]->n_nodes;
        if (fs[k]->n_nodes > 0) nnf += fs[k]->node_off[fs[k]->n_nodes] - fs[k]->node_off[0];
        o.max_feat = std::max(o.max_feat, fs[k]->n);
    }
    o.feat_off = P.reserve(4 * (nkf + 1));
    o.keys = P.reserve(sizeof(orbx_keypoint) * (size_t)nf);
    o.desc = P.reserve(32 * (size_t)nf);
    o.u_right = P.reserve(4 * (size_t)nf);
    o.flag = P.reserve((size_t)nf);
    o.node_off = P.reserve(4 * (nkf + 1));
    o.node_id = P.reserve(4 * (size_t)nn);
    o.node_feat_off = P.reserve(4 * ((size_t)nn + 1));
    o.node_feat = P.reserve(4 * (size_t)nnf);
    int f0 = 0, n0 = 0, e0 = 0;
    for (int k = 0; k < nkf; ++k) {
        const orbx_featureset* f = fs[k];
        P.at<int32_t>(o.feat_off)[k] = f0;
        P.at<int32_t>(o.node_off)[k] = n0;
        if (f->n > 0) {
            std::memcpy(P.at<orbx_keypoint>(o.keys) + f0, f->keys, sizeof(orbx_keypoint) * f->n);
            std::memcpy(P.at<uint8_t>(o.desc) + 32 * (size_t)f0, f->desc, 32 * (size_t)f->n);
            float* ur = P.at<float>(o.u_right) + f0;
            for (int i = 0; i < f->n; ++i) ur[i] = f->u_right ? f->u_right[i] : -1.0f;
            uint8_t* fl = P.at<uint8_t>(o.flag) + f0;
            for (int i = 0; i < f->n; ++i) fl[i] = (flags && flags[k]) ? (flags[k][i] != 0) : 0;
        }
        for (int j = 0; j < f->n_nodes; ++j) {
            P.at<uint32_t>(o.node_id)[n0 + j] = f->node_id[j];
            P.at<int32_t>(o.node_feat_off)[n0 + j] = e0 + f->node_off[j] - f->node_off[0];
        }
        if (f->n_nodes > 0) {
            const int cnt = f->node_off[f->n_nodes] - f->node_off[0];
            std::memcpy(P.at<int32_t>(o.node_feat) + e0, f->node_feat + f->node_off[0], 4 * (size_t)cnt);
            e0 += cnt;
        }
        f0 += f->n;
        n0 += f->n_nodes;
    }
    P.at<int32_t>(o.feat_off)[nkf] = f0;
    P.at<int32_t>(o.node_off)[nkf] = n0;
    P.at<int32_t>(o.node_feat_off)[n0] = e0;
    return o;
}

orbx_kf_db dev_db(const DbOffsets& o, uint8_t* base) {
    orbx_kf_db d{};
    d.nkf = o.nkf;
    d.max_feat = o.max_feat;
    d.feat_off = (const int32_t*)(base + o.feat_off);
    d.keys = (const orbx_keypoint*)(base + o.keys);
    d.desc = base + o.desc;
    d.u_right = (const float*)(base + o.u_right);
    d.flag = base + o.flag;
    d.node_off = (const int32_t*)(base + o.node_off);
    d.node_id = (const uint32_t*)(base + o.node_id);
    d.node_feat_off = (const int32_t*)(base + o.node_feat_off);
    d.node_feat = (const int32_t*)(base + o.node_feat);
    return d;
}

// A single featureset with its grid (projection searches).
struct FeatOffsets {
    size_t keys, desc, u_right, grid_off, grid_feat;
};

FeatOffsets pack_feat(Packer& P, const orbx_featureset* f) {
    FeatOffsets o{};
    o.keys = P.add(f->keys, sizeof(orbx_keypoint) * (size_t)f->n);
    o.desc = P.add(f->desc, 32 * (size_t)f->n);
    o.u_right = P.reserve(4 * (size_t)f->n);
    float* ur = P.at<float>(o.u_right);
    for (int i = 0; i < f->n; ++i) ur[i] = f->u_right ? f->u_right[i] : -1.0f;
    const size_t cells = (size_t)f->grid_cols * f->grid_rows;
    o.grid_off = P.add(f->grid_off, 4 * (cells + 1));
    o.grid_feat = P.add(f->grid_feat, 4 * (size_t)f->grid_off[cells]);
    return o;
}

orbx_featureset dev_feat(const orbx_featureset* f, const FeatOffsets& o, uint8_t* base) {
    orbx_featureset d = *f;
    d.keys = (const orbx_keypoint*)(base + o.keys);
    d.desc = base + o.desc;
    d.u_right = (const float*)(base + o.u_right);
    d.n_nodes = 0;
    d.node_id = nullptr;
    d.node_off = nullptr;
    d.node_feat = nullptr;
    d.grid_off = (const int32_t*)(base + o.grid_off);
    d.grid_feat = (const int32_t*)(base + o.grid_feat);
    return d;
}

orbx_status upload(orbx_matcher* m) {
    if (!m->d_in.ensure(m->staging.size())) return ORBX_ERR_DEVICE;
    if (!HIPOK(hipMemcpyAsync(m->d_in.p, m->staging.data(), m->staging.size(),
                              hipMemcpyHostToDevice, m->stream)))
        return ORBX_ERR_DEVICE;
    if (!HIPOK(hipMemsetAsync(m->d_err, 0, sizeof(int), m->stream))) return ORBX_ERR_DEVICE;
    return ORBX_OK;
}

// Copies `bytes` from the device output block to `dst` and waits; checks the error word.
orbx_status finish(orbx_matcher* m, void* dst, const void* src, size_t bytes) {
    int err = 0;
    if (bytes && !HIPOK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, m->stream)))
        return ORBX_ERR_DEVICE;
    if (!HIPOK(hipMemcpyAsync(&err, m->d_err, sizeof(int), hipMemcpyDeviceToHost, m->stream)) ||
        !HIPOK(hipStreamSynchronize(m->stream)))
        return ORBX_ERR_DEVICE;
    return err ? ORBX_ERR_CAPACITY : ORBX_OK;
}

orbx_status bow_common(orbx_matcher* m, const orbx_featureset* a, const uint8_t* va,
                       const orbx_featureset* b, const uint8_t* vb, int kf_kf, int32_t* out,
                       int32_t* nmatches) {
    if (!m || !out || !nmatches || !va || (kf_kf && !vb)) return ORBX_ERR_INVALID;
    if (!valid_feat(a, true, false) || !valid_feat(b, true, false)) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(m->mu);
    if (!HIPOK(hipSetDevice(m->prm.device))) return ORBX_ERR_DEVICE;
    Packer P(m->staging);
    const orbx_featureset* fa[1] = {a};
    const orbx_featureset* fb[1] = {b};
    const uint8_t* la[1] = {va};
    const uint8_t* lb[1] = {vb};
    const DbOffsets oa = pack_db(P, fa, la, 1), ob = pack_db(P, fb, lb, 1);
    orbx_status s = upload(m);
    if (s != ORBX_OK) return s;
    const int nout = kf_kf ? a->n : b->n;
    if (!m->d_out.ensure(4 * ((size_t)nout + 64))) return ORBX_ERR_DEVICE;
    BowLaunch L{};
    L.A = dev_db(oa, m->d_in.as<uint8_t>());
    L.B = dev_db(ob, m->d_in.as<uint8_t>());
    L.a_fixed = 1;
    L.b_fixed = 1;
    L.kf_kf = kf_kf;
    L.njobs = 1;
    L.ratio = m->prm.nnratio;
    L.check_ori = m->prm.check_orientation;
    L.out = m->d_out.as<int32_t>() + 64;
    L.out_stride = nout;
    L.nmatches = m->d_out.as<int32_t>();
    L.err = m->d_err;
    if (bow_lds_bytes(L) > MATCH_MAX_LDS) return ORBX_ERR_UNSUPPORTED;
    hipEvent_t e = m->timer.start(m->stream);
    if (!HIPOK(launch_bow(L, m->stream))) return ORBX_ERR_DEVICE;
    m->timer.stop(ORBX_MK_BOW, e, m->stream);
    std::vector<int32_t> res((size_t)nout + 64);
    s = finish(m, res.data(), m->d_out.p, 4 * res.size());
    if (s != ORBX_OK) return s;
    std::memcpy(out, res.data() + 64, 4 * (size_t)nout);
    *nmatches = res[0];
    return ORBX_OK;
}

orbx_status proj_common(orbx_matcher* m, int mode, const orbx_featureset* T,
                        const uint8_t* claimed, const uint8_t* qdesc, const orbx_proj_query* q,
                        int nq, const float* inv_sigma2, int nlevels, int orb_dist, int32_t* out,
                        int32_t* nmatches, const uint8_t* qflags = nullptr, int flags = 0) {
    if (!m || !out || !nmatches || nq < 0 || nq > (1 << 22)) return ORBX_ERR_INVALID;
    if (nq > 0 && (!qdesc || !q)) return ORBX_ERR_INVALID;
    if (!valid_feat(T, false, true)) return ORBX_ERR_INVALID;
    if (mode == ORBX_PROJ_FUSE && (!inv_sigma2 || nlevels <= 0)) return ORBX_ERR_INVALID;
    if (nlevels > MATCH_MAX_LEVELS) return ORBX_ERR_UNSUPPORTED;
    if (proj_mode_greedy(mode) && proj_resolve_lds_bytes(mode, T->n, nq) > MATCH_MAX_LDS)
        return ORBX_ERR_UNSUPPORTED;
    std::lock_guard<std::mutex> lk(m->mu);
    if (!HIPOK(hipSetDevice(m->prm.device))) return ORBX_ERR_DEVICE;
    Packer P(m->staging);
    const FeatOffsets ot = pack_feat(P, T);
    const size_t oq = P.add(q, sizeof(orbx_proj_query) * (size_t)nq);
    const size_t od = P.add(qdesc, 32 * (size_t)nq);
    size_t oc = 0, of = 0;
    if (claimed) oc = P.add(claimed, (size_t)T->n);
    if (qflags) of = P.add(qflags, (size_t)nq);
    orbx_status s = upload(m);
    if (s != ORBX_OK) return s;
    // outputs: nmatches(64 ints) | out[nq] | hist[32] | top2[nq] | bins[nq] | cand | ncand
    const size_t o_out = 256, o_hist = align256(o_out + 4 * (size_t)nq),
                 o_top = align256(o_hist + 128), o_bin = align256(o_top + 16 * (size_t)nq),
                 o_cand = align256(o_bin + (size_t)nq),
                 o_nc = align256(o_cand + 8 * PROJ_K * (size_t)nq),
                 o_end = align256(o_nc + 4 * (size_t)nq);
    if (!m->d_out.ensure(o_end)) return ORBX_ERR_DEVICE;
    uint8_t* base = m->d_in.as<uint8_t>();
    uint8_t* ob = m->d_out.as<uint8_t>();
    ProjLaunch L{};
    L.mode = mode;
    L.T = dev_feat(T, ot, base);
    L.njobs = 1;
    L.max_t = T->n;
    L.qdesc = base + od;
    L.q = (const orbx_proj_query*)(base + oq);
    L.nq = nq;
    for (int l = 0; l < MATCH_MAX_LEVELS; ++l)
        L.inv_sigma2[l] = (inv_sigma2 && l < nlevels) ? inv_sigma2[l] : 0.f;
    L.orb_dist = orb_dist;
    L.ratio = m->prm.nnratio;
    L.check_ori = m->prm.check_orientation;
    L.claimed_in = claimed ? base + oc : nullptr;
    L.qflags = qflags ? base + of : nullptr;
    L.prefilter = (flags & ORBX_PROJ_PREFILTER) != 0;
    L.out = (int32_t*)(ob + o_out);
    L.top2 = (int4*)(ob + o_top);
    L.cand = (int2*)(ob + o_cand);
    L.ncand = (int32_t*)(ob + o_nc);
    L.out_bin = (int8_t*)(ob + o_bin);
    L.hist = (int32_t*)(ob + o_hist);
    L.nmatches = (int32_t*)ob;
    L.err = m->d_err;
    if (nq == 0) {
        *nmatches = 0;
        return ORBX_OK;
    }
    if (!HIPOK(launch_proj(L, m->stream, &m->timer))) return ORBX_ERR_DEVICE;
    std::vector<int32_t> res(64 + (size_t)nq);
    s = finish(m, res.data(), ob, 4 * res.size());
    if (s != ORBX_OK) return s;
    std::memcpy(out, res.data() + 64, 4 * (size_t)nq);
    *nmatches = res[0];
    return ORBX_OK;
}

}  // namespace

extern "C" {

orbx_status orbx_matcher_create(const orbx_matcher_params* params, orbx_matcher** out) {
    if (!out) return ORBX_ERR_INVALID;
    *out = nullptr;
    orbx_matcher_params p{0.6f, 1, 0};
    if (params) p = *params;
    if (!(p.nnratio > 0.f) || p.device < 0) return ORBX_ERR_INVALID;
    int ndev = 0;
    if (!HIPOK(hipGetDeviceCount(&ndev)) || ndev <= 0) return ORBX_ERR_DEVICE;
    if (p.device >= ndev) return ORBX_ERR_INVALID;
    orbx_matcher* m = new orbx_matcher();
    m->prm = p;
    if (!HIPOK(hipSetDevice(p.device)) ||
        !HIPOK(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking)) ||
        !HIPOK(hipMalloc((void**)&m->d_err, 64)) || !HIPOK(hipMemset(m->d_err, 0, 64)) ||
        !HIPOK(hipEventCreateWithFlags(&m->bf_done, hipEventDisableTiming)) ||
        !HIPOK(prepare_match_kernels())) {
        orbx_matcher_destroy(m);
        return ORBX_ERR_DEVICE;
    }
    hipDeviceProp_t prop;
    if (HIPOK(hipGetDeviceProperties(&prop, p.device)) && prop.multiProcessorCount > 0)
        m->ncu = prop.multiProcessorCount;
    *out = m;
    return ORBX_OK;
}

orbx_status orbx_matcher_destroy(orbx_matcher* m) {
    if (!m) return ORBX_ERR_INVALID;
    (void)hipSetDevice(m->prm.device);
    if (m->stream) (void)hipStreamSynchronize(m->stream);
    if (m->have_bf) (void)hipEventSynchronize(m->bf_done);
    if (m->bf_done) (void)hipEventDestroy(m->bf_done);
    m->d_in.release();
    m->d_out.release();
    m->d_aux.release();
    m->d_proj.release();
    m->d_bf.release();
    if (m->d_err) (void)hipFree(m->d_err);
    m->timer.destroy();
    if (m->stream) (void)hipStreamDestroy(m->stream);
    delete m;
    return ORBX_OK;
}

void orbx_compute_three_maxima(const int32_t* histo, int32_t L, int32_t* ind1, int32_t* ind2,
                               int32_t* ind3) {
    int max1 = 0, max2 = 0, max3 = 0;
    int a = ind1 ? *ind1 : -1, b = ind2 ? *ind2 : -1, c = ind3 ? *ind3 : -1;
    for (int i = 0; histo && i < L; i++) {
        const int s = histo[i];
        if (s > max1) {
            max3 = max2; max2 = max1; max1 = s;
            c = b; b = a; a = i;
        } else if (s > max2) {
            max3 = max2; max2 = s;
            c = b; b = i;
        } else if (s > max3) {
            max3 = s; c = i;
        }
    }
    if (max2 < 0.1f * (float)max1) {
        b = -1; c = -1;
    } else if (max3 < 0.1f * (float)max1) {
        c = -1;
    }
    if (ind1) *ind1 = a;
    if (ind2) *ind2 = b;
    if (ind3) *ind3 = c;
}

orbx_status orbx_search_by_bow_kf_frame(orbx_matcher* m, const orbx_featureset* kf,
                                        const uint8_t* kf_valid, const orbx_featureset* f,
                                        int32_t* match_f, int32_t* nmatches) {
    return bow_common(m, kf, kf_valid, f, nullptr, 0, match_f, nmatches);
}

orbx_status orbx_search_by_bow_kf_kf(orbx_matcher* m, const orbx_featureset* kf1,
                                     const uint8_t* valid1, const orbx_featureset* kf2,
                                     const uint8_t* valid2, int32_t* match12, int32_t* nmatches) {
    return bow_common(m, kf1, valid1, kf2, valid2, 1, match12, nmatches);
}

orbx_status orbx_search_for_triangulation(orbx_matcher* m, const orbx_featureset* kf1,
                                          const uint8_t* has_mp1, const orbx_featureset* kf2,
                                          const uint8_t* has_mp2, const float* F12, float ex,
                                          float ey, const float* sigma2_2, const float* scale_2,
                                          int32_t nlevels, int32_t only_stereo, int32_t* pairs,
                                          int32_t pair_cap, int32_t* nmatches) {
    if (!m || !has_mp1 || !has_mp2 || !F12 || !sigma2_2 || !scale_2 || !nmatches ||
        nlevels <= 0 || pair_cap < 0 || (pair_cap > 0 && !pairs))
        return ORBX_ERR_INVALID;
    if (nlevels > MATCH_MAX_LEVELS) return ORBX_ERR_UNSUPPORTED;
    if (!valid_feat(kf1, true, false) || !valid_feat(kf2, true, false)) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(m->mu);
    if (!HIPOK(hipSetDevice(m->prm.device))) return ORBX_ERR_DEVICE;
    Packer P(m->staging);
    const orbx_featureset* fs[2] = {kf1, kf2};
    const uint8_t* fl[2] = {has_mp1, has_mp2};
    const DbOffsets od = pack_db(P, fs, fl, 2);
    const size_t ojob = P.reserve(4 * 4);
    int32_t* jb = P.at<int32_t>(ojob);
    jb[0] = 0;       // kf1
    jb[1] = 1;       // kf2
    jb[2] = 0;       // job_off[0]
    jb[3] = kf1->n;  // job_off[1]
    const size_t of = P.add(F12, 9 * sizeof(float));
    const float epi[2] = {ex, ey};
    const size_t oe = P.add(epi, sizeof(epi));
    orbx_status s = upload(m);
    if (s != ORBX_OK) return s;
    if (!m->d_out.ensure(4 * ((size_t)kf1->n + 64))) return ORBX_ERR_DEVICE;
    uint8_t* base = m->d_in.as<uint8_t>();
    TriLaunch L{};
    L.db = dev_db(od, base);
    L.njobs = 1;
    L.kf1 = (const int32_t*)(base + ojob);
    L.kf2 = (const int32_t*)(base + ojob) + 1;
    L.F12 = (const float*)(base + of);
    L.epi = (const float*)(base + oe);
    for (int l = 0; l < MATCH_MAX_LEVELS; ++l) {
        L.sigma2[l] = l < nlevels ? sigma2_2[l] : 0.f;
        L.scale[l] = l < nlevels ? scale_2[l] : 0.f;
    }
    L.only_stereo = only_stereo;
    L.check_ori = m->prm.check_orientation;
    L.job_off = (const int32_t*)(base + ojob) + 2;
    L.out = m->d_out.as<int32_t>() + 64;
    L.nmatches = m->d_out.as<int32_t>();
    L.err = m->d_err;
    if (tri_lds_bytes(L.db.max_feat) > TRI_MAX_LDS) return ORBX_ERR_UNSUPPORTED;
    hipEvent_t e = m->timer.start(m->stream);
    if (!HIPOK(launch_triangulate(L, m->stream))) return ORBX_ERR_DEVICE;
    m->timer.stop(ORBX_MK_TRIANGULATE, e, m->stream);
    std::vector<int32_t> res((size_t)kf1->n + 64);
    s = finish(m, res.data(), m->d_out.p, 4 * res.size());
    if (s != ORBX_OK) return s;
    // vMatchedPairs in idx1 order (:861-869)
    int np = 0;
    for (int i = 0; i < kf1->n; ++i) {
        const int j = res[64 + i];
        if (j < 0) continue;
        if (np < pair_cap) {
            pairs[2 * np] = i;
            pairs[2 * np + 1] = j;
        }
        ++np;
    }
    *nmatches = res[0];
    return np > pair_cap ? ORBX_ERR_CAPACITY : ORBX_OK;
}

orbx_status orbx_search_by_projection(orbx_matcher* m, int32_t mode,
                                      const orbx_featureset* target, const uint8_t* claimed,
                                      const uint8_t* qdesc, const orbx_proj_query* q,
                                      int32_t nq, const float* inv_sigma2, int32_t nlevels,
                                      int32_t orb_dist, int32_t* match_q, int32_t* nmatches) {
    if (mode < 0 || mode >= ORBX_PROJ_MODE_COUNT) return ORBX_ERR_INVALID;
    return proj_common(m, mode, target, claimed, qdesc, q, nq, inv_sigma2, nlevels, orb_dist,
                       match_q, nmatches);
}

orbx_status orbx_search_by_projection_ex(orbx_matcher* m, int32_t mode,
                                         const orbx_featureset* target, const uint8_t* claimed,
                                         const uint8_t* qdesc, const orbx_proj_query* q,
                                         const uint8_t* qflags, int32_t nq,
                                         const float* inv_sigma2, int32_t nlevels,
                                         int32_t orb_dist, int32_t flags, int32_t* match_q,
                                         int32_t* nmatches) {
    if (mode < 0 || mode >= ORBX_PROJ_MODE_COUNT || (flags & ~ORBX_PROJ_PREFILTER) || !m)
        return ORBX_ERR_INVALID;
    // LAST_FRAME's rotation filter runs per feature in the reference (:1516-1535): with
    // no-claim queries a feature can be matched twice and sit in two bins, which a per-query
    // filter cannot reproduce, so that combination needs the caller's own filter (PREFILTER)
    if (mode == ORBX_PROJ_LAST_FRAME && m->prm.check_orientation && !(flags & ORBX_PROJ_PREFILTER) &&
        qflags && nq > 0)
        for (int32_t i = 0; i < nq; ++i)
            if (qflags[i] & ORBX_QF_NO_CLAIM) return ORBX_ERR_INVALID;
    return proj_common(m, mode, target, claimed, qdesc, q, nq, inv_sigma2, nlevels, orb_dist,
                       match_q, nmatches, qflags, flags);
}

orbx_status orbx_search_by_sim3(orbx_matcher* m, const orbx_featureset* kf1,
                                const orbx_featureset* kf2, const uint8_t* qdesc1,
                                const orbx_proj_query* q12, int32_t n1, const uint8_t* qdesc2,
                                const orbx_proj_query* q21, int32_t n2, int32_t* match12,
                                int32_t* nmatches) {
    if (!kf1 || !kf2 || !match12 || !nmatches || n1 < 0 || n2 < 0) return ORBX_ERR_INVALID;
    std::vector<int32_t> v1((size_t)n1 + 1), v2((size_t)n2 + 1);
    int32_t c1 = 0, c2 = 0;
    orbx_status s = proj_common(m, ORBX_PROJ_SIM3, kf2, nullptr, qdesc1, q12, n1, nullptr, 0, 0,
                                v1.data(), &c1);
    if (s != ORBX_OK) return s;
    s = proj_common(m, ORBX_PROJ_SIM3, kf1, nullptr, qdesc2, q21, n2, nullptr, 0, 0, v2.data(),
                    &c2);
    if (s != ORBX_OK) return s;
    int nFound = 0;
    for (int i1 = 0; i1 < n1; ++i1) {   // :1366-1379
        match12[i1] = -1;
        const int idx2 = v1[i1];
        if (idx2 >= 0 && idx2 < n2 && v2[idx2] == i1) {
            match12[i1] = idx2;
            ++nFound;
        }
    }
    *nmatches = nFound;
    return ORBX_OK;
}

orbx_status orbx_search_for_initialization(orbx_matcher* m, const orbx_featureset* f1,
                                           const orbx_featureset* f2, float* prev_matched,
                                           int32_t window_size, int32_t* match12,
                                           int32_t* nmatches) {
    if (!f1 || !f2 || !prev_matched || !match12 || !nmatches) return ORBX_ERR_INVALID;
    if (!valid_feat(f1, false, false)) return ORBX_ERR_INVALID;
    const int n1 = f1->n;
    // one query per F1 feature (:459-466): level-0 features search F2 around vbPrevMatched
    std::vector<orbx_proj_query> q((size_t)n1);
    for (int i = 0; i < n1; ++i) {
        const int level1 = f1->keys[i].octave;
        q[i].u = prev_matched[2 * i];
        q[i].v = prev_matched[2 * i + 1];
        q[i].ur = 0.f;
        q[i].radius = level1 > 0 ? -1.0f : (float)window_size;
        q[i].min_level = level1;
        q[i].max_level = level1;
        q[i].pred_level = 0;
        q[i].angle = f1->keys[i].angle;
    }
    orbx_status s = proj_common(m, PROJ_INIT, f2, nullptr, f1->desc, q.data(), n1, nullptr, 0,
                                0, match12, nmatches);
    if (s != ORBX_OK) return s;
    for (int i = 0; i < n1; ++i)   // :555-558
        if (match12[i] >= 0) {
            prev_matched[2 * i] = f2->keys[match12[i]].x;
            prev_matched[2 * i + 1] = f2->keys[match12[i]].y;
        }
    return ORBX_OK;
}

orbx_status orbx_search_by_bow_kf_frame_batch_device(orbx_matcher* m, const orbx_kf_db* db,
                                                     const orbx_featureset* f,
                                                     int32_t* d_match, int32_t* d_nmatches,
                                                     void* stream) {
    if (!m || !db || !f || !d_match || !d_nmatches) return ORBX_ERR_INVALID;
    if (db->nkf < 0 || db->max_feat < 0 || db->max_feat > MAX_FEAT || f->n < 0 || f->n > MAX_FEAT)
        return ORBX_ERR_INVALID;
    if (db->nkf == 0) return ORBX_OK;
    if (!db->feat_off || !db->keys || !db->desc || !db->flag || !db->node_off || !db->node_id ||
        !db->node_feat_off || !db->node_feat || (f->n > 0 && (!f->keys || !f->desc)) ||
        (f->n_nodes > 0 && (!f->node_id || !f->node_off || !f->node_feat)))
        return ORBX_ERR_INVALID;
    if (((uintptr_t)db->desc & 15) || ((uintptr_t)f->desc & 15)) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(m->mu);
    if (!HIPOK(hipSetDevice(m->prm.device))) return ORBX_ERR_DEVICE;
    hipStream_t st = (hipStream_t)stream;
    // The frame as a one-keyframe database: its CSR offsets are already absolute.
    if (!m->d_aux.ensure(64)) return ORBX_ERR_DEVICE;
    int32_t offs[4] = {0, f->n, 0, f->n_nodes};
    if (!HIPOK(hipMemcpyAsync(m->d_aux.p, offs, sizeof(offs), hipMemcpyHostToDevice, st)))
        return ORBX_ERR_DEVICE;
    BowLaunch L{};
    L.A = *db;
    L.B.nkf = 1;
    L.B.max_feat = f->n;
    L.B.feat_off = m->d_aux.as<int32_t>();
    L.B.keys = f->keys;
    L.B.desc = f->desc;
    L.B.u_right = f->u_right;
    L.B.flag = db->flag;   // not read for SearchByBoW(KeyFrame*, Frame&)
    L.B.node_off = m->d_aux.as<int32_t>() + 2;
    L.B.node_id = f->node_id;
    L.B.node_feat_off = f->node_off;
    L.B.node_feat = f->node_feat;
    L.a_fixed = 0;
    L.b_fixed = 1;
    L.kf_kf = 0;
    L.njobs = db->nkf;
    L.ratio = m->prm.nnratio;
    L.check_ori = m->prm.check_orientation;
    L.out = d_match;
    L.out_stride = f->n;
    L.nmatches = d_nmatches;
    L.err = m->d_err;
    if (bow_lds_bytes(L) > MATCH_MAX_LDS) return ORBX_ERR_UNSUPPORTED;
    hipEvent_t e = m->timer.start(st);
    if (!HIPOK(launch_bow(L, st))) return ORBX_ERR_DEVICE;
    m->timer.stop(ORBX_MK_BOW, e, st);
    return ORBX_OK;
}

orbx_status orbx_search_for_triangulation_batch_device(
    orbx_matcher* m, const orbx_kf_db* db, int32_t njobs, const int32_t* d_kf1,
    const int32_t* d_kf2, const float* d_F12, const float* d_epi, const float* sigma2,
    const float* scale, int32_t nlevels, int32_t only_stereo, const int32_t* d_job_off,
    int32_t* d_match12, int32_t* d_nmatches, void* stream) {
    if (!m || !db || njobs < 0 || !sigma2 || !scale || nlevels <= 0) return ORBX_ERR_INVALID;
    if (nlevels > MATCH_MAX_LEVELS) return ORBX_ERR_UNSUPPORTED;
    if (db->max_feat < 0 || db->max_feat > MAX_FEAT) return ORBX_ERR_INVALID;
    if (njobs == 0) return ORBX_OK;
    if (!d_kf1 || !d_kf2 || !d_F12 || !d_epi || !d_job_off || !d_match12 || !d_nmatches ||
        !db->feat_off || !db->keys || !db->desc || !db->flag || !db->node_off || !db->node_id ||
        !db->node_feat_off || !db->node_feat)
        return ORBX_ERR_INVALID;
    if ((uintptr_t)db->desc & 15) return ORBX_ERR_INVALID;
    const bool nord = db->node_keys || db->node_desc || db->node_flag || db->node_u_right;
    if (nord && (!db->node_keys || !db->node_desc || !db->node_flag ||
                 (db->u_right != nullptr) != (db->node_u_right != nullptr) ||
                 ((uintptr_t)db->node_desc & 15)))
        return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(m->mu);
    if (!HIPOK(hipSetDevice(m->prm.device))) return ORBX_ERR_DEVICE;
    TriLaunch L{};
    L.db = *db;
    L.njobs = njobs;
    L.kf1 = d_kf1;
    L.kf2 = d_kf2;
    L.F12 = d_F12;
    L.epi = d_epi;
    for (int l = 0; l < MATCH_MAX_LEVELS; ++l) {
        L.sigma2[l] = l < nlevels ? sigma2[l] : 0.f;
        L.scale[l] = l < nlevels ? scale[l] : 0.f;
    }
    L.only_stereo = only_stereo;
    L.check_ori = m->prm.check_orientation;
    L.job_off = d_job_off;
    L.out = d_match12;
    L.nmatches = d_nmatches;
    L.err = m->d_err;
    if (tri_lds_bytes(db->max_feat) > TRI_MAX_LDS) return ORBX_ERR_UNSUPPORTED;
    hipStream_t st = (hipStream_t)stream;
    hipEvent_t e = m->timer.start(st);
    if (!HIPOK(launch_triangulate(L, st))) return ORBX_ERR_DEVICE;
    m->timer.stop(ORBX_MK_TRIANGULATE, e, st);
    return ORBX_OK;
}

orbx_status orbx_search_by_projection_batch_device(
    orbx_matcher* m, int32_t mode, const orbx_featureset* frames, int32_t njobs,
    const int32_t* d_feat_off, const int32_t* d_grid_off, int32_t max_feat,
    const uint8_t* d_claimed, const uint8_t* d_qdesc, const orbx_proj_query* d_q,
    const int32_t* d_q_off, int32_t nq, const float* inv_sigma2, int32_t nlevels,
    int32_t orb_dist, int32_t* d_match, int32_t* d_nmatches, void* stream) {
    if (!m || !frames || njobs < 0 || nq < 0 || nq > (1 << 24)) return ORBX_ERR_INVALID;
    if (mode < 0 || mode >= ORBX_PROJ_MODE_COUNT) return ORBX_ERR_INVALID;
    if (max_feat < 0 || max_feat > MAX_FEAT) return ORBX_ERR_INVALID;
    if (mode == ORBX_PROJ_FUSE && (!inv_sigma2 || nlevels <= 0)) return ORBX_ERR_INVALID;
    if (nlevels > MATCH_MAX_LEVELS) return ORBX_ERR_UNSUPPORTED;
    if (frames->grid_cols <= 0 || frames->grid_rows <= 0 ||
        (long long)frames->grid_cols * frames->grid_rows > (1 << 20))
        return ORBX_ERR_INVALID;
    if (njobs == 0) return ORBX_OK;
    if (!d_feat_off || !d_grid_off || !d_q_off || !d_match || !d_nmatches || !frames->keys ||
        !frames->desc || !frames->grid_off || !frames->grid_feat || (nq > 0 && (!d_qdesc || !d_q)))
        return ORBX_ERR_INVALID;
    if (((uintptr_t)frames->desc & 15) || ((uintptr_t)d_qdesc & 15)) return ORBX_ERR_INVALID;
    if (proj_mode_greedy(mode) && proj_resolve_lds_bytes(mode, max_feat, 0) > MATCH_MAX_LDS)
        return ORBX_ERR_UNSUPPORTED;
    std::lock_guard<std::mutex> lk(m->mu);
    if (!HIPOK(hipSetDevice(m->prm.device))) return ORBX_ERR_DEVICE;
    hipStream_t st = (hipStream_t)stream;
    // scratch: hist[32 * njobs] | top2[nq] | bins[nq] | cand[nq * PROJ_K] | ncand[nq]
    const size_t o_top = align256(128 * (size_t)njobs), o_bin = align256(o_top + 16 * (size_t)nq),
                 o_cand = align256(o_bin + (size_t)nq),
                 o_nc = align256(o_cand + 8 * PROJ_K * (size_t)nq),
                 o_end = align256(o_nc + 4 * (size_t)nq);
    if (!m->d_proj.ensure(o_end)) return ORBX_ERR_DEVICE;
    uint8_t* sb = m->d_proj.as<uint8_t>();
    ProjLaunch L{};
    L.mode = mode;
    L.T = *frames;
    L.T.n = max_feat;
    L.T.n_nodes = 0;
    L.T.node_id = nullptr;
    L.T.node_off = nullptr;
    L.T.node_feat = nullptr;
    L.njobs = njobs;
    L.t_off = d_feat_off;
    L.g_off = d_grid_off;
    L.q_off = d_q_off;
    L.max_t = max_feat;
    L.qdesc = d_qdesc;
    L.q = d_q;
    L.nq = nq;
    for (int l = 0; l < MATCH_MAX_LEVELS; ++l)
        L.inv_sigma2[l] = (inv_sigma2 && l < nlevels) ? inv_sigma2[l] : 0.f;
    L.orb_dist = orb_dist;
    L.ratio = m->prm.nnratio;
    L.check_ori = m->prm.check_orientation;
    L.claimed_in = d_claimed;
    L.out = d_match;
    L.top2 = (int4*)(sb + o_top);
    L.cand = (int2*)(sb + o_cand);
    L.ncand = (int32_t*)(sb + o_nc);
    L.out_bin = (int8_t*)(sb + o_bin);
    L.hist = (int32_t*)sb;
    L.nmatches = d_nmatches;
    L.err = m->d_err;
    if (nq == 0) {   // every job: no queries, no matches
        if (!HIPOK(hipMemsetAsync(d_nmatches, 0, 4 * (size_t)njobs, st))) return ORBX_ERR_DEVICE;
        return ORBX_OK;
    }
    if (!HIPOK(launch_proj(L, st, &m->timer))) return ORBX_ERR_DEVICE;
    return ORBX_OK;
}

orbx_status orbx_compute_distinctive_descriptors(orbx_matcher* m, const uint8_t* desc,
                                                 const int32_t* off, int32_t npoints,
                                                 int32_t* best) {
    if (!m || !off || !best || npoints < 0) return ORBX_ERR_INVALID;
    if (npoints == 0) return ORBX_OK;
    if (off[0] < 0) return ORBX_ERR_INVALID;
    for (int p = 0; p < npoints; ++p) {
        if (off[p + 1] < off[p]) return ORBX_ERR_INVALID;
        if (off[p + 1] - off[p] > ORBX_MAX_OBSERVATIONS) return ORBX_ERR_UNSUPPORTED;
    }
    const int n = off[npoints] - off[0];
    if (n > 0 && !desc) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(m->mu);
    if (!HIPOK(hipSetDevice(m->prm.device))) return ORBX_ERR_DEVICE;
    Packer P(m->staging);
    const size_t od = P.add(n > 0 ? desc + 32 * (size_t)off[0] : nullptr, 32 * (size_t)n);
    std::vector<int32_t> rel((size_t)npoints + 1);
    for (int p = 0; p <= npoints; ++p) rel[p] = off[p] - off[0];
    const size_t oo = P.add(rel.data(), 4 * rel.size());
    orbx_status s = upload(m);
    if (s != ORBX_OK) return s;
    if (!m->d_out.ensure(4 * (size_t)npoints)) return ORBX_ERR_DEVICE;
    uint8_t* base = m->d_in.as<uint8_t>();
    hipEvent_t e = m->timer.start(m->stream);
    if (!HIPOK(launch_distinctive(base + od, (const int32_t*)(base + oo),
                                  npoints, m->d_out.as<int32_t>(), m->d_err, m->stream)))
        return ORBX_ERR_DEVICE;
    m->timer.stop(ORBX_MK_DISTINCTIVE, e, m->stream);
    return finish(m, best, m->d_out.p, 4 * (size_t)npoints);
}

orbx_status orbx_compute_distinctive_descriptors_device(orbx_matcher* m, const uint8_t* d_desc,
                                                        const int32_t* d_off, int32_t npoints,
                                                        int32_t* d_best, void* stream) {
    if (!m || !d_off || !d_best || !d_desc || npoints < 0) return ORBX_ERR_INVALID;
    if (npoints == 0) return ORBX_OK;
    std::lock_guard<std::mutex> lk(m->mu);
    if (!HIPOK(hipSetDevice(m->prm.device))) return ORBX_ERR_DEVICE;
    hipStream_t st = (hipStream_t)stream;
    hipEvent_t e = m->timer.start(st);
    if (!HIPOK(launch_distinctive(d_desc, d_off, npoints, d_best, m->d_err, st)))
        return ORBX_ERR_DEVICE;
    m->timer.stop(ORBX_MK_DISTINCTIVE, e, st);
    return ORBX_OK;
}

namespace {
orbx_status bf_run(orbx_matcher* m, const uint8_t* d_q, int nq, const uint8_t* d_db,
                   long long ndb, long long idx_base, int32_t* bi, int32_t* bd, int32_t* sd,
                   hipStream_t st) {
    BfLaunch a{};
    a.q = d_q;
    a.nq = nq;
    a.db = d_db;
    a.ndb = ndb;
    a.idx_base = idx_base;
    a.chunk = bf_chunk_rows(ndb, nq, m->ncu, m->bf_kernel);
    const size_t need = bf_partial_bytes(ndb, nq, a.chunk);
    // growing frees the scratch an earlier launch (any stream) may still use
    if (need > m->d_bf.n && m->have_bf && !HIPOK(hipEventSynchronize(m->bf_done)))
        return ORBX_ERR_DEVICE;
    if (!m->d_bf.ensure(need)) return ORBX_ERR_DEVICE;
    // the previous launch on another stream must be done with the scratch
    if (m->have_bf && m->bf_stream != st && !HIPOK(hipStreamWaitEvent(st, m->bf_done, 0)))
        return ORBX_ERR_DEVICE;
    a.part = m->d_bf.p;
    a.best_idx = bi;
    a.best_dist = bd;
    a.second_dist = sd;
    a.kernel = m->bf_kernel;
    if (!HIPOK(launch_bf_top2(a, st, &m->timer)) || !HIPOK(hipEventRecord(m->bf_done, st)))
        return ORBX_ERR_DEVICE;
    m->bf_stream = st;
    m->have_bf = true;
    return ORBX_OK;
}
}  // namespace

orbx_status orbx_hamming_bf_top2(orbx_matcher* m, const uint8_t* q, int32_t nq,
                                 const uint8_t* db, int64_t ndb, int32_t* best_idx,
                                 int32_t* best_dist, int32_t* second_dist) {
    if (!m || nq < 0 || ndb < 0 || ndb >= INT32_MAX) return ORBX_ERR_INVALID;
    if (nq == 0) return ORBX_OK;
    if (!q || !best_idx || !best_dist || !second_dist || (ndb > 0 && !db)) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(m->mu);
    if (!HIPOK(hipSetDevice(m->prm.device))) return ORBX_ERR_DEVICE;
    const size_t qb = 32 * (size_t)nq, dbb = 32 * (size_t)ndb, ob = 4 * (size_t)nq;
    if (!m->d_in.ensure(align256(qb) + std::max<size_t>(dbb, 32)) || !m->d_out.ensure(3 * align256(ob)))
        return ORBX_ERR_DEVICE;
    uint8_t* din = m->d_in.as<uint8_t>();
    uint8_t* dout = m->d_out.as<uint8_t>();
    if (!HIPOK(hipMemcpyAsync(din, q, qb, hipMemcpyHostToDevice, m->stream)) ||
        (dbb && !HIPOK(hipMemcpyAsync(din + align256(qb), db, dbb, hipMemcpyHostToDevice, m->stream))))
        return ORBX_ERR_DEVICE;
    int32_t* bi = (int32_t*)dout;
    int32_t* bd = (int32_t*)(dout + align256(ob));
    int32_t* sd = (int32_t*)(dout + 2 * align256(ob));
    orbx_status s = bf_run(m, din, nq, din + align256(qb), ndb, 0, bi, bd, sd, m->stream);
    if (s != ORBX_OK) return s;
    if (!HIPOK(hipMemcpyAsync(best_idx, bi, ob, hipMemcpyDeviceToHost, m->stream)) ||
        !HIPOK(hipMemcpyAsync(best_dist, bd, ob, hipMemcpyDeviceToHost, m->stream)) ||
        !HIPOK(hipMemcpyAsync(second_dist, sd, ob, hipMemcpyDeviceToHost, m->stream)) ||
        !HIPOK(hipStreamSynchronize(m->stream)))
        return ORBX_ERR_DEVICE;
    return ORBX_OK;
}

const char* orbx_bf_kernel(void) { return orbx::bf_kernel_name(ORBX_BF_MFMA); }

const char* orbx_bf_kernel_name(int32_t kernel) { return orbx::bf_kernel_name(kernel); }

orbx_status orbx_matcher_set_bf_kernel(orbx_matcher* m, int32_t kernel) {
    if (!m || !orbx::bf_kernel_name(kernel)) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(m->mu);
    m->bf_kernel = kernel;
    return ORBX_OK;
}

orbx_status orbx_hamming_bf_top2_device(orbx_matcher* m, const uint8_t* d_q, int32_t nq,
                                        const uint8_t* d_db, int64_t ndb, int64_t idx_base,
                                        int32_t* d_best_idx, int32_t* d_best_dist,
                                        int32_t* d_second_dist, void* stream) {
    if (!m || nq < 0 || ndb < 0 || idx_base < 0 || ndb + idx_base >= INT32_MAX)
        return ORBX_ERR_INVALID;
    if (nq == 0) return ORBX_OK;
    if (!d_q || !d_best_idx || !d_best_dist || !d_second_dist || (ndb > 0 && !d_db))
        return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(m->mu);
    if (!HIPOK(hipSetDevice(m->prm.device))) return ORBX_ERR_DEVICE;
    return bf_run(m, d_q, nq, d_db, ndb, idx_base, d_best_idx, d_best_dist, d_second_dist,
                  (hipStream_t)stream);
}

orbx_status orbx_kf_db_node_order(orbx_matcher* m, const orbx_kf_db* db, int32_t n,
                                  orbx_keypoint* d_keys, uint8_t* d_desc, float* d_u_right,
                                  uint8_t* d_flag, void* stream) {
    if (!m || !db || n < 0 || db->nkf < 0) return ORBX_ERR_INVALID;
    if (db->nkf == 0 || n == 0) return ORBX_OK;
    if (!db->feat_off || !db->keys || !db->desc || !db->flag || !db->node_off ||
        !db->node_feat_off || !db->node_feat || !d_keys || !d_desc || !d_flag ||
        (db->u_right && !d_u_right) || ((uintptr_t)d_desc & 15) || ((uintptr_t)db->desc & 15))
        return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(m->mu);
    if (!HIPOK(hipSetDevice(m->prm.device))) return ORBX_ERR_DEVICE;
    orbx_kf_db d = *db;
    d.node_keys = nullptr;
    d.node_desc = nullptr;
    d.node_u_right = nullptr;
    d.node_flag = nullptr;
    if (!HIPOK(launch_node_order(d, n, d_keys, d_desc, db->u_right ? d_u_right : nullptr, d_flag,
                                 (hipStream_t)stream)))
        return ORBX_ERR_DEVICE;
    return ORBX_OK;
}

orbx_status orbx_matcher_sync(orbx_matcher* m, void* stream) {
    if (!m) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(m->mu);
    if (!HIPOK(hipSetDevice(m->prm.device))) return ORBX_ERR_DEVICE;
    int err = 0;
    hipStream_t st = (hipStream_t)stream;
    if (!HIPOK(hipMemcpyAsync(&err, m->d_err, sizeof(int), hipMemcpyDeviceToHost, st)) ||
        !HIPOK(hipStreamSynchronize(st)) || !HIPOK(hipMemset(m->d_err, 0, sizeof(int))))
        return ORBX_ERR_DEVICE;
    return err ? ORBX_ERR_CAPACITY : ORBX_OK;
}

orbx_status orbx_matcher_profile_enable(orbx_matcher* m, int on) {
    if (!m) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(m->mu);
    m->timer.on = on != 0;
    return ORBX_OK;
}

orbx_status orbx_matcher_profile_collect(orbx_matcher* m, double* total_ms, int64_t* launches) {
    if (!m) return ORBX_ERR_INVALID;
    std::lock_guard<std::mutex> lk(m->mu);
    m->timer.collect();
    for (int k = 0; k < ORBX_MK_COUNT; ++k) {
        if (total_ms) total_ms[k] = m->timer.ms[k];
        if (launches) launches[k] = m->timer.n[k];
        m->timer.ms[k] = 0;
        m->timer.n[k] = 0;
    }
    return ORBX_OK;
}

const char* orbx_match_kernel_name(int id) {
    static const char* names[ORBX_MK_COUNT] = {"k_bow", "k_triangulate", "k_proj_search",
                                               "k_proj_resolve", "k_distinctive"};
    return (id >= 0 && id < ORBX_MK_COUNT) ? names[id] : "";
}

}  // extern "C"
