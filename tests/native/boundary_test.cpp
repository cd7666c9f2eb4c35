// boundary_test.cpp — a C++ consumer of the drop-in boundary, compiled by g++ against
// include/orbx*.h only and linked to liborbx.so (no HIP headers, no torch, no ctypes).
//
//   boundary_test layout        struct sizes / field offsets as JSON (no GPU; the CPU suite
//                               compares them with the Python ctypes mirrors)
//   boundary_test run DIR       the sequence INTEGRATION.md installs into ORB-SLAM2, on the GPU:
//     * two ORBextractor handles, the left and right images extracted on two std::threads
//       (Frame::Frame stereo, src/Frame.cc:89-92) through orbx_extract;
//     * Frame::ComputeStereoMatches (src/Frame.cc:102) through orbx_stereo_match;
//     * ORBmatcher(0.75, true).SearchByBoW(KF = right view, F = left view) (src/ORBmatcher.cc:
//       182-319, single-node FeatureVector: the brute-force anchor of SURVEY 8c);
//     * ORBmatcher(0.6, false).SearchForTriangulation(left, right, F12) (:702-872).
//   DIR holds left.raw / right.raw (W*H bytes) and params.txt ("W H nfeatures mbf mb ex ey
//   F12[9]"); the outputs are written back to DIR as raw little-endian arrays.
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "orbx.h"
#include "orbx_frame.h"
#include "orbx_kfdb.h"
#include "orbx_match.h"
#include "orbx_vocab.h"

// cv::KeyPoint as OpenCV 3.2 lays it out (core/types.hpp: Point2f pt; float size, angle,
// response; int octave, class_id): the facade of INTEGRATION.md hands a
// std::vector<cv::KeyPoint>'s buffer to orbx_extract, so the layouts must agree byte for byte.
struct CvPoint2f { float x, y; };
struct CvKeyPointShape {
    CvPoint2f pt;
    float size, angle, response;
    int octave, class_id;
};
static_assert(sizeof(orbx_keypoint) == 28, "orbx_keypoint is 28 bytes");
static_assert(sizeof(orbx_keypoint) == sizeof(CvKeyPointShape), "cv::KeyPoint size");
static_assert(offsetof(orbx_keypoint, x) == offsetof(CvKeyPointShape, pt) + offsetof(CvPoint2f, x), "pt.x");
static_assert(offsetof(orbx_keypoint, y) == offsetof(CvKeyPointShape, pt) + offsetof(CvPoint2f, y), "pt.y");
static_assert(offsetof(orbx_keypoint, size) == offsetof(CvKeyPointShape, size), "size");
static_assert(offsetof(orbx_keypoint, angle) == offsetof(CvKeyPointShape, angle), "angle");
static_assert(offsetof(orbx_keypoint, response) == offsetof(CvKeyPointShape, response), "response");
static_assert(offsetof(orbx_keypoint, octave) == offsetof(CvKeyPointShape, octave), "octave");
static_assert(offsetof(orbx_keypoint, class_id) == offsetof(CvKeyPointShape, class_id), "class_id");
static_assert(alignof(orbx_keypoint) == alignof(CvKeyPointShape), "alignment");

#define FIELD(T, f) std::printf("%s\"%s\": [%zu, %zu]", first ? "" : ", ", #f, offsetof(T, f), sizeof(((T*)0)->f)), first = false
#define STRUCT(T, ...)                                                     \
    do {                                                                   \
        std::printf("%s\"%s\": {\"size\": %zu, \"fields\": {", nfirst ? "" : ", ", #T, sizeof(T)); \
        bool first = true;                                                 \
        __VA_ARGS__;                                                       \
        std::printf("}}");                                                 \
        nfirst = false;                                                    \
    } while (0)

static int layout() {
    bool nfirst = true;
    std::printf("{");
    STRUCT(orbx_keypoint, FIELD(orbx_keypoint, x); FIELD(orbx_keypoint, y); FIELD(orbx_keypoint, size);
           FIELD(orbx_keypoint, angle); FIELD(orbx_keypoint, response); FIELD(orbx_keypoint, octave);
           FIELD(orbx_keypoint, class_id));
    STRUCT(orbx_extractor_params, FIELD(orbx_extractor_params, nfeatures);
           FIELD(orbx_extractor_params, scale_factor); FIELD(orbx_extractor_params, nlevels);
           FIELD(orbx_extractor_params, ini_th_fast); FIELD(orbx_extractor_params, min_th_fast);
           FIELD(orbx_extractor_params, cv_simd); FIELD(orbx_extractor_params, max_batch);
           FIELD(orbx_extractor_params, device));
    STRUCT(orbx_batch_view, FIELD(orbx_batch_view, batch); FIELD(orbx_batch_view, kp_cap);
           FIELD(orbx_batch_view, kps); FIELD(orbx_batch_view, desc); FIELD(orbx_batch_view, nkp);
           FIELD(orbx_batch_view, pyramid); FIELD(orbx_batch_view, pyr_bytes);
           FIELD(orbx_batch_view, level_w); FIELD(orbx_batch_view, level_h);
           FIELD(orbx_batch_view, level_pitch); FIELD(orbx_batch_view, level_off));
    STRUCT(orbx_featureset, FIELD(orbx_featureset, n); FIELD(orbx_featureset, keys);
           FIELD(orbx_featureset, desc); FIELD(orbx_featureset, u_right);
           FIELD(orbx_featureset, n_nodes); FIELD(orbx_featureset, node_id);
           FIELD(orbx_featureset, node_off); FIELD(orbx_featureset, node_feat);
           FIELD(orbx_featureset, grid_cols); FIELD(orbx_featureset, grid_rows);
           FIELD(orbx_featureset, grid_off); FIELD(orbx_featureset, grid_feat);
           FIELD(orbx_featureset, min_x); FIELD(orbx_featureset, min_y);
           FIELD(orbx_featureset, max_x); FIELD(orbx_featureset, max_y);
           FIELD(orbx_featureset, grid_inv_w); FIELD(orbx_featureset, grid_inv_h));
    STRUCT(orbx_matcher_params, FIELD(orbx_matcher_params, nnratio);
           FIELD(orbx_matcher_params, check_orientation); FIELD(orbx_matcher_params, device));
    STRUCT(orbx_kf_db, FIELD(orbx_kf_db, nkf); FIELD(orbx_kf_db, max_feat); FIELD(orbx_kf_db, feat_off);
           FIELD(orbx_kf_db, keys); FIELD(orbx_kf_db, desc); FIELD(orbx_kf_db, u_right);
           FIELD(orbx_kf_db, flag); FIELD(orbx_kf_db, node_off); FIELD(orbx_kf_db, node_id);
           FIELD(orbx_kf_db, node_feat_off); FIELD(orbx_kf_db, node_feat);
           FIELD(orbx_kf_db, node_keys); FIELD(orbx_kf_db, node_desc);
           FIELD(orbx_kf_db, node_u_right); FIELD(orbx_kf_db, node_flag));
    STRUCT(orbx_proj_query, FIELD(orbx_proj_query, u); FIELD(orbx_proj_query, v);
           FIELD(orbx_proj_query, ur); FIELD(orbx_proj_query, radius);
           FIELD(orbx_proj_query, min_level); FIELD(orbx_proj_query, max_level);
           FIELD(orbx_proj_query, pred_level); FIELD(orbx_proj_query, angle));
    STRUCT(orbx_kfdb_params, FIELD(orbx_kfdb_params, covisibles); FIELD(orbx_kfdb_params, device));
    std::printf("}\n");
    return 0;
}

static bool read_file(const std::string& path, std::vector<uint8_t>& out) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    out.resize((size_t)n);
    const bool ok = std::fread(out.data(), 1, out.size(), f) == out.size();
    std::fclose(f);
    return ok;
}

static bool write_file(const std::string& path, const void* p, size_t n) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    const bool ok = n == 0 || std::fwrite(p, 1, n, f) == n;
    std::fclose(f);
    return ok;
}

#define CHECK(call)                                                                      \
    do {                                                                                 \
        const orbx_status s_ = (call);                                                   \
        if (s_ != ORBX_OK) {                                                             \
            std::fprintf(stderr, "%s failed: %d [%s]\n", #call, (int)s_, orbx_last_error()); \
            return 1;                                                                    \
        }                                                                                \
    } while (0)

// One view as ORB_SLAM2::Frame holds it after ExtractORB (mvKeys, mDescriptors).
struct View {
    std::vector<orbx_keypoint> kps;
    std::vector<uint8_t> desc;
    int n = 0;
    orbx_status st = ORBX_OK;
};

static void extract(orbx_extractor* h, const uint8_t* img, int w, int hgt, View* v) {
    // the facade's ORBextractor::operator(): size the vectors from the call's count
    int n = 0;
    v->kps.resize(4096);
    v->desc.resize(4096 * 32);
    v->st = orbx_extract(h, img, w, hgt, (size_t)w, v->kps.data(), 4096, v->desc.data(), &n);
    if (v->st == ORBX_ERR_CAPACITY) {
        v->kps.resize((size_t)n);
        v->desc.resize((size_t)n * 32);
        v->st = orbx_extract(h, img, w, hgt, (size_t)w, v->kps.data(), n, v->desc.data(), &n);
    }
    v->n = n;
    v->kps.resize((size_t)std::max(n, 0));
    v->desc.resize((size_t)std::max(n, 0) * 32);
}

static orbx_featureset single_node(const View& v, std::vector<int32_t>& feat, const uint32_t* id,
                                   const int32_t* off) {
    orbx_featureset f;
    std::memset(&f, 0, sizeof(f));
    feat.resize((size_t)v.n);
    for (int i = 0; i < v.n; ++i) feat[(size_t)i] = i;
    f.n = v.n;
    f.keys = v.kps.data();
    f.desc = v.desc.data();
    f.u_right = nullptr;
    f.n_nodes = 1;
    f.node_id = id;
    f.node_off = off;
    f.node_feat = feat.data();
    return f;
}

static int run(const std::string& dir) {
    int W = 0, H = 0, nfeat = 0;
    float mbf = 0, mb = 0, ex = 0, ey = 0, F12[9];
    {
        FILE* f = std::fopen((dir + "/params.txt").c_str(), "r");
        if (!f) return 2;
        int got = std::fscanf(f, "%d %d %d %f %f %f %f", &W, &H, &nfeat, &mbf, &mb, &ex, &ey);
        for (int i = 0; i < 9; ++i) got += std::fscanf(f, "%f", &F12[i]);
        std::fclose(f);
        if (got != 16) return 2;
    }
    std::vector<uint8_t> L, R;
    if (!read_file(dir + "/left.raw", L) || !read_file(dir + "/right.raw", R) ||
        L.size() != (size_t)W * H || R.size() != (size_t)W * H)
        return 2;
    std::printf("%s\n", orbx_version());

    // Tracking.cc:136-139: one extractor per camera, same parameters
    orbx_extractor_params p = {nfeat, 1.2f, 8, 20, 7, 1, 1, 0};
    orbx_extractor *hl = nullptr, *hr = nullptr;
    CHECK(orbx_extractor_create(&p, &hl));
    CHECK(orbx_extractor_create(&p, &hr));
    View vl, vr;
    {   // Frame.cc:89-92
        std::thread tl(extract, hl, L.data(), W, H, &vl);
        std::thread tr(extract, hr, R.data(), W, H, &vr);
        tl.join();
        tr.join();
    }
    CHECK(vl.st);
    CHECK(vr.st);
    std::vector<float> uR((size_t)vl.n), depth((size_t)vl.n);
    int nvalid = 0;
    CHECK(orbx_stereo_match(hl, hr, mbf, mb, uR.data(), depth.data(), vl.n, &nvalid));

    // matchers (LocalMapping / Tracking own their ORBmatcher objects)
    const uint32_t node_id[1] = {0};
    std::vector<int32_t> fl, fr;
    const int32_t offl[2] = {0, vl.n}, offr[2] = {0, vr.n};
    const orbx_featureset F = single_node(vl, fl, node_id, offl);
    const orbx_featureset KF = single_node(vr, fr, node_id, offr);
    orbx_matcher *mbow = nullptr, *mtri = nullptr;
    const orbx_matcher_params pb = {0.75f, 1, 0}, pt = {0.6f, 0, 0};
    CHECK(orbx_matcher_create(&pb, &mbow));
    CHECK(orbx_matcher_create(&pt, &mtri));
    std::vector<uint8_t> valid((size_t)vr.n, 1);
    std::vector<int32_t> bow(1 + (size_t)vl.n);
    CHECK(orbx_search_by_bow_kf_frame(mbow, &KF, valid.data(), &F, bow.data() + 1, bow.data()));
    // scale tables of the extractor (mvLevelSigma2 / mvScaleFactors of KF2)
    float scale[8], sigma2[8];
    CHECK(orbx_extractor_tables(hr, scale, nullptr, sigma2, nullptr, nullptr));
    std::vector<uint8_t> has1((size_t)vl.n, 0), has2((size_t)vr.n, 0);
    std::vector<int32_t> tri(1 + 2 * (size_t)vl.n);
    CHECK(orbx_search_for_triangulation(mtri, &F, has1.data(), &KF, has2.data(), F12, ex, ey,
                                        sigma2, scale, 8, 0, tri.data() + 1, vl.n, tri.data()));

    // the schedule inside an extraction (orbx_extractor_set_overlap) does not change results:
    // the left view again with every kernel on the caller's stream
    {
        orbx_extractor* h1 = nullptr;
        CHECK(orbx_extractor_create(&p, &h1));
        CHECK(orbx_extractor_set_overlap(h1, 0, 0, 1));
        int mode = -1, fork_level = -1, levels = -1;
        CHECK(orbx_extractor_get_overlap(h1, &mode, &fork_level, &levels));
        View v1;
        extract(h1, L.data(), W, H, &v1);
        CHECK(v1.st);
        orbx_extractor_destroy(h1);
        if (mode != 0 || v1.n != vl.n || v1.desc != vl.desc ||
            std::memcmp(v1.kps.data(), vl.kps.data(), (size_t)vl.n * sizeof(orbx_keypoint)) != 0) {
            std::printf("boundary_test: the one-stream extraction differs\n");
            return 4;
        }
    }

    const int nl = vl.n, nr = vr.n;
    bool ok = write_file(dir + "/n.bin", &nl, 4) && write_file(dir + "/nr.bin", &nr, 4) &&
              write_file(dir + "/nvalid.bin", &nvalid, 4) &&
              write_file(dir + "/kps_left.bin", vl.kps.data(), vl.kps.size() * 28) &&
              write_file(dir + "/desc_left.bin", vl.desc.data(), vl.desc.size()) &&
              write_file(dir + "/kps_right.bin", vr.kps.data(), vr.kps.size() * 28) &&
              write_file(dir + "/desc_right.bin", vr.desc.data(), vr.desc.size()) &&
              write_file(dir + "/uRight.bin", uR.data(), uR.size() * 4) &&
              write_file(dir + "/depth.bin", depth.data(), depth.size() * 4) &&
              write_file(dir + "/bow.bin", bow.data(), bow.size() * 4) &&
              write_file(dir + "/tri.bin", tri.data(), (1 + 2 * (size_t)tri[0]) * 4);
    orbx_matcher_destroy(mbow);
    orbx_matcher_destroy(mtri);
    orbx_extractor_destroy(hl);
    orbx_extractor_destroy(hr);
    std::printf("boundary_test: %d / %d keypoints, %d stereo, %d bow, %d triangulation\n", nl, nr,
                nvalid, bow[0], tri[0]);
    return ok ? 0 : 3;
}

// Per-stereo-frame latency of the drop-in path as ORB-SLAM2's Tracking thread sees it
// (bench.py --workload dropin): per frame, Frame::Frame's two std::threads run ExtractORB on
// the left and right images (Frame.cc:89-92), then ComputeStereoMatches (:102); host images
// in, host keypoints / descriptors / uRight / depth out.  DIR holds P pairs
// (pair_<i>_left.raw, pair_<i>_right.raw) and params.txt ("W H nfeatures mbf mb P"); frame f
// uses pair f % P.  `trackers` independent tracking threads (K SLAM sessions sharing the GPU,
// System.cc:91-101 per session), each with its own left / right handle pair, each running
// warmup + nframes frames; they start together after every session's warm-up.  Prints one JSON
// line: every timed frame's latency (steady_clock like Examples/Stereo/stereo_kitti.cc:80-98),
// the wall time of the timed frames over all trackers, and a digest per tracker of its frames'
// outputs (the sessions see the same pairs, so equal digests mean equal results).
static uint64_t fnv1a(uint64_t h, const void* p, size_t n) {
    const uint8_t* b = (const uint8_t*)p;
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

static int bench(const std::string& dir, int nframes, int warmup, int trackers) {
    int W = 0, H = 0, nfeat = 0, P = 0;
    float mbf = 0, mb = 0;
    {
        FILE* f = std::fopen((dir + "/params.txt").c_str(), "r");
        if (!f) return 2;
        const int got = std::fscanf(f, "%d %d %d %f %f %d", &W, &H, &nfeat, &mbf, &mb, &P);
        std::fclose(f);
        if (got != 6 || P < 1) return 2;
    }
    std::vector<std::vector<uint8_t>> Ls((size_t)P), Rs((size_t)P);
    for (int i = 0; i < P; ++i) {
        const std::string b = dir + "/pair_" + std::to_string(i);
        if (!read_file(b + "_left.raw", Ls[(size_t)i]) || !read_file(b + "_right.raw", Rs[(size_t)i]) ||
            Ls[(size_t)i].size() != (size_t)W * H || Rs[(size_t)i].size() != (size_t)W * H)
            return 2;
    }
    trackers = std::max(trackers, 1);
    struct Session {
        orbx_extractor *hl = nullptr, *hr = nullptr;
        std::vector<double> ms;
        long long kp_sum = 0, nv_sum = 0;
        uint64_t digest = 1469598103934665603ull;
        orbx_status st = ORBX_OK;
    };
    std::vector<Session> ss((size_t)trackers);
    orbx_extractor_params p = {nfeat, 1.2f, 8, 20, 7, 1, 1, 0};
    for (Session& s : ss) {
        CHECK(orbx_extractor_create(&p, &s.hl));
        CHECK(orbx_extractor_create(&p, &s.hr));
    }
    std::mutex mu;
    std::condition_variable cv;
    int warm_done = 0;
    bool go = false;
    auto track = [&](Session* s) {
        std::vector<float> uR(4096), depth(4096);
        for (int f = 0; f < warmup + nframes; ++f) {
            if (f == warmup) {   // every session warm, then all timed frames start together
                std::unique_lock<std::mutex> lk(mu);
                if (++warm_done == trackers) { go = true; cv.notify_all(); }
                cv.wait(lk, [&] { return go; });
            }
            const int i = f % P;
            View vl, vr;
            const auto t0 = std::chrono::steady_clock::now();
            std::thread tl(extract, s->hl, Ls[(size_t)i].data(), W, H, &vl);
            std::thread tr(extract, s->hr, Rs[(size_t)i].data(), W, H, &vr);
            tl.join();
            tr.join();
            if (vl.st != ORBX_OK || vr.st != ORBX_OK) { s->st = vl.st != ORBX_OK ? vl.st : vr.st; return; }
            int nvalid = 0;
            if ((int)uR.size() < vl.n) { uR.resize((size_t)vl.n); depth.resize((size_t)vl.n); }
            s->st = orbx_stereo_match(s->hl, s->hr, mbf, mb, uR.data(), depth.data(), vl.n, &nvalid);
            if (s->st != ORBX_OK) return;
            const auto t1 = std::chrono::steady_clock::now();
            if (f >= warmup) {
                s->ms.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
                s->kp_sum += vl.n;
                s->nv_sum += nvalid;
                uint64_t h = fnv1a(s->digest, &vl.n, 4);
                h = fnv1a(h, vl.kps.data(), vl.kps.size() * sizeof(orbx_keypoint));
                h = fnv1a(h, vl.desc.data(), vl.desc.size());
                h = fnv1a(h, vr.kps.data(), vr.kps.size() * sizeof(orbx_keypoint));
                h = fnv1a(h, vr.desc.data(), vr.desc.size());
                h = fnv1a(h, uR.data(), (size_t)vl.n * 4);
                h = fnv1a(h, depth.data(), (size_t)vl.n * 4);
                s->digest = fnv1a(h, &nvalid, 4);
            }
        }
    };
    std::vector<std::thread> th;
    std::chrono::steady_clock::time_point t_go;
    for (Session& s : ss) th.emplace_back(track, &s);
    {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return go; });
        t_go = std::chrono::steady_clock::now();
    }
    for (std::thread& t : th) t.join();
    const double wall_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_go).count();
    long long kp_sum = 0, nv_sum = 0;
    for (Session& s : ss) {
        CHECK(s.st);
        kp_sum += s.kp_sum;
        nv_sum += s.nv_sum;
        orbx_extractor_destroy(s.hl);
        orbx_extractor_destroy(s.hr);
    }
    const long long nt = (long long)nframes * trackers;
    std::printf("{\"frames\": %d, \"warmup\": %d, \"trackers\": %d, \"wall_ms\": %.4f, "
                "\"mean_keypoints_left\": %.3f, \"mean_stereo_matches\": %.3f, \"digests\": [",
                nframes, warmup, trackers, wall_ms, (double)kp_sum / std::max(nt, 1LL),
                (double)nv_sum / std::max(nt, 1LL));
    for (size_t k = 0; k < ss.size(); ++k)
        std::printf("%s\"%016llx\"", k ? ", " : "", (unsigned long long)ss[k].digest);
    std::printf("], \"latency_ms\": [");
    bool first = true;
    for (Session& s : ss)
        for (double v : s.ms) {
            std::printf("%s%.4f", first ? "" : ", ", v);
            first = false;
        }
    std::printf("]}\n");
    return 0;
}

// configs[0] as Tracking::TrackReferenceKeyFrame runs it on one frame (Tracking.cc:805-847):
// ExtractORB of the frame (Frame.cc:204), Frame::ComputeBoW (Frame.cc:420-427, DBoW2 transform
// with levelsup), then ORBmatcher(0.7, true).SearchByBoW(reference keyframe, frame)
// (ORBmatcher.cc:182-319), timed per frame.  DIR: pair_<i>_left.raw (the reference keyframes'
// images, extracted and transformed once, untimed) and pair_<i>_right.raw (the frames), and
// params.txt ("W H nfeatures P levelsup vocabulary_path").  Frame f is matched against
// keyframe f % P; 85 % of a keyframe's features carry a MapPoint (seeded mask).  With DUMPDIR
// the first P frames' keyframe / frame features, BoW / FeatureVectors and matches are written
// there for the parity test (tests/test_boundary_cpp.py).
struct BowFrame {
    View v;
    std::vector<uint32_t> bow_w, fv_node;
    std::vector<double> bow_v;
    std::vector<int32_t> fv_off, fv_feat;
    int32_t nb = 0;
    orbx_featureset fs;
};

// one BowFrame's extraction and transform as raw arrays: PREFIX_kps.bin (28-byte keypoints),
// _desc.bin, _bow_w.bin / _bow_v.bin (nb entries), _fv_node.bin, _fv_off.bin (nodes + 1),
// _fv_feat.bin
static bool dump_bow_frame(const std::string& prefix, const BowFrame& f) {
    const size_t nf = (size_t)f.fs.n_nodes;
    return write_file(prefix + "_kps.bin", f.v.kps.data(), (size_t)f.v.n * 28) &&
           write_file(prefix + "_desc.bin", f.v.desc.data(), (size_t)f.v.n * 32) &&
           write_file(prefix + "_bow_w.bin", f.bow_w.data(), (size_t)f.nb * 4) &&
           write_file(prefix + "_bow_v.bin", f.bow_v.data(), (size_t)f.nb * 8) &&
           write_file(prefix + "_fv_node.bin", f.fv_node.data(), nf * 4) &&
           write_file(prefix + "_fv_off.bin", f.fv_off.data(), (nf + 1) * 4) &&
           write_file(prefix + "_fv_feat.bin", f.fv_feat.data(), (size_t)f.fv_off[nf] * 4);
}

static orbx_status make_bow_frame(orbx_extractor* h, orbx_vocabulary* voc, int levelsup,
                                  const uint8_t* img, int W, int H, BowFrame* f) {
    extract(h, img, W, H, &f->v);
    if (f->v.st != ORBX_OK) return f->v.st;
    const int n = f->v.n;
    f->bow_w.resize((size_t)n + 1);
    f->bow_v.resize((size_t)n + 1);
    f->fv_node.resize((size_t)n + 1);
    f->fv_off.resize((size_t)n + 2);
    f->fv_feat.resize((size_t)n + 1);
    int32_t nb = 0, nf = 0;
    const orbx_status s = orbx_vocabulary_transform(voc, f->v.desc.data(), n, levelsup, nullptr,
                                                    nullptr, f->bow_w.data(), f->bow_v.data(), &nb,
                                                    f->fv_node.data(), f->fv_off.data(),
                                                    f->fv_feat.data(), &nf);
    f->nb = nb;
    std::memset(&f->fs, 0, sizeof(f->fs));
    f->fs.n = n;
    f->fs.keys = f->v.kps.data();
    f->fs.desc = f->v.desc.data();
    f->fs.n_nodes = nf;
    f->fs.node_id = f->fv_node.data();
    f->fs.node_off = f->fv_off.data();
    f->fs.node_feat = f->fv_feat.data();
    return s;
}

static int tum(const std::string& dir, int nframes, int warmup, const std::string& dump) {
    int W = 0, H = 0, nfeat = 0, P = 0, levelsup = 4;
    char vpath[4096] = {0};
    {
        FILE* f = std::fopen((dir + "/params.txt").c_str(), "r");
        if (!f) return 2;
        const int got = std::fscanf(f, "%d %d %d %d %d %4095s", &W, &H, &nfeat, &P, &levelsup, vpath);
        std::fclose(f);
        if (got != 6 || P < 1) return 2;
    }
    std::vector<std::vector<uint8_t>> Ls((size_t)P), Rs((size_t)P);
    for (int i = 0; i < P; ++i) {
        const std::string b = dir + "/pair_" + std::to_string(i);
        if (!read_file(b + "_left.raw", Ls[(size_t)i]) || !read_file(b + "_right.raw", Rs[(size_t)i]))
            return 2;
    }
    orbx_vocabulary* voc = nullptr;
    CHECK(orbx_vocabulary_load_text(vpath, 0, &voc));
    orbx_extractor_params p = {nfeat, 1.2f, 8, 20, 7, 1, 1, 0};
    orbx_extractor *hk = nullptr, *hf = nullptr;
    CHECK(orbx_extractor_create(&p, &hk));
    CHECK(orbx_extractor_create(&p, &hf));
    orbx_matcher* m = nullptr;
    const orbx_matcher_params mp = {0.7f, 1, 0};   // Tracking.cc:812
    CHECK(orbx_matcher_create(&mp, &m));
    std::vector<BowFrame> kfs((size_t)P);
    std::vector<std::vector<uint8_t>> valid((size_t)P);
    uint32_t rng = 12345u;
    for (int i = 0; i < P; ++i) {
        CHECK(make_bow_frame(hk, voc, levelsup, Ls[(size_t)i].data(), W, H, &kfs[(size_t)i]));
        valid[(size_t)i].resize((size_t)kfs[(size_t)i].v.n);
        for (auto& b : valid[(size_t)i]) {
            rng = rng * 1664525u + 1013904223u;
            b = (rng >> 8) % 100 < 85;
        }
    }
    std::vector<double> ms;
    long long matches = 0, kps = 0;
    std::vector<int32_t> out;
    for (int f = 0; f < warmup + nframes; ++f) {
        const int i = f % P;
        BowFrame fr;
        const auto t0 = std::chrono::steady_clock::now();
        CHECK(make_bow_frame(hf, voc, levelsup, Rs[(size_t)i].data(), W, H, &fr));
        out.resize((size_t)std::max(fr.v.n, 1));
        int32_t nm = 0;
        CHECK(orbx_search_by_bow_kf_frame(m, &kfs[(size_t)i].fs, valid[(size_t)i].data(), &fr.fs,
                                          out.data(), &nm));
        const auto t1 = std::chrono::steady_clock::now();
        if (f >= warmup) {
            ms.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
            matches += nm;
            kps += fr.v.n;
        }
        // parity dump (outside the timed interval): the first pass over the P pairs
        if (!dump.empty() && f < P) {
            const std::string b = dump + "/frame_" + std::to_string(i);
            const std::string k = dump + "/kf_" + std::to_string(i);
            if (!dump_bow_frame(b, fr) || !dump_bow_frame(k, kfs[(size_t)i]) ||
                !write_file(k + "_valid.bin", valid[(size_t)i].data(), valid[(size_t)i].size()) ||
                !write_file(b + "_nm.bin", &nm, 4) ||
                !write_file(b + "_matches.bin", out.data(), (size_t)fr.v.n * 4))
                return 3;
        }
    }
    orbx_matcher_destroy(m);
    orbx_extractor_destroy(hk);
    orbx_extractor_destroy(hf);
    orbx_vocabulary_destroy(voc);
    std::printf("{\"frames\": %d, \"warmup\": %d, \"mean_keypoints\": %.3f, "
                "\"mean_bow_matches\": %.3f, \"latency_ms\": [",
                nframes, warmup, (double)kps / std::max(nframes, 1),
                (double)matches / std::max(nframes, 1));
    for (size_t k = 0; k < ms.size(); ++k) std::printf("%s%.4f", k ? ", " : "", ms[k]);
    std::printf("]}\n");
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 2 && std::string(argv[1]) == "layout") return layout();
    if (argc >= 3 && std::string(argv[1]) == "run") return run(argv[2]);
    if (argc >= 5 && std::string(argv[1]) == "bench")
        return bench(argv[2], std::atoi(argv[3]), std::atoi(argv[4]), argc >= 6 ? std::atoi(argv[5]) : 1);
    if (argc >= 5 && std::string(argv[1]) == "tum")
        return tum(argv[2], std::atoi(argv[3]), std::atoi(argv[4]), argc >= 6 ? argv[5] : "");
    std::fprintf(stderr, "usage: %s layout | run DIR | bench DIR NFRAMES WARMUP [TRACKERS] | tum DIR NFRAMES WARMUP [DUMPDIR]\n",
                 argv[0]);
    return 2;
}
