// facade_test — the drop-in facade of INTEGRATION.md compiled and run as ORB-SLAM2 would use it:
// integration/ORBextractor.h (ORB_SLAM2::ORBextractor over liborbx) and
// integration/orbx_slam2_glue.h (Frame::ComputeStereoMatches, the featureset views,
// ORBmatcher::SearchByBoW), with Frame / KeyFrame / MapPoint reduced to the members the facade
// reads.  cv:: comes from tests/native/cv_standin (this image has no OpenCV).
//
//   facade_test nogpu     the ORBextractor constructor on a host without a GPU: must throw
//                         std::runtime_error naming the failing call (no silent fallback)
//   facade_test run DIR   DIR holds left.raw / right.raw (W*H bytes) and params.txt
//                         ("W H nfeatures mbf"); writes the same raw arrays as boundary_test
//                         `run` (n, nr, nvalid, kps/desc of both views, uRight, depth, bow)
//   facade_test bench DIR FRAMES WARMUP K
//                         the stereo Frame constructor's extraction and stereo (Frame.cc:66-120:
//                         two ExtractORB threads, then ComputeStereoMatches) per frame, timed
//                         (steady_clock, as Examples/Stereo/stereo_kitti.cc:80-98), on K
//                         independent tracking threads (K SLAM sessions sharing the GPU); DIR as
//                         boundary_test `bench` (pair_<i>_left/right.raw, params.txt
//                         "W H nfeatures mbf mb P").  Prints boundary_test bench's JSON line.
//   a trailing "frame" on run / bench: each stereo frame through orbx_glue::ExtractStereo
//   (both views as one two-image submission with the stereo match appended); a trailing "pyr"
//   on bench: the two ExtractORB threads keep refreshing mvImagePyramid (the host pyramid copy
//   on, as for an unchanged Frame::ComputeStereoMatches) and the stereo match runs through the
//   C ABI directly, so the line prices operator()'s pyramid copy
//
// `run` (threads) also checks the mvImagePyramid contract (ORBextractor.h:85, ORBextractor.cc:433,
// 1129-1154): both extractors' levels after operator() go to pyr_left.bin / pyr_right.bin (every
// level, rows tightly packed) for the oracle comparison, and the reference's own stereo body
// (Frame.cc:496-686, restated below over those cv::Mat levels) must give the same uRight / depth
// as orbx_glue::ComputeStereoMatches.
#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "ORBextractor.h"
#include "orbx_slam2_glue.h"

namespace {

constexpr int FRAME_GRID_COLS = 64;  // Frame.h:33-34
constexpr int FRAME_GRID_ROWS = 48;

struct MapPoint {
    bool bad = false;
    bool isBad() const { return bad; }
};

// The members of ORB_SLAM2::Frame (Frame.h) the facade reads or writes.
struct Frame {
    ORB_SLAM2::ORBextractor* mpORBextractorLeft = nullptr;
    ORB_SLAM2::ORBextractor* mpORBextractorRight = nullptr;
    float fx = 0.f, mbf = 0.f;
    int N = 0;
    std::vector<cv::KeyPoint> mvKeys, mvKeysRight, mvKeysUn;
    cv::Mat mDescriptors, mDescriptorsRight;
    std::vector<float> mvuRight, mvDepth;
    std::map<unsigned int, std::vector<unsigned int>> mFeatVec;
    std::vector<std::size_t> mGrid[FRAME_GRID_COLS][FRAME_GRID_ROWS];
    float mnMinX = 0.f, mnMinY = 0.f, mnMaxX = 0.f, mnMaxY = 0.f;
    float mfGridElementWidthInv = 0.f, mfGridElementHeightInv = 0.f;

    // Frame.cc:240-249
    void ExtractORB(int flag, const cv::Mat& im) {
        if (flag == 0)
            (*mpORBextractorLeft)(im, cv::Mat(), mvKeys, mDescriptors);
        else
            (*mpORBextractorRight)(im, cv::Mat(), mvKeysRight, mDescriptorsRight);
    }

    // Frame::ComputeStereoMatches as the reference has it (Frame.cc:496-686), restated over the
    // extractors' mvImagePyramid (the drop-in must keep that member valid for exactly this
    // body).  mb is passed (the reference reads it before it is set, Frame.cc:534 / :127).  An
    // empty vDistIdx skips the cut (the reference takes the median of an empty vector, UB).
    int ComputeStereoMatchesReference(float mb) {
        mvuRight = std::vector<float>(N, -1.0f);
        mvDepth = std::vector<float>(N, -1.0f);
        const std::vector<float> sf = mpORBextractorLeft->GetScaleFactors();
        const std::vector<float> isf = mpORBextractorLeft->GetInverseScaleFactors();
        const int TH_HIGH = 100, TH_LOW = 50;
        const int thOrbDist = (TH_HIGH + TH_LOW) / 2;
        const int nRows = mpORBextractorLeft->mvImagePyramid[0].rows;
        std::vector<std::vector<size_t>> rows((size_t)nRows);
        const int Nr = (int)mvKeysRight.size();
        for (int iR = 0; iR < Nr; iR++) {
            const cv::KeyPoint& kp = mvKeysRight[(size_t)iR];
            const float r = 2.0f * sf[(size_t)kp.octave];
            const int maxr = (int)std::ceil(kp.pt.y + r), minr = (int)std::floor(kp.pt.y - r);
            for (int yi = minr; yi <= maxr; yi++) rows[(size_t)yi].push_back((size_t)iR);
        }
        const float minZ = mb, minD = 0, maxD = mbf / minZ;
        std::vector<std::pair<int, int>> vDistIdx;
        for (int iL = 0; iL < N; iL++) {
            const cv::KeyPoint& kpL = mvKeys[(size_t)iL];
            const int levelL = kpL.octave;
            const float vL = kpL.pt.y, uL = kpL.pt.x;
            const std::vector<size_t>& cand = rows[(size_t)vL];
            if (cand.empty()) continue;
            const float minU = uL - maxD, maxU = uL - minD;
            if (maxU < 0) continue;
            int bestDist = TH_HIGH;
            size_t bestIdxR = 0;
            for (size_t iR : cand) {
                const cv::KeyPoint& kpR = mvKeysRight[iR];
                if (kpR.octave < levelL - 1 || kpR.octave > levelL + 1) continue;
                const float uR = kpR.pt.x;
                if (uR >= minU && uR <= maxU) {
                    const uint32_t* a = (const uint32_t*)mDescriptors.ptr(iL);
                    const uint32_t* b = (const uint32_t*)mDescriptorsRight.ptr((int)iR);
                    int dist = 0;   // ORBmatcher::DescriptorDistance (:1715-1731)
                    for (int k = 0; k < 8; ++k) dist += __builtin_popcount(a[k] ^ b[k]);
                    if (dist < bestDist) { bestDist = dist; bestIdxR = iR; }
                }
            }
            if (bestDist >= thOrbDist) continue;
            const float uR0 = mvKeysRight[bestIdxR].pt.x;
            const float scaleFactor = isf[(size_t)kpL.octave];
            const float scaleduL = std::round(kpL.pt.x * scaleFactor);
            const float scaledvL = std::round(kpL.pt.y * scaleFactor);
            const float scaleduR0 = std::round(uR0 * scaleFactor);
            const int w = 5;
            const cv::Mat& PL = mpORBextractorLeft->mvImagePyramid[(size_t)kpL.octave];
            const cv::Mat& PR = mpORBextractorRight->mvImagePyramid[(size_t)kpL.octave];
            cv::Mat IL = PL.rowRange((int)scaledvL - w, (int)scaledvL + w + 1)
                             .colRange((int)scaleduL - w, (int)scaleduL + w + 1);
            IL.convertTo(IL, CV_32F);
            IL = IL - IL.at<float>(w, w) * cv::Mat::ones(IL.rows, IL.cols, CV_32F);
            int bestSad = INT_MAX, bestincR = 0;
            const int L = 5;
            std::vector<float> vDists(2 * L + 1);
            const float iniu = scaleduR0 + L - w, endu = scaleduR0 + L + w + 1;
            if (iniu < 0 || endu >= PR.cols) continue;
            for (int incR = -L; incR <= +L; incR++) {
                cv::Mat IR = PR.rowRange((int)scaledvL - w, (int)scaledvL + w + 1)
                                 .colRange((int)scaleduR0 + incR - w, (int)scaleduR0 + incR + w + 1);
                IR.convertTo(IR, CV_32F);
                IR = IR - IR.at<float>(w, w) * cv::Mat::ones(IR.rows, IR.cols, CV_32F);
                const float dist = (float)cv::norm(IL, IR, cv::NORM_L1);
                if (dist < bestSad) { bestSad = (int)dist; bestincR = incR; }
                vDists[(size_t)(L + incR)] = dist;
            }
            if (bestincR == -L || bestincR == L) continue;
            const float dist1 = vDists[(size_t)(L + bestincR - 1)];
            const float dist2 = vDists[(size_t)(L + bestincR)];
            const float dist3 = vDists[(size_t)(L + bestincR + 1)];
            const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
            if (deltaR < -1 || deltaR > 1) continue;
            float bestuR = sf[(size_t)kpL.octave] * ((float)scaleduR0 + (float)bestincR + deltaR);
            float disparity = (uL - bestuR);
            if (disparity >= minD && disparity < maxD) {
                if (disparity <= 0) {
                    disparity = 0.01f;
                    bestuR = uL - 0.01f;
                }
                mvDepth[(size_t)iL] = mbf / disparity;
                mvuRight[(size_t)iL] = bestuR;
                vDistIdx.push_back(std::pair<int, int>(bestSad, iL));
            }
        }
        std::sort(vDistIdx.begin(), vDistIdx.end());
        int nvalid = (int)vDistIdx.size();
        if (vDistIdx.empty()) return 0;
        const float median = (float)vDistIdx[vDistIdx.size() / 2].first;
        const float thDist = 1.5f * 1.4f * median;
        for (int i = (int)vDistIdx.size() - 1; i >= 0; i--) {
            if (vDistIdx[(size_t)i].first < thDist) break;
            mvuRight[(size_t)vDistIdx[(size_t)i].second] = -1;
            mvDepth[(size_t)vDistIdx[(size_t)i].second] = -1;
            --nvalid;
        }
        return nvalid;
    }
};

// Every level of an extractor's mvImagePyramid, rows tightly packed, level after level.
bool dump_pyramid(const ORB_SLAM2::ORBextractor& ex, std::vector<uint8_t>& out) {
    out.clear();
    if (ex.mvImagePyramid.size() != 8) return false;
    for (const cv::Mat& m : ex.mvImagePyramid) {
        if (m.empty() || m.type() != CV_8U) return false;
        for (int y = 0; y < m.rows; ++y) out.insert(out.end(), m.ptr(y), m.ptr(y) + m.cols);
    }
    return true;
}

// The members of ORB_SLAM2::KeyFrame SearchByBoW reads.
struct KeyFrame {
    int N = 0;
    std::vector<MapPoint*> mvpMapPoints;
    std::vector<MapPoint*> GetMapPointMatches() const { return mvpMapPoints; }
};

bool read_file(const std::string& path, std::vector<uint8_t>& out) {
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

bool write_file(const std::string& path, const void* p, size_t n) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    const bool ok = n == 0 || std::fwrite(p, 1, n, f) == n;
    std::fclose(f);
    return ok;
}

int nogpu() {
    try {
        ORB_SLAM2::ORBextractor ex(1000, 1.2f, 8, 20, 7);
    } catch (const std::runtime_error& e) {
        std::printf("facade_test: constructor threw: %s\n", e.what());
        return std::strstr(e.what(), "orbx_extractor_create") ? 0 : 5;
    }
    std::printf("facade_test: constructor succeeded without a GPU\n");
    return 6;
}

int run(const std::string& dir, bool frame_call) {
    int W = 0, H = 0, nfeat = 0;
    float mbf = 0.f;
    {
        FILE* f = std::fopen((dir + "/params.txt").c_str(), "r");
        if (!f) return 2;
        const int got = std::fscanf(f, "%d %d %d %f", &W, &H, &nfeat, &mbf);
        std::fclose(f);
        if (got != 4) return 2;
    }
    std::vector<uint8_t> L, R;
    if (!read_file(dir + "/left.raw", L) || !read_file(dir + "/right.raw", R) ||
        L.size() != (size_t)W * H || R.size() != (size_t)W * H)
        return 2;

    // Tracking.cc:136-139: one extractor per camera
    ORB_SLAM2::ORBextractor left(nfeat, 1.2f, 8, 20, 7), right(nfeat, 1.2f, 8, 20, 7);
    if (left.GetLevels() != 8 || left.GetScaleFactors().size() != 8 ||
        left.GetScaleFactor() != 1.2f || left.GetScaleSigmaSquares()[1] != 1.2f * 1.2f) {
        std::printf("facade_test: scale tables differ\n");
        return 4;
    }
    // an empty image returns without touching the outputs (ORBextractor.cc:1068-1069)
    {
        std::vector<cv::KeyPoint> kp(3);
        cv::Mat d;
        left(cv::Mat(), cv::Mat(), kp, d);
        if (kp.size() != 3 || !d.empty()) {
            std::printf("facade_test: empty image changed the outputs\n");
            return 4;
        }
    }
    Frame F;
    F.mpORBextractorLeft = &left;
    F.mpORBextractorRight = &right;
    F.mbf = mbf;
    F.fx = 718.856f;  // KITTI 00-02 (Examples/Stereo/KITTI00-02.yaml)
    // the image rows are W bytes apart; a Mat over a wider buffer checks `step` handling
    const size_t pitch = (size_t)W + 24;
    std::vector<uint8_t> Lp(pitch * H, 0xA5);
    for (int y = 0; y < H; ++y) std::memcpy(&Lp[(size_t)y * pitch], &L[(size_t)y * W], (size_t)W);
    const cv::Mat imL(H, W, CV_8UC1, Lp.data(), pitch), imR(H, W, CV_8UC1, R.data());
    int nvalid = 0;
    if (frame_call) {   // Frame.cc:89-102 as one two-image submission
        // without KeepPyramid no pyramid is left (a fixed state, solo or served) ...
        nvalid = orbx_glue::ExtractStereo(F, imL, imR);
        try {
            left.MaterializePyramid();
            std::printf("facade_test: a pyramid after ExtractStereo without KeepPyramid\n");
            return 4;
        } catch (const std::runtime_error&) {
        }
        // ... with it both views' pyramids (checked below); the outputs are the same
        left.KeepPyramid(true);
        nvalid = orbx_glue::ExtractStereo(F, imL, imR);
        // an empty view: the extractors return silently (ORBextractor.cc:1068-1069)
        Frame E;
        E.mpORBextractorLeft = &left;
        E.mpORBextractorRight = &right;
        E.mbf = F.mbf;
        E.fx = F.fx;
        if (orbx_glue::ExtractStereo(E, cv::Mat(), imR) != 0 || E.N != 0 || !E.mvKeys.empty() ||
            E.mvKeysRight.empty()) {
            std::printf("facade_test: ExtractStereo with an empty left image\n");
            return 4;
        }
        nvalid = orbx_glue::ExtractStereo(F, imL, imR);
        {   // the right view's pyramid source is the left handle: another call on it first
            // makes MaterializePyramid throw instead of returning another frame's levels
            Frame G;
            G.mpORBextractorLeft = &left;
            G.mpORBextractorRight = &right;
            G.mbf = F.mbf;
            G.fx = F.fx;
            orbx_glue::ExtractStereo(G, imL, imR);
            std::vector<cv::KeyPoint> k2;
            cv::Mat d2;
            left(imR, cv::Mat(), k2, d2);   // the left handle moves on
            try {
                right.MaterializePyramid();
                std::printf("facade_test: a stale pyramid source was not detected\n");
                return 4;
            } catch (const std::runtime_error&) {
            }
        }
        nvalid = orbx_glue::ExtractStereo(F, imL, imR);
    } else {   // Frame.cc:89-92
        // the constructor sized mvImagePyramid (ORBextractor.cc:433)
        if (left.mvImagePyramid.size() != 8 || !left.HostPyramid()) {
            std::printf("facade_test: mvImagePyramid not sized / host pyramid off after the constructor\n");
            return 4;
        }
        std::thread tl(&Frame::ExtractORB, &F, 0, std::cref(imL));
        std::thread tr(&Frame::ExtractORB, &F, 1, std::cref(imR));
        tl.join();
        tr.join();
    }
    F.N = (int)F.mvKeys.size();
    const int nr = (int)F.mvKeysRight.size();
    if (F.N == 0 || nr == 0 || F.mDescriptors.rows != F.N || F.mDescriptors.cols != 32 ||
        !F.mDescriptors.isContinuous()) {
        std::printf("facade_test: bad extraction outputs\n");
        return 4;
    }
    // mvImagePyramid on request: level 0 is the input image (both views after ExtractStereo)
    for (int v = 0; v < (frame_call ? 2 : 1); ++v) {
        std::vector<cv::Mat>& pyr = (v ? right : left).MaterializePyramid();
        const std::vector<uint8_t>& img = v ? R : L;
        if (pyr.size() != 8 || pyr[0].rows != H || pyr[0].cols != W) return 4;
        for (int y = 0; y < H; ++y)
            if (std::memcmp(pyr[0].ptr(y), &img[(size_t)y * W], (size_t)W) != 0) {
                std::printf("facade_test: mvImagePyramid[0] of view %d differs from the input\n", v);
                return 4;
            }
    }
    if (!frame_call) {
        // every level of both views straight after operator() (the oracle compares them) ...
        std::vector<uint8_t> pl, pr;
        if (!dump_pyramid(left, pl) || !dump_pyramid(right, pr) ||
            !write_file(dir + "/pyr_left.bin", pl.data(), pl.size()) ||
            !write_file(dir + "/pyr_right.bin", pr.data(), pr.size())) {
            std::printf("facade_test: mvImagePyramid incomplete after operator()\n");
            return 4;
        }
        // ... and the reference's own stereo body over them equals the glue's device match
        const int nref = F.ComputeStereoMatchesReference(F.mbf / F.fx);
        const std::vector<float> uref = F.mvuRight, dref = F.mvDepth;
        nvalid = orbx_glue::ComputeStereoMatches(F);
        if (nref != nvalid || uref.size() != F.mvuRight.size() ||
            std::memcmp(uref.data(), F.mvuRight.data(), uref.size() * 4) != 0 ||
            std::memcmp(dref.data(), F.mvDepth.data(), dref.size() * 4) != 0) {
            std::printf("facade_test: Frame.cc's stereo body over mvImagePyramid (%d) differs "
                        "from orbx_glue::ComputeStereoMatches (%d)\n", nref, nvalid);
            return 4;
        }
        if (!write_file(dir + "/nvalid_ref.bin", &nref, 4)) return 3;
        // the glue turned the host copy off (it reads the device pyramids): the next
        // operator() leaves empty levels, MaterializePyramid() fills them on request
        if (left.HostPyramid() || right.HostPyramid()) {
            std::printf("facade_test: host pyramid still on after the glue's stereo match\n");
            return 4;
        }
        std::vector<cv::KeyPoint> k2;
        cv::Mat d2;
        left(imL, cv::Mat(), k2, d2);
        if (left.mvImagePyramid.size() != 8 || !left.mvImagePyramid[0].empty()) {
            std::printf("facade_test: stale mvImagePyramid after the opt-out\n");
            return 4;
        }
        std::vector<uint8_t> pl2;
        left.MaterializePyramid();
        if (!dump_pyramid(left, pl2) || pl2 != pl) {
            std::printf("facade_test: MaterializePyramid after the opt-out differs\n");
            return 4;
        }
        // the source check: the right extractor's view does not outlive its handle's next call
        left.SetHostPyramid(true);
        left(imL, cv::Mat(), k2, d2);
        if (!dump_pyramid(left, pl2) || pl2 != pl) {
            std::printf("facade_test: mvImagePyramid after re-enabling differs\n");
            return 4;
        }
    }

    // SearchByBoW(KF = right view, F = left view), one vocabulary node holding every feature
    F.mvKeysUn = F.mvKeys;
    for (int i = 0; i < F.N; ++i) F.mFeatVec[0].push_back((unsigned)i);
    Frame KFf;
    KFf.N = nr;
    KFf.mvKeysUn = F.mvKeysRight;
    KFf.mDescriptors = F.mDescriptorsRight;
    for (int i = 0; i < nr; ++i) KFf.mFeatVec[0].push_back((unsigned)i);
    orbx_glue::OrbxView fv, kv;
    orbx_glue::BuildView(F, fv, FRAME_GRID_COLS, FRAME_GRID_ROWS);
    orbx_glue::BuildView(KFf, kv, FRAME_GRID_COLS, FRAME_GRID_ROWS);
    kv.fs.u_right = nullptr;
    fv.fs.u_right = nullptr;
    std::vector<MapPoint> points((size_t)nr);
    KeyFrame KF;
    KF.N = nr;
    for (MapPoint& p : points) KF.mvpMapPoints.push_back(&p);
    orbx_matcher* m = nullptr;
    const orbx_matcher_params mp = {0.75f, 1, 0};
    orbx_glue::check(orbx_matcher_create(&mp, &m), "orbx_matcher_create");
    std::vector<MapPoint*> matches;
    const int nbow = orbx_glue::SearchByBoW(m, &KF, kv, F, fv, matches);
    orbx_matcher_destroy(m);
    std::vector<int32_t> bow(1 + (size_t)F.N, -1);
    bow[0] = nbow;
    for (int i = 0; i < F.N; ++i)
        if (matches[(size_t)i]) bow[1 + (size_t)i] = (int32_t)(matches[(size_t)i] - points.data());

    const bool ok =
        write_file(dir + "/n.bin", &F.N, 4) && write_file(dir + "/nr.bin", &nr, 4) &&
        write_file(dir + "/nvalid.bin", &nvalid, 4) &&
        write_file(dir + "/kps_left.bin", F.mvKeys.data(), F.mvKeys.size() * 28) &&
        write_file(dir + "/desc_left.bin", F.mDescriptors.data, (size_t)F.N * 32) &&
        write_file(dir + "/kps_right.bin", F.mvKeysRight.data(), F.mvKeysRight.size() * 28) &&
        write_file(dir + "/desc_right.bin", F.mDescriptorsRight.data, (size_t)nr * 32) &&
        write_file(dir + "/uRight.bin", F.mvuRight.data(), F.mvuRight.size() * 4) &&
        write_file(dir + "/depth.bin", F.mvDepth.data(), F.mvDepth.size() * 4) &&
        write_file(dir + "/bow.bin", bow.data(), bow.size() * 4);
    std::printf("facade_test: %d / %d keypoints, %d stereo, %d bow\n", F.N, nr, nvalid, nbow);
    return ok ? 0 : 3;
}

uint64_t fnv1a(uint64_t h, const void* p, size_t n) {
    const uint8_t* b = (const uint8_t*)p;
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

int bench(const std::string& dir, int nframes, int warmup, int trackers, bool frame_call,
          bool host_pyr) {
    int W = 0, H = 0, nfeat = 0, P = 0;
    float mbf = 0.f, mb = 0.f;
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
        std::unique_ptr<ORB_SLAM2::ORBextractor> left, right;   // Tracking.cc:136-139
        std::vector<double> ms;
        long long kp_sum = 0, nv_sum = 0;
        uint64_t digest = 1469598103934665603ull;
        std::string err;
    };
    // Frame::fx such that the glue's mbf / fx is the params' mb exactly (boundary_test `bench`
    // passes mb itself)
    float fx = mbf / mb;
    for (int t = 0; t < 8 && mbf / fx != mb; ++t)
        fx = std::nextafter(fx, mbf / fx > mb ? 1e30f : 0.f);
    if (mbf / fx != mb) return 2;
    std::vector<Session> ss((size_t)trackers);
    for (Session& s : ss) {
        s.left.reset(new ORB_SLAM2::ORBextractor(nfeat, 1.2f, 8, 20, 7));
        s.right.reset(new ORB_SLAM2::ORBextractor(nfeat, 1.2f, 8, 20, 7));
    }
    std::mutex mu;
    std::condition_variable cv;
    int warm_done = 0;
    bool go = false;
    auto track = [&](Session* s) {
        try {
            for (int f = 0; f < warmup + nframes; ++f) {
                if (f == warmup) {   // every session warm, then all timed frames start together
                    std::unique_lock<std::mutex> lk(mu);
                    if (++warm_done == trackers) { go = true; cv.notify_all(); }
                    cv.wait(lk, [&] { return go; });
                }
                const int i = f % P;
                const cv::Mat imL(H, W, CV_8UC1, Ls[(size_t)i].data()),
                    imR(H, W, CV_8UC1, Rs[(size_t)i].data());
                const auto t0 = std::chrono::steady_clock::now();
                Frame F;   // the stereo Frame constructor (Frame.cc:66-120)
                F.mpORBextractorLeft = s->left.get();
                F.mpORBextractorRight = s->right.get();
                F.mbf = mbf;
                F.fx = fx;
                int nvalid = 0;
                if (frame_call) {   // Frame.cc:89-102 as one two-image submission
                    nvalid = orbx_glue::ExtractStereo(F, imL, imR);
                } else if (host_pyr) {   // mvImagePyramid refreshed by every operator()
                    std::thread tl(&Frame::ExtractORB, &F, 0, std::cref(imL));
                    std::thread tr(&Frame::ExtractORB, &F, 1, std::cref(imR));
                    tl.join();
                    tr.join();
                    F.N = (int)F.mvKeys.size();
                    if (F.mpORBextractorLeft->mvImagePyramid[0].empty())
                        throw std::runtime_error("bench pyr: no mvImagePyramid");
                    F.mvuRight.assign((size_t)F.N, -1.f);
                    F.mvDepth.assign((size_t)F.N, -1.f);
                    orbx_glue::check(orbx_stereo_match(F.mpORBextractorLeft->handle(),
                                                       F.mpORBextractorRight->handle(), F.mbf,
                                                       F.mbf / F.fx, F.mvuRight.data(),
                                                       F.mvDepth.data(), F.N, &nvalid),
                                     "orbx_stereo_match");
                } else {
                    std::thread tl(&Frame::ExtractORB, &F, 0, std::cref(imL));
                    std::thread tr(&Frame::ExtractORB, &F, 1, std::cref(imR));
                    tl.join();
                    tr.join();
                    F.N = (int)F.mvKeys.size();
                    nvalid = orbx_glue::ComputeStereoMatches(F);
                }
                const auto t1 = std::chrono::steady_clock::now();
                if (f >= warmup) {
                    s->ms.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
                    s->kp_sum += F.N;
                    s->nv_sum += nvalid;
                    const int nr = (int)F.mvKeysRight.size();
                    uint64_t h = fnv1a(s->digest, &F.N, 4);
                    h = fnv1a(h, F.mvKeys.data(), (size_t)F.N * sizeof(cv::KeyPoint));
                    h = fnv1a(h, F.mDescriptors.data, (size_t)F.N * 32);
                    h = fnv1a(h, F.mvKeysRight.data(), (size_t)nr * sizeof(cv::KeyPoint));
                    h = fnv1a(h, F.mDescriptorsRight.data, (size_t)nr * 32);
                    h = fnv1a(h, F.mvuRight.data(), (size_t)F.N * 4);
                    h = fnv1a(h, F.mvDepth.data(), (size_t)F.N * 4);
                    s->digest = fnv1a(h, &nvalid, 4);
                }
            }
        } catch (const std::exception& e) {
            s->err = e.what();
            std::unique_lock<std::mutex> lk(mu);
            if (!go) { ++warm_done; if (warm_done == trackers) { go = true; cv.notify_all(); } }
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
        if (!s.err.empty()) {
            std::fprintf(stderr, "facade_test bench: %s\n", s.err.c_str());
            return 1;
        }
        kp_sum += s.kp_sum;
        nv_sum += s.nv_sum;
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

}  // namespace

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "";
    try {
        if (mode == "nogpu") return nogpu();
        // a trailing "frame": the stereo Frame's extraction and matching as one call
        // (orbx_glue::ExtractStereo) instead of two ExtractORB threads + ComputeStereoMatches
        const bool frame_call = std::string(argv[argc - 1]) == "frame";
        const bool host_pyr = std::string(argv[argc - 1]) == "pyr";
        if (mode == "run" && argc > 2) return run(argv[2], frame_call);
        if (mode == "bench" && argc > 5)
            return bench(argv[2], std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5]),
                         frame_call, host_pyr);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "facade_test: %s\n", e.what());
        return 1;
    }
    std::fprintf(stderr, "usage: facade_test nogpu | run DIR [frame] | bench DIR FRAMES WARMUP K [frame|pyr]\n");
    return 2;
}
