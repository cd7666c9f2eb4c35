// orbx_slam2_glue.h — the Frame / ORBmatcher side of the drop-in, as
// templates over the reference's own Frame, KeyFrame and MapPoint classes so that this header
// needs nothing from ORB-SLAM2 beyond the members it names.
//
//   ComputeStereoMatches(F)         replaces Frame::ComputeStereoMatches (src/Frame.cc:496-686)
//   ExtractStereo(F, imL, imR)      replaces Frame.cc:89-102 (both ExtractORB threads + the
//                                   stereo match) by one two-image submission
//   OrbxView / BuildView(f, view)   the orbx_featureset of a Frame / KeyFrame (mFeatVec, mGrid)
//   SearchByBoW(m, pKF, F, out)     ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...) (:182-319)
//
// ORB_SLAM2::ORBextractor is the one of integration/ORBextractor.h (handle()).
#ifndef ORBX_INTEGRATION_SLAM2_GLUE_H
#define ORBX_INTEGRATION_SLAM2_GLUE_H

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include <opencv2/core/core.hpp>

#include "orbx.h"
#include "orbx_match.h"

namespace orbx_glue {

inline void check(orbx_status s, const char* what) {
    if (s != ORBX_OK) throw std::runtime_error(std::string(what) + ": " + orbx_last_error());
}

// Frame.cc:496-686 for the last extraction of both cameras.  The reference reads the member
// mb uninitialised at Frame.cc:534 (it is set only after ComputeStereoMatches returns in the
// stereo constructor, Frame.cc:66-120); the intended value mbf / fx is passed instead.
// It reads the device pyramids, so it turns the extractors' host pyramid copy off for the
// frames after this one (integration/ORBextractor.h, the opt-out).
template <class Frame>
int ComputeStereoMatches(Frame& F) {
    if (F.mpORBextractorLeft->HostPyramid()) F.mpORBextractorLeft->SetHostPyramid(false);
    if (F.mpORBextractorRight->HostPyramid()) F.mpORBextractorRight->SetHostPyramid(false);
    F.mvuRight = std::vector<float>(F.N, -1.0f);
    F.mvDepth = std::vector<float>(F.N, -1.0f);
    int nvalid = 0;
    check(orbx_stereo_match(F.mpORBextractorLeft->handle(), F.mpORBextractorRight->handle(),
                            F.mbf, F.mbf / F.fx, F.mvuRight.data(), F.mvDepth.data(), F.N,
                            &nvalid),
          "orbx_stereo_match");
    return nvalid;
}

// Frame.cc:89-102 in one call (the stereo Frame constructor's two ExtractORB threads, then
// ComputeStereoMatches): both views as one two-image batch on the LEFT extractor's handle with
// the stereo match appended, one submission and one wait (orbx_stereo_frame_view).  Fills
// mvKeys / mDescriptors, mvKeysRight / mDescriptorsRight, N, mvuRight / mvDepth with the same
// values as the two-thread form.  The right extractor's handle is not used.
//
// An empty image: each ExtractORB returns without touching its outputs (ORBextractor.cc:
// 1068-1069), so the views go through the extractors' operator() one by one and no stereo
// match is made (the reference would take the median of an empty vector, Frame.cc:673).
// mvImagePyramid afterwards: see integration/ORBextractor.h (KeepPyramid on the left one).
template <class Frame>
int ExtractStereo(Frame& F, const cv::Mat& imLeft, const cv::Mat& imRight) {
    static_assert(sizeof(cv::KeyPoint) == sizeof(orbx_keypoint), "cv::KeyPoint layout");
    if (imLeft.empty() || imRight.empty()) {
        (*F.mpORBextractorLeft)(imLeft, cv::Mat(), F.mvKeys, F.mDescriptors);
        (*F.mpORBextractorRight)(imRight, cv::Mat(), F.mvKeysRight, F.mDescriptorsRight);
        F.N = (int)F.mvKeys.size();
        F.mvuRight.assign((size_t)F.N, -1.0f);
        F.mvDepth.assign((size_t)F.N, -1.0f);
        return 0;
    }
    if (imLeft.rows != imRight.rows || imLeft.cols != imRight.cols)
        throw std::invalid_argument("ExtractStereo: left and right sizes differ");
    // the match reads the device pyramids: no host copy from the extractors' operator()
    // (empty images above) either
    if (F.mpORBextractorLeft->HostPyramid()) F.mpORBextractorLeft->SetHostPyramid(false);
    if (F.mpORBextractorRight->HostPyramid()) F.mpORBextractorRight->SetHostPyramid(false);
    orbx_stereo_frame_out o{};
    check(orbx_stereo_frame_view(F.mpORBextractorLeft->handle(), imLeft.data,
                                 (size_t)imLeft.step, imRight.data, (size_t)imRight.step,
                                 imLeft.cols, imLeft.rows, F.mbf, F.mbf / F.fx, &o),
          "orbx_stereo_frame_view");
    F.mpORBextractorLeft->SetPyramidSource(F.mpORBextractorLeft, 0);
    F.mpORBextractorRight->SetPyramidSource(F.mpORBextractorLeft, 1);
    auto keys = [](const orbx_keypoint* k, int n) {
        const cv::KeyPoint* c = reinterpret_cast<const cv::KeyPoint*>(k);
        return std::vector<cv::KeyPoint>(c, c + n);
    };
    auto desc = [](const uint8_t* d, int n, cv::Mat& m) {
        if (n == 0) {
            m.release();
            return;
        }
        m.create(n, 32, CV_8U);
        if (m.isContinuous())
            std::memcpy(m.data, d, (size_t)n * 32);
        else
            for (int i = 0; i < n; ++i) std::memcpy(m.ptr(i), d + (size_t)i * 32, 32);
    };
    F.mvKeys = keys(o.kps[0], o.n[0]);
    F.mvKeysRight = keys(o.kps[1], o.n[1]);
    desc(o.desc[0], o.n[0], F.mDescriptors);
    desc(o.desc[1], o.n[1], F.mDescriptorsRight);
    F.N = o.n[0];
    F.mvuRight.assign(o.u_right, o.u_right + o.n[0]);
    F.mvDepth.assign(o.depth, o.depth + o.n[0]);
    return o.n_valid;
}

// CSR copies of mFeatVec (after ComputeBoW) and mGrid (after AssignFeaturesToGrid); the other
// arrays are the frame's own (mvKeysUn, mDescriptors, mvuRight).  Rebuild after either changes.
struct OrbxView {
    std::vector<uint32_t> node_id;
    std::vector<int32_t> node_off, node_feat;
    std::vector<int32_t> grid_off, grid_feat;
    orbx_featureset fs{};
};

template <class F>
void BuildView(const F& f, OrbxView& v, int grid_cols, int grid_rows) {
    v.node_id.clear();
    v.node_off.assign(1, 0);
    v.node_feat.clear();
    for (const auto& kv : f.mFeatVec) {  // std::map: ascending node id
        v.node_id.push_back((uint32_t)kv.first);
        for (auto i : kv.second) v.node_feat.push_back((int32_t)i);
        v.node_off.push_back((int32_t)v.node_feat.size());
    }
    v.grid_off.assign(1, 0);
    v.grid_feat.clear();
    for (int ix = 0; ix < grid_cols; ++ix)  // cell c = ix * rows + iy
        for (int iy = 0; iy < grid_rows; ++iy) {
            for (auto i : f.mGrid[ix][iy]) v.grid_feat.push_back((int32_t)i);
            v.grid_off.push_back((int32_t)v.grid_feat.size());
        }
    static_assert(sizeof(*f.mvKeysUn.data()) == sizeof(orbx_keypoint),
                  "mvKeysUn elements must be cv::KeyPoint (orbx_keypoint's layout)");
    orbx_featureset& s = v.fs;
    s.n = f.N;
    s.keys = reinterpret_cast<const orbx_keypoint*>(f.mvKeysUn.data());
    s.desc = f.mDescriptors.data;  // N x 32, continuous
    s.u_right = f.mvuRight.empty() ? nullptr : f.mvuRight.data();
    s.n_nodes = (int32_t)v.node_id.size();
    s.node_id = v.node_id.data();
    s.node_off = v.node_off.data();
    s.node_feat = v.node_feat.data();
    s.grid_cols = grid_cols;
    s.grid_rows = grid_rows;
    s.grid_off = v.grid_off.data();
    s.grid_feat = v.grid_feat.data();
    s.min_x = f.mnMinX;
    s.min_y = f.mnMinY;
    s.max_x = f.mnMaxX;
    s.max_y = f.mnMaxY;
    s.grid_inv_w = f.mfGridElementWidthInv;
    s.grid_inv_h = f.mfGridElementHeightInv;
}

// ORBmatcher.cc:182-319.  `m` is the ORBmatcher's orbx_matcher (one per thread); kf_view /
// f_view are the BuildView results of pKF and F.
template <class KeyFrame, class Frame, class MapPoint>
int SearchByBoW(orbx_matcher* m, KeyFrame* pKF, const OrbxView& kf_view, Frame& F,
                const OrbxView& f_view, std::vector<MapPoint*>& vpMapPointMatches) {
    const std::vector<MapPoint*> vpMapPointsKF = pKF->GetMapPointMatches();
    std::vector<uint8_t> valid((size_t)pKF->N);
    for (int i = 0; i < pKF->N; ++i)
        valid[(size_t)i] = vpMapPointsKF[(size_t)i] && !vpMapPointsKF[(size_t)i]->isBad();
    std::vector<int32_t> match((size_t)F.N);
    int32_t n = 0;
    check(orbx_search_by_bow_kf_frame(m, &kf_view.fs, valid.data(), &f_view.fs, match.data(), &n),
          "orbx_search_by_bow_kf_frame");
    vpMapPointMatches.assign((size_t)F.N, static_cast<MapPoint*>(nullptr));
    for (int i = 0; i < F.N; ++i)
        if (match[(size_t)i] >= 0) vpMapPointMatches[(size_t)i] = vpMapPointsKF[(size_t)match[(size_t)i]];
    return n;
}

}  // namespace orbx_glue

#endif  // ORBX_INTEGRATION_SLAM2_GLUE_H
