// ORBextractor.h — drop-in replacement for ORB-SLAM2's include/ORBextractor.h (:45-111) and
// src/ORBextractor.cc, header-only, over liborbx's C ABI (include/orbx.h).
//
// A maintainer copies this file over include/ORBextractor.h, deletes src/ORBextractor.cc from
// the ORB_SLAM2 library sources, adds <repo>/include to the include path and links
// <repo>/my_orb_slam2_amd/liborbx.so.  Callers (Frame.cc:80-86, :140-146, :195-201 and the
// ExtractORB threads at Frame.cc:89-92) compile unchanged: the constructor, operator() and the
// getters keep the reference's signatures and results.
//
// mvImagePyramid keeps the reference's contract: sized nlevels in the constructor
// (ORBextractor.cc:433) and refilled by every operator() (:1129-1154), so the reference's own
// Frame::ComputeStereoMatches (Frame.cc:503-619) runs unchanged on it.  Its levels are cv::Mat
// headers over liborbx's pinned host copy of the pyramid (orbx_extractor_host_pyramid: one DMA
// inside the extraction's device sequence, beside its FAST / octree / descriptor kernels), valid
// until this extractor's next operator(), like the reference's, which views into a bordered
// image that the next call replaces.
//
// Opt-out: the glue in orbx_slam2_glue.h replaces that only reader with the device-resident
// orbx_stereo_match (ComputeStereoMatches) or the one-call stereo Frame (ExtractStereo), and
// turns the copy off on the extractors it drives (SetHostPyramid(false)).  operator() then
// leaves nlevels empty Mats, and code that still needs the host pyramid calls
// MaterializePyramid() after the call.  After ExtractStereo both extractors'
// MaterializePyramid() return their view's levels when the LEFT extractor has KeepPyramid(true),
// and throw otherwise, whether the frame ran alone or in a frame-server batch (include/orbx.h
// orbx_extractor_keep_pyramid).
#ifndef ORBX_INTEGRATION_ORBEXTRACTOR_H
#define ORBX_INTEGRATION_ORBEXTRACTOR_H

#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include <opencv2/core/core.hpp>

#include "orbx.h"

namespace ORB_SLAM2 {

class ORBextractor {
public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

    // ORBextractor.cc:410-470: the scale / sigma tables and per-level feature budget come
    // from liborbx (same float arithmetic as the reference constructor).
    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST)
        : nfeatures(nfeatures), scaleFactor(scaleFactor), nlevels(nlevels),
          iniThFAST(iniThFAST), minThFAST(minThFAST) {
        orbx_extractor_params p{nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST,
                                /*cv_simd=*/1, /*max_batch=*/1, /*device=*/0};
        check(orbx_extractor_create(&p, &h), "orbx_extractor_create");
        mvScaleFactor.resize(nlevels);
        mvInvScaleFactor.resize(nlevels);
        mvLevelSigma2.resize(nlevels);
        mvInvLevelSigma2.resize(nlevels);
        mnFeaturesPerLevel.resize(nlevels);
        check(orbx_extractor_tables(h, mvScaleFactor.data(), mvInvScaleFactor.data(),
                                    mvLevelSigma2.data(), mvInvLevelSigma2.data(),
                                    mnFeaturesPerLevel.data()),
              "orbx_extractor_tables");
        mvImagePyramid.resize(nlevels);  // :433
        SetHostPyramid(true);
    }
    ~ORBextractor() { orbx_extractor_destroy(h); }
    ORBextractor(const ORBextractor&) = delete;
    ORBextractor& operator=(const ORBextractor&) = delete;

    // ORBextractor.cc:1065-1127.  The mask is ignored, as in the reference.
    void operator()(cv::InputArray _image, cv::InputArray /*mask*/,
                    std::vector<cv::KeyPoint>& keypoints, cv::OutputArray _descriptors) {
        if (_image.empty()) return;  // :1068-1069
        cv::Mat image = _image.getMat();
        if (image.type() != CV_8UC1)  // :1072 (an assert in the reference)
            throw std::invalid_argument("ORBextractor: image must be CV_8UC1");
        static_assert(sizeof(cv::KeyPoint) == sizeof(orbx_keypoint),
                      "cv::KeyPoint and orbx_keypoint must share their 28-byte layout");
        // the outputs stay in liborbx's pinned block; one copy each into the caller's vector
        // and descriptor Mat
        const orbx_keypoint* kp = nullptr;
        const uint8_t* dsc = nullptr;
        int n = 0;
        check(orbx_extract_view(h, image.data, image.cols, image.rows, (size_t)image.step, &kp,
                                &dsc, &n),
              "orbx_extract_view");
        pyramid_valid = false;
        pyr_src = h;
        pyr_index = 0;
        pyr_owner = alive;
        pyr_serial = orbx_extractor_serial(h);
        if (n < 0) {  // empty image inside liborbx as well
            keypoints.clear();
            return;
        }
        // :1129-1154: this call's levels, headers over liborbx's pinned copy
        orbx_host_pyramid hp{};
        if (host_pyramid && orbx_host_pyramid_view(h, &hp) == ORBX_OK) {
            for (int l = 0; l < nlevels; ++l)
                mvImagePyramid[l] = cv::Mat(hp.height[l], hp.width[l], CV_8U,
                                            const_cast<uint8_t*>(hp.data[l]), hp.step[l]);
            pyramid_valid = true;
        } else {
            for (int l = 0; l < nlevels; ++l) mvImagePyramid[l] = cv::Mat();
        }
        const cv::KeyPoint* k = reinterpret_cast<const cv::KeyPoint*>(kp);
        keypoints.assign(k, k + n);
        if (n == 0) {  // :1086-1088
            _descriptors.release();
            return;
        }
        _descriptors.create(n, 32, CV_8U);  // :1090-1091
        cv::Mat d = _descriptors.getMat();
        if (d.isContinuous()) {
            std::memcpy(d.data, dsc, (size_t)n * 32);
        } else {
            for (int i = 0; i < n; ++i) std::memcpy(d.ptr(i), dsc + (size_t)i * 32, 32);
        }
    }

    int inline GetLevels() { return nlevels; }
    float inline GetScaleFactor() { return (float)scaleFactor; }
    std::vector<float> inline GetScaleFactors() { return mvScaleFactor; }
    std::vector<float> inline GetInverseScaleFactors() { return mvInvScaleFactor; }
    std::vector<float> inline GetScaleSigmaSquares() { return mvLevelSigma2; }
    std::vector<float> inline GetInverseScaleSigmaSquares() { return mvInvLevelSigma2; }

    // Fills mvImagePyramid with the last call's pyramid (ORBextractor.cc:1129-1155's levels,
    // the unblurred images); a no-op when it is already current (after operator() with the
    // host pyramid on).  Throws when the last call left no pyramid (a stereo Frame without
    // KeepPyramid, see the file comment).
    std::vector<cv::Mat>& MaterializePyramid() {
        if (!pyramid_valid) {
            // the source of this view's pyramid must still be the call that set it (after
            // ExtractStereo the right view's source is the left extractor's handle)
            if (pyr_owner.expired())
                throw std::runtime_error("MaterializePyramid: the pyramid's extractor is gone");
            if (orbx_extractor_serial(pyr_src) != pyr_serial)
                throw std::runtime_error("MaterializePyramid: the pyramid's extractor ran "
                                         "another call since this view's frame");
            mvImagePyramid.resize(nlevels);
            for (int l = 0; l < nlevels; ++l) {
                int w = 0, hh = 0;
                check(orbx_pyramid_level(pyr_src, pyr_index, l, nullptr, &w, &hh),
                      "orbx_pyramid_level");
                mvImagePyramid[l].create(hh, w, CV_8U);
                check(orbx_pyramid_level(pyr_src, pyr_index, l, mvImagePyramid[l].data, &w, &hh),
                      "orbx_pyramid_level");
            }
            pyramid_valid = true;
        }
        return mvImagePyramid;
    }

    // Whether operator() refreshes mvImagePyramid (orbx_extractor_host_pyramid; on from the
    // constructor).  The glue switches it off where it replaces the pyramid's only reader.
    void SetHostPyramid(bool on) {
        check(orbx_extractor_host_pyramid(h, on ? 1 : 0), "orbx_extractor_host_pyramid");
        host_pyramid = on;
    }
    bool HostPyramid() const { return host_pyramid; }

    // orbx_extractor_keep_pyramid on this extractor's handle: a stereo Frame extracted through
    // it (orbx_glue::ExtractStereo, this being the LEFT extractor) leaves both views' pyramids.
    void KeepPyramid(bool on) { check(orbx_extractor_keep_pyramid(h, on ? 1 : 0), "orbx_extractor_keep_pyramid"); }

    // Where MaterializePyramid reads from after a call this extractor did not make itself: the
    // stereo Frame ran on `from`'s handle, this view is image `index` of it (the glue sets it).
    void SetPyramidSource(const ORBextractor* from, int index) {
        pyramid_valid = false;
        pyr_src = from->h;
        pyr_index = index;
        pyr_owner = from->alive;
        pyr_serial = orbx_extractor_serial(from->h);
    }

    // The liborbx handle, for orbx_stereo_match (orbx_slam2_glue.h).
    orbx_extractor* handle() const { return h; }

    std::vector<cv::Mat> mvImagePyramid;

protected:
    static void check(orbx_status s, const char* what) {
        if (s != ORBX_OK)
            throw std::runtime_error(std::string(what) + ": " + orbx_last_error());
    }

    orbx_extractor* h = nullptr;
    int nfeatures;
    double scaleFactor;
    int nlevels;
    int iniThFAST;
    int minThFAST;
    std::vector<int> mnFeaturesPerLevel;
    std::vector<float> mvScaleFactor;
    std::vector<float> mvInvScaleFactor;
    std::vector<float> mvLevelSigma2;
    std::vector<float> mvInvLevelSigma2;

private:
    bool host_pyramid = false;
    bool pyramid_valid = false;
    orbx_extractor* pyr_src = nullptr;   // the handle and image holding this view's pyramid
    int pyr_index = 0;
    uint64_t pyr_serial = 0;             // pyr_src's orbx_extractor_serial when it was set
    std::shared_ptr<int> alive = std::make_shared<int>(0);   // expires with this extractor
    std::weak_ptr<int> pyr_owner;        // ... and with pyr_src's
};

}  // namespace ORB_SLAM2

#endif  // ORBX_INTEGRATION_ORBEXTRACTOR_H
