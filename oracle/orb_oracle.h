// orb_oracle.h — CPU restatement of the reference ORB hot path.  TEST INFRASTRUCTURE ONLY.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this code,
// and only as the checker / the timed CPU baseline.  The product (my_orb_slam2_amd/) never
// links it.
//
// What it restates (file:line relative to the reference root):
//   ORBextractor ctor tables       src/ORBextractor.cc:410-470
//   ComputePyramid                 src/ORBextractor.cc:1129-1154
//   ComputeKeyPointsOctTree        src/ORBextractor.cc:776-875
//   ExtractorNode::DivideNode      src/ORBextractor.cc:481-537
//   DistributeOctTree              src/ORBextractor.cc:539-765
//   IC_Angle / computeOrientation  src/ORBextractor.cc:77-104, 472-479
//   computeOrbDescriptor           src/ORBextractor.cc:108-147, 1056-1063
//   operator()                     src/ORBextractor.cc:1065-1127
//   Frame::ComputeStereoMatches    src/Frame.cc:496-686
// and the OpenCV 3.2 primitives those call (cv::FAST TYPE_9_16 with NMS, cv::resize
// INTER_LINEAR 8U, cv::GaussianBlur 7x7 sigma 2 8U, cv::fastAtan2, cvRound), restated from
// OpenCV's published algorithm — OpenCV is not in this image, so those are PARITY UNPINNED
// against the real library (see DESIGN.md "Oracle").  glibc cosf/sinf are called directly
// (the reference calls them too).
//
// Two documented conventions where the reference itself is not deterministic:
//   * DistributeOctTree phase 2 sorts (size, ExtractorNode*) — ties by heap address.  Here
//     ties go by allocation (push) order, i.e. a never-reusing bump allocator.
//   * ComputeStereoMatches reads Frame::mb before it is assigned (Frame.cc:534 vs :127);
//     the caller passes mb (normally mbf/fx).  An empty match list skips the median step
//     (the reference indexes an empty vector there, Frame.cc:673).
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// cv::KeyPoint field order (28 bytes).
typedef struct {
    float x, y, size, angle, response;
    int octave, class_id;
} okp_t;

// simd = 1: emulate OpenCV 3.2's x86-64 SSE2 vector loops in resize / GaussianBlur (their
//           vertical passes round differently from the scalar tails);
// simd = 0: OpenCV's scalar C++ formulas everywhere.
void* oracle_extractor_create(int nfeatures, float scaleFactor, int nlevels, int iniThFAST,
                              int minThFAST, int simd);
void oracle_extractor_destroy(void* h);
// Returns the keypoint count, or -1 for an empty image (outputs untouched).
int oracle_extract(void* h, const uint8_t* img, int width, int height, int stride);
int oracle_num_keypoints(void* h);
int oracle_get_keypoints(void* h, okp_t* out, int cap);
int oracle_get_descriptors(void* h, uint8_t* out, int cap_rows);
int oracle_num_levels(void* h);
int oracle_level_size(void* h, int level, int* w, int* hgt);
// which: 0 = pyramid level (mvImagePyramid), 1 = Gaussian-blurred level.
int oracle_get_level(void* h, int level, int which, uint8_t* out);
// Per-level FAST candidates (vToDistributeKeys, coordinates relative to minBorder).
int oracle_get_candidates(void* h, int level, okp_t* out, int cap);
// Per-level keypoints after octree + border + orientation (level coordinates).
int oracle_get_level_keypoints(void* h, int level, okp_t* out, int cap);
void oracle_get_tables(void* h, float* scale, float* inv_scale, float* sigma2, float* inv_sigma2,
                       int* features_per_level, int* umax16);

// Frame::ComputeStereoMatches over the last extraction of hL (left) and hR (right).
// uRight / depth: N_left floats each (-1 = no match).  Returns number of valid matches.
int oracle_stereo_match(void* hL, void* hR, float mbf, float mb, float* uRight, float* depth);

// Standalone primitives for unit tests.
void oracle_resize(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst, int dw, int dh,
                   int simd);
void oracle_gaussian7(const uint8_t* src, int w, int h, int stride, uint8_t* dst, int simd);
int oracle_fast(const uint8_t* img, int stride, int rows, int cols, int threshold, okp_t* out,
                int cap);
float oracle_fast_atan2(float y, float x);
void oracle_gaussian_taps(int* taps7);
int oracle_descriptor_distance(const uint8_t* a, const uint8_t* b);

#ifdef __cplusplus
}
#endif
