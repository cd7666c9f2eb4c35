/* orbx_frame.h — per-frame geometry helpers around the matchers (src/Frame.cc).
 *
 * Frame::UndistortKeyPoints (src/Frame.cc:429-459) and Frame::ComputeImageBounds (:461-489)
 * call cv::undistortPoints(points, K, DistCoef, noArgument, K).  The OpenCV 3.2 algorithm is
 * restated (modules/imgproc/src/undistort.cpp, cvUndistortPoints): normalise with 1/fx,
 * 1/fy in double, 5 fixed-point iterations of the inverse distortion (k1 k2 p1 p2 [k3 [k4 k5
 * k6]]), re-project with P = K, store as float.  PARITY UNPINNED against the real OpenCV
 * (absent from this image); bit-exact between GPU and the CPU restatement.
 * K is passed as (fx, fy, cx, cy): the reference's K is diag(fx, fy, 1) with (cx, cy) in the
 * last column (Tracking.cc:56-64).
 */
#ifndef ORBX_FRAME_H
#define ORBX_FRAME_H

#include "orbx.h"
#include "orbx_match.h"

#ifdef __cplusplus
extern "C" {
#endif

/* mvKeysUn from mvKeys: a copy when dist[0] == 0 (Frame.cc:431-435), else every keypoint's
 * pt undistorted (other fields copied).  ndist: 4, 5 or 8. */
orbx_status orbx_undistort_keypoints(const float* K4, const float* dist, int32_t ndist,
                                     const orbx_keypoint* kps, int32_t n,
                                     orbx_keypoint* kps_un, int device);
/* Same on device keypoints (n entries, in place allowed), on the caller's stream. */
orbx_status orbx_undistort_keypoints_device(const float* K4, const float* dist, int32_t ndist,
                                            const orbx_keypoint* d_kps, int32_t n,
                                            orbx_keypoint* d_kps_un, void* stream);
/* Frame::ComputeImageBounds: bounds = (mnMinX, mnMaxX, mnMinY, mnMaxY). */
orbx_status orbx_image_bounds(const float* K4, const float* dist, int32_t ndist, int32_t width,
                              int32_t height, float* bounds);

/* Frame::AssignFeaturesToGrid (Frame.cc:243-258, PosInGrid :407-417) on device keypoints:
 * grid_off (cols*rows + 1) and grid_feat (n; features outside the grid are dropped) in the
 * orbx_featureset layout (cell c = ix*rows + iy, indices ascending within a cell). */
orbx_status orbx_assign_grid_device(const orbx_keypoint* d_kps, int32_t n, int32_t cols,
                                    int32_t rows, float min_x, float min_y, float inv_w,
                                    float inv_h, int32_t* d_grid_off, int32_t* d_grid_feat,
                                    void* stream);

/* Batched forms for frames laid out like orbx_batch_view (frame f's keypoints at
 * d_kps + f*kp_stride, d_n[f] of them, device counts).  Grid: frame f's grid_off block at
 * d_grid_off + f*(cols*rows+1), its grid_feat (frame-local indices) at
 * d_grid_feat + f*kp_stride.  Undistort: slots past d_n[f] are left untouched. */
orbx_status orbx_assign_grid_batch_device(const orbx_keypoint* d_kps, int32_t kp_stride,
                                          const int32_t* d_n, int32_t batch, int32_t cols,
                                          int32_t rows, float min_x, float min_y, float inv_w,
                                          float inv_h, int32_t* d_grid_off,
                                          int32_t* d_grid_feat, void* stream);
orbx_status orbx_undistort_keypoints_batch_device(const float* K4, const float* dist,
                                                  int32_t ndist, const orbx_keypoint* d_kps,
                                                  int32_t kp_stride, const int32_t* d_n,
                                                  int32_t batch, orbx_keypoint* d_kps_un,
                                                  void* stream);

/* ---- Frame::isInFrustum + MapPoint::PredictScale (Tracking::SearchLocalPoints' projection of
 * the local map, src/Tracking.cc:1297-1335; src/Frame.cc:285-349; src/MapPoint.cc:394-444) ----
 *
 * One MapPoint as isInFrustum reads it: GetWorldPos(), GetNormal(), and mfMinDistance /
 * mfMaxDistance (the invariance limits 0.8f * min and 1.2f * max are applied here,
 * MapPoint.cc:394-404).  32 bytes. */
typedef struct {
    float pos[3];
    float min_dist;
    float normal[3];
    float max_dist;
} orbx_map_point;

/* A frame's pose and camera as isInFrustum reads them: mRcw (row-major 3x3), mtcw, mOw,
 * fx fy cx cy, mbf, the image bounds (mnMinX, mnMaxX, mnMinY, mnMaxY), mvScaleFactors (nlevels
 * entries) and mfLogScaleFactor (= logf(mfScaleFactor), Frame.cc:82).  The projection query
 * of a MapPoint in view is the one SearchByProjection(Frame&, vpMapPoints, th) builds from
 * mTrackProjX / mTrackProjY / mTrackProjXR / mnTrackScaleLevel / mTrackViewCos
 * (ORBmatcher.cc:46-80). */
typedef struct {
    float Rcw[9];
    float tcw[3];
    float Ow[3];
    float fx, fy, cx, cy, mbf;
    float min_x, max_x, min_y, max_y;
    float log_scale_factor;
    int32_t nlevels;
    float scale[16];
} orbx_frame_pose;

/* For every MapPoint i of every frame f (frame f's MapPoints at [d_mp_off[f], d_mp_off[f+1])
 * of d_mps, d_mp_off on the device): isInFrustum(pMP, viewing_cos_limit) with
 *   Pc = mRcw*P + mtcw as OpenCV 3.2's cv::gemm small-matrix path evaluates it (float
 *        products and sums, + tcw in double, rounded to float),
 *   dist = cv::norm(P - mOw) (squares summed in double, sqrt, float),
 *   viewCos = (P - mOw).dot(normal) / dist (double), rounded to float,
 *   level = PredictScale: ceilf(logf(max_dist / dist) / mfLogScaleFactor) clamped to
 *           [0, nlevels - 1] (glibc 2.35 logf, restated bit for bit, orbx_math.h),
 * and, when in view, the SearchByProjection query d_q[i] = {u, v, ur = u - mbf*invz,
 * radius = RadiusByViewingCos(viewCos) [* th if th != 1] * scale[level], level - 1, level,
 * level, 0}; not in view (or d_skip[i] != 0: the MapPoint is bad or already matched in this
 * frame, Tracking.cc:1316-1320): radius = -1 (the matcher skips it).  d_nvisible[f] (optional)
 * = nToMatch, the frame's MapPoints in view.  max_mps >= every frame's MapPoint count. */
orbx_status orbx_is_in_frustum_batch_device(const orbx_frame_pose* d_frames, int32_t nframes,
                                            const orbx_map_point* d_mps,
                                            const int32_t* d_mp_off, int32_t max_mps,
                                            const uint8_t* d_skip, float viewing_cos_limit,
                                            float th, orbx_proj_query* d_q,
                                            int32_t* d_nvisible, void* stream);
/* One frame, host arrays (copied to the device for the call). */
orbx_status orbx_is_in_frustum(const orbx_frame_pose* frame, const orbx_map_point* mps,
                               int32_t n, const uint8_t* skip, float viewing_cos_limit,
                               float th, orbx_proj_query* q, int32_t* nvisible, int device);

/* Tracking's colour input (src/Tracking.cc:189-214): cv::cvtColor(*2GRAY) for 3- or 4-channel
 * 8-bit images, OpenCV 3.2's integer path RGB2Gray<uchar> (Y = (R*4899 + G*9617 + B*1868 +
 * 8192) >> 14).  rgb = 1 for RGB/RGBA order (mbRGB), 0 for BGR/BGRA.  OpenCV builds with IPP
 * may route BGR2GRAY through ippiColorToGray instead: PARITY UNPINNED against the library. */
orbx_status orbx_cvt_color_device(const uint8_t* d_src, int32_t width, int32_t height,
                                  size_t src_stride, int32_t channels, int32_t rgb,
                                  uint8_t* d_dst, size_t dst_stride, void* stream);
orbx_status orbx_cvt_color(const uint8_t* src, int32_t width, int32_t height, size_t src_stride,
                           int32_t channels, int32_t rgb, uint8_t* dst, size_t dst_stride,
                           int device);

#ifdef __cplusplus
}
#endif
#endif /* ORBX_FRAME_H */
