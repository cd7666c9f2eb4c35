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
