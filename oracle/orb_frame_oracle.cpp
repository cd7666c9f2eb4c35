// orb_frame_oracle.cpp — CPU restatement of Frame::UndistortKeyPoints / ComputeImageBounds
// (src/Frame.cc:429-489) with OpenCV 3.2's cvUndistortPoints (TEST INFRASTRUCTURE ONLY).
// OpenCV is absent from this image: the undistortion is restated from OpenCV 3.2's published
// modules/imgproc/src/undistort.cpp (PARITY UNPINNED against the library).
#include <algorithm>
#include <cstdint>

extern "C" {

// cvUndistortPoints with cameraMatrix = P = K(fx, fy, cx, cy), R = I, 5 iterations.
void oracle_undistort_points(const float* K4, const float* dist, int ndist, const float* xy,
                             int n, float* out) {
    double k[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < ndist && i < 8; ++i) k[i] = dist[i];
    const double A00 = K4[0], A11 = K4[1], A02 = K4[2], A12 = K4[3];
    const double fx = A00, fy = A11, ifx = 1. / fx, ify = 1. / fy, cx = A02, cy = A12;
    // RR = PP * I (cvMatMul), PP = K
    const double RR[3][3] = {{A00, 0, A02}, {0, A11, A12}, {0, 0, 1}};
    const int iters = 5;
    for (int i = 0; i < n; i++) {
        double x, y, x0, y0;
        x = xy[2 * i];
        y = xy[2 * i + 1];
        x0 = x = (x - cx) * ifx;
        y0 = y = (y - cy) * ify;
        for (int j = 0; j < iters; j++) {
            double r2 = x * x + y * y;
            double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) /
                            (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
            double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x);
            double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y;
            x = (x0 - deltaX) * icdist;
            y = (y0 - deltaY) * icdist;
        }
        double xx = RR[0][0] * x + RR[0][1] * y + RR[0][2];
        double yy = RR[1][0] * x + RR[1][1] * y + RR[1][2];
        double ww = 1. / (RR[2][0] * x + RR[2][1] * y + RR[2][2]);
        x = xx * ww;
        y = yy * ww;
        out[2 * i] = (float)x;
        out[2 * i + 1] = (float)y;
    }
}

// Frame::UndistortKeyPoints (Frame.cc:429-459): copy when k1 == 0.
void oracle_undistort_keypoints(const float* K4, const float* dist, int ndist, const float* xy,
                                int n, float* out) {
    if (dist[0] == 0.0) {
        std::copy(xy, xy + 2 * n, out);
        return;
    }
    oracle_undistort_points(K4, dist, ndist, xy, n, out);
}

// Frame::ComputeImageBounds (Frame.cc:461-489): out = minX, maxX, minY, maxY.
void oracle_image_bounds(const float* K4, const float* dist, int ndist, int cols, int rows,
                         float* out) {
    if (dist[0] != 0.0) {
        const float m[8] = {0.0f, 0.0f, (float)cols, 0.0f, 0.0f, (float)rows, (float)cols, (float)rows};
        float u[8];
        oracle_undistort_points(K4, dist, ndist, m, 4, u);
        out[0] = std::min(u[0], u[4]);
        out[1] = std::max(u[2], u[6]);
        out[2] = std::min(u[1], u[3]);
        out[3] = std::max(u[5], u[7]);
    } else {
        out[0] = 0.0f;
        out[1] = cols;
        out[2] = 0.0f;
        out[3] = rows;
    }
}

}  // extern "C"

extern "C" {
// cvtColor(*2GRAY), OpenCV 3.2 RGB2Gray<uchar> (imgproc/src/color.cpp): tab-based integer
// path, yuv_shift = 14, R2Y = 4899, G2Y = 9617, B2Y = 1868, rounding 1 << 13 in the third
// table.  blueIdx = 0 for BGR, 2 for RGB.
void oracle_cvt_gray(const uint8_t* src, int w, int h, int scn, int rgb, uint8_t* dst) {
    const int coeffs[3] = {4899, 9617, 1868};   // R2Y, G2Y, B2Y
    const int blueIdx = rgb ? 2 : 0;
    int tab[256 * 3];
    int b = 0, g = 0, r = (1 << 13);
    const int db = coeffs[blueIdx ^ 2], dg = coeffs[1], dr = coeffs[blueIdx];
    for (int i = 0; i < 256; i++, b += db, g += dg, r += dr) {
        tab[i] = b;
        tab[i + 256] = g;
        tab[i + 512] = r;
    }
    for (int i = 0; i < w * h; i++) {
        const uint8_t* s = src + (size_t)i * scn;
        dst[i] = (uint8_t)((tab[s[0]] + tab[s[1] + 256] + tab[s[2] + 512]) >> 14);
    }
}
}

// ---- Frame::isInFrustum (src/Frame.cc:285-349) + MapPoint::PredictScale (MapPoint.cc:430-444),
// and the query SearchByProjection(Frame&, vpMapPoints, th) builds (ORBmatcher.cc:55-80) -------
// The cv::Mat arithmetic is restated from OpenCV 3.2 (PARITY UNPINNED against the library):
//   mRcw*P + mtcw   MatExpr folds into cv::gemm(Rcw, P, 1, tcw, 1); its small-matrix path
//                   (matmul.cpp, len 3, one output column) sums a_r0*b0 + a_r1*b1 + a_r2*b2 in
//                   float and stores (float)(t*alpha + c*beta) computed in double
//   cv::norm(PO)    normL2_<float, double>: squares summed in double, std::sqrt
//   PO.dot(Pn)      dotProd_32f -> dotProd_<float>: (double)a*b summed in double
// std::log / std::ceil of floats are logf / ceilf: TemplatedVocabulary.h:36 puts `using
// namespace std` in scope of MapPoint.cc and Frame.cc, so the float overloads are chosen.
#include <cmath>
#include <climits>
#include <cstring>

namespace {
struct OMapPoint {
    float pos[3], min_dist, normal[3], max_dist;
};
struct OFrame {
    float Rcw[9], tcw[3], Ow[3];
    float fx, fy, cx, cy, mbf;
    float mnMinX, mnMaxX, mnMinY, mnMaxY;
    float mfLogScaleFactor;
    int mnScaleLevels;
    float mvScaleFactors[16];
};
struct OQuery {
    float u, v, ur, radius;
    int min_level, max_level, pred_level;
    float angle;
};

// MapPoint::PredictScale(const float& currentDist, Frame* pF)
int predict_scale(const OMapPoint& mp, float currentDist, const OFrame& F) {
    float ratio = mp.max_dist / currentDist;
    const float q = std::ceil(std::log(ratio) / F.mfLogScaleFactor);
    // int nScale = ceil(...): the x86 conversion (cvttss2si) gives INT_MIN out of range
    int nScale = (q >= -2147483648.0f && q < 2147483648.0f) ? (int)q : INT_MIN;
    if (nScale < 0)
        nScale = 0;
    else if (nScale >= F.mnScaleLevels)
        nScale = F.mnScaleLevels - 1;
    return nScale;
}

// Frame::isInFrustum(MapPoint* pMP, float viewingCosLimit); fills the mTrack* members
bool is_in_frustum(const OFrame& F, const OMapPoint& mp, float viewingCosLimit, float& u_out,
                   float& v_out, float& ur_out, int& level_out, float& viewcos_out) {
    // const cv::Mat Pc = mRcw*P+mtcw;
    float Pc[3];
    for (int r = 0; r < 3; ++r) {
        const float* a = F.Rcw + 3 * r;
        const float t0 = a[0] * mp.pos[0] + a[1] * mp.pos[1] + a[2] * mp.pos[2];
        const double alpha = 1.0, beta = 1.0;
        Pc[r] = (float)(t0 * alpha + F.tcw[r] * beta);
    }
    const float& PcX = Pc[0];
    const float& PcY = Pc[1];
    const float& PcZ = Pc[2];
    if (PcZ < 0.0f) return false;
    const float invz = 1.0f / PcZ;
    const float u = F.fx * PcX * invz + F.cx;
    const float v = F.fy * PcY * invz + F.cy;
    if (u < F.mnMinX || u > F.mnMaxX) return false;
    if (v < F.mnMinY || v > F.mnMaxY) return false;
    const float maxDistance = 1.2f * mp.max_dist;   // GetMaxDistanceInvariance
    const float minDistance = 0.8f * mp.min_dist;   // GetMinDistanceInvariance
    float PO[3];
    for (int k = 0; k < 3; ++k) PO[k] = mp.pos[k] - F.Ow[k];
    double s = 0;
    for (int k = 0; k < 3; ++k) {
        const double vk = PO[k];
        s += vk * vk;
    }
    const float dist = (float)std::sqrt(s);
    if (dist < minDistance || dist > maxDistance) return false;
    double dot = 0;
    for (int k = 0; k < 3; ++k) dot += (double)PO[k] * mp.normal[k];
    const float viewCos = dot / dist;
    if (viewCos < viewingCosLimit) return false;
    const int nPredictedLevel = predict_scale(mp, dist, F);
    u_out = u;
    ur_out = u - F.mbf * invz;
    v_out = v;
    level_out = nPredictedLevel;
    viewcos_out = viewCos;
    return true;
}

// ORBmatcher::RadiusByViewingCos (ORBmatcher.cc:134-140)
float radius_by_viewing_cos(const float& viewCos) {
    if (viewCos > 0.998)
        return 2.5;
    else
        return 4.0;
}
}  // namespace

extern "C" {
// Tracking::SearchLocalPoints' projection loop (Tracking.cc:1322-1335) over n MapPoints of one
// frame, and the window each in-view MapPoint gets in SearchByProjection (ORBmatcher.cc:55-80):
// q[i] as orbx_proj_query (radius -1 when skip[i] or not in view).  Returns nToMatch.
int oracle_is_in_frustum(const void* frame, const void* mps, int n, const uint8_t* skip,
                         float viewingCosLimit, float th, void* q_out) {
    OFrame F;
    std::memcpy(&F, frame, sizeof(F));
    const OMapPoint* M = (const OMapPoint*)mps;
    OQuery* Q = (OQuery*)q_out;
    const bool bFactor = th != 1.0;
    int nToMatch = 0;
    for (int i = 0; i < n; ++i) {
        OQuery q = {0.0f, 0.0f, 0.0f, -1.0f, -1, -1, -1, 0.0f};
        float u, v, ur, viewCos;
        int level;
        if (!(skip && skip[i]) && is_in_frustum(F, M[i], viewingCosLimit, u, v, ur, level, viewCos)) {
            nToMatch++;
            float r = radius_by_viewing_cos(viewCos);
            if (bFactor) r *= th;
            q = {u, v, ur, r * F.mvScaleFactors[level], level - 1, level, level, 0.0f};
        }
        Q[i] = q;
    }
    return nToMatch;
}
}
