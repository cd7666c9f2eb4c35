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
