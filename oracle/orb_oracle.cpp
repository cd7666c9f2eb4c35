// orb_oracle.cpp — CPU restatement of the reference ORB extractor + stereo matcher.
// TEST INFRASTRUCTURE ONLY (see orb_oracle.h for scope, citations and conventions).
//
// The structure deliberately follows the reference's own control flow (per-cell FAST calls,
// std::list octree, per-keypoint loops) so that each block can be read against the cited
// reference lines; it is not meant to be fast.
#include "orb_oracle.h"

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstring>
#include <list>
#include <utility>
#include <vector>

namespace {

typedef okp_t KeyPoint;

KeyPoint make_kp(float x, float y, float size, float angle, float response, int octave = 0) {
    KeyPoint k;
    k.x = x; k.y = y; k.size = size; k.angle = angle; k.response = response;
    k.octave = octave; k.class_id = -1;
    return k;
}

// ------------------------------------------------------------------------------------------
// OpenCV 3.2 scalar helpers [restated; x86-64 SSE2 semantics]
// ------------------------------------------------------------------------------------------
inline int cvRound(double v) { return (int)lrint(v); }   // cvtsd2si: round half to even
inline int cvRound(float v) { return (int)lrintf(v); }   // cvtss2si
inline int cvFloor(float v) { int i = cvRound(v); float diff = (float)(v - i); return i - (diff < 0); }
inline int cvCeil(float v) { int i = cvRound(v); float diff = (float)(i - v); return i + (diff < 0); }
inline short sat_short_from_float(float v) {
    int i = cvRound(v);
    return (short)(i < SHRT_MIN ? SHRT_MIN : i > SHRT_MAX ? SHRT_MAX : i);
}
inline uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

// cv::borderInterpolate for BORDER_REFLECT_101.
int reflect101(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p - 1 + 1;
        else p = len - 1 - (p - len) - 1;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

// cv::fastAtan2 (core/src/mathfuncs.cpp, OpenCV 3.2).
float fastAtan2(float y, float x) {
    static const float k = (float)(180 / 3.14159265358979323846);
    static const float atan2_p1 = 0.9997878412794807f * k;
    static const float atan2_p3 = -0.3258083974640975f * k;
    static const float atan2_p5 = 0.1555786518463281f * k;
    static const float atan2_p7 = -0.04432655554792128f * k;
    float ax = std::fabs(x), ay = std::fabs(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((atan2_p7 * c2 + atan2_p5) * c2 + atan2_p3) * c2 + atan2_p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((atan2_p7 * c2 + atan2_p5) * c2 + atan2_p3) * c2 + atan2_p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

struct Mat8 {
    int w = 0, h = 0;
    std::vector<uint8_t> d;
    void create(int W, int H) { w = W; h = H; d.assign((size_t)W * H, 0); }
    uint8_t* row(int y) { return &d[(size_t)y * w]; }
    const uint8_t* row(int y) const { return &d[(size_t)y * w]; }
    uint8_t at(int y, int x) const { return d[(size_t)y * w + x]; }
};

// ------------------------------------------------------------------------------------------
// cv::resize(src, dst, dsize, 0, 0, INTER_LINEAR) for CV_8UC1 (imgwarp.cpp, OpenCV 3.2).
// Horizontal pass: HResizeLinear<uchar,int,short,2048> — exact int32.
// Vertical pass: VResizeLinear + FixedPtCast<int,uchar,22> (scalar), or the SSE2
// VResizeLinearVec_32s8u loop ((S>>4)*b >>16 per row, +2 >>2) for x below its loop end.
// ------------------------------------------------------------------------------------------
int vresize_simd_end(int width) {
    int x = 0;
    for (; x <= width - 16; x += 16) {}
    for (; x < width - 4; x += 4) {}
    return x;
}

void resize_linear(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst, int dw, int dh,
                   int dstride, bool simd) {
    if (sw == dw && sh == dh) {
        for (int y = 0; y < sh; ++y) memcpy(dst + (size_t)y * dstride, src + (size_t)y * sstride, sw);
        return;
    }
    const double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
    const double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
    {
        int iscale_x = cvRound(scale_x), iscale_y = cvRound(scale_y);
        bool is_area_fast = std::abs(scale_x - iscale_x) < DBL_EPSILON &&
                            std::abs(scale_y - iscale_y) < DBL_EPSILON;
        if (is_area_fast && iscale_x == 2 && iscale_y == 2) {
            // INTER_LINEAR at exactly 1/2 is routed to the INTER_AREA fast path (2x2 mean).
            for (int y = 0; y < dh; ++y)
                for (int x = 0; x < dw; ++x) {
                    const uint8_t* s0 = src + (size_t)(2 * y) * sstride + 2 * x;
                    const uint8_t* s1 = s0 + sstride;
                    dst[(size_t)y * dstride + x] = (uint8_t)((s0[0] + s0[1] + s1[0] + s1[1] + 2) >> 2);
                }
            return;
        }
    }
    std::vector<int> xofs(dw), yofs(dh);
    std::vector<short> ialpha(2 * dw), ibeta(2 * dh);
    int xmax = dw;
    for (int dx = 0; dx < dw; ++dx) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cvFloor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0, sx = 0; }
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) fx = 0, sx = sw - 1;
        }
        xofs[dx] = sx;
        float cbuf0 = 1.f - fx, cbuf1 = fx;
        ialpha[2 * dx] = sat_short_from_float(cbuf0 * 2048);
        ialpha[2 * dx + 1] = sat_short_from_float(cbuf1 * 2048);
    }
    for (int dy = 0; dy < dh; ++dy) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cvFloor(fy);
        fy -= sy;
        yofs[dy] = sy;
        float cbuf0 = 1.f - fy, cbuf1 = fy;
        ibeta[2 * dy] = sat_short_from_float(cbuf0 * 2048);
        ibeta[2 * dy + 1] = sat_short_from_float(cbuf1 * 2048);
    }
    auto clip = [](int x, int a, int b) { return x >= a ? (x < b ? x : b - 1) : a; };
    std::vector<int> H0(dw), H1(dw);
    auto hresize = [&](const uint8_t* S, int* D) {
        int dx = 0;
        for (; dx < xmax; ++dx) {
            int sx = xofs[dx];
            D[dx] = S[sx] * ialpha[2 * dx] + S[sx + 1] * ialpha[2 * dx + 1];
        }
        for (; dx < dw; ++dx) D[dx] = S[xofs[dx]] * 2048;
    };
    const int xs = simd ? vresize_simd_end(dw) : 0;
    for (int dy = 0; dy < dh; ++dy) {
        int sy0 = yofs[dy];
        int r0 = clip(sy0, 0, sh), r1 = clip(sy0 + 1, 0, sh);
        hresize(src + (size_t)r0 * sstride, H0.data());
        hresize(src + (size_t)r1 * sstride, H1.data());
        const int b0 = ibeta[2 * dy], b1 = ibeta[2 * dy + 1];
        uint8_t* D = dst + (size_t)dy * dstride;
        for (int x = 0; x < xs; ++x) {
            int s0 = std::min(std::max(H0[x] >> 4, -32768), 32767);   // packs_epi32
            int s1 = std::min(std::max(H1[x] >> 4, -32768), 32767);
            int m0 = (s0 * b0) >> 16, m1 = (s1 * b1) >> 16;              // mulhi_epi16
            int t = std::min(std::max(m0 + m1, -32768), 32767);           // adds_epi16
            t = std::min(std::max(t + 2, -32768), 32767);
            D[x] = sat_u8(t >> 2);                                        // srai + packus
        }
        for (int x = xs; x < dw; ++x) D[x] = sat_u8((H0[x] * b0 + H1[x] * b1 + (1 << 21)) >> 22);
    }
}

// ------------------------------------------------------------------------------------------
// cv::GaussianBlur(img, img, Size(7,7), 2, 2, BORDER_REFLECT_101) for CV_8UC1.
// getGaussianKernel(7, 2, CV_32F) -> fixed point x256 (Σ=257); row pass exact int32
// (RowFilter<uchar,int>); column pass SymmColumnFilter<FixedPtCastEx<int,uchar>> with
// bits=16, whose SSE2 vector loop (SymmColumnVec_32s8u) runs in float (k/65536) and rounds
// half-even with cvtps2dq for x < 4*floor(w/4); the scalar tail uses (s + 2^15) >> 16.
// ------------------------------------------------------------------------------------------
void gaussian_taps(int taps[7]) {
    float cf[7];
    double sigmaX = 2.0, scale2X = -0.5 / (sigmaX * sigmaX), sum = 0;
    for (int i = 0; i < 7; ++i) {
        double x = i - (7 - 1) * 0.5;
        double t = std::exp(scale2X * x * x);
        cf[i] = (float)t;
        sum += cf[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < 7; ++i) cf[i] = (float)(cf[i] * sum);
    for (int i = 0; i < 7; ++i) taps[i] = cvRound(cf[i] * 256.f);
}

void gaussian7(const uint8_t* src, int w, int h, int sstride, uint8_t* dst, int dstride, bool simd) {
    int taps[7];
    gaussian_taps(taps);
    float kf[4];
    for (int k = 0; k < 4; ++k) kf[k] = (float)taps[3 + k] * (1.f / 65536.f);
    // Row pass over every source row.
    std::vector<int> R((size_t)w * h);
    for (int y = 0; y < h; ++y) {
        const uint8_t* s = src + (size_t)y * sstride;
        for (int x = 0; x < w; ++x) {
            int acc = 0;
            for (int k = 0; k < 7; ++k) acc += taps[k] * s[reflect101(x + k - 3, w)];
            R[(size_t)y * w + x] = acc;
        }
    }
    const int xs = simd ? (w / 4) * 4 : 0;
    for (int y = 0; y < h; ++y) {
        const int* rows[7];
        for (int k = 0; k < 7; ++k) rows[k] = &R[(size_t)reflect101(y + k - 3, h) * w];
        uint8_t* D = dst + (size_t)y * dstride;
        for (int x = 0; x < xs; ++x) {
            float s = (float)rows[3][x] * kf[0];
            s = s + 0.0f;
            for (int k = 1; k <= 3; ++k) {
                int pair = rows[3 + k][x] + rows[3 - k][x];
                float t = (float)pair * kf[k];
                s = s + t;
            }
            int v = (int)lrintf(s);                           // cvtps2dq (half-even)
            v = std::min(std::max(v, -32768), 32767);         // packs_epi32
            D[x] = sat_u8(v);                                 // packus_epi16
        }
        for (int x = xs; x < w; ++x) {
            int s0 = taps[3] * rows[3][x];
            for (int k = 1; k <= 3; ++k) s0 += taps[3 + k] * (rows[3 + k][x] + rows[3 - k][x]);
            D[x] = sat_u8((s0 + (1 << 15)) >> 16);
        }
    }
}

// ------------------------------------------------------------------------------------------
// cv::FAST(img, kps, threshold, nonmaxSuppression=true) — FAST_t<16> (fast.cpp, OpenCV 3.2),
// scalar loop; the SSE2 loop of that function is an exact restatement of the same test.
// ------------------------------------------------------------------------------------------
int corner_score16(const uint8_t* ptr, const int pixel[], int threshold) {
    const int K = 8, N = K * 3 + 1;
    int k, v = ptr[0];
    short d[N];
    for (k = 0; k < N; k++) d[k] = (short)(v - ptr[pixel[k]]);
    int a0 = threshold;
    for (k = 0; k < 16; k += 2) {
        int a = std::min((int)d[k + 1], (int)d[k + 2]);
        a = std::min(a, (int)d[k + 3]);
        if (a <= a0) continue;
        a = std::min(a, (int)d[k + 4]);
        a = std::min(a, (int)d[k + 5]);
        a = std::min(a, (int)d[k + 6]);
        a = std::min(a, (int)d[k + 7]);
        a = std::min(a, (int)d[k + 8]);
        a0 = std::max(a0, std::min(a, (int)d[k]));
        a0 = std::max(a0, std::min(a, (int)d[k + 9]));
    }
    int b0 = -a0;
    for (k = 0; k < 16; k += 2) {
        int b = std::max((int)d[k + 1], (int)d[k + 2]);
        b = std::max(b, (int)d[k + 3]);
        b = std::max(b, (int)d[k + 4]);
        b = std::max(b, (int)d[k + 5]);
        if (b >= b0) continue;
        b = std::max(b, (int)d[k + 6]);
        b = std::max(b, (int)d[k + 7]);
        b = std::max(b, (int)d[k + 8]);
        b0 = std::min(b0, std::max(b, (int)d[k]));
        b0 = std::min(b0, std::max(b, (int)d[k + 9]));
    }
    return -b0 - 1;
}

void fast9(const uint8_t* img, int stride, int rows, int cols, int threshold,
           std::vector<KeyPoint>& keypoints) {
    const int K = 8, N = 16 + K + 1;
    static const int offsets16[16][2] = {{0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1},
                                         {2, -2}, {1, -3}, {0, -3}, {-1, -3}, {-2, -2},
                                         {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};
    int pixel[25];
    for (int k = 0; k < 16; ++k) pixel[k] = offsets16[k][0] + offsets16[k][1] * stride;
    for (int k = 16; k < 25; ++k) pixel[k] = pixel[k - 16];
    keypoints.clear();
    threshold = std::min(std::max(threshold, 0), 255);
    uint8_t threshold_tab[512];
    for (int i = -255; i <= 255; i++)
        threshold_tab[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);
    if (cols <= 0 || rows <= 0) return;
    std::vector<uint8_t> bufv((size_t)cols * 3, 0);
    std::vector<int> cpv((size_t)(cols + 1) * 3 + 4, 0);
    uint8_t* buf[3] = {&bufv[0], &bufv[cols], &bufv[2 * cols]};
    int* cpbuf[3] = {&cpv[1], &cpv[1] + cols + 1, &cpv[1] + 2 * (cols + 1)};
    for (int i = 3; i < rows - 2; i++) {
        const uint8_t* ptr = img + (size_t)i * stride + 3;
        uint8_t* curr = buf[(i - 3) % 3];
        int* cornerpos = cpbuf[(i - 3) % 3];
        memset(curr, 0, cols);
        int ncorners = 0;
        if (i < rows - 3) {
            for (int j = 3; j < cols - 3; j++, ptr++) {
                int v = ptr[0];
                const uint8_t* tab = &threshold_tab[0] - v + 255;
                int d = tab[ptr[pixel[0]]] | tab[ptr[pixel[8]]];
                if (d == 0) continue;
                d &= tab[ptr[pixel[2]]] | tab[ptr[pixel[10]]];
                d &= tab[ptr[pixel[4]]] | tab[ptr[pixel[12]]];
                d &= tab[ptr[pixel[6]]] | tab[ptr[pixel[14]]];
                if (d == 0) continue;
                d &= tab[ptr[pixel[1]]] | tab[ptr[pixel[9]]];
                d &= tab[ptr[pixel[3]]] | tab[ptr[pixel[11]]];
                d &= tab[ptr[pixel[5]]] | tab[ptr[pixel[13]]];
                d &= tab[ptr[pixel[7]]] | tab[ptr[pixel[15]]];
                if (d & 1) {
                    int vt = v - threshold, count = 0;
                    for (int k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x < vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else
                            count = 0;
                    }
                }
                if (d & 2) {
                    int vt = v + threshold, count = 0;
                    for (int k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x > vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else
                            count = 0;
                    }
                }
            }
        }
        cornerpos[-1] = ncorners;
        if (i == 3) continue;
        const uint8_t* prev = buf[(i - 4 + 3) % 3];
        const uint8_t* pprev = buf[(i - 5 + 3) % 3];
        cornerpos = cpbuf[(i - 4 + 3) % 3];
        ncorners = cornerpos[-1];
        for (int k = 0; k < ncorners; k++) {
            int j = cornerpos[k];
            int score = prev[j];
            if (score > prev[j + 1] && score > prev[j - 1] && score > pprev[j - 1] &&
                score > pprev[j] && score > pprev[j + 1] && score > curr[j - 1] &&
                score > curr[j] && score > curr[j + 1])
                keypoints.push_back(make_kp((float)j, (float)(i - 1), 7.f, -1, (float)score));
        }
    }
}

// ------------------------------------------------------------------------------------------
// The ORB extractor (src/ORBextractor.cc)
// ------------------------------------------------------------------------------------------
const int PATCH_SIZE = 31;
const int HALF_PATCH_SIZE = 15;
const int EDGE_THRESHOLD = 19;

const signed char kPattern[1024] = {
#include "../my_orb_slam2_amd/csrc/orbx_pattern.inc"
};

struct ExtractorNode;
typedef std::list<ExtractorNode> NodeList;

struct ExtractorNode {
    std::vector<KeyPoint> vKeys;
    int ULx = 0, ULy = 0, URx = 0, URy = 0, BLx = 0, BLy = 0, BRx = 0, BRy = 0;
    NodeList::iterator lit;
    bool bNoMore = false;
    long long seq = 0;   // allocation order (stands in for the node's heap address)

    // src/ORBextractor.cc:481-537
    void DivideNode(ExtractorNode& n1, ExtractorNode& n2, ExtractorNode& n3, ExtractorNode& n4) {
        const int halfX = (int)std::ceil(static_cast<float>(URx - ULx) / 2);
        const int halfY = (int)std::ceil(static_cast<float>(BRy - ULy) / 2);
        n1.ULx = ULx; n1.ULy = ULy;
        n1.URx = ULx + halfX; n1.URy = ULy;
        n1.BLx = ULx; n1.BLy = ULy + halfY;
        n1.BRx = ULx + halfX; n1.BRy = ULy + halfY;
        n1.vKeys.reserve(vKeys.size());
        n2.ULx = n1.URx; n2.ULy = n1.URy;
        n2.URx = URx; n2.URy = URy;
        n2.BLx = n1.BRx; n2.BLy = n1.BRy;
        n2.BRx = URx; n2.BRy = ULy + halfY;
        n2.vKeys.reserve(vKeys.size());
        n3.ULx = n1.BLx; n3.ULy = n1.BLy;
        n3.URx = n1.BRx; n3.URy = n1.BRy;
        n3.BLx = BLx; n3.BLy = BLy;
        n3.BRx = n1.BRx; n3.BRy = BLy;
        n3.vKeys.reserve(vKeys.size());
        n4.ULx = n3.URx; n4.ULy = n3.URy;
        n4.URx = n2.BRx; n4.URy = n2.BRy;
        n4.BLx = n3.BRx; n4.BLy = n3.BRy;
        n4.BRx = BRx; n4.BRy = BRy;
        n4.vKeys.reserve(vKeys.size());
        for (size_t i = 0; i < vKeys.size(); i++) {
            const KeyPoint& kp = vKeys[i];
            if (kp.x < n1.URx) {
                if (kp.y < n1.BRy) n1.vKeys.push_back(kp);
                else n3.vKeys.push_back(kp);
            } else if (kp.y < n1.BRy)
                n2.vKeys.push_back(kp);
            else
                n4.vKeys.push_back(kp);
        }
        if (n1.vKeys.size() == 1) n1.bNoMore = true;
        if (n2.vKeys.size() == 1) n2.bNoMore = true;
        if (n3.vKeys.size() == 1) n3.bNoMore = true;
        if (n4.vKeys.size() == 1) n4.bNoMore = true;
    }
};

struct SizePtr {
    int size;
    ExtractorNode* node;
    bool operator<(const SizePtr& o) const {
        if (size != o.size) return size < o.size;
        return node->seq < o.node->seq;
    }
};

class Extractor {
  public:
    Extractor(int nfeatures_, float scaleFactor_, int nlevels_, int iniTh, int minTh, bool simd_)
        : nfeatures(nfeatures_), scaleFactor(scaleFactor_), nlevels(nlevels_), iniThFAST(iniTh),
          minThFAST(minTh), simd(simd_) {
        // src/ORBextractor.cc:410-470
        mvScaleFactor.resize(nlevels);
        mvLevelSigma2.resize(nlevels);
        mvScaleFactor[0] = 1.0f;
        mvLevelSigma2[0] = 1.0f;
        for (int i = 1; i < nlevels; i++) {
            mvScaleFactor[i] = (float)(mvScaleFactor[i - 1] * scaleFactor);
            mvLevelSigma2[i] = mvScaleFactor[i] * mvScaleFactor[i];
        }
        mvInvScaleFactor.resize(nlevels);
        mvInvLevelSigma2.resize(nlevels);
        for (int i = 0; i < nlevels; i++) {
            mvInvScaleFactor[i] = 1.0f / mvScaleFactor[i];
            mvInvLevelSigma2[i] = 1.0f / mvLevelSigma2[i];
        }
        pyr.resize(nlevels);
        blurred.resize(nlevels);
        cand.resize(nlevels);
        mnFeaturesPerLevel.resize(nlevels);
        float factor = (float)(1.0f / scaleFactor);
        float nDesiredFeaturesPerScale =
            nfeatures * (1 - factor) / (1 - (float)pow((double)factor, (double)nlevels));
        int sumFeatures = 0;
        for (int level = 0; level < nlevels - 1; level++) {
            mnFeaturesPerLevel[level] = cvRound(nDesiredFeaturesPerScale);
            sumFeatures += mnFeaturesPerLevel[level];
            nDesiredFeaturesPerScale *= factor;
        }
        mnFeaturesPerLevel[nlevels - 1] = std::max(nfeatures - sumFeatures, 0);

        umax.resize(HALF_PATCH_SIZE + 1);
        int v, v0, vmax = cvFloor((float)(HALF_PATCH_SIZE * std::sqrt(2.f) / 2 + 1));
        int vmin = cvCeil((float)(HALF_PATCH_SIZE * std::sqrt(2.f) / 2));
        const double hp2 = HALF_PATCH_SIZE * HALF_PATCH_SIZE;
        for (v = 0; v <= vmax; ++v) umax[v] = cvRound(std::sqrt(hp2 - v * v));
        for (v = HALF_PATCH_SIZE, v0 = 0; v >= vmin; --v) {
            while (umax[v0] == umax[v0 + 1]) ++v0;
            umax[v] = v0;
            ++v0;
        }
    }

    // src/ORBextractor.cc:1129-1154 (the padded border is never read on the path; the level
    // images are stored unpadded here).
    void ComputePyramid(const uint8_t* img, int w, int h, int stride) {
        for (int level = 0; level < nlevels; ++level) {
            float scale = mvInvScaleFactor[level];
            int sw = cvRound((float)w * scale), sh = cvRound((float)h * scale);
            pyr[level].create(sw, sh);
            if (level != 0) {
                resize_linear(pyr[level - 1].d.data(), pyr[level - 1].w, pyr[level - 1].h,
                              pyr[level - 1].w, pyr[level].d.data(), sw, sh, sw, simd);
            } else {
                for (int y = 0; y < h; ++y) memcpy(pyr[0].row(y), img + (size_t)y * stride, w);
            }
        }
    }

    // src/ORBextractor.cc:539-765
    std::vector<KeyPoint> DistributeOctTree(const std::vector<KeyPoint>& vToDistributeKeys,
                                            const int& minX, const int& maxX, const int& minY,
                                            const int& maxY, const int& N) {
        long long seq = 0;
        // Guard (documented in DESIGN.md): with no candidates the reference returns an empty
        // list whenever its root count is well defined; with nIni < 1 it indexes an empty
        // vector (undefined).  Both return empty here.
        if (vToDistributeKeys.empty()) return std::vector<KeyPoint>();
        if (!(maxY - minY > 0) || std::round(static_cast<float>(maxX - minX) / (maxY - minY)) < 1)
            return std::vector<KeyPoint>();
        const int nIni = (int)std::round(static_cast<float>(maxX - minX) / (maxY - minY));
        const float hX = static_cast<float>(maxX - minX) / nIni;
        NodeList lNodes;
        std::vector<ExtractorNode*> vpIniNodes;
        vpIniNodes.resize(nIni);
        for (int i = 0; i < nIni; i++) {
            ExtractorNode ni;
            ni.ULx = (int)(hX * static_cast<float>(i)); ni.ULy = 0;
            ni.URx = (int)(hX * static_cast<float>(i + 1)); ni.URy = 0;
            ni.BLx = ni.ULx; ni.BLy = maxY - minY;
            ni.BRx = ni.URx; ni.BRy = maxY - minY;
            ni.vKeys.reserve(vToDistributeKeys.size());
            ni.seq = seq++;
            lNodes.push_back(ni);
            vpIniNodes[i] = &lNodes.back();
        }
        for (size_t i = 0; i < vToDistributeKeys.size(); i++) {
            const KeyPoint& kp = vToDistributeKeys[i];
            vpIniNodes[(size_t)(kp.x / hX)]->vKeys.push_back(kp);
        }
        NodeList::iterator lit = lNodes.begin();
        while (lit != lNodes.end()) {
            if (lit->vKeys.size() == 1) {
                lit->bNoMore = true;
                lit++;
            } else if (lit->vKeys.empty())
                lit = lNodes.erase(lit);
            else
                lit++;
        }
        bool bFinish = false;
        std::vector<SizePtr> vSizeAndPointerToNode;
        vSizeAndPointerToNode.reserve(lNodes.size() * 4);
        auto push_child = [&](ExtractorNode& n, bool track, std::vector<SizePtr>& v) {
            n.seq = seq++;
            lNodes.push_front(n);
            if (n.vKeys.size() > 1) {
                if (track) v.push_back(SizePtr{(int)n.vKeys.size(), &lNodes.front()});
                lNodes.front().lit = lNodes.begin();
                return 1;
            }
            return 0;
        };
        while (!bFinish) {
            int prevSize = (int)lNodes.size();
            lit = lNodes.begin();
            int nToExpand = 0;
            vSizeAndPointerToNode.clear();
            while (lit != lNodes.end()) {
                if (lit->bNoMore) {
                    lit++;
                    continue;
                } else {
                    ExtractorNode n1, n2, n3, n4;
                    lit->DivideNode(n1, n2, n3, n4);
                    if (n1.vKeys.size() > 0) nToExpand += push_child(n1, true, vSizeAndPointerToNode);
                    if (n2.vKeys.size() > 0) nToExpand += push_child(n2, true, vSizeAndPointerToNode);
                    if (n3.vKeys.size() > 0) nToExpand += push_child(n3, true, vSizeAndPointerToNode);
                    if (n4.vKeys.size() > 0) nToExpand += push_child(n4, true, vSizeAndPointerToNode);
                    lit = lNodes.erase(lit);
                    continue;
                }
            }
            if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) {
                bFinish = true;
            } else if (((int)lNodes.size() + nToExpand * 3) > N) {
                while (!bFinish) {
                    prevSize = (int)lNodes.size();
                    std::vector<SizePtr> vPrevSizeAndPointerToNode = vSizeAndPointerToNode;
                    vSizeAndPointerToNode.clear();
                    std::sort(vPrevSizeAndPointerToNode.begin(), vPrevSizeAndPointerToNode.end());
                    for (int j = (int)vPrevSizeAndPointerToNode.size() - 1; j >= 0; j--) {
                        ExtractorNode n1, n2, n3, n4;
                        vPrevSizeAndPointerToNode[j].node->DivideNode(n1, n2, n3, n4);
                        if (n1.vKeys.size() > 0) push_child(n1, true, vSizeAndPointerToNode);
                        if (n2.vKeys.size() > 0) push_child(n2, true, vSizeAndPointerToNode);
                        if (n3.vKeys.size() > 0) push_child(n3, true, vSizeAndPointerToNode);
                        if (n4.vKeys.size() > 0) push_child(n4, true, vSizeAndPointerToNode);
                        lNodes.erase(vPrevSizeAndPointerToNode[j].node->lit);
                        if ((int)lNodes.size() >= N) break;
                    }
                    if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) bFinish = true;
                }
            }
        }
        std::vector<KeyPoint> vResultKeys;
        vResultKeys.reserve(nfeatures);
        for (NodeList::iterator it = lNodes.begin(); it != lNodes.end(); it++) {
            std::vector<KeyPoint>& vNodeKeys = it->vKeys;
            KeyPoint* pKP = &vNodeKeys[0];
            float maxResponse = pKP->response;
            for (size_t k = 1; k < vNodeKeys.size(); k++) {
                if (vNodeKeys[k].response > maxResponse) {
                    pKP = &vNodeKeys[k];
                    maxResponse = vNodeKeys[k].response;
                }
            }
            vResultKeys.push_back(*pKP);
        }
        return vResultKeys;
    }

    // src/ORBextractor.cc:77-104
    float IC_Angle(const Mat8& image, float ptx, float pty) const {
        int m_01 = 0, m_10 = 0;
        const uint8_t* center = &image.d[(size_t)cvRound(pty) * image.w + cvRound(ptx)];
        for (int u = -HALF_PATCH_SIZE; u <= HALF_PATCH_SIZE; ++u) m_10 += u * center[u];
        int step = image.w;
        for (int v = 1; v <= HALF_PATCH_SIZE; ++v) {
            int v_sum = 0;
            int d = umax[v];
            for (int u = -d; u <= d; ++u) {
                int val_plus = center[u + v * step], val_minus = center[u - v * step];
                v_sum += (val_plus - val_minus);
                m_10 += u * (val_plus + val_minus);
            }
            m_01 += v * v_sum;
        }
        return fastAtan2((float)m_01, (float)m_10);
    }

    // src/ORBextractor.cc:776-875
    void ComputeKeyPointsOctTree(std::vector<std::vector<KeyPoint>>& allKeypoints) {
        allKeypoints.resize(nlevels);
        const float W = 30;
        for (int level = 0; level < nlevels; ++level) {
            const int minBorderX = EDGE_THRESHOLD - 3;
            const int minBorderY = minBorderX;
            const int maxBorderX = pyr[level].w - EDGE_THRESHOLD + 3;
            const int maxBorderY = pyr[level].h - EDGE_THRESHOLD + 3;
            std::vector<KeyPoint>& vToDistributeKeys = cand[level];
            vToDistributeKeys.clear();
            vToDistributeKeys.reserve(nfeatures * 10);
            const float width = (maxBorderX - minBorderX);
            const float height = (maxBorderY - minBorderY);
            const int nCols = (int)(width / W);
            const int nRows = (int)(height / W);
            const int wCell = (int)std::ceil(width / nCols);
            const int hCell = (int)std::ceil(height / nRows);
            std::vector<KeyPoint> vKeysCell;
            for (int i = 0; i < nRows; i++) {
                const float iniY = minBorderY + i * hCell;
                float maxY = iniY + hCell + 6;
                if (iniY >= maxBorderY - 3) continue;
                if (maxY > maxBorderY) maxY = maxBorderY;
                for (int j = 0; j < nCols; j++) {
                    const float iniX = minBorderX + j * wCell;
                    float maxX = iniX + wCell + 6;
                    if (iniX >= maxBorderX - 6) continue;
                    if (maxX > maxBorderX) maxX = maxBorderX;
                    const int r0 = (int)iniY, r1 = (int)maxY, c0 = (int)iniX, c1 = (int)maxX;
                    const uint8_t* roi = pyr[level].d.data() + (size_t)r0 * pyr[level].w + c0;
                    fast9(roi, pyr[level].w, r1 - r0, c1 - c0, iniThFAST, vKeysCell);
                    if (vKeysCell.empty())
                        fast9(roi, pyr[level].w, r1 - r0, c1 - c0, minThFAST, vKeysCell);
                    for (auto& k : vKeysCell) {
                        k.x += j * wCell;
                        k.y += i * hCell;
                        vToDistributeKeys.push_back(k);
                    }
                }
            }
            std::vector<KeyPoint>& keypoints = allKeypoints[level];
            keypoints.reserve(nfeatures);
            // (the reference prints vToDistributeKeys.size() here, src/ORBextractor.cc:854)
            keypoints = DistributeOctTree(vToDistributeKeys, minBorderX, maxBorderX, minBorderY,
                                          maxBorderY, mnFeaturesPerLevel[level]);
            const int scaledPatchSize = (int)(PATCH_SIZE * mvScaleFactor[level]);
            const int nkps = (int)keypoints.size();
            for (int i = 0; i < nkps; i++) {
                keypoints[i].x += minBorderX;
                keypoints[i].y += minBorderY;
                keypoints[i].octave = level;
                keypoints[i].size = (float)scaledPatchSize;
            }
        }
        for (int level = 0; level < nlevels; ++level)
            for (auto& kp : allKeypoints[level]) kp.angle = IC_Angle(pyr[level], kp.x, kp.y);
    }

    // src/ORBextractor.cc:108-147
    void computeOrbDescriptor(const KeyPoint& kpt, const Mat8& img, uint8_t* desc) const {
        const float factorPI = (float)(3.14159265358979323846 / 180.f);
        float angle = (float)kpt.angle * factorPI;
        float a = cosf(angle), b = sinf(angle);
        const uint8_t* center = &img.d[(size_t)cvRound(kpt.y) * img.w + cvRound(kpt.x)];
        const int step = img.w;
        const signed char* pattern = kPattern;
        auto get = [&](int idx) {
            float px = (float)pattern[2 * idx], py = (float)pattern[2 * idx + 1];
            float ry = px * b;
            float ry2 = py * a;
            float rx = px * a;
            float rx2 = py * b;
            return (int)center[cvRound(ry + ry2) * step + cvRound(rx - rx2)];
        };
        for (int i = 0; i < 32; ++i, pattern += 32) {
            int val = 0;
            for (int bit = 0; bit < 8; ++bit) {
                int t0 = get(2 * bit), t1 = get(2 * bit + 1);
                val |= (t0 < t1) << bit;
            }
            desc[i] = (uint8_t)val;
        }
    }

    // src/ORBextractor.cc:1065-1127
    int run(const uint8_t* img, int w, int h, int stride) {
        if (!img || w <= 0 || h <= 0) return -1;
        ComputePyramid(img, w, h, stride);
        std::vector<std::vector<KeyPoint>> allKeypoints;
        ComputeKeyPointsOctTree(allKeypoints);
        levelKps = allKeypoints;
        int nkeypoints = 0;
        for (int level = 0; level < nlevels; ++level) nkeypoints += (int)allKeypoints[level].size();
        descriptors.assign((size_t)nkeypoints * 32, 0);
        keypoints.clear();
        keypoints.reserve(nkeypoints);
        int offset = 0;
        for (int level = 0; level < nlevels; ++level) {
            std::vector<KeyPoint>& kps = allKeypoints[level];
            int nkeypointsLevel = (int)kps.size();
            if (nkeypointsLevel == 0) { blurred[level].create(0, 0); continue; }
            Mat8& working = blurred[level];
            working.create(pyr[level].w, pyr[level].h);
            gaussian7(pyr[level].d.data(), pyr[level].w, pyr[level].h, pyr[level].w,
                      working.d.data(), working.w, simd);
            for (int i = 0; i < nkeypointsLevel; ++i)
                computeOrbDescriptor(kps[i], working, &descriptors[(size_t)(offset + i) * 32]);
            offset += nkeypointsLevel;
            if (level != 0) {
                float scale = mvScaleFactor[level];
                for (auto& kp : kps) { kp.x = kp.x * scale; kp.y = kp.y * scale; }
            }
            keypoints.insert(keypoints.end(), kps.begin(), kps.end());
        }
        return nkeypoints;
    }

    int nfeatures;
    double scaleFactor;
    int nlevels, iniThFAST, minThFAST;
    bool simd;
    std::vector<int> mnFeaturesPerLevel, umax;
    std::vector<float> mvScaleFactor, mvInvScaleFactor, mvLevelSigma2, mvInvLevelSigma2;
    std::vector<Mat8> pyr, blurred;
    std::vector<std::vector<KeyPoint>> cand, levelKps;
    std::vector<KeyPoint> keypoints;
    std::vector<uint8_t> descriptors;
};

int DescriptorDistance(const uint8_t* a8, const uint8_t* b8) {
    // src/ORBmatcher.cc:1715-1731 (SWAR popcount of the XOR; equal to a plain popcount).
    const int32_t* pa = (const int32_t*)a8;
    const int32_t* pb = (const int32_t*)b8;
    int dist = 0;
    for (int i = 0; i < 8; i++, pa++, pb++) {
        unsigned int v = *pa ^ *pb;
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
    }
    return dist;
}

// src/Frame.cc:496-686
int ComputeStereoMatches(const Extractor& L, const Extractor& R, float mbf, float mb,
                         float* mvuRight, float* mvDepth) {
    const int N = (int)L.keypoints.size();
    for (int i = 0; i < N; ++i) { mvuRight[i] = -1.0f; mvDepth[i] = -1.0f; }
    const int TH_HIGH = 100, TH_LOW = 50;
    const int thOrbDist = (TH_HIGH + TH_LOW) / 2;
    const int nRows = L.pyr[0].h;
    std::vector<std::vector<size_t>> vRowIndices(nRows, std::vector<size_t>());
    for (int i = 0; i < nRows; i++) vRowIndices[i].reserve(200);
    const int Nr = (int)R.keypoints.size();
    const std::vector<float>& mvScaleFactors = L.mvScaleFactor;
    const std::vector<float>& mvInvScaleFactors = L.mvInvScaleFactor;
    for (int iR = 0; iR < Nr; iR++) {
        const KeyPoint& kp = R.keypoints[iR];
        const float& kpY = kp.y;
        const float r = 2.0f * mvScaleFactors[kp.octave];
        const int maxr = (int)std::ceil(kpY + r);
        const int minr = (int)std::floor(kpY - r);
        for (int yi = minr; yi <= maxr; yi++) vRowIndices[yi].push_back(iR);
    }
    const float minZ = mb;
    const float minD = 0;
    const float maxD = mbf / minZ;
    std::vector<std::pair<int, int>> vDistIdx;
    vDistIdx.reserve(N);
    for (int iL = 0; iL < N; iL++) {
        const KeyPoint& kpL = L.keypoints[iL];
        const int& levelL = kpL.octave;
        const float& vL = kpL.y;
        const float& uL = kpL.x;
        const std::vector<size_t>& vCandidates = vRowIndices[(size_t)vL];
        if (vCandidates.empty()) continue;
        const float minU = uL - maxD;
        const float maxU = uL - minD;
        if (maxU < 0) continue;
        int bestDist = TH_HIGH;
        size_t bestIdxR = 0;
        const uint8_t* dL = &L.descriptors[(size_t)iL * 32];
        for (size_t iC = 0; iC < vCandidates.size(); iC++) {
            const size_t iR = vCandidates[iC];
            const KeyPoint& kpR = R.keypoints[iR];
            if (kpR.octave < levelL - 1 || kpR.octave > levelL + 1) continue;
            const float& uR = kpR.x;
            if (uR >= minU && uR <= maxU) {
                const uint8_t* dR = &R.descriptors[iR * 32];
                const int dist = DescriptorDistance(dL, dR);
                if (dist < bestDist) {
                    bestDist = dist;
                    bestIdxR = iR;
                }
            }
        }
        if (bestDist < thOrbDist) {
            const float uR0 = R.keypoints[bestIdxR].x;
            const float scaleFactor = mvInvScaleFactors[kpL.octave];
            const float scaleduL = std::round(kpL.x * scaleFactor);
            const float scaledvL = std::round(kpL.y * scaleFactor);
            const float scaleduR0 = std::round(uR0 * scaleFactor);
            const int w = 5;
            const Mat8& PL = L.pyr[kpL.octave];
            const Mat8& PR = R.pyr[kpL.octave];
            const int yl0 = (int)(scaledvL - w), xl0 = (int)(scaleduL - w);
            const float cL = (float)PL.at(yl0 + w, xl0 + w);
            int bestDist2 = INT_MAX;
            int bestincR = 0;
            const int L5 = 5;
            std::vector<float> vDists;
            vDists.resize(2 * L5 + 1);
            const float iniu = scaleduR0 + L5 - w;
            const float endu = scaleduR0 + L5 + w + 1;
            if (iniu < 0 || endu >= PR.w) continue;
            for (int incR = -L5; incR <= +L5; incR++) {
                const int xr0 = (int)(scaleduR0 + incR - w);
                const float cR = (float)PR.at(yl0 + w, xr0 + w);
                double s = 0;
                for (int yy = 0; yy < 2 * w + 1; ++yy)
                    for (int xx = 0; xx < 2 * w + 1; ++xx) {
                        float il = (float)PL.at(yl0 + yy, xl0 + xx) - cL;
                        float ir = (float)PR.at(yl0 + yy, xr0 + xx) - cR;
                        s += std::abs((double)(il - ir));
                    }
                float dist = (float)s;
                if (dist < bestDist2) {
                    bestDist2 = (int)dist;
                    bestincR = incR;
                }
                vDists[L5 + incR] = dist;
            }
            if (bestincR == -L5 || bestincR == L5) continue;
            const float dist1 = vDists[L5 + bestincR - 1];
            const float dist2 = vDists[L5 + bestincR];
            const float dist3 = vDists[L5 + bestincR + 1];
            const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
            if (deltaR < -1 || deltaR > 1) continue;
            float bestuR = mvScaleFactors[kpL.octave] * ((float)scaleduR0 + (float)bestincR + deltaR);
            float disparity = (uL - bestuR);
            if (disparity >= minD && disparity < maxD) {
                if (disparity <= 0) {
                    disparity = 0.01;
                    bestuR = uL - 0.01;
                }
                mvDepth[iL] = mbf / disparity;
                mvuRight[iL] = bestuR;
                vDistIdx.push_back(std::pair<int, int>(bestDist2, iL));
            }
        }
    }
    if (vDistIdx.empty()) return 0;
    std::sort(vDistIdx.begin(), vDistIdx.end());
    const float median = vDistIdx[vDistIdx.size() / 2].first;
    const float thDist = 1.5f * 1.4f * median;
    int valid = (int)vDistIdx.size();
    for (int i = (int)vDistIdx.size() - 1; i >= 0; i--) {
        if (vDistIdx[i].first < thDist) break;
        mvuRight[vDistIdx[i].second] = -1;
        mvDepth[vDistIdx[i].second] = -1;
        --valid;
    }
    return valid;
}

}  // namespace

extern "C" {

void* oracle_extractor_create(int nfeatures, float scaleFactor, int nlevels, int iniThFAST,
                              int minThFAST, int simd) {
    return new Extractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, simd != 0);
}
void oracle_extractor_destroy(void* h) { delete (Extractor*)h; }
int oracle_extract(void* h, const uint8_t* img, int width, int height, int stride) {
    return ((Extractor*)h)->run(img, width, height, stride);
}
int oracle_num_keypoints(void* h) { return (int)((Extractor*)h)->keypoints.size(); }
int oracle_get_keypoints(void* h, okp_t* out, int cap) {
    auto& k = ((Extractor*)h)->keypoints;
    int n = std::min(cap, (int)k.size());
    if (n > 0) memcpy(out, k.data(), sizeof(okp_t) * n);
    return (int)k.size();
}
int oracle_get_descriptors(void* h, uint8_t* out, int cap_rows) {
    auto& d = ((Extractor*)h)->descriptors;
    int rows = (int)(d.size() / 32);
    int n = std::min(cap_rows, rows);
    if (n > 0) memcpy(out, d.data(), (size_t)n * 32);
    return rows;
}
int oracle_num_levels(void* h) { return ((Extractor*)h)->nlevels; }
int oracle_level_size(void* h, int level, int* w, int* hgt) {
    auto* e = (Extractor*)h;
    if (level < 0 || level >= e->nlevels) return -1;
    *w = e->pyr[level].w;
    *hgt = e->pyr[level].h;
    return 0;
}
int oracle_get_level(void* h, int level, int which, uint8_t* out) {
    auto* e = (Extractor*)h;
    if (level < 0 || level >= e->nlevels) return -1;
    const Mat8& m = which ? e->blurred[level] : e->pyr[level];
    if (m.d.empty()) return 0;
    memcpy(out, m.d.data(), m.d.size());
    return (int)m.d.size();
}
int oracle_get_candidates(void* h, int level, okp_t* out, int cap) {
    auto* e = (Extractor*)h;
    auto& c = e->cand[level];
    int n = std::min(cap, (int)c.size());
    if (n > 0) memcpy(out, c.data(), sizeof(okp_t) * n);
    return (int)c.size();
}
int oracle_get_level_keypoints(void* h, int level, okp_t* out, int cap) {
    auto* e = (Extractor*)h;
    auto& c = e->levelKps[level];   // copied before run() scales to level-0 coordinates
    int n = std::min(cap, (int)c.size());
    if (n > 0) memcpy(out, c.data(), sizeof(okp_t) * n);
    return (int)c.size();
}
void oracle_get_tables(void* h, float* scale, float* inv_scale, float* sigma2, float* inv_sigma2,
                       int* features_per_level, int* umax16) {
    auto* e = (Extractor*)h;
    for (int i = 0; i < e->nlevels; ++i) {
        scale[i] = e->mvScaleFactor[i];
        inv_scale[i] = e->mvInvScaleFactor[i];
        sigma2[i] = e->mvLevelSigma2[i];
        inv_sigma2[i] = e->mvInvLevelSigma2[i];
        features_per_level[i] = e->mnFeaturesPerLevel[i];
    }
    for (int i = 0; i < 16; ++i) umax16[i] = e->umax[i];
}
int oracle_stereo_match(void* hL, void* hR, float mbf, float mb, float* uRight, float* depth) {
    return ComputeStereoMatches(*(Extractor*)hL, *(Extractor*)hR, mbf, mb, uRight, depth);
}
void oracle_resize(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst, int dw, int dh,
                   int simd) {
    resize_linear(src, sw, sh, sstride, dst, dw, dh, dw, simd != 0);
}
void oracle_gaussian7(const uint8_t* src, int w, int h, int stride, uint8_t* dst, int simd) {
    gaussian7(src, w, h, stride, dst, w, simd != 0);
}
int oracle_fast(const uint8_t* img, int stride, int rows, int cols, int threshold, okp_t* out,
                int cap) {
    std::vector<KeyPoint> k;
    fast9(img, stride, rows, cols, threshold, k);
    int n = std::min(cap, (int)k.size());
    if (n > 0) memcpy(out, k.data(), sizeof(okp_t) * n);
    return (int)k.size();
}
float oracle_fast_atan2(float y, float x) { return fastAtan2(y, x); }
void oracle_gaussian_taps(int* taps7) { gaussian_taps(taps7); }
int oracle_descriptor_distance(const uint8_t* a, const uint8_t* b) { return DescriptorDistance(a, b); }

}  // extern "C"
