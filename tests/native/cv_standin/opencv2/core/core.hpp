// A stand-in for the OpenCV 3.2 core types the drop-in facades (integration/ORBextractor.h,
// integration/orbx_slam2_glue.h, integration/ORBmatcher.h) and the ORB-SLAM2 stand-in classes of
// tests/native/slam2_standin touch: cv::Mat (2-D, CV_8UC1 or CV_32FC1), its expressions (MatExpr:
// scaled, transposed, matrix products with an added term), cv::norm, Mat::dot, cv::KeyPoint,
// cv::Point2f and the InputArray / OutputArray proxies.  It exists only so that the native tests
// can compile and run the facades in this image, which has no OpenCV.  Members keep OpenCV's
// names, types and semantics (refcounted data, row / column views sharing data, continuity,
// `step` in bytes), so code that compiles here compiles against the real headers; an ORB-SLAM2
// build uses OpenCV itself.
//
// Arithmetic follows OpenCV 3.2 as this repository restates it (PARITY UNPINNED against the
// library; the same model as oracle/orb_frame_oracle.cpp):
//   A*B (+ C)      cv::gemm's small-matrix path: each element sums its products in float, left
//                  to right, and stores (float)(t*alpha + c*beta) evaluated in double
//   s*A, A/s, -A   Mat::convertTo(alpha): (float)(x * (float)alpha + 0.0f)
//   A.t()          transpose (then convertTo when scaled)
//   A + B, A - B   element-wise float add / subtract
//   norm(A)        sqrt of the squares summed in double;  A.dot(B): (double)a*b summed in double
//   norm(A, B, NORM_L1)  |a - b| in float, summed in double (normDiffL1_<float, double>)
//   A.convertTo(D, CV_32F)  8U -> 32F element by element (a new buffer, so D may be A)
#ifndef ORBX_CV_STANDIN_CORE_HPP
#define ORBX_CV_STANDIN_CORE_HPP

#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>

#define CV_8U 0
#define CV_8UC1 0
#define CV_32F 5
#define CV_32FC1 5

namespace cv {

typedef unsigned char uchar;

struct Point2f {
    float x = 0.f, y = 0.f;
    Point2f() = default;
    Point2f(float x_, float y_) : x(x_), y(y_) {}
};

// core/types.hpp: Point2f pt; float size, angle, response; int octave, class_id
class KeyPoint {
public:
    Point2f pt;
    float size = 0.f;
    float angle = -1.f;
    float response = 0.f;
    int octave = 0;
    int class_id = -1;
};

class _OutputArray;
class MatExpr;

class Mat {
public:
    int rows = 0, cols = 0;
    uchar* data = nullptr;
    size_t step = 0;  // bytes per row (MatStep converts to this in OpenCV)

    Mat() = default;
    Mat(int r, int c, int type) { create(r, c, type); }
    Mat(int r, int c, int type, void* ext, size_t st = 0)
        : rows(r), cols(c), data((uchar*)ext), type_(check_type(type)) {
        step = st ? st : (size_t)c * elemSize();
    }
    Mat& operator=(const MatExpr& e);

    void create(int r, int c, int type) {
        check_type(type);
        if (owner && r == rows && c == cols && type == type_ &&
            step == (size_t)c * elemSize())
            return;
        type_ = type;
        const size_t es = elemSize();
        owner.reset(new uchar[(size_t)r * c * es + 1], std::default_delete<uchar[]>());
        data = owner.get();
        rows = r;
        cols = c;
        step = (size_t)c * es;
    }
    void release() {
        owner.reset();
        data = nullptr;
        rows = cols = 0;
        step = 0;
    }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    int type() const { return type_; }
    size_t elemSize() const { return type_ == CV_32F ? 4 : 1; }
    size_t total() const { return (size_t)rows * cols; }
    bool isContinuous() const { return rows <= 1 || step == (size_t)cols * elemSize(); }
    uchar* ptr(int r = 0) { return data + (size_t)r * step; }
    const uchar* ptr(int r = 0) const { return data + (size_t)r * step; }
    template <class T> T* ptr(int r = 0) { return (T*)ptr(r); }
    template <class T> const T* ptr(int r = 0) const { return (const T*)ptr(r); }
    // at(i) on a single row or column (OpenCV's 1-index form); at(r, c) in general
    template <class T> T& at(int i) {
        return rows == 1 ? ((T*)data)[i] : *(T*)(data + (size_t)i * step);
    }
    template <class T> const T& at(int i) const {
        return rows == 1 ? ((const T*)data)[i] : *(const T*)(data + (size_t)i * step);
    }
    template <class T> T& at(int r, int c) { return ((T*)ptr(r))[c]; }
    template <class T> const T& at(int r, int c) const { return ((const T*)ptr(r))[c]; }

    Mat rowRange(int a, int b) const {
        if (a < 0 || b > rows || a > b) throw std::out_of_range("cv::Mat::rowRange");
        Mat m(*this);
        m.data = data + (size_t)a * step;
        m.rows = b - a;
        return m;
    }
    Mat colRange(int a, int b) const {
        if (a < 0 || b > cols || a > b) throw std::out_of_range("cv::Mat::colRange");
        Mat m(*this);
        m.data = data + (size_t)a * elemSize();
        m.cols = b - a;
        return m;
    }
    Mat row(int r) const { return rowRange(r, r + 1); }
    Mat col(int c) const { return colRange(c, c + 1); }
    Mat clone() const {
        Mat m(rows, cols, type_);
        for (int r = 0; r < rows; ++r) std::memcpy(m.ptr(r), ptr(r), (size_t)cols * elemSize());
        return m;
    }
    inline void copyTo(const _OutputArray& dst) const;
    void copyTo(Mat& dst) const {
        Mat c = clone();
        if (!dst.empty() && dst.rows == rows && dst.cols == cols && dst.type_ == type_) {
            for (int r = 0; r < rows; ++r) std::memcpy(dst.ptr(r), c.ptr(r), (size_t)cols * elemSize());
        } else {
            dst = c;
        }
    }
    inline MatExpr t() const;
    // Mat::dot for CV_32F (dotProd_32f: (double)a*b accumulated in double over the elements in
    // row-major order)
    double dot(const Mat& m) const {
        if (type_ != CV_32F || m.type_ != CV_32F || total() != m.total())
            throw std::invalid_argument("cv stand-in: dot of CV_32F arrays of one size");
        double s = 0;
        for (size_t k = 0; k < total(); ++k) s += (double)fel(k) * m.fel(k);
        return s;
    }
    static Mat zeros(int r, int c, int type) {
        Mat m(r, c, type);
        for (int i = 0; i < r; ++i) std::memset(m.ptr(i), 0, (size_t)c * m.elemSize());
        return m;
    }
    static Mat ones(int r, int c, int type) {
        Mat m(r, c, type);
        for (int i = 0; i < r; ++i)
            for (int k = 0; k < c; ++k) {
                if (type == CV_32F) m.at<float>(i, k) = 1.f;
                else m.at<uchar>(i, k) = 1;
            }
        return m;
    }
    // convertTo(m, rtype) with alpha 1, beta 0: CV_8U -> CV_32F, or a copy of the same type
    void convertTo(Mat& dst, int rtype) const {
        if (rtype == type_) {
            Mat c = clone();
            dst = c;
            return;
        }
        if (type_ != CV_8U || rtype != CV_32F)
            throw std::invalid_argument("cv stand-in: convertTo CV_8U -> CV_32F only");
        Mat d(rows, cols, CV_32F);
        for (int r = 0; r < rows; ++r)
            for (int k = 0; k < cols; ++k) d.at<float>(r, k) = (float)at<uchar>(r, k);
        dst = d;
    }
    static Mat eye(int r, int c, int type) {
        Mat m = zeros(r, c, type);
        for (int i = 0; i < r && i < c; ++i) {
            if (type == CV_32F) m.at<float>(i, i) = 1.f;
            else m.at<uchar>(i, i) = 1;
        }
        return m;
    }
    // element k in row-major order (CV_32F)
    float fel(size_t k) const { return at<float>((int)(k / cols), (int)(k % cols)); }
    float& fel(size_t k) { return at<float>((int)(k / cols), (int)(k % cols)); }

private:
    static int check_type(int type) {
        if (type != CV_8UC1 && type != CV_32FC1)
            throw std::invalid_argument("cv stand-in: CV_8UC1 or CV_32FC1 only");
        return type;
    }
    std::shared_ptr<uchar> owner;
    int type_ = CV_8UC1;
};

// A matrix expression (OpenCV's MatExpr, reduced to the forms the facades build):
//   SCALED  alpha * a            (MatOp_AddEx with one operand)
//   TRANS   alpha * a^T          (MatOp_T)
//   GEMM    alpha * op(a) * b + beta * c   (MatOp_GEMM; op = transpose when a_t)
class MatExpr {
public:
    enum Kind { SCALED, TRANS, GEMM };
    Kind kind = SCALED;
    Mat a, b, c;
    double alpha = 1.0, beta = 0.0;
    bool a_t = false;

    operator Mat() const { return eval(); }  // NOLINT: implicit, as in OpenCV
    MatExpr t() const { return MatExpr::trans(eval(), 1.0); }

    static MatExpr scaled(const Mat& a, double s) {
        MatExpr e;
        e.kind = SCALED;
        e.a = a;
        e.alpha = s;
        return e;
    }
    static MatExpr trans(const Mat& a, double s) {
        MatExpr e;
        e.kind = TRANS;
        e.a = a;
        e.alpha = s;
        return e;
    }
    static MatExpr gemm(const Mat& a, bool a_t, const Mat& b, double s) {
        MatExpr e;
        e.kind = GEMM;
        e.a = a;
        e.a_t = a_t;
        e.b = b;
        e.alpha = s;
        return e;
    }

    // convertTo(alpha, beta = 0) on CV_32F (cvtScale_<float, float, float>)
    static Mat convert_scaled(const Mat& src, double alpha) {
        if (src.type() != CV_32F) throw std::invalid_argument("cv stand-in: CV_32F arithmetic only");
        Mat d(src.rows, src.cols, CV_32F);
        if (std::fabs(alpha - 1) < 2.220446049250313e-16) {   // noScale: a copy
            for (int r = 0; r < src.rows; ++r) std::memcpy(d.ptr(r), src.ptr(r), (size_t)src.cols * 4);
            return d;
        }
        const float s = (float)alpha, shift = 0.0f;
        for (int r = 0; r < src.rows; ++r)
            for (int k = 0; k < src.cols; ++k) d.at<float>(r, k) = src.at<float>(r, k) * s + shift;
        return d;
    }

    Mat eval() const {
        if (kind == SCALED) return convert_scaled(a, alpha);
        if (kind == TRANS) {
            Mat t(a.cols, a.rows, CV_32F);
            for (int r = 0; r < a.rows; ++r)
                for (int k = 0; k < a.cols; ++k) t.at<float>(k, r) = a.at<float>(r, k);
            return alpha == 1.0 ? t : convert_scaled(t, alpha);
        }
        const int m = a_t ? a.cols : a.rows, len = a_t ? a.rows : a.cols;
        if (a.type() != CV_32F || b.type() != CV_32F || b.rows != len)
            throw std::invalid_argument("cv stand-in: gemm operand sizes");
        const bool has_c = !c.empty();
        if (has_c && (c.rows != m || c.cols != b.cols))
            throw std::invalid_argument("cv stand-in: gemm added term size");
        Mat d(m, b.cols, CV_32F);
        for (int i = 0; i < m; ++i)
            for (int j = 0; j < b.cols; ++j) {
                float t = 0.f;
                for (int k = 0; k < len; ++k) {
                    const float av = a_t ? a.at<float>(k, i) : a.at<float>(i, k);
                    t = k == 0 ? av * b.at<float>(k, j) : t + av * b.at<float>(k, j);
                }
                d.at<float>(i, j) = has_c ? (float)(t * alpha + c.at<float>(i, j) * beta)
                                          : (float)(t * alpha);
            }
        return d;
    }
};

inline Mat& Mat::operator=(const MatExpr& e) { return *this = e.eval(); }
inline MatExpr Mat::t() const { return MatExpr::trans(*this, 1.0); }

// operand of a product: the matrix, its scale and whether it is transposed (MatOp::matmul)
struct MulOperand {
    Mat m;
    double s;
    bool t;
    MulOperand(const Mat& x) : m(x), s(1.0), t(false) {}  // NOLINT: implicit
    MulOperand(const MatExpr& e) : s(1.0), t(false) {      // NOLINT: implicit
        if (e.kind == MatExpr::SCALED) { m = e.a; s = e.alpha; }
        else if (e.kind == MatExpr::TRANS) { m = e.a; s = e.alpha; t = true; }
        else m = e.eval();
    }
};

inline MatExpr mat_mul(const MulOperand& x, const MulOperand& y) {
    Mat b = y.t ? MatExpr::trans(y.m, 1.0).eval() : y.m;
    return MatExpr::gemm(x.m, x.t, b, x.s * y.s);
}
inline MatExpr operator*(const Mat& x, const Mat& y) { return mat_mul(x, y); }
inline MatExpr operator*(const MatExpr& x, const Mat& y) { return mat_mul(x, y); }
inline MatExpr operator*(const Mat& x, const MatExpr& y) { return mat_mul(x, y); }
inline MatExpr operator*(const MatExpr& x, const MatExpr& y) { return mat_mul(x, y); }

inline MatExpr operator*(double s, const Mat& a) { return MatExpr::scaled(a, s); }
inline MatExpr operator*(const Mat& a, double s) { return MatExpr::scaled(a, s); }
inline MatExpr operator/(const Mat& a, double s) { return MatExpr::scaled(a, 1.0 / s); }
inline MatExpr operator-(const Mat& a) { return MatExpr::scaled(a, -1.0); }
inline MatExpr operator*(double s, const MatExpr& e) {
    MatExpr r = e;
    r.alpha *= s;
    if (r.kind == MatExpr::GEMM) r.beta *= s;
    return r;
}
inline MatExpr operator*(const MatExpr& e, double s) { return s * e; }
inline MatExpr operator-(const MatExpr& e) { return -1.0 * e; }

// element-wise float add / subtract of two CV_32F matrices of one size
inline Mat elementwise(const Mat& x, const Mat& y, float sign) {
    if (x.type() != CV_32F || y.type() != CV_32F || x.rows != y.rows || x.cols != y.cols)
        throw std::invalid_argument("cv stand-in: element-wise operands");
    Mat d(x.rows, x.cols, CV_32F);
    for (int r = 0; r < x.rows; ++r)
        for (int k = 0; k < x.cols; ++k)
            d.at<float>(r, k) = sign > 0 ? x.at<float>(r, k) + y.at<float>(r, k)
                                         : x.at<float>(r, k) - y.at<float>(r, k);
    return d;
}
// a product plus / minus a matrix folds into the gemm (MatOp_GEMM::add / subtract)
inline MatExpr gemm_add(const MatExpr& e, const Mat& c, double beta) {
    if (e.kind != MatExpr::GEMM || !e.c.empty()) return MatExpr::scaled(elementwise(e.eval(), c, (float)beta), 1.0);
    MatExpr r = e;
    r.c = c;
    r.beta = beta;
    return r;
}
inline Mat operator+(const Mat& x, const Mat& y) { return elementwise(x, y, 1.f); }
inline Mat operator-(const Mat& x, const Mat& y) { return elementwise(x, y, -1.f); }
inline MatExpr operator+(const MatExpr& e, const Mat& c) { return gemm_add(e, c, 1.0); }
inline MatExpr operator+(const Mat& c, const MatExpr& e) { return gemm_add(e, c, 1.0); }
inline MatExpr operator-(const MatExpr& e, const Mat& c) { return gemm_add(e, c, -1.0); }
inline Mat operator-(const Mat& x, const MatExpr& y) { return elementwise(x, y.eval(), -1.f); }

// cv::norm(src) = NORM_L2 for CV_32F: normL2_<float, double>
inline double norm(const Mat& a) {
    double s = 0;
    for (size_t k = 0; k < a.total(); ++k) {
        const double v = a.fel(k);
        s += v * v;
    }
    return std::sqrt(s);
}

enum { NORM_L1 = 2 };
// cv::norm(a, b, NORM_L1) for CV_32F: normDiffL1_<float, double>, |a - b| accumulated in double
inline double norm(const Mat& a, const Mat& b, int type) {
    if (type != NORM_L1 || a.type() != CV_32F || b.type() != CV_32F || a.rows != b.rows ||
        a.cols != b.cols)
        throw std::invalid_argument("cv stand-in: norm(a, b, NORM_L1) of CV_32F arrays of one size");
    double s = 0;
    for (int r = 0; r < a.rows; ++r)
        for (int k = 0; k < a.cols; ++k) s += std::fabs(a.at<float>(r, k) - b.at<float>(r, k));
    return s;
}

class _InputArray {
public:
    _InputArray(const Mat& m) : m_(&m) {}  // NOLINT: implicit, as in OpenCV
    Mat getMat() const { return *m_; }
    bool empty() const { return m_->empty(); }

private:
    const Mat* m_;
};

class _OutputArray {
public:
    _OutputArray(Mat& m) : m_(&m) {}  // NOLINT: implicit, as in OpenCV
    void create(int r, int c, int type) const { m_->create(r, c, type); }
    Mat getMat() const { return *m_; }
    void release() const { m_->release(); }

private:
    Mat* m_;
};

typedef const _InputArray& InputArray;
typedef const _OutputArray& OutputArray;

inline void Mat::copyTo(const _OutputArray& dst) const {
    dst.create(rows, cols, type_);
    Mat d = dst.getMat();
    for (int r = 0; r < rows; ++r) std::memcpy(d.ptr(r), ptr(r), (size_t)cols * elemSize());
}

}  // namespace cv

#endif  // ORBX_CV_STANDIN_CORE_HPP
