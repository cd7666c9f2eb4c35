// A stand-in for the few OpenCV 3.2 core types the drop-in facade (integration/ORBextractor.h,
// integration/orbx_slam2_glue.h) touches: cv::Mat (8-bit, 2-D), cv::KeyPoint, cv::Point2f and
// the InputArray / OutputArray proxies.  It exists only so that tests/native/facade_test.cpp
// can compile and run the facade's marshalling in this image, which has no OpenCV; the members
// keep OpenCV's names, types and semantics (refcounted data, row views, continuity, `step` in
// bytes), so code that compiles here compiles against the real headers.  An ORB-SLAM2 build
// uses OpenCV itself.
#ifndef ORBX_CV_STANDIN_CORE_HPP
#define ORBX_CV_STANDIN_CORE_HPP

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>

#define CV_8U 0
#define CV_8UC1 0

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

class Mat {
public:
    int rows = 0, cols = 0;
    uchar* data = nullptr;
    size_t step = 0;  // bytes per row (MatStep converts to this in OpenCV)

    Mat() = default;
    Mat(int r, int c, int type) { create(r, c, type); }
    Mat(int r, int c, int type, void* ext, size_t st = 0) : rows(r), cols(c), data((uchar*)ext) {
        check_type(type);
        step = st ? st : (size_t)c;
    }

    void create(int r, int c, int type) {
        check_type(type);
        if (owner && r == rows && c == cols && step == (size_t)c) return;
        owner.reset(new uchar[(size_t)r * c + 1], std::default_delete<uchar[]>());
        data = owner.get();
        rows = r;
        cols = c;
        step = (size_t)c;
    }
    void release() {
        owner.reset();
        data = nullptr;
        rows = cols = 0;
        step = 0;
    }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    int type() const { return CV_8UC1; }
    bool isContinuous() const { return rows <= 1 || step == (size_t)cols; }
    uchar* ptr(int r = 0) { return data + (size_t)r * step; }
    const uchar* ptr(int r = 0) const { return data + (size_t)r * step; }
    template <class T> T* ptr(int r = 0) { return (T*)ptr(r); }
    Mat rowRange(int a, int b) const {
        if (a < 0 || b > rows || a > b) throw std::out_of_range("cv::Mat::rowRange");
        Mat m(*this);
        m.data = data + (size_t)a * step;
        m.rows = b - a;
        return m;
    }
    Mat clone() const {
        Mat m(rows, cols, CV_8UC1);
        for (int r = 0; r < rows; ++r) std::memcpy(m.ptr(r), ptr(r), (size_t)cols);
        return m;
    }
    inline void copyTo(const _OutputArray& dst) const;

private:
    static void check_type(int type) {
        if (type != CV_8UC1) throw std::invalid_argument("cv stand-in: 8-bit single channel only");
    }
    std::shared_ptr<uchar> owner;
};

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
    dst.create(rows, cols, CV_8UC1);
    Mat d = dst.getMat();
    for (int r = 0; r < rows; ++r) std::memcpy(d.ptr(r), ptr(r), (size_t)cols);
}

}  // namespace cv

#endif  // ORBX_CV_STANDIN_CORE_HPP
