// cvlite.hpp -- the few OpenCV-2.4 core types the drop-in adapter headers
// use (cv::Mat, cv::KeyPoint, cv::Point2f, Input/OutputArray), so the
// adapter can be compiled and exercised in this repo's tests without
// OpenCV.  Test scaffolding for OUR headers only; selected with
// -DORBGPU_CV_HEADER='"cvlite.hpp"'.  Layouts follow OpenCV 2.4's public
// headers (KeyPoint: pt, size, angle, response, octave, class_id).
#ifndef ORBGPU_TESTS_CVLITE_HPP
#define ORBGPU_TESTS_CVLITE_HPP

#include <cstddef>
#include <memory>
#include <vector>

#define CV_8U 0
#define CV_8UC1 0

namespace cv {

struct Point2f {
    float x = 0.f, y = 0.f;
    Point2f() = default;
    Point2f(float x_, float y_) : x(x_), y(y_) {}
};

struct KeyPoint {
    Point2f pt;
    float size = 0.f, angle = -1.f, response = 0.f;
    int octave = 0, class_id = -1;
    KeyPoint() = default;
    KeyPoint(float x, float y, float size_, float angle_ = -1.f, float response_ = 0.f, int octave_ = 0,
             int class_id_ = -1)
        : pt(x, y), size(size_), angle(angle_), response(response_), octave(octave_), class_id(class_id_) {}
};

class Mat {
public:
    int rows = 0, cols = 0;
    size_t step = 0;
    unsigned char* data = nullptr;
    Mat() = default;
    Mat(int r, int c, int /*type*/, void* ext, size_t st = 0)
        : rows(r), cols(c), step(st ? st : (size_t)c), data(static_cast<unsigned char*>(ext)) {}
    void create(int r, int c, int /*type*/) {
        if (r == rows && c == cols && buf_) return;
        buf_ = std::make_shared<std::vector<unsigned char>>((size_t)r * c);
        rows = r; cols = c; step = (size_t)c; data = buf_->data();
    }
    void release() { buf_.reset(); rows = cols = 0; step = 0; data = nullptr; }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    int type() const { return CV_8UC1; }
    template <class T> T* ptr(int r) { return reinterpret_cast<T*>(data + (size_t)r * step); }
    template <class T> const T* ptr(int r) const { return reinterpret_cast<const T*>(data + (size_t)r * step); }

private:
    std::shared_ptr<std::vector<unsigned char>> buf_;
};

class _InputArray {
public:
    _InputArray(const Mat& m) : m_(&m) {}
    Mat getMat() const { return *m_; }
    bool empty() const { return m_->empty(); }

private:
    const Mat* m_;
};

class _OutputArray {
public:
    _OutputArray(Mat& m) : m_(&m) {}
    void create(int r, int c, int t) const { m_->create(r, c, t); }
    void release() const { m_->release(); }
    Mat getMat() const { return *m_; }

private:
    Mat* m_;
};

typedef const _InputArray& InputArray;
typedef const _OutputArray& OutputArray;

}  // namespace cv

#endif
