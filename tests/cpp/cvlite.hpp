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
#define CV_32F 5
#define CV_64F 6

namespace cv {

struct Point2f {
    float x = 0.f, y = 0.f;
    Point2f() = default;
    Point2f(float x_, float y_) : x(x_), y(y_) {}
};

struct Point3f {
    float x = 0.f, y = 0.f, z = 0.f;
    Point3f() = default;
    Point3f(float x_, float y_, float z_) : x(x_), y(y_), z(z_) {}
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
    Mat(int r, int c, int t, void* ext, size_t st = 0)
        : rows(r), cols(c), step(st ? st : (size_t)c * esize(t)), data(static_cast<unsigned char*>(ext)), type_(t) {}
    Mat(int r, int c, int t) { create(r, c, t); }
    void create(int r, int c, int t) {
        if (r == rows && c == cols && t == type_ && buf_) return;
        buf_ = std::make_shared<std::vector<unsigned char>>((size_t)r * c * esize(t));
        rows = r; cols = c; type_ = t; step = (size_t)c * esize(t); data = buf_->data();
    }
    void release() { buf_.reset(); rows = cols = 0; step = 0; data = nullptr; }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    int type() const { return type_; }
    Mat clone() const {
        Mat m(rows, cols, type_);
        for (int r = 0; r < rows; ++r)
            for (size_t b = 0; b < (size_t)cols * esize(type_); ++b) m.data[r * m.step + b] = data[r * step + b];
        return m;
    }
    static Mat eye(int r, int c, int t) {
        Mat m(r, c, t);
        for (int i = 0; i < r; ++i)
            for (int j = 0; j < c; ++j) {
                if (t == CV_32F) m.at<float>(i, j) = i == j ? 1.f : 0.f;
                else if (t == CV_64F) m.at<double>(i, j) = i == j ? 1.0 : 0.0;
                else m.at<unsigned char>(i, j) = i == j ? 1 : 0;
            }
        return m;
    }
    template <class T> T* ptr(int r) { return reinterpret_cast<T*>(data + (size_t)r * step); }
    template <class T> const T* ptr(int r) const { return reinterpret_cast<const T*>(data + (size_t)r * step); }
    template <class T> T& at(int r, int c) { return ptr<T>(r)[c]; }
    template <class T> const T& at(int r, int c) const { return ptr<T>(r)[c]; }
    template <class T> T& at(int i) { return rows == 1 ? at<T>(0, i) : at<T>(i, 0); }
    template <class T> const T& at(int i) const { return rows == 1 ? at<T>(0, i) : at<T>(i, 0); }

private:
    static size_t esize(int t) { return t == CV_32F ? 4 : t == CV_64F ? 8 : 1; }
    std::shared_ptr<std::vector<unsigned char>> buf_;
    int type_ = CV_8UC1;
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
