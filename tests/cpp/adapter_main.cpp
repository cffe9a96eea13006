// adapter_main.cpp -- drives the drop-in C++ adapter headers
// (include/orbslam2_amd/ORBextractor.h, ORBmatcher.h) the way Frame.cpp and
// Initializer use them; tests/test_adapter.py checks its output.
//
//   adapter_main scales <nfeatures> <scale> <nlevels>
//       print the ORBextractor scale tables (no device needed)
//   adapter_main empty
//       operator() on an empty image must return leaving outputs untouched
//   adapter_main extract <w> <h> <nfeat> <img0.raw> <img1.raw> <out.bin>
//       extract two frames, SearchForInitialization(F0, F1), write
//       [n0, kps0 (28 B each), desc0, n1, kps1, desc1, nmatches, matches12,
//        level-1 pyramid of frame 1]
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <iterator>
#include <vector>

#include "orbslam2_amd/ORBextractor.h"
#include "orbslam2_amd/ORBmatcher.h"

namespace {

struct MiniFrame {  // the members of ORB_SLAM2::Frame the matcher reads
    std::vector<cv::KeyPoint> mvKeysUn;
    cv::Mat mDescriptors;
    float mnMinX = 0.f, mnMaxX = 0.f, mnMinY = 0.f, mnMaxY = 0.f;
};

std::vector<unsigned char> read_file(const char* path) {
    std::ifstream f(path, std::ios::binary);
    return std::vector<unsigned char>(std::istreambuf_iterator<char>(f), {});
}

void put_frame(FILE* out, const MiniFrame& F) {
    const int n = (int)F.mvKeysUn.size();
    fwrite(&n, 4, 1, out);
    for (const cv::KeyPoint& k : F.mvKeysUn) {
        const float f5[5] = {k.pt.x, k.pt.y, k.size, k.angle, k.response};
        const int i2[2] = {k.octave, k.class_id};
        fwrite(f5, 4, 5, out);
        fwrite(i2, 4, 2, out);
    }
    for (int i = 0; i < n; ++i) fwrite(F.mDescriptors.ptr<unsigned char>(i), 1, 32, out);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc >= 5 && !strcmp(argv[1], "scales")) {
        ORB_SLAM2::ORBextractor ex(atoi(argv[2]), (float)atof(argv[3]), atoi(argv[4]), 20, 7);
        const auto s = ex.GetScaleFactors(), is = ex.GetInverseScaleFactors();
        const auto s2 = ex.GetScaleSigmaSquares(), is2 = ex.GetInverseScaleSigmaSquares();
        printf("%d %.9g\n", ex.GetLevels(), ex.GetScaleFactor());
        for (size_t i = 0; i < s.size(); ++i) printf("%a %a %a %a\n", s[i], is[i], s2[i], is2[i]);
        return 0;
    }
    if (argc >= 2 && !strcmp(argv[1], "empty")) {
        ORB_SLAM2::ORBextractor ex(1000, 1.2f, 8, 20, 7);
        std::vector<cv::KeyPoint> kps(3);
        cv::Mat desc, img;
        ex(img, cv::Mat(), kps, desc);
        printf("%zu %d\n", kps.size(), desc.empty() ? 1 : 0);
        return kps.size() == 3 && desc.empty() ? 0 : 1;
    }
    if (argc >= 8 && !strcmp(argv[1], "extract")) {
        const int w = atoi(argv[2]), h = atoi(argv[3]), nf = atoi(argv[4]);
        std::vector<unsigned char> im[2] = {read_file(argv[5]), read_file(argv[6])};
        if (im[0].size() != (size_t)w * h || im[1].size() != (size_t)w * h) {
            fprintf(stderr, "bad image size\n");
            return 2;
        }
        try {
            ORB_SLAM2::ORBextractor ex(nf, 1.2f, 8, 20, 7);
            MiniFrame F[2];
            for (int f = 0; f < 2; ++f) {
                cv::Mat img(h, w, CV_8UC1, im[f].data(), (size_t)w);
                ex(img, cv::Mat(), F[f].mvKeysUn, F[f].mDescriptors);
                F[f].mnMaxX = (float)w;
                F[f].mnMaxY = (float)h;
            }
            std::vector<cv::Point2f> prev;
            for (const cv::KeyPoint& k : F[0].mvKeysUn) prev.push_back(k.pt);
            std::vector<int> m12;
            const int nm = orbslam2_amd::SearchForInitialization(0.9f, true, F[0], F[1], prev, m12, 100);
            FILE* out = fopen(argv[7], "wb");
            put_frame(out, F[0]);
            put_frame(out, F[1]);
            fwrite(&nm, 4, 1, out);
            fwrite(m12.data(), 4, m12.size(), out);
            const cv::Mat& L1 = ex.mvImagePyramid[1];
            const int lw = L1.cols, lh = L1.rows;
            fwrite(&lw, 4, 1, out);
            fwrite(&lh, 4, 1, out);
            for (int y = 0; y < lh; ++y) fwrite(L1.ptr<unsigned char>(y), 1, (size_t)lw, out);
            fclose(out);
        } catch (const std::exception& e) {
            fprintf(stderr, "exception: %s\n", e.what());
            return 3;
        }
        return 0;
    }
    if (argc >= 2 && !strcmp(argv[1], "nodevice")) {  // must throw, not fall back
        try {
            ORB_SLAM2::ORBextractor ex(1000, 1.2f, 8, 20, 7);
            std::vector<unsigned char> buf(640 * 480, 7);
            cv::Mat img(480, 640, CV_8UC1, buf.data());
            std::vector<cv::KeyPoint> kps;
            cv::Mat desc;
            ex(img, cv::Mat(), kps, desc);
        } catch (const std::runtime_error& e) {
            printf("threw: %s\n", e.what());
            return 0;
        }
        return 1;
    }
    fprintf(stderr, "usage: see header\n");
    return 2;
}
