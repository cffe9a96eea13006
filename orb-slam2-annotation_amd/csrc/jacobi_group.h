// jacobi_group.h -- one-sided (Hestenes) Jacobi for a matrix whose ROWS are
// spread over a G-lane group: lane r holds row r of A in a[NC] (rows past the
// matrix hold zeros) and row r of V in v[NC] (lanes r < NC; V starts as the
// identity).  On return the columns of A V are mutually orthogonal, so the
// column norms are the singular values and the columns of V the right
// singular vectors (cv::SVDecomp's vt rows, cvSVD's V).  Used by
// init_models.hip (the 9-column DLT matrices of ComputeH21 / ComputeF21) and
// epnp_wave.h (the 12 x 12 M^T M of EPnP).
//
// Two choices make it fast on a wave:
//   * round-robin (tournament) order: a sweep is M-1 rounds of M/2 DISJOINT
//     column pairs (M = NC rounded up to even), so the pairs of a round have
//     independent reductions and rotation parameters and their dependent
//     div/sqrt chains interleave, where the cyclic order ran them one after
//     another (66 chains per 12-column sweep on one wave with nothing else
//     to issue);
//   * a column whose squared norm is below 1e-28 ||A||_F^2 is numerically
//     null and takes no rotation.  Without this floor an exactly rank-deficient
//     matrix (the 8 x 9 ComputeF21 system always is; EPnP's M^T M of a
//     minimal set; noise-free correspondences) never meets the relative
//     test: its null column is rounding noise whose cosine with the others
//     stays O(1e-15) after every rotation, and the sweep loop ran to its cap
//     of 60 (measured: 779 us for the 400 models of one Initialize).
// The relative test itself is the usual |gamma| <= 1e-15 sqrt(alpha beta),
// evaluated squared (no sqrt on the chain).
#pragma once

#include <hip/hip_runtime.h>

#include "group_sum.h"

namespace orbgpu {

constexpr double kJacobiTol2 = 1e-30;  // (1e-15)^2
constexpr double kJacobiNegl = 1e-28;  // squared column norm, relative to ||A||_F^2

// rotation (c, s) that orthogonalises columns p, q with squared norms alpha,
// beta and dot product gamma; false (identity) when they already are, or one
// of them is numerically null
__host__ __device__ __forceinline__ bool jacobi_rotation(double alpha, double beta, double gamma, double negl,
                                                         double& c, double& s) {
    c = 1.0;
    s = 0.0;
    if (gamma == 0.0 || gamma * gamma <= kJacobiTol2 * alpha * beta || alpha <= negl || beta <= negl) return false;
    const double zeta = (beta - alpha) / (2.0 * gamma);
    const double t = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
    c = 1.0 / sqrt(1.0 + t * t);
    s = c * t;
    return true;
}

// column at position `pos` in round k of the circle method over M positions
// (position 0 fixed, the others rotate); a column index >= NC is a bye
__host__ __device__ constexpr int jacobi_col(int pos, int k, int M) {
    return pos == 0 ? 0 : (pos - 1 + k) % (M - 1) + 1;
}

template <int NC, int G>
__device__ __forceinline__ void hestenes_group(double (&a)[NC], double (&v)[NC], int max_sweeps = 60) {
    constexpr int M = NC + (NC & 1);
    constexpr int P = M / 2;
    double fro = 0.0;
#pragma unroll
    for (int j = 0; j < NC; ++j) fro += a[j] * a[j];
    const double negl = kJacobiNegl * group_sum_dpp<G>(fro);
    for (int sweep = 0; sweep < max_sweeps; ++sweep) {
        bool rotated = false;
#pragma unroll
        for (int k = 0; k < M - 1; ++k) {
            double al[P], be[P], ga[P], cs[P], sn[P];
#pragma unroll
            for (int i = 0; i < P; ++i) {
                const int p = jacobi_col(i, k, M), q = jacobi_col(M - 1 - i, k, M);
                if (p >= NC || q >= NC) continue;
                al[i] = group_sum_dpp<G>(a[p] * a[p]);
                be[i] = group_sum_dpp<G>(a[q] * a[q]);
                ga[i] = group_sum_dpp<G>(a[p] * a[q]);
            }
#pragma unroll
            for (int i = 0; i < P; ++i) {
                const int p = jacobi_col(i, k, M), q = jacobi_col(M - 1 - i, k, M);
                if (p >= NC || q >= NC) continue;
                rotated |= jacobi_rotation(al[i], be[i], ga[i], negl, cs[i], sn[i]);
            }
#pragma unroll
            for (int i = 0; i < P; ++i) {
                const int p = jacobi_col(i, k, M), q = jacobi_col(M - 1 - i, k, M);
                if (p >= NC || q >= NC) continue;
                const double x = a[p], y = a[q];
                a[p] = cs[i] * x - sn[i] * y;
                a[q] = sn[i] * x + cs[i] * y;
                const double vx = v[p], vy = v[q];
                v[p] = cs[i] * vx - sn[i] * vy;
                v[q] = sn[i] * vx + cs[i] * vy;
            }
        }
        if (!__any(rotated)) break;  // wave-uniform: converged groups rotate by the identity
    }
}

}  // namespace orbgpu
