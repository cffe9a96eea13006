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
// evaluated squared (no sqrt on the chain); the column norms are carried
// through the rotations, and the rotation parameters use the hardware
// reciprocal estimates with Newton steps.
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

// 1/x and 1/sqrt(x) from the hardware estimates (v_rcp_f64, v_rsq_f64) and
// two Newton steps each: full double accuracy for the finite positive
// arguments of a rotation, at a fraction of the IEEE div / sqrt sequences
__device__ __forceinline__ double rcp_nr(double x) {
    double r = __builtin_amdgcn_rcp(x);
    r = fma(r, fma(-x, r, 1.0), r);
    return fma(r, fma(-x, r, 1.0), r);
}
__device__ __forceinline__ double rsq_nr(double x) {
    double r = __builtin_amdgcn_rsq(x);
    r = fma(0.5 * r, fma(-x * r, r, 1.0), r);
    return fma(0.5 * r, fma(-x * r, r, 1.0), r);
}

// the rotation of jacobi_rotation with t = tan(theta) too (for the norm
// update).  t itself is computed in single precision (v_rcp_f32 /
// v_sqrt_f32 on the float-rounded zeta): an angle off by ~1e-7 relative
// leaves a residual cosine of ~1e-7 times the old one, which the next sweep
// removes, while c = 1/sqrt(1 + t^2) (double, Newton-refined) and s = c t
// keep every rotation orthogonal to double precision, so V stays
// orthonormal and the converged singular vectors are as accurate as with an
// exact angle.  |zeta| >= 1e18 takes t = gamma / (beta - alpha) in double.
__device__ __forceinline__ bool jacobi_rotation_fast(double alpha, double beta, double gamma, double negl, double& c,
                                                     double& s, double& t) {
    // branch-free (every value computed, the identity selected at the end):
    // a round's pairs are then one basic block and their chains interleave
    const bool skip = gamma == 0.0 || gamma * gamma <= kJacobiTol2 * alpha * beta || alpha <= negl || beta <= negl;
    const double dba = beta - alpha;
    const float zeta = (float)dba * __builtin_amdgcn_rcpf((float)(2.0 * gamma));
    const float root = __builtin_amdgcn_sqrtf(fmaf(zeta, zeta, 1.0f));
    const float tf = copysignf(__builtin_amdgcn_rcpf(fabsf(zeta) + root), zeta);
    const double t_small = zeta == 0.0f ? 1.0 : (double)tf;
    // zeta^2 beyond float range (or 2 gamma below it): t = 1/(2 zeta) in
    // double; a zero t there would leave the pair unrotated and the sweep
    // loop running to its cap
    const double t_big = dba == 0.0 ? 1.0 : gamma * rcp_nr(dba);
    const double tt = fabsf(zeta) < 1e18f ? t_small : t_big;
    const double cc = rsq_nr(fma(tt, tt, 1.0));
    t = skip ? 0.0 : tt;
    c = skip ? 1.0 : cc;
    s = skip ? 0.0 : cc * tt;
    return !skip;
}

// the rotation the sequential Jacobis (epnp.h) use: IEEE on the host, the
// fast reciprocals on the device (HIP host/device overloading)
__host__ inline bool jacobi_rot(double alpha, double beta, double gamma, double negl, double& c, double& s) {
    return jacobi_rotation(alpha, beta, gamma, negl, c, s);
}
__device__ inline bool jacobi_rot(double alpha, double beta, double gamma, double negl, double& c, double& s) {
    double t;
    return jacobi_rotation_fast(alpha, beta, gamma, negl, c, s, t);
}

// returns the number of sweeps run.  The squared column norms are kept
// current through the rotations (alpha' = alpha - t gamma, beta' = beta + t
// gamma) and recomputed from the columns at the start of every sweep, so a
// pair costs one group reduction (its dot product) instead of three.  The
// circle method moves the COLUMNS, not the pairing: every round pairs
// positions (i, M-1-i), then positions 1..M-1 rotate left by one (after M-1
// rounds every column is back in place), so the round body has static
// register indices and stays a loop (a fully unrolled sweep of 66 pairs
// inflated register pressure until the kernel spilled).  An odd NC gets a
// zero column, which every test skips.
template <int NC, int G>
__device__ __forceinline__ int hestenes_group(double (&a_in)[NC], double (&v_in)[NC], int max_sweeps = 60) {
    constexpr int M = NC + (NC & 1);
    constexpr int P = M / 2;
    double a[M], v[M], nrm[M];
#pragma unroll
    for (int j = 0; j < M; ++j) {
        a[j] = j < NC ? a_in[j] : 0.0;
        v[j] = j < NC ? v_in[j] : 0.0;
    }
    double fro = 0.0;
#pragma unroll
    for (int j = 0; j < NC; ++j) fro += a[j] * a[j];
    const double negl = kJacobiNegl * group_sum_dpp<G>(fro);
    int sweep = 0;
    while (sweep < max_sweeps) {
        ++sweep;
        bool rotated = false;
#pragma unroll
        for (int j = 0; j < M; ++j) nrm[j] = group_sum_dpp<G>(a[j] * a[j]);
#pragma unroll 1
        for (int k = 0; k < M - 1; ++k) {
            double ga[P], cs[P], sn[P], tn[P];
#pragma unroll
            for (int i = 0; i < P; ++i) ga[i] = group_sum_dpp<G>(a[i] * a[M - 1 - i]);
#pragma unroll
            for (int i = 0; i < P; ++i) {
                rotated |= jacobi_rotation_fast(nrm[i], nrm[M - 1 - i], ga[i], negl, cs[i], sn[i], tn[i]);
                nrm[i] = fma(-tn[i], ga[i], nrm[i]);
                nrm[M - 1 - i] = fma(tn[i], ga[i], nrm[M - 1 - i]);
            }
#pragma unroll
            for (int i = 0; i < P; ++i) {  // explicit FMAs: two instructions per updated value
                const int q = M - 1 - i;
                const double x = a[i], y = a[q];
                a[i] = fma(cs[i], x, -sn[i] * y);
                a[q] = fma(sn[i], x, cs[i] * y);
                const double vx = v[i], vy = v[q];
                v[i] = fma(cs[i], vx, -sn[i] * vy);
                v[q] = fma(sn[i], vx, cs[i] * vy);
            }
            // positions 1..M-1 rotate left by one
            const double a1 = a[1], v1 = v[1], n1 = nrm[1];
#pragma unroll
            for (int j = 1; j < M - 1; ++j) {
                a[j] = a[j + 1];
                v[j] = v[j + 1];
                nrm[j] = nrm[j + 1];
            }
            a[M - 1] = a1;
            v[M - 1] = v1;
            nrm[M - 1] = n1;
        }
        if (!__any(rotated)) break;  // wave-uniform: converged groups rotate by the identity
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        a_in[j] = a[j];
        v_in[j] = v[j];
    }
    return sweep;
}

}  // namespace orbgpu
