// jacobi_lds.h -- one-sided (Hestenes) Jacobi for ONE wave working on a
// small dense matrix held in LDS, with the disjoint column pairs of a
// round-robin round spread over the wave: pair i of the round is owned by
// lanes 8i..8i+7, and lane s of the pair holds rows s, s+8, ... of both
// columns (A and V).  A round is then ~20 wave instructions per lane (two
// column loads, an 8-lane DPP dot product, the rotation, the updates, two
// stores) instead of the ~400 of jacobi_group.h's rows-on-lanes form, where
// one lane carries a whole row of A and V and every pair of the round runs
// through its instruction stream (EPnP's Refine: 3.1 k cycles per round on
// one wave, 136 us per 12 x 12 decomposition).
//
// Same rotation (jacobi_rotation_fast), same tournament order
// (jacobi_col), same convergence and null-column tests as hestenes_group;
// only the association of each dot product differs (8-lane partial sums of
// rows s, s+8, ...), so results agree to rounding.
//
// Layout (caller-initialised, all in LDS, doubles):
//   A: M columns of NRP rows (column c at A + c*NRP), rows >= NR and the
//      extra column of an odd NC are zero;
//   V: M columns of NVP rows (column c at V + c*NVP), the NC x NC identity
//      in the first NC rows, zero elsewhere;
//   nrm: M doubles, overwritten: on return the squared column norms of A V.
// On return the columns of A V are mutually orthogonal and the columns of V
// the right singular vectors (unsorted), as hestenes_group's.
#pragma once

#include <hip/hip_runtime.h>

#include "group_sum.h"
#include "jacobi_group.h"

namespace orbgpu {

// sum over the lane's 8-lane group on DPP (quad sums, then the other quad of
// the half row); every lane of the group gets the same bits
__device__ __forceinline__ double oct_sum(double x) {
    x += dpp_f64<kDppXor1>(x);
    x += dpp_f64<kDppXor2>(x);
    x += dpp_f64<kDppHalfMirror>(x);
    return x;
}

// LP lanes per column pair (8 or 4); one problem per GW-lane group of the
// wave (GW = 64: the whole wave, or 16: four independent problems per wave,
// each on its own LDS matrices).
template <int LP>
__device__ __forceinline__ double lp_sum(double x) {
    static_assert(LP == 4 || LP == 8, "4 or 8 lanes per pair");
    if constexpr (LP == 8) return oct_sum(x);
    x += dpp_f64<kDppXor1>(x);
    x += dpp_f64<kDppXor2>(x);
    return x;
}

template <int NC, int NR, int LP = 8, int GW = 64>
struct JacobiLds {
    static constexpr int M = NC + (NC & 1);  // positions of the circle method
    static constexpr int P = M / 2;          // pairs per round
    static_assert(NC >= 2 && P * LP <= GW, "every column pair of a round needs its own LP lanes in the group");
    static constexpr int RA = (NR + LP - 1) / LP;  // rows of A per lane
    static constexpr int RV = (NC + LP - 1) / LP;  // rows of V per lane
    static constexpr int NRP = LP * RA;            // column stride of A
    static constexpr int NVP = LP * RV;            // column stride of V
    static constexpr int kDoubles = M * NRP + M * NVP + M;

    // the wave's LDS writes visible to its later reads (one wave, no block
    // barrier): release/acquire workgroup fences around the wave barrier so
    // the compiler cannot move or reuse LDS loads across it (the intrinsics
    // alone are IntrNoMem), then the stores retired
    static __device__ __forceinline__ void sync() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }

    // A <- the NR x NC matrix a(r, c), V <- I (every lane of the group calls)
    template <class F>
    static __device__ void init(double* A, double* V, int lane, F a) {
        lane %= GW;
        for (int idx = lane; idx < M * NRP; idx += GW) {
            const int c = idx / NRP, r = idx - c * NRP;
            A[idx] = (r < NR && c < NC) ? a(r, c) : 0.0;
        }
        for (int idx = lane; idx < M * NVP; idx += GW) {
            const int c = idx / NVP, r = idx - c * NVP;
            V[idx] = (r == c && c < NC) ? 1.0 : 0.0;
        }
        sync();
    }

    // returns the number of sweeps run
    // `store` false: the group computes but never writes (a duplicate problem)
    static __device__ int run(double* A, double* V, double* nrm, int lane, int max_sweeps = 60, bool store = true) {
        const int lg = lane % GW, pair = lg / LP, s = lg % LP;
        const bool active = pair < P && store;
        const int i = pair < P ? pair : 0;  // idle lanes shadow pair 0 and never store
        double fro = 0.0;
        for (int idx = lg; idx < M * NRP; idx += GW) fro += A[idx] * A[idx];
        const double negl = kJacobiNegl * group_sum_dpp<GW>(fro);
        int sweep = 0;
        while (sweep < max_sweeps) {
            ++sweep;
            bool rotated = false;
            {  // the squared column norms, carried through the rotations of the sweep
                const int p = i, q = M - 1 - i;
                double np = 0.0, nq = 0.0;
#pragma unroll
                for (int k = 0; k < RA; ++k) {
                    const double x = A[p * NRP + s + LP * k], y = A[q * NRP + s + LP * k];
                    np += x * x;
                    nq += y * y;
                }
                np = lp_sum<LP>(np);
                nq = lp_sum<LP>(nq);
                if (active && s == 0) {
                    nrm[p] = np;
                    nrm[q] = nq;
                }
                sync();
            }
#pragma unroll 1
            for (int k = 0; k < M - 1; ++k) {
                const int p = jacobi_col(i, k, M), q = jacobi_col(M - 1 - i, k, M);
                double* Ap = A + p * NRP + s;
                double* Aq = A + q * NRP + s;
                double* Vp = V + p * NVP + s;
                double* Vq = V + q * NVP + s;
                double ap[RA], aq[RA], vp[RV], vq[RV];
#pragma unroll
                for (int j = 0; j < RA; ++j) {
                    ap[j] = Ap[LP * j];
                    aq[j] = Aq[LP * j];
                }
#pragma unroll
                for (int j = 0; j < RV; ++j) {
                    vp[j] = Vp[LP * j];
                    vq[j] = Vq[LP * j];
                }
                const double alpha = nrm[p], beta = nrm[q];
                double g = ap[0] * aq[0];
#pragma unroll
                for (int j = 1; j < RA; ++j) g = fma(ap[j], aq[j], g);
                g = lp_sum<LP>(g);
                double c, sn, t;
                rotated |= jacobi_rotation_fast(alpha, beta, g, negl, c, sn, t);
#pragma unroll
                for (int j = 0; j < RA; ++j) {
                    const double x = ap[j], y = aq[j];
                    ap[j] = fma(c, x, -sn * y);
                    aq[j] = fma(sn, x, c * y);
                }
#pragma unroll
                for (int j = 0; j < RV; ++j) {
                    const double x = vp[j], y = vq[j];
                    vp[j] = fma(c, x, -sn * y);
                    vq[j] = fma(sn, x, c * y);
                }
                if (active) {
#pragma unroll
                    for (int j = 0; j < RA; ++j) {
                        Ap[LP * j] = ap[j];
                        Aq[LP * j] = aq[j];
                    }
#pragma unroll
                    for (int j = 0; j < RV; ++j) {
                        Vp[LP * j] = vp[j];
                        Vq[LP * j] = vq[j];
                    }
                    if (s == 0) {
                        nrm[p] = fma(-t, g, alpha);
                        nrm[q] = fma(t, g, beta);
                    }
                }
                sync();
            }
            if (!__any(rotated)) break;  // wave-uniform
        }
        {  // exact squared norms of the converged columns
            const int p = i, q = M - 1 - i;
            double np = 0.0, nq = 0.0;
#pragma unroll
            for (int k = 0; k < RA; ++k) {
                const double x = A[p * NRP + s + LP * k], y = A[q * NRP + s + LP * k];
                np += x * x;
                nq += y * y;
            }
            np = lp_sum<LP>(np);
            nq = lp_sum<LP>(nq);
            if (active && s == 0) {
                nrm[p] = np;
                nrm[q] = nq;
            }
            sync();
        }
        return sweep;
    }
};

}  // namespace orbgpu
