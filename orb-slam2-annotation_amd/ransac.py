"""Host-side mirror of the reference's RANSAC solvers over the C ABI in
include/orbgpu_ransac.h.

* glibc-compatible random stream: ``srand``, ``rand``, ``random_int``
  (DUtils::Random, Thirdparty/DBoW2/DUtils/Random.cpp:33-50), with state
  save/restore so hypotheses can be evaluated speculatively on the GPU while
  the stream advances exactly as the reference's sequential loop.
* ``Sim3Solver`` -- Sim3Solver (src/Sim3Solver.cpp:37-447): the same
  constructor data (camera-frame points of both keyframes, level sigmas,
  intrinsics), ``set_ransac_parameters``, ``iterate``, ``find`` and the
  ``get_estimated_*`` accessors; the hypotheses are solved and scored by
  csrc/sim3.hip.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np

import orbgpu

RAND_MAX = 2147483647


class RandState(ctypes.Structure):
    _fields_ = [("r", ctypes.c_int32 * 31), ("f", ctypes.c_int32), ("b", ctypes.c_int32)]


class Sim3Problem(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("offset", ctypes.c_int), ("fix_scale", ctypes.c_int),
                ("min_inliers", ctypes.c_int), ("best_inliers", ctypes.c_int), ("n_hyp", ctypes.c_int),
                ("sample_offset", ctypes.c_int), ("pad", ctypes.c_int),
                ("K1", ctypes.c_float * 4), ("K2", ctypes.c_float * 4)]


class Sim3Result(ctypes.Structure):
    _fields_ = [("found", ctypes.c_int), ("consumed", ctypes.c_int), ("best_inliers", ctypes.c_int),
                ("best_hyp", ctypes.c_int), ("T12", ctypes.c_float * 16), ("R12", ctypes.c_float * 9),
                ("t12", ctypes.c_float * 3), ("s12", ctypes.c_float)]


def srand(seed: int) -> None:
    orbgpu.lib().orbgpu_srand(seed & 0xFFFFFFFF)


def rand() -> int:
    return orbgpu.lib().orbgpu_rand()


def random_int(lo: int, hi: int) -> int:
    return orbgpu.lib().orbgpu_random_int(lo, hi)


def get_state() -> RandState:
    st = RandState()
    orbgpu.lib().orbgpu_rand_get_state(ctypes.byref(st))
    return st


def set_state(st: RandState) -> None:
    orbgpu.lib().orbgpu_rand_set_state(ctypes.byref(st))


def draw_triplets(n: int, n_iter: int) -> np.ndarray:
    """The minimal sets of n_iter Sim3 iterations from the global stream:
    vAvailableIndices = all; 3 x (RandomInt(0, size-1), swap with back, pop)
    (Sim3Solver.cpp:172-183)."""
    out = np.zeros((n_iter, 3), np.int32)
    for it in range(n_iter):
        avail = list(range(n))
        for k in range(3):
            r = random_int(0, len(avail) - 1)
            out[it, k] = avail[r]
            avail[r] = avail[-1]
            avail.pop()
    return out


def sim3_ransac_batch(problems, X1, X2, maxerr1, maxerr2, samples, inliers):
    """Host form of orbgpu_sim3_ransac_batch: problems is a ctypes array of
    Sim3Problem; returns a ctypes array of Sim3Result; inliers updated in place."""
    L = orbgpu.lib()
    B = len(problems)
    res = (Sim3Result * max(B, 1))()
    X1 = np.ascontiguousarray(X1, np.float32)
    X2 = np.ascontiguousarray(X2, np.float32)
    e1 = np.ascontiguousarray(maxerr1, np.float32)
    e2 = np.ascontiguousarray(maxerr2, np.float32)
    smp = np.ascontiguousarray(samples, np.int32).reshape(-1, 3)
    orbgpu._check(L.orbgpu_sim3_ransac_batch(B, ctypes.addressof(problems), len(X1), X1.ctypes.data, X2.ctypes.data,
                                             e1.ctypes.data, e2.ctypes.data, len(smp), smp.ctypes.data,
                                             ctypes.addressof(res), inliers.ctypes.data),
                  "orbgpu_sim3_ransac_batch")
    return res


def max_error(sigma2: np.ndarray) -> np.ndarray:
    """mvnMaxError = 9.210*sigma^2 stored in a vector<size_t> (truncated),
    compared as float (Sim3Solver.cpp:92-93, :350)."""
    return np.floor(9.210 * np.asarray(sigma2, np.float64)).astype(np.float32)


class Sim3Solver:
    """Sim3Solver(pKF1, pKF2, vpMatched12, bFixScale) on the correspondence
    data the reference gathers in its constructor (Sim3Solver.cpp:37-107):
    X1, X2 = camera-frame points (mvX3Dc1/2), sigma2_1/2 = level sigma^2 of the
    matched keypoints, K1/K2 = (fx, fy, cx, cy), indices1 = mvnIndices1 (the
    vpMatched12 slot of each correspondence), n1 = vpMatched12.size()."""

    def __init__(self, X1, X2, sigma2_1, sigma2_2, K1, K2, fix_scale=True, indices1=None, n1=None):
        self.X1 = np.ascontiguousarray(X1, np.float32).reshape(-1, 3)
        self.X2 = np.ascontiguousarray(X2, np.float32).reshape(-1, 3)
        self.e1 = max_error(sigma2_1)
        self.e2 = max_error(sigma2_2)
        self.K1 = [float(v) for v in K1]
        self.K2 = [float(v) for v in K2]
        self.fix_scale = bool(fix_scale)
        self.N = len(self.X1)
        self.indices1 = np.arange(self.N) if indices1 is None else np.asarray(indices1)
        self.n1 = self.N if n1 is None else int(n1)
        self.iterations = 0
        self.best_inliers = 0
        self.best_mask = np.zeros(self.N, np.uint8)
        self.best_T12 = self.best_R = self.best_t = None
        self.best_s = 0.0
        self.set_ransac_parameters()

    def set_ransac_parameters(self, probability=0.99, min_inliers=6, max_iterations=300):
        """Sim3Solver.cpp:111-141."""
        self.prob, self.min_inliers, self.max_its = probability, min_inliers, max_iterations
        N = self.N
        eps = np.float32(min_inliers) / np.float32(N) if N else np.float32(np.inf)
        if min_inliers == N:
            n_it = 1
        else:
            with np.errstate(all="ignore"):
                v = math.log(1 - probability) / math.log(1 - float(eps) ** 3) if 0 < float(eps) < 1 else float("nan")
            n_it = int(math.ceil(v)) if math.isfinite(v) else -(2 ** 31)
        self.max_its = max(1, min(n_it, max_iterations))
        self.iterations = 0

    def iterate(self, n_iterations):
        """Sim3Solver::iterate (Sim3Solver.cpp:147-221): returns (T12 or None,
        no_more, inliers[n1] bool, n_inliers)."""
        inl = np.zeros(self.n1, bool)
        if self.N < self.min_inliers:
            return None, True, inl, 0
        n_hyp = max(0, min(n_iterations, self.max_its - self.iterations))
        snap = get_state()
        samples = draw_triplets(self.N, n_hyp)
        prob = (Sim3Problem * 1)()
        p = prob[0]
        p.n, p.offset, p.fix_scale = self.N, 0, int(self.fix_scale)
        p.min_inliers, p.best_inliers, p.n_hyp, p.sample_offset = self.min_inliers, self.best_inliers, n_hyp, 0
        p.K1[:] = self.K1
        p.K2[:] = self.K2
        mask = self.best_mask.copy()
        r = sim3_ransac_batch(prob, self.X1, self.X2, self.e1, self.e2, samples if n_hyp else np.zeros((0, 3)),
                              mask)[0]
        # consume exactly the draws of the iterations the reference ran
        set_state(snap)
        draw_triplets(self.N, r.consumed)
        self.iterations += r.consumed
        self.best_inliers = r.best_inliers
        if r.best_hyp >= 0:
            self.best_mask = mask
            self.best_T12 = np.array(r.T12, np.float32).reshape(4, 4)
            self.best_R = np.array(r.R12, np.float32).reshape(3, 3)
            self.best_t = np.array(r.t12, np.float32)
            self.best_s = float(r.s12)
        if r.found:
            inl[self.indices1[self.best_mask.astype(bool)]] = True
            return self.best_T12.copy(), False, inl, r.best_inliers
        return None, self.iterations >= self.max_its, inl, 0

    def find(self):
        T, _, inl, n = self.iterate(self.max_its)
        return T, inl, n

    def get_estimated_rotation(self):
        return None if self.best_R is None else self.best_R.copy()

    def get_estimated_translation(self):
        return None if self.best_t is None else self.best_t.copy()

    def get_estimated_scale(self):
        return self.best_s


# --------------------------------------------------------------------------
# PnPsolver
# --------------------------------------------------------------------------
class PnPProblem(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("offset", ctypes.c_int), ("min_inliers", ctypes.c_int),
                ("best_inliers", ctypes.c_int), ("n_hyp", ctypes.c_int), ("sample_offset", ctypes.c_int),
                ("fu", ctypes.c_float), ("fv", ctypes.c_float), ("uc", ctypes.c_float), ("vc", ctypes.c_float)]


class PnPResult(ctypes.Structure):
    _fields_ = [("found", ctypes.c_int), ("consumed", ctypes.c_int), ("best_inliers", ctypes.c_int),
                ("best_hyp", ctypes.c_int), ("refined_inliers", ctypes.c_int),
                ("best_Tcw", ctypes.c_float * 16), ("refined_Tcw", ctypes.c_float * 16)]


def draw_sets(n: int, n_iter: int, k: int) -> np.ndarray:
    """Minimal sets of n_iter iterations: k x (RandomInt(0, size-1), swap
    with back, pop) from all indices (PnPsolver.cpp:229-244, k = minSet)."""
    out = np.zeros((n_iter, k), np.int32)
    for it in range(n_iter):
        avail = list(range(n))
        for j in range(k):
            r = random_int(0, len(avail) - 1)
            out[it, j] = avail[r]
            avail[r] = avail[-1]
            avail.pop()
    return out


def pnp_ransac_batch(problems, P3w, P2, maxerr, samples, best_mask, refined_mask):
    """Host form of orbgpu_pnp_ransac_batch; masks updated in place."""
    L = orbgpu.lib()
    B = len(problems)
    res = (PnPResult * max(B, 1))()
    P3w = np.ascontiguousarray(P3w, np.float32)
    P2 = np.ascontiguousarray(P2, np.float32)
    e = np.ascontiguousarray(maxerr, np.float32)
    smp = np.ascontiguousarray(samples, np.int32).reshape(-1, 4)
    orbgpu._check(L.orbgpu_pnp_ransac_batch(B, ctypes.addressof(problems), len(P3w), P3w.ctypes.data, P2.ctypes.data,
                                            e.ctypes.data, len(smp), smp.ctypes.data, ctypes.addressof(res),
                                            best_mask.ctypes.data, refined_mask.ctypes.data),
                  "orbgpu_pnp_ransac_batch")
    return res


class PnPsolver:
    """PnPsolver(F, vpMapPointMatches) on the data its constructor gathers
    (PnPsolver.cpp:104-139): P3w = world positions of the matched MapPoints
    (mvP3Dw), P2 = their undistorted keypoints (mvP2D), sigma2 = level sigma^2
    of those keypoints (mvSigma2), (fu, fv, uc, vc) = F.fx, fy, cx, cy,
    indices = mvKeyPointIndices, n_matches = vpMapPointMatches.size()."""

    def __init__(self, P3w, P2, sigma2, fu, fv, uc, vc, indices=None, n_matches=None):
        self.P3w = np.ascontiguousarray(P3w, np.float32).reshape(-1, 3)
        self.P2 = np.ascontiguousarray(P2, np.float32).reshape(-1, 2)
        self.sigma2 = np.asarray(sigma2, np.float32)
        self.cam = (float(fu), float(fv), float(uc), float(vc))
        self.N = len(self.P3w)
        self.indices = np.arange(self.N) if indices is None else np.asarray(indices)
        self.n_matches = self.N if n_matches is None else int(n_matches)
        self.iterations = 0
        self.best_inliers = 0
        self.best_mask = np.zeros(self.N, np.uint8)
        self.best_Tcw = None
        self.set_ransac_parameters()

    def set_ransac_parameters(self, probability=0.99, min_inliers=8, max_iterations=300, min_set=4, epsilon=0.4,
                              th2=5.991):
        """PnPsolver.cpp:159-195."""
        N = self.N
        eps = np.float32(epsilon)
        n_min = int(np.float32(N) * eps)
        n_min = max(n_min, min_inliers, min_set)
        self.min_inliers, self.min_set, self.prob = n_min, min_set, probability
        if N and eps < np.float32(n_min) / np.float32(N):
            eps = np.float32(n_min) / np.float32(N)
        if n_min == N:
            n_it = 1
        else:
            with np.errstate(all="ignore"):
                v = math.log(1 - probability) / math.log(1 - float(eps) ** 3) if 0 < float(eps) < 1 else float("nan")
            n_it = int(math.ceil(v)) if math.isfinite(v) else -(2 ** 31)
        self.max_its = max(1, min(n_it, max_iterations))
        self.maxerr = (self.sigma2 * np.float32(th2)).astype(np.float32)

    def iterate(self, n_iterations):
        """PnPsolver::iterate (PnPsolver.cpp:203-301): returns (Tcw or None,
        no_more, inliers[n_matches] bool, n_inliers)."""
        inl = np.zeros(self.n_matches, bool)
        if self.N < self.min_inliers:
            return None, True, np.zeros(0, bool), 0
        # while (mnIterations < maxIts || nCurrentIterations < nIterations)
        n_hyp = max(self.max_its - self.iterations, n_iterations)
        snap = get_state()
        samples = draw_sets(self.N, n_hyp, self.min_set)
        prob = (PnPProblem * 1)()
        p = prob[0]
        p.n, p.offset, p.min_inliers, p.best_inliers = self.N, 0, self.min_inliers, self.best_inliers
        p.n_hyp, p.sample_offset = n_hyp, 0
        p.fu, p.fv, p.uc, p.vc = self.cam
        bm = self.best_mask.copy()
        rm = np.zeros(self.N, np.uint8)
        r = pnp_ransac_batch(prob, self.P3w, self.P2, self.maxerr, samples, bm, rm)[0]
        set_state(snap)  # consume exactly the draws of the iterations run
        draw_sets(self.N, r.consumed, self.min_set)
        self.iterations += r.consumed
        self.best_inliers = r.best_inliers
        if r.best_hyp >= 0:
            self.best_mask = bm
            self.best_Tcw = np.array(r.best_Tcw, np.float32).reshape(4, 4)
        if r.found:
            inl[self.indices[rm.astype(bool)]] = True
            return np.array(r.refined_Tcw, np.float32).reshape(4, 4), False, inl, r.refined_inliers
        no_more = self.iterations >= self.max_its
        if no_more and self.best_inliers >= self.min_inliers:
            inl[self.indices[self.best_mask.astype(bool)]] = True
            return self.best_Tcw.copy(), True, inl, self.best_inliers
        return None, no_more, np.zeros(0, bool), 0

    def find(self):
        T, _, inl, n = self.iterate(self.max_its)
        return T, inl, n
