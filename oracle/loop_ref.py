"""CPU restatement of LoopClosing::ComputeSim3's hot loop.

TEST INFRASTRUCTURE ONLY: the parity oracle for csrc/loop.hip (and the
large-vocabulary DBoW2 transform of csrc/bow.hip); imported by tests/ and
nothing else.  Citations: LC = /root/reference/ORB-SLAM2/src/LoopClosing.cpp,
S3 = .../src/Sim3Solver.cpp, T = .../Thirdparty/DBoW2/DBoW2/
TemplatedVocabulary.h, R = .../Thirdparty/DBoW2/DUtils/Random.cpp.

* ``ArrayVocabulary.transform`` -- TemplatedVocabulary::transform (T:1151-1283)
  vectorised over features for trees of a million nodes (same walk as
  bow_ref.Vocabulary.transform_one: first minimum among the children in file
  order, direct-index node at level L - levelsup, FeatureVector entries for
  features with weight > 0).
* ``sim3_setup`` -- the Sim3Solver constructor (S3:37-107): correspondences in
  vpMatched12 order, camera-frame points Rcw*Xw + tcw with double-accumulated
  products (OpenCV's float gemm), truncated 9.210*sigma^2 error bounds.
* ``compute_sim3`` -- the round-robin loop (LC:339-356) over Sim3Solver
  objects whose iterate() (S3:147-221) is oracle/ransac_ref.cpp's
  orbref_sim3_ransac, drawing every minimal set with the HOST glibc rand()
  (srand(seed) per query) through RandomInt (R:33-50) -- the random stream
  is pinned to the real libc, not to a restatement.  The SearchBySim3 /
  OptimizeSim3 verification (LC:358-392) is outside the hot path and taken
  to pass: a query ends at the first iterate() that returns a Sim3.

Parity of the Sim3 arithmetic itself against the reference's OpenCV build
is unpinned; the GPU is compared with this oracle on integer
outcomes exactly and on the pose to the tolerance of tests/test_ransac.py.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import math

import numpy as np

import orbref

POP8 = np.array([bin(i).count("1") for i in range(256)], np.int32)


class ArrayVocabulary:
    """TemplatedVocabulary nodes from the arrays of synth.synthetic_vocabulary*
    (node i+1 = parent[i], is_leaf[i], desc[i], weight[i]; node 0 = root)."""

    def __init__(self, k, L, scoring, weighting, parent, is_leaf, desc, weight):
        self.k, self.L, self.scoring, self.weighting = k, L, scoring, weighting
        n = len(parent) + 1
        self.desc = np.concatenate([np.zeros((1, 32), np.uint8), np.asarray(desc, np.uint8)])
        self.weight = np.concatenate([[0.0], np.asarray(weight, np.float64)])
        leaf = np.concatenate([[0], np.asarray(is_leaf, np.int32)])
        self.word_id = np.zeros(n, np.int64)
        self.word_id[leaf > 0] = np.arange(int((leaf > 0).sum()))
        par = np.asarray(parent, np.int64)
        order = np.argsort(par, kind="stable")  # children grouped by parent, file order kept
        self.children = (order + 1).astype(np.int64)
        self.child_count = np.bincount(par, minlength=n).astype(np.int64)
        self.child_start = np.concatenate([[0], np.cumsum(self.child_count)[:-1]]).astype(np.int64)

    def transform(self, D: np.ndarray, levelsup: int = 4):
        """(words, nodes, weights, fv dict node -> [features]) for descriptors D."""
        D = np.asarray(D, np.uint8).reshape(-1, 32)
        n = len(D)
        final = np.zeros(n, np.int64)
        nid = np.zeros(n, np.int64)
        nid_level = self.L - levelsup
        active = np.ones(n, bool) if self.child_count[0] > 0 else np.zeros(n, bool)
        level = 0
        while active.any():
            level += 1
            idx = np.nonzero(active)[0]
            f = final[idx]
            cs, cc = self.child_start[f], self.child_count[f]
            w = int(cc.max())
            slot = np.arange(w)[None, :]
            cand = self.children[np.minimum(cs[:, None] + slot, len(self.children) - 1)]
            d = POP8[D[idx, None, :] ^ self.desc[cand]].sum(-1)
            d[slot >= cc[:, None]] = 1 << 20
            best = np.argmin(d, axis=1)  # first minimum, children in file order
            final[idx] = cand[np.arange(len(idx)), best]
            if level == nid_level:
                nid[idx] = final[idx]
            active[idx] = self.child_count[final[idx]] > 0
        words, weights = self.word_id[final], self.weight[final]
        fv = {}
        for i in range(n):
            if weights[i] > 0:
                fv.setdefault(int(nid[i]), []).append(i)
        return words, nid, weights, dict(sorted(fv.items()))


def _gemv_f32(R, X):
    """float 3x3 * float 3-vector with double accumulation, rounded to float
    (OpenCV 2.4 GEMMSingleMul<float,double> for a small product)."""
    R = R.astype(np.float64)
    X = X.astype(np.float64)
    return ((R[:, 0] * X[0] + R[:, 1] * X[1]) + R[:, 2] * X[2]).astype(np.float32)


def sim3_setup(match12, valid1, valid2, mp1, mp2, Tcw1, Tcw2, oct1, oct2, sigma2):
    """Sim3Solver::Sim3Solver (S3:37-107) -> (X1, X2, e1, e2, idx1)."""
    R1, t1 = np.asarray(Tcw1[:9], np.float32).reshape(3, 3), np.asarray(Tcw1[9:12], np.float32)
    R2, t2 = np.asarray(Tcw2[:9], np.float32).reshape(3, 3), np.asarray(Tcw2[9:12], np.float32)
    X1, X2, e1, e2, idx = [], [], [], [], []
    for i1, i2 in enumerate(match12):
        if i2 < 0 or not valid1[i1] or not valid2[i2]:
            continue
        X1.append((_gemv_f32(R1, mp1[i1]) + t1).astype(np.float32))
        X2.append((_gemv_f32(R2, mp2[i2]) + t2).astype(np.float32))
        # mvnMaxError = 9.210*sigma^2 in a vector<size_t> (S3:92-93)
        e1.append(np.float32(math.floor(9.210 * float(np.float32(sigma2[oct1[i1]])))))
        e2.append(np.float32(math.floor(9.210 * float(np.float32(sigma2[oct2[i2]])))))
        idx.append(i1)
    f = lambda a, s: np.array(a, np.float32).reshape(s)  # noqa: E731
    return f(X1, (-1, 3)), f(X2, (-1, 3)), f(e1, (-1,)), f(e2, (-1,)), np.array(idx, np.int32)


_LIBC = None


def libc():
    global _LIBC
    if _LIBC is None:
        _LIBC = ctypes.CDLL(ctypes.util.find_library("c"))
        _LIBC.srand.argtypes = [ctypes.c_uint]
        _LIBC.rand.restype = ctypes.c_int
    return _LIBC


def random_int(lo, hi):
    """DUtils::Random::RandomInt on the host glibc rand() (R:33-50)."""
    d = hi - lo + 1
    return int((libc().rand() / (2147483647 + 1.0)) * d) + lo


def max_iterations(N, min_inliers=20, probability=0.99, max_its=300):
    """Sim3Solver::SetRansacParameters (S3:111-141)."""
    eps = float(np.float32(min_inliers) / np.float32(N))
    if min_inliers == N:
        n_it = 1
    else:
        with np.errstate(all="ignore"):
            den = math.log(1 - eps ** 3) if eps < 1 else float("nan")
            v = math.log(1 - probability) / den if den == den and den != 0 else float("nan")
        n_it = int(math.ceil(v)) if math.isfinite(v) and abs(v) < 2 ** 31 else -(2 ** 31)
    return max(1, min(n_it, max_its))


class Sim3SolverRef:
    """One Sim3Solver over the set-up correspondences."""

    def __init__(self, corr, K1, K2, fix_scale, min_inliers=20, probability=0.99, max_its=300):
        self.X1, self.X2, self.e1, self.e2, self.idx = corr
        self.N = len(self.X1)
        self.K1, self.K2 = np.asarray(K1, np.float32), np.asarray(K2, np.float32)
        self.fix_scale, self.min_inliers = fix_scale, min_inliers
        self.max_its = max_iterations(self.N, min_inliers, probability, max_its) if self.N > 0 else 0
        self.iterations = 0
        self.best = 0
        self.best_pose = None
        self.best_mask = None

    def iterate(self, n_iterations):
        """(found, no_more, n_inliers) -- S3:147-221."""
        if self.N < self.min_inliers:
            return False, True, 0
        n_hyp = max(0, min(n_iterations, self.max_its - self.iterations))
        samples = np.zeros((n_hyp, 3), np.int32)
        found = False
        for h in range(n_hyp):
            avail = list(range(self.N))
            for k in range(3):
                r = random_int(0, len(avail) - 1)
                samples[h, k] = avail[r]
                avail[r] = avail[-1]
                avail.pop()
            out = orbref.sim3_ransac(self.X1, self.X2, self.e1, self.e2, self.K1, self.K2, self.fix_scale,
                                     self.min_inliers, self.best, samples[h:h + 1])
            self.iterations += 1
            if out["best_hyp"] >= 0:
                self.best = out["best_inliers"]
                self.best_pose = out
                self.best_mask = out["inliers"].astype(bool)
            if out["found"]:
                found = True
                break
        if found:
            return True, False, self.best
        return False, self.iterations >= self.max_its, 0


def compute_sim3(solvers, seed, iterations_per_call=5):
    """The while/for loop of ComputeSim3 (LC:339-356) from srand(seed).
    solvers: Sim3SolverRef or None (discarded before RANSAC, LC:314-318).
    Returns dict(matched, round, n_inliers, hypotheses, solver)."""
    libc().srand(seed)
    discarded = [s is None for s in solvers]
    n_cand = sum(not d for d in discarded)
    rnd = -1
    while n_cand > 0:
        rnd += 1
        for i, s in enumerate(solvers):
            if discarded[i]:
                continue
            found, no_more, nin = s.iterate(iterations_per_call)
            if no_more:
                discarded[i] = True
                n_cand -= 1
            if found:
                return {"matched": i, "round": rnd, "n_inliers": nin, "discarded": discarded,
                        "hypotheses": sum(x.iterations for x in solvers if x is not None)}
    return {"matched": -1, "round": -1, "n_inliers": 0, "discarded": discarded,
            "hypotheses": sum(x.iterations for x in solvers if x is not None)}
