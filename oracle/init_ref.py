"""CPU restatement of the monocular Initializer's model scoring -- TEST
INFRASTRUCTURE ONLY: imported by tests/ as the checker, never by the product
path (orb-slam2-annotation_amd/initializer.py -> csrc/init.hip).

  check_homography   Initializer::CheckHomography   src/Initializer.cpp:390-495
  check_fundamental  Initializer::CheckFundamental  src/Initializer.cpp:497-594
  select_best        FindHomography / FindFundamental's `if(currentScore>score)`
                     (src/Initializer.cpp:207-212, :264-269)

Float32 throughout, evaluated in the reference's expression order (numpy does
not contract a*b+c into an FMA); `1.0/x` is a double division rounded to float
as the reference's double literal makes it; the score is the sequential float
sum of the loop.

Parity unpinned against the reference itself: the reference ships no tests or
fixtures for the Initializer and its sources need OpenCV (cv::Mat,
cv::KeyPoint), which this image lacks, so they cannot be compiled here
(DESIGN.md §6).  The restatement follows the quoted lines term for term.
"""
from __future__ import annotations

import numpy as np

F = np.float32
TH_H = F(5.991)   # :409
TH_F = F(3.841)   # :514
TH_SCORE = F(5.991)  # :515


def inv_sigma_square(sigma: float) -> np.float32:
    """invSigmaSquare = 1.0/(sigma*sigma) (:411, :516)"""
    s = F(sigma)
    return F(1.0 / np.float64(s * s))


def _recip(w: np.ndarray) -> np.ndarray:
    return (1.0 / w.astype(np.float64)).astype(F)


def _seq_score(t1: np.ndarray, t2: np.ndarray) -> np.float32:
    score = F(0.0)
    for a, b in zip(t1.tolist(), t2.tolist()):
        score = F(score + F(a))
        score = F(score + F(b))
    return score


def homography_terms(pts: np.ndarray, H21: np.ndarray, H12: np.ndarray, sigma: float):
    """per-match chi-square pair of CheckHomography (:417-480)"""
    u1, v1, u2, v2 = (pts[:, k].astype(F) for k in range(4))
    h = H21.astype(F).reshape(9)
    g = H12.astype(F).reshape(9)
    inv = inv_sigma_square(sigma)
    w2in1inv = _recip(g[6] * u2 + g[7] * v2 + g[8])
    u2in1 = (g[0] * u2 + g[1] * v2 + g[2]) * w2in1inv
    v2in1 = (g[3] * u2 + g[4] * v2 + g[5]) * w2in1inv
    chi1 = ((u1 - u2in1) * (u1 - u2in1) + (v1 - v2in1) * (v1 - v2in1)) * inv
    w1in2inv = _recip(h[6] * u1 + h[7] * v1 + h[8])
    u1in2 = (h[0] * u1 + h[1] * v1 + h[2]) * w1in2inv
    v1in2 = (h[3] * u1 + h[4] * v1 + h[5]) * w1in2inv
    chi2 = ((u2 - u1in2) * (u2 - u1in2) + (v2 - v1in2) * (v2 - v1in2)) * inv
    return chi1.astype(F), chi2.astype(F)


def fundamental_terms(pts: np.ndarray, F21: np.ndarray, sigma: float):
    """per-match chi-square pair of CheckFundamental (:522-580)"""
    u1, v1, u2, v2 = (pts[:, k].astype(F) for k in range(4))
    f = F21.astype(F).reshape(9)
    inv = inv_sigma_square(sigma)
    a2 = f[0] * u1 + f[1] * v1 + f[2]
    b2 = f[3] * u1 + f[4] * v1 + f[5]
    c2 = f[6] * u1 + f[7] * v1 + f[8]
    num2 = a2 * u2 + b2 * v2 + c2
    chi1 = (num2 * num2 / (a2 * a2 + b2 * b2)) * inv
    a1 = f[0] * u2 + f[3] * v2 + f[6]
    b1 = f[1] * u2 + f[4] * v2 + f[7]
    c1 = f[2] * u2 + f[5] * v2 + f[8]
    num1 = a1 * u1 + b1 * v1 + c1
    chi2 = (num1 * num1 / (a1 * a1 + b1 * b1)) * inv
    return chi1.astype(F), chi2.astype(F)


def _score(chi1, chi2, th, ths):
    with np.errstate(invalid="ignore"):
        out1, out2 = chi1 > th, chi2 > th
        t1 = np.where(out1, F(0), ths - chi1).astype(F)
        t2 = np.where(out2, F(0), ths - chi2).astype(F)
    return _seq_score(t1, t2), ~(out1 | out2)


def check_homography(pts, H21, H12, sigma=1.0):
    """(score, vbMatchesInliers) of CheckHomography; pts = (n, 4) u1 v1 u2 v2"""
    with np.errstate(all="ignore"):
        chi1, chi2 = homography_terms(np.asarray(pts), np.asarray(H21), np.asarray(H12), sigma)
    return _score(chi1, chi2, TH_H, TH_H)


def check_fundamental(pts, F21, sigma=1.0):
    """(score, vbMatchesInliers) of CheckFundamental"""
    with np.errstate(all="ignore"):
        chi1, chi2 = fundamental_terms(np.asarray(pts), np.asarray(F21), sigma)
    return _score(chi1, chi2, TH_F, TH_SCORE)


def select_best(scores) -> int:
    """index of the kept iteration (first strict maximum above 0), or -1"""
    best, idx = F(0), -1
    for h, s in enumerate(np.asarray(scores, F).tolist()):
        if F(s) > best:
            best, idx = F(s), h
    return idx


# ---- model hypotheses (Normalize, ComputeH21/F21, FindHomography/Fundamental)
# The 8-point SVDs are restated with numpy's LAPACK SVD in double (cv::SVDecomp
# of the float DLT matrix is not reproducible here): H/F are compared with the
# GPU to a tolerance, the kept iteration exactly.

def normalize(pts: np.ndarray):
    """Normalize (Initializer.cpp:965-1015): sequential float sums; returns
    (normalised (n, 2) float32, T (3, 3) float32)."""
    pts = np.asarray(pts, F).reshape(-1, 2)
    n = len(pts)
    out = np.zeros_like(pts)
    T = np.eye(3, dtype=F)
    for ax in range(2):
        mean = F(0.0)
        for v in pts[:, ax].tolist():
            mean = F(mean + F(v))
        mean = F(mean / F(n))
        dev = F(0.0)
        for v in pts[:, ax].tolist():
            dev = F(dev + F(abs(F(F(v) - mean))))
        dev = F(dev / F(n))
        s = F(1.0 / np.float64(dev))
        out[:, ax] = ((pts[:, ax] - mean) * s).astype(F)
        T[ax, ax] = s
        T[ax, 2] = F(-mean * s)
    return out, T


def mul3(a, b):
    """float 3x3 product with double accumulation (OpenCV's small float gemm)"""
    a64, b64 = np.asarray(a, F).astype(np.float64), np.asarray(b, F).astype(np.float64)
    c = np.zeros((3, 3), np.float64)
    for i in range(3):
        for j in range(3):
            c[i, j] = (a64[i, 0] * b64[0, j] + a64[i, 1] * b64[1, j]) + a64[i, 2] * b64[2, j]
    return c.astype(F)


def inv3(m):
    """cv::Mat::inv() of a 3x3 CV_32F (closed form, double, rounded to float)"""
    S = np.asarray(m, F).astype(np.float64)
    d0 = (S[0, 0] * (S[1, 1] * S[2, 2] - S[1, 2] * S[2, 1]) - S[0, 1] * (S[1, 0] * S[2, 2] - S[1, 2] * S[2, 0]) +
          S[0, 2] * (S[1, 0] * S[2, 1] - S[1, 1] * S[2, 0]))
    if d0 == 0.0:
        return np.zeros((3, 3), F)
    d = 1.0 / d0
    t = [(S[1, 1] * S[2, 2] - S[1, 2] * S[2, 1]) * d, (S[0, 2] * S[2, 1] - S[0, 1] * S[2, 2]) * d,
         (S[0, 1] * S[1, 2] - S[0, 2] * S[1, 1]) * d, (S[1, 2] * S[2, 0] - S[1, 0] * S[2, 2]) * d,
         (S[0, 0] * S[2, 2] - S[0, 2] * S[2, 0]) * d, (S[0, 2] * S[1, 0] - S[0, 0] * S[1, 2]) * d,
         (S[1, 0] * S[2, 1] - S[1, 1] * S[2, 0]) * d, (S[0, 1] * S[2, 0] - S[0, 0] * S[2, 1]) * d,
         (S[0, 0] * S[1, 1] - S[0, 1] * S[1, 0]) * d]
    return np.array(t, np.float64).astype(F).reshape(3, 3)


def _null_vector(A):
    _, _, vt = np.linalg.svd(A.astype(np.float64))
    return vt[-1].astype(F)


def compute_h21(p1, p2):
    """ComputeH21 (:292-330): the float DLT matrix, vt.row(8)"""
    u1, v1, u2, v2 = p1[:, 0], p1[:, 1], p2[:, 0], p2[:, 1]
    A = np.zeros((2 * len(p1), 9), F)
    A[0::2, 3], A[0::2, 4], A[0::2, 5] = -u1, -v1, -1
    A[0::2, 6], A[0::2, 7], A[0::2, 8] = v2 * u1, v2 * v1, v2
    A[1::2, 0], A[1::2, 1], A[1::2, 2] = u1, v1, 1
    A[1::2, 6], A[1::2, 7], A[1::2, 8] = -u2 * u1, -u2 * v1, -u2
    return _null_vector(A).reshape(3, 3)


def compute_f21(p1, p2):
    """ComputeF21 (:332-388): vt.row(8) of the float DLT matrix, then the
    rank-2 projection (w(2) = 0)"""
    u1, v1, u2, v2 = p1[:, 0], p1[:, 1], p2[:, 0], p2[:, 1]
    A = np.stack([u2 * u1, u2 * v1, u2, v2 * u1, v2 * v1, v2, u1, v1, np.ones_like(u1)], 1).astype(F)
    if A.shape[0] < 9:
        A = np.vstack([A, np.zeros((9 - A.shape[0], 9), F)])
    Fpre = _null_vector(A).reshape(3, 3)
    u, w, vt = np.linalg.svd(Fpre.astype(np.float64))
    w[2] = 0.0
    return (u @ np.diag(w) @ vt).astype(F)


def find_models(kp1, kp2, pairs, sets, sigma=1.0):
    """Normalize + FindHomography + FindFundamental (:160-269) over the given
    minimal sets.  Returns dict with H21/H12/F21 per iteration, scores,
    kept iterations (best_h, best_f) and the score ratio RH (:140)."""
    pn1, T1 = normalize(kp1)
    pn2, T2 = normalize(kp2)
    pairs = np.asarray(pairs).reshape(-1, 2)
    pts = np.concatenate([np.asarray(kp1, F)[pairs[:, 0]], np.asarray(kp2, F)[pairs[:, 1]]], 1)
    T2inv, T2t = inv3(T2), T2.T.copy()
    n_it = len(sets)
    H21 = np.zeros((n_it, 3, 3), F)
    H12 = np.zeros((n_it, 3, 3), F)
    F21 = np.zeros((n_it, 3, 3), F)
    sh = np.zeros(n_it, F)
    sf = np.zeros(n_it, F)
    for it, s in enumerate(sets):
        a, b = pn1[pairs[s, 0]], pn2[pairs[s, 1]]
        H21[it] = mul3(mul3(T2inv, compute_h21(a, b)), T1)
        H12[it] = inv3(H21[it])
        F21[it] = mul3(mul3(T2t, compute_f21(a, b)), T1)
        sh[it] = check_homography(pts, H21[it], H12[it], sigma)[0]
        sf[it] = check_fundamental(pts, F21[it], sigma)[0]
    bh, bf = select_best(sh), select_best(sf)
    SH = sh[bh] if bh >= 0 else F(0)
    SF = sf[bf] if bf >= 0 else F(0)
    return {"pts": pts, "H21": H21, "H12": H12, "F21": F21, "scores_h": sh, "scores_f": sf, "best_h": bh,
            "best_f": bf, "RH": F(SH / F(SH + SF)) if SH + SF > 0 else F(0), "T1": T1, "T2": T2, "pn1": pn1,
            "pn2": pn2}


# ---- ReconstructH / ReconstructF (Initializer.cpp:596-963, CheckRT :1017-1118) ----
def _det3(m):
    S = np.asarray(m, F).astype(np.float64)
    return (S[0, 0] * (S[1, 1] * S[2, 2] - S[1, 2] * S[2, 1]) - S[0, 1] * (S[1, 0] * S[2, 2] - S[1, 2] * S[2, 0]) +
            S[0, 2] * (S[1, 0] * S[2, 1] - S[1, 1] * S[2, 0]))


def _svd3(M):
    """cv::SVD::compute of a 3x3 float Mat: (w, U, Vt) as floats (LAPACK in
    double; sign conventions only reorder the hypotheses)"""
    u, w, vt = np.linalg.svd(np.asarray(M, F).astype(np.float64))
    return w.astype(F), u.astype(F), vt.astype(F)


def _unit(t):
    t = np.asarray(t, F)
    nrm = np.sqrt(np.sum(t.astype(np.float64) ** 2))
    return (t.astype(np.float64) * (1.0 / nrm)).astype(F)


def _gemv(A, x):
    A64, x64 = np.asarray(A, F).astype(np.float64), np.asarray(x, F).astype(np.float64)
    return np.array([(A64[i, 0] * x64[0] + A64[i, 1] * x64[1]) + A64[i, 2] * x64[2] for i in range(3)]).astype(F)


def homography_hypotheses(H21, K):
    """ReconstructH's eight (R, t) (:700-850), or [] when d1/d2 or d2/d3 < 1.00001"""
    A = mul3(mul3(inv3(K), H21), K)
    w, U, Vt = _svd3(A)
    s = F(_det3(U) * _det3(Vt))
    d1, d2, d3 = w
    if float(F(d1 / d2)) < 1.00001 or float(F(d2 / d3)) < 1.00001:
        return []
    aux1 = F(np.sqrt(F(F(d1 * d1 - d2 * d2) / F(d1 * d1 - d3 * d3))))
    aux3 = F(np.sqrt(F(F(d2 * d2 - d3 * d3) / F(d1 * d1 - d3 * d3))))
    x1, x3 = [aux1, aux1, -aux1, -aux1], [aux3, -aux3, aux3, -aux3]
    ast = F(F(np.sqrt(F(F(d1 * d1 - d2 * d2) * F(d2 * d2 - d3 * d3)))) / F(F(d1 + d3) * d2))
    cth = F(F(F(d2 * d2) + F(d1 * d3)) / F(F(d1 + d3) * d2))
    asp = F(F(np.sqrt(F(F(d1 * d1 - d2 * d2) * F(d2 * d2 - d3 * d3)))) / F(F(d1 - d3) * d2))
    cph = F(F(F(d1 * d3) - F(d2 * d2)) / F(F(d1 - d3) * d2))
    st, sp = [ast, -ast, -ast, ast], [asp, -asp, -asp, asp]
    out = []
    for pas in range(2):
        for i in range(4):
            Rp = np.eye(3, dtype=F)
            if pas == 0:
                Rp[0, 0], Rp[0, 2], Rp[2, 0], Rp[2, 2] = cth, -st[i], st[i], cth
                tp = np.array([x1[i], 0, -x3[i]], F) * F(d1 - d3)
            else:
                Rp[0, 0], Rp[0, 2], Rp[1, 1], Rp[2, 0], Rp[2, 2] = cph, sp[i], -1, sp[i], -cph
                tp = np.array([x1[i], 0, x3[i]], F) * F(d1 + d3)
            URp = (U.astype(np.float64) @ Rp.astype(np.float64) * float(s)).astype(F)
            out.append((mul3(URp, Vt), _unit(_gemv(U, tp.astype(F)))))
    return out


def fundamental_hypotheses(F21, K):
    """DecomposeE (:1120-1150) of E21 = K^T F21 K; ReconstructF's order
    (R1, t), (R2, t), (R1, -t), (R2, -t)"""
    E = mul3(mul3(np.asarray(K, F).T.copy(), F21), K)
    w, U, Vt = _svd3(E)
    t = _unit(U[:, 2])
    W = np.array([[0, -1, 0], [1, 0, 0], [0, 0, 1]], F)
    R1 = mul3(mul3(U, W), Vt)
    if _det3(R1) < 0:
        R1 = -R1
    R2 = mul3(mul3(U, W.T.copy()), Vt)
    if _det3(R2) < 0:
        R2 = -R2
    return [(R1, t), (R2, t), (R1, -t), (R2, -t)]


def check_rt(R, t, pts, inliers, K, th2):
    """CheckRT (:1017-1118) for one hypothesis: (nGood, parallax, counted[n],
    good[n], p3d (n, 3)) per match (the reference indexes the last three by
    the match's first keypoint)."""
    K = np.asarray(K, F)
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    Rt = np.concatenate([np.asarray(R, F), np.asarray(t, F).reshape(3, 1)], 1)
    P2 = (K.astype(np.float64) @ Rt.astype(np.float64)).astype(F)
    O2 = (-(np.asarray(R, F).T.astype(np.float64) @ np.asarray(t, F).astype(np.float64))).astype(F)
    P1 = np.zeros((3, 4), F)
    P1[:, :3] = K
    n = len(pts)
    counted, good = np.zeros(n, bool), np.zeros(n, bool)
    p3d = np.zeros((n, 3), F)
    cosv = []
    for m in range(n):
        if not inliers[m]:
            continue
        u1, v1, u2, v2 = (F(x) for x in pts[m])
        A = np.stack([u1 * P1[2] - P1[0], v1 * P1[2] - P1[1], u2 * P2[2] - P2[0], v2 * P2[2] - P2[1]]).astype(F)
        _, _, vt = np.linalg.svd(A.astype(np.float64))
        x = vt[3].astype(F)
        X = (x[:3] / x[3]).astype(F)
        if not np.all(np.isfinite(X)):
            continue
        d1 = F(np.sqrt(np.sum(X.astype(np.float64) ** 2)))
        n2 = (X - O2).astype(F)
        d2 = F(np.sqrt(np.sum(n2.astype(np.float64) ** 2)))
        cp = F(float(np.dot(X.astype(np.float64), n2.astype(np.float64))) / float(F(d1 * d2)))
        if X[2] <= 0 and float(cp) < 0.99998:
            continue
        Xc2 = (_gemv(R, X) + np.asarray(t, F)).astype(F)
        if Xc2[2] <= 0 and float(cp) < 0.99998:
            continue
        iz1 = F(F(1.0) / X[2])
        im1x, im1y = F(F(fx * X[0]) * iz1 + cx), F(F(fy * X[1]) * iz1 + cy)
        if F(F((im1x - u1) * (im1x - u1)) + F((im1y - v1) * (im1y - v1))) > th2:
            continue
        iz2 = F(F(1.0) / Xc2[2])
        im2x, im2y = F(F(fx * Xc2[0]) * iz2 + cx), F(F(fy * Xc2[1]) * iz2 + cy)
        if F(F((im2x - u2) * (im2x - u2)) + F((im2y - v2) * (im2y - v2))) > th2:
            continue
        cosv.append(cp)
        counted[m] = True
        p3d[m] = X
        good[m] = float(cp) < 0.99998
    ng = int(counted.sum())
    if ng:
        cosv.sort()
        par = F(float(F(np.arccos(cosv[min(50, ng - 1)]) * F(180))) / np.pi)
    else:
        par = F(0)
    return ng, par, counted, good, p3d


def reconstruct(model, kp1, kp2, pairs, inliers, M21, K, sigma=1.0, min_parallax=1.0, min_triangulated=50):
    """ReconstructH (model 0) / ReconstructF (model 1): dict with ok, best,
    hyps [(R, t)], n_good, parallax, R21, t21, p3d (n1, 3), triangulated (n1)."""
    pairs = np.asarray(pairs).reshape(-1, 2)
    pts = np.concatenate([np.asarray(kp1, F)[pairs[:, 0]], np.asarray(kp2, F)[pairs[:, 1]]], 1)
    N = int(np.sum(np.asarray(inliers) != 0))
    hy = homography_hypotheses(M21, K) if model == 0 else fundamental_hypotheses(M21, K)
    th2 = F(4.0 * float(F(F(sigma) * F(sigma))))
    res = [check_rt(R, t, pts, inliers, K, th2) for R, t in hy]
    ng = [r[0] for r in res]
    par = [r[1] for r in res]
    best, ok = -1, False
    if model == 0 and hy:
        bg, sbg, bp = 0, 0, F(-1)
        for i in range(len(hy)):
            if ng[i] > bg:
                sbg, bg, best, bp = bg, ng[i], i, par[i]
            elif ng[i] > sbg:
                sbg = ng[i]
        ok = sbg < 0.75 * bg and bp >= min_parallax and bg > min_triangulated and bg > 0.9 * N
    elif model == 1:
        mg = max(ng)
        nmin = max(int(0.9 * N), min_triangulated)
        nsim = sum(1 for g in ng if g > 0.7 * mg)
        if not (mg < nmin or nsim > 1):
            best = ng.index(mg)
            ok = par[best] > min_parallax
    n1 = len(kp1)
    p3d, tri = np.zeros((n1, 3), F), np.zeros(n1, bool)
    if ok:
        _, _, counted, good, P = res[best]
        for m in np.nonzero(counted)[0]:
            p3d[pairs[m, 0]] = P[m]
            tri[pairs[m, 0]] = good[m]
    return {"ok": bool(ok), "best": best, "hyps": hy, "n_good": ng, "parallax": par,
            "R21": hy[best][0] if best >= 0 else None, "t21": hy[best][1] if best >= 0 else None,
            "p3d": p3d, "triangulated": tri}
