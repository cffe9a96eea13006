"""CPU restatement of PnPsolver (EPnP + RANSAC) in numpy.

TEST INFRASTRUCTURE ONLY: the parity oracle for csrc/pnp.hip (imported by
tests/ and nothing else).  Citations: P = /root/reference/ORB-SLAM2/src/
PnPsolver.cpp.  The reference's OpenCV-1 linear algebra (cvSVD, cvInvert and
cvSolve with CV_SVD) is restated with numpy's LAPACK SVD/eigh; its own
qr_solve is restated line by line.  PARITY STATUS: vs OpenCV unpinned; GPU
vs this oracle to a stated pose tolerance (tests/test_pnp.py).
"""
from __future__ import annotations

import numpy as np


def _sym_eig_desc(a):
    """cvSVD(A, D, U^T) of a symmetric PSD matrix: eigenvalues descending,
    eigenvectors as rows."""
    w, v = np.linalg.eigh(a)
    order = np.argsort(-w, kind="stable")
    return w[order], v[:, order].T


def _qr_solve(A, b, X=None):
    """PnPsolver::qr_solve (P:955-1047), Householder QR least squares, letter
    for letter: the eta scan starts at |A[k,k]| and covers rows k .. nr-2 (the
    pointer loop P:975-980 reads before it advances, so the last row never
    takes part); the column is scaled by `*= inv_eta`, inv_eta = 1./eta
    (P:987-990); a zero eta returns with X untouched (P:982-985)."""
    A = A.copy()
    b = b.copy()
    nr, nc = A.shape
    X = np.zeros(nc) if X is None else X.copy()
    A1 = np.zeros(nc)
    A2 = np.zeros(nc)
    for k in range(nc):
        eta = abs(A[k, k])
        for i in range(k + 1, nr):
            elt = abs(A[i - 1, k])
            if eta < elt:
                eta = elt
        if eta == 0:
            return X
        inv_eta = 1.0 / eta
        s = 0.0
        for i in range(k, nr):
            A[i, k] *= inv_eta
            s += A[i, k] * A[i, k]
        sigma = np.sqrt(s)
        if A[k, k] < 0:
            sigma = -sigma
        A[k, k] += sigma
        A1[k] = sigma * A[k, k]
        A2[k] = -eta * sigma
        for j in range(k + 1, nc):
            t = 0.0
            for i in range(k, nr):
                t += A[i, k] * A[i, j]
            tau = t / A1[k]
            for i in range(k, nr):
                A[i, j] -= tau * A[i, k]
    for j in range(nc):
        tau = 0.0
        for i in range(j, nr):
            tau += A[i, j] * b[i]
        tau /= A1[j]
        for i in range(j, nr):
            b[i] -= tau * A[i, j]
    X[nc - 1] = b[nc - 1] / A2[nc - 1]
    for i in range(nc - 2, -1, -1):
        s = 0.0
        for j in range(i + 1, nc):
            s += A[i, j] * X[j]
        X[i] = (b[i] - s) / A2[i]
    return X


W_NULL = np.array([[((i * 7 + j * 13 + i * j * 5 + 3) % 17 - 8) / 8.0 for j in range(4)] for i in range(12)])


def canonicalize_null_space(ut, k):
    """Spec decision: the k = 12 - 2n exact null-space vectors of
    M (rows 11, 10, ... of ut) are replaced by the orthonormal basis Q of the
    same subspace with W^T Q upper triangular: Gram-Schmidt of V (W^T V)^-1."""
    ut = ut.copy()
    V = np.stack([ut[11 - c] for c in range(k)], 1)
    B = V @ np.linalg.inv(W_NULL[:, :k].T @ V)
    for c in range(k):
        for j in range(c):
            B[:, c] -= (B[:, j] @ B[:, c]) * B[:, j]
        B[:, c] /= np.linalg.norm(B[:, c])
    for c in range(k):
        ut[11 - c] = B[:, c]
    return ut


def compute_pose(pws, us, cam):
    """PnPsolver::compute_pose (P:523-580).  pws (n,3), us (n,2) float64,
    cam = (fu, fv, uc, vc).  Returns (R 3x3, t 3, mean reprojection error)."""
    fu, fv, uc, vc = cam
    n = len(pws)
    # choose_control_points (P:423-455)
    c0 = pws.mean(axis=0)
    d = pws - c0
    dc, uct = _sym_eig_desc(d.T @ d)
    for i in range(3):  # spec decision: largest-magnitude component positive
        if uct[i, np.argmax(np.abs(uct[i]))] < 0:
            uct[i] = -uct[i]
    cws = np.zeros((4, 3))
    cws[0] = c0
    for i in range(1, 4):
        cws[i] = c0 + np.sqrt(dc[i - 1] / n) * uct[i - 1]
    # compute_barycentric_coordinates (P:457-481), cvInvert(CV_SVD) = pinv
    cc = (cws[1:] - cws[0]).T
    ci = np.linalg.pinv(cc)
    alphas = np.zeros((n, 4))
    alphas[:, 1:] = (pws - cws[0]) @ ci.T
    alphas[:, 0] = 1.0 - alphas[:, 1] - alphas[:, 2] - alphas[:, 3]
    # fill_M (P:483-497), M^T M, cvSVD
    M = np.zeros((2 * n, 12))
    for k in range(4):
        M[0::2, 3 * k] = alphas[:, k] * fu
        M[0::2, 3 * k + 2] = alphas[:, k] * (uc - us[:, 0])
        M[1::2, 3 * k + 1] = alphas[:, k] * fv
        M[1::2, 3 * k + 2] = alphas[:, k] * (vc - us[:, 1])
    _, ut = _sym_eig_desc(M.T @ M)
    if 12 - 2 * n > 0:
        ut = canonicalize_null_space(ut, min(4, 12 - 2 * n))
    # compute_L_6x10 (P:863-898), compute_rho (P:900-908)
    v = [ut[11 - i] for i in range(4)]
    pairs = [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]
    dv = np.array([[v[i][3 * a:3 * a + 3] - v[i][3 * b:3 * b + 3] for (a, b) in pairs] for i in range(4)])
    L = np.zeros((6, 10))
    for j in range(6):
        D = dv[:, j]
        L[j] = [D[0] @ D[0], 2 * D[0] @ D[1], D[1] @ D[1], 2 * D[0] @ D[2], 2 * D[1] @ D[2], D[2] @ D[2],
                2 * D[0] @ D[3], 2 * D[1] @ D[3], 2 * D[2] @ D[3], D[3] @ D[3]]
    rho = np.array([((cws[a] - cws[b]) ** 2).sum() for (a, b) in pairs])

    def gauss_newton(betas):  # P:942-963, compute_A_and_b_gauss_newton P:910-940
        x = np.zeros(4)  # gauss_newton's x, kept by a singular qr_solve
        for _ in range(5):
            A = np.zeros((6, 4))
            bb = np.zeros(6)
            for i in range(6):
                r = L[i]
                b0, b1, b2, b3 = betas
                A[i] = [2 * r[0] * b0 + r[1] * b1 + r[3] * b2 + r[6] * b3,
                        r[1] * b0 + 2 * r[2] * b1 + r[4] * b2 + r[7] * b3,
                        r[3] * b0 + r[4] * b1 + 2 * r[5] * b2 + r[8] * b3,
                        r[6] * b0 + r[7] * b1 + r[8] * b2 + 2 * r[9] * b3]
                bb[i] = rho[i] - (r[0] * b0 * b0 + r[1] * b0 * b1 + r[2] * b1 * b1 + r[3] * b0 * b2 + r[4] * b1 * b2 +
                                  r[5] * b2 * b2 + r[6] * b0 * b3 + r[7] * b1 * b3 + r[8] * b2 * b3 + r[9] * b3 * b3)
            x = _qr_solve(A, bb, x)
            betas = betas + x
        return betas

    def r_and_t(betas):  # compute_R_and_t (P:735-745)
        ccs = np.zeros((4, 3))
        for i in range(4):
            ccs += betas[i] * ut[11 - i].reshape(4, 3)
        pcs = alphas @ ccs
        if pcs[0, 2] < 0:  # solve_for_sign (P:715-733)
            ccs = -ccs
            pcs = -pcs
        pc0, pw0 = pcs.mean(axis=0), pws.mean(axis=0)  # estimate_R_and_t (P:636-700)
        abt = (pcs - pc0).T @ (pws - pw0)
        U, _, Vt = np.linalg.svd(abt)
        R = U @ Vt
        if np.linalg.det(R) < 0:
            R[2] = -R[2]
        t = pc0 - R @ pw0
        Xc = pws @ R.T + t  # reprojection_error (P:612-634)
        ue = uc + fu * Xc[:, 0] / Xc[:, 2]
        ve = vc + fv * Xc[:, 1] / Xc[:, 2]
        err = np.sqrt((us[:, 0] - ue) ** 2 + (us[:, 1] - ve) ** 2).mean()
        return R, t, err

    sols = []
    b4 = np.linalg.lstsq(L[:, [0, 1, 3, 6]], rho, rcond=None)[0]  # find_betas_approx_1 (P:747-781)
    if b4[0] < 0:
        B = np.array([np.sqrt(-b4[0]), 0, 0, 0])
        B[1:] = -b4[1:] / B[0]
    else:
        B = np.array([np.sqrt(b4[0]), 0, 0, 0])
        B[1:] = b4[1:] / B[0]
    sols.append(r_and_t(gauss_newton(B)))
    b3 = np.linalg.lstsq(L[:, :3], rho, rcond=None)[0]  # find_betas_approx_2 (P:783-815)
    if b3[0] < 0:
        B = np.array([np.sqrt(-b3[0]), np.sqrt(-b3[2]) if b3[2] < 0 else 0.0, 0, 0])
    else:
        B = np.array([np.sqrt(b3[0]), np.sqrt(b3[2]) if b3[2] > 0 else 0.0, 0, 0])
    if b3[1] < 0:
        B[0] = -B[0]
    sols.append(r_and_t(gauss_newton(B)))
    b5 = np.linalg.lstsq(L[:, :5], rho, rcond=None)[0]  # find_betas_approx_3 (P:817-851)
    if b5[0] < 0:
        B = np.array([np.sqrt(-b5[0]), np.sqrt(-b5[2]) if b5[2] < 0 else 0.0, 0, 0])
    else:
        B = np.array([np.sqrt(b5[0]), np.sqrt(b5[2]) if b5[2] > 0 else 0.0, 0, 0])
    if b5[1] < 0:
        B[0] = -B[0]
    B[2] = b5[3] / B[0]
    sols.append(r_and_t(gauss_newton(B)))
    best = 0
    if sols[1][2] < sols[0][2]:
        best = 1
    if sols[2][2] < sols[best][2]:
        best = 2
    return sols[best]


def check_inliers(R, t, P3w, P2, maxerr, cam):
    """PnPsolver::CheckInliers (P:352-386) with its float/double mix."""
    fu, fv, uc, vc = cam
    X = P3w.astype(np.float64)
    Xc = (R[0, 0] * X[:, 0] + R[0, 1] * X[:, 1] + R[0, 2] * X[:, 2] + t[0]).astype(np.float32)
    Yc = (R[1, 0] * X[:, 0] + R[1, 1] * X[:, 1] + R[1, 2] * X[:, 2] + t[1]).astype(np.float32)
    invZc = (1 / (R[2, 0] * X[:, 0] + R[2, 1] * X[:, 1] + R[2, 2] * X[:, 2] + t[2])).astype(np.float32)
    ue = uc + fu * Xc.astype(np.float64) * invZc.astype(np.float64)
    ve = vc + fv * Yc.astype(np.float64) * invZc.astype(np.float64)
    dx = (P2[:, 0].astype(np.float64) - ue).astype(np.float32)
    dy = (P2[:, 1].astype(np.float64) - ve).astype(np.float32)
    e2 = dx * dx + dy * dy
    return e2 < maxerr


def ransac_call(P3w, P2, maxerr, cam, min_inliers, best_inliers, best_mask, samples):
    """The loop body of PnPsolver::iterate (P:224-299) over the given
    4-tuples, with Refine (P:303-349).  Returns dict(found, consumed,
    best_inliers, best_hyp, best_R, best_t, best_mask, refined_R, refined_t,
    refined_inliers, refined_mask)."""
    cam = tuple(float(c) for c in cam)
    pw_all = P3w.astype(np.float64)
    us_all = P2.astype(np.float64)
    best = best_inliers
    best_hyp = -1
    bmask = np.asarray(best_mask, bool).copy()
    bR = bt = None
    tried = False
    out = {"found": 0, "consumed": len(samples), "refined_inliers": 0, "refined_R": None, "refined_t": None,
           "refined_mask": None}
    for h, idx in enumerate(samples):
        R, t, _ = compute_pose(pw_all[idx], us_all[idx], cam)
        mask = check_inliers(R, t, P3w, P2, maxerr, cam)
        c = int(mask.sum())
        if c < min_inliers:
            continue
        if c > best:
            best, best_hyp, bmask, bR, bt, tried = c, h, mask, R, t, False
        if not tried:
            sel = np.nonzero(bmask)[0]
            Rr, tr, _ = compute_pose(pw_all[sel], us_all[sel], cam)
            rmask = check_inliers(Rr, tr, P3w, P2, maxerr, cam)
            tried = True
            out.update(refined_R=Rr, refined_t=tr, refined_mask=rmask, refined_inliers=int(rmask.sum()))
            if rmask.sum() > min_inliers:
                out.update(found=1, consumed=h + 1)
                break
    out.update(best_inliers=best, best_hyp=best_hyp, best_mask=bmask, best_R=bR, best_t=bt)
    if not out["found"]:
        out["refined_inliers"] = 0
    return out
