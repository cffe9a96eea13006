"""CPU restatement of LocalMapping::CreateNewMapPoints' per-match
triangulation (src/LocalMapping.cpp:369-515, KeyFrame::UnprojectStereo
src/KeyFrame.cpp:747-775).

TEST INFRASTRUCTURE ONLY: the oracle for csrc/mapping.hip.  numpy float32
scalars in the reference's expression order; cv::Mat float products with
double accumulation (the repo's convention); the 4x4
SVD by LAPACK in double (OpenCV's float Jacobi SVD is not reproducible:
parity by tolerance, parity against the reference binary unpinned).
"""
from __future__ import annotations

import math

import numpy as np

F, D = np.float32, np.float64


def _rwc(T, v):
    T = np.asarray(T, F).reshape(3, 4)
    return [F(D(T[0, j]) * D(v[0]) + D(T[1, j]) * D(v[1]) + D(T[2, j]) * D(v[2])) for j in range(3)]


def _rowdot_t(T, r, x):
    T = np.asarray(T, F).reshape(3, 4)
    return F(D(T[r, 0]) * D(x[0]) + D(T[r, 1]) * D(x[1]) + D(T[r, 2]) * D(x[2]) + D(T[r, 3]))


def _norm_d(v):  # cv::norm: double
    return math.sqrt(D(v[0]) * D(v[0]) + D(v[1]) * D(v[1]) + D(v[2]) * D(v[2]))


def _norm(v):  # float dist = cv::norm(...)
    return F(_norm_d(v))


def _unproject(K, i):
    z = F(K["depth"][i])
    if not z > 0:
        return None
    u, v = F(K["kps"]["x"][i]), F(K["kps"]["y"][i])
    xc = [F(F(F(u - F(K["cx"])) * z) * F(K["invfx"])), F(F(F(v - F(K["cy"])) * z) * F(K["invfy"])), z]
    r = _rwc(K["Tcw"], xc)
    return [F(r[j] + F(K["Ow"][j])) for j in range(3)]


def _reproj_ok(K, X, kp, ur, stereo, mbf, z):
    s2 = F(K["level_sigma2"][int(kp["octave"]) & 15])
    x, y = _rowdot_t(K["Tcw"], 0, X), _rowdot_t(K["Tcw"], 1, X)
    invz = F(F(1.0) / z)
    u = F(F(F(F(K["fx"]) * x) * invz) + F(K["cx"]))
    v = F(F(F(F(K["fy"]) * y) * invz) + F(K["cy"]))
    ex, ey = F(u - F(kp["x"])), F(v - F(kp["y"]))
    e2 = F(F(ex * ex) + F(ey * ey))
    if not stereo:
        return not D(e2) > 5.991 * D(s2)
    er = F(F(u - F(F(mbf) * invz)) - F(ur))
    return not D(F(e2 + F(er * er))) > 7.8 * D(s2)


def triangulate_matches(kf1, kf2, pairs, scale_factor):
    """-> (x3d (n, 3) float32, ok (n,) bool) per matched pair (idx1, idx2)."""
    n = len(pairs)
    out, ok = np.zeros((n, 3), F), np.zeros(n, bool)
    ratio_factor = F(F(1.5) * F(scale_factor))
    for m, (i1, i2) in enumerate(np.asarray(pairs).reshape(-1, 2)):
        A, B = kf1, kf2
        kp1, kp2 = A["kps_un"][i1], B["kps_un"][i2]
        ur1 = F(A["u_right"][i1]) if A.get("u_right") is not None else F(-1)
        ur2 = F(B["u_right"][i2]) if B.get("u_right") is not None else F(-1)
        st1, st2 = ur1 >= 0, ur2 >= 0
        xn1 = [F(F(F(kp1["x"]) - F(A["cx"])) * F(A["invfx"])), F(F(F(kp1["y"]) - F(A["cy"])) * F(A["invfy"])), F(1)]
        xn2 = [F(F(F(kp2["x"]) - F(B["cx"])) * F(B["invfx"])), F(F(F(kp2["y"]) - F(B["cy"])) * F(B["invfy"])), F(1)]
        r1, r2 = _rwc(A["Tcw"], xn1), _rwc(B["Tcw"], xn2)
        dot = D(r1[0]) * D(r2[0]) + D(r1[1]) * D(r2[1]) + D(r1[2]) * D(r2[2])
        cos_rays = F(dot / (_norm_d(r1) * _norm_d(r2)))  # LocalMapping.cpp:410, all double
        cs = F(cos_rays + F(1))
        cs1 = cs2 = cs
        if st1:
            cs1 = F(np.cos(F(F(2) * np.arctan2(F(F(A["b"]) / F(2)), F(A["depth"][i1])))))
        elif st2:
            cs2 = F(np.cos(F(F(2) * np.arctan2(F(F(B["b"]) / F(2)), F(B["depth"][i2])))))
        cs = min(cs1, cs2)
        if cos_rays < cs and cos_rays > 0 and (st1 or st2 or D(cos_rays) < 0.9998):
            T1, T2 = np.asarray(A["Tcw"], F).reshape(3, 4), np.asarray(B["Tcw"], F).reshape(3, 4)
            M = np.stack([xn1[0] * T1[2] - T1[0], xn1[1] * T1[2] - T1[1],
                          xn2[0] * T2[2] - T2[0], xn2[1] * T2[2] - T2[1]]).astype(F)
            _, _, vt = np.linalg.svd(M.astype(D))
            x = vt[3].astype(F)
            if x[3] == 0:
                continue
            X = [F(x[k] / x[3]) for k in range(3)]
        elif st1 and cs1 < cs2:
            X = _unproject(A, i1)
        elif st2 and cs2 < cs1:
            X = _unproject(B, i2)
        else:
            continue
        if X is None:
            continue
        z1 = _rowdot_t(A["Tcw"], 2, X)
        if z1 <= 0:
            continue
        z2 = _rowdot_t(B["Tcw"], 2, X)
        if z2 <= 0:
            continue
        if not _reproj_ok(A, X, kp1, ur1, st1, A["bf"], z1) or not _reproj_ok(B, X, kp2, ur2, st2, A["bf"], z2):
            continue
        d1 = _norm([F(X[k] - F(A["Ow"][k])) for k in range(3)])
        d2 = _norm([F(X[k] - F(B["Ow"][k])) for k in range(3)])
        if d1 == 0 or d2 == 0:
            continue
        ratio_dist = F(d2 / d1)
        ratio_oct = F(F(A["scale_factors"][int(kp1["octave"]) & 15]) / F(B["scale_factors"][int(kp2["octave"]) & 15]))
        if F(ratio_dist * ratio_factor) < ratio_oct or ratio_dist > F(ratio_oct * ratio_factor):
            continue
        out[m] = X
        ok[m] = True
    return out, ok
