"""CPU restatement of the projection matchers: Frame::isInFrustum and the four
ORBmatcher::SearchByProjection overloads, with Frame::GetFeaturesInArea,
MapPoint::PredictScale and RadiusByViewingCos.

TEST INFRASTRUCTURE ONLY: the parity oracle for csrc/proj.hip.  Citations:
M = /root/reference/ORB-SLAM2/src/ORBmatcher.cpp, F = .../src/Frame.cpp,
MP = .../src/MapPoint.cpp.  Float arithmetic is restated in numpy float32
scalars, with cv::Mat products of float matrices accumulated in double as
OpenCV's small-matrix gemm does.  Bar: bit-exact matches and counts.
"""
from __future__ import annotations

import math

import numpy as np

f32, f64 = np.float32, np.float64
GC, GR, HL, TH_LOW, TH_HIGH = 64, 48, 30, 50, 100
VALID, HAS_OBS, IN_VIEW = 1, 2, 4
LOCAL, SIM3, LAST_FRAME, KEYFRAME = 0, 1, 2, 3


def dotd3(a, x):
    return f32(f64(a[0]) * f64(x[0]) + f64(a[1]) * f64(x[1]) + f64(a[2]) * f64(x[2]))


def transform(T, x):
    return [f32(dotd3(T[i, :3], x) + f32(T[i, 3])) for i in range(3)]


def camera_center(T):
    t = T[:3, 3]
    return [f32(-dotd3(T[:3, j], t)) for j in range(3)]


def norm3(v):
    return f32(math.sqrt(f64(v[0]) * f64(v[0]) + f64(v[1]) * f64(v[1]) + f64(v[2]) * f64(v[2])))


def c_round(v):
    v = float(v)
    return int(math.copysign(math.floor(abs(v) + 0.5), v))


def predict_scale(max_dist, dist, tgt):
    """MapPoint::PredictScale (MP:481-508)."""
    ratio = f32(f32(max_dist) / f32(dist))
    lg = f32(math.log(f64(ratio)))
    s = math.ceil(f32(lg / f32(tgt["log_scale_factor"])))
    return 0 if s < 0 else min(s, tgt["n_levels"] - 1)


class Grid:
    """Frame::AssignFeaturesToGrid / GetFeaturesInArea (F:241-259, 379-443)."""

    def __init__(self, tgt):
        self.t = tgt
        self.invW = f32(f32(GC) / f32(f32(tgt["max_x"]) - f32(tgt["min_x"])))
        self.invH = f32(f32(GR) / f32(f32(tgt["max_y"]) - f32(tgt["min_y"])))
        self.cells = [[[] for _ in range(GR)] for _ in range(GC)]
        k = tgt["kps"]
        for i in range(len(k)):
            px = c_round(f32(f32(k["x"][i]) - f32(tgt["min_x"])) * self.invW)
            py = c_round(f32(f32(k["y"][i]) - f32(tgt["min_y"])) * self.invH)
            if 0 <= px < GC and 0 <= py < GR:
                self.cells[px][py].append(i)

    def area(self, x, y, r, min_level=-1, max_level=-1):
        t, k = self.t, self.t["kps"]
        x, y, r = f32(x), f32(y), f32(r)
        mnx, mny = f32(t["min_x"]), f32(t["min_y"])
        cx0 = max(0, math.floor(f32(f32(x - mnx) - r) * self.invW))
        if cx0 >= GC:
            return []
        cx1 = min(GC - 1, math.ceil(f32(f32(x - mnx) + r) * self.invW))
        if cx1 < 0:
            return []
        cy0 = max(0, math.floor(f32(f32(y - mny) - r) * self.invH))
        if cy0 >= GR:
            return []
        cy1 = min(GR - 1, math.ceil(f32(f32(y - mny) + r) * self.invH))
        if cy1 < 0:
            return []
        check = min_level > 0 or max_level >= 0
        out = []
        for ix in range(cx0, cx1 + 1):
            for iy in range(cy0, cy1 + 1):
                for i in self.cells[ix][iy]:
                    o = int(k["octave"][i])
                    if check:
                        if o < min_level:
                            continue
                        if max_level >= 0 and o > max_level:
                            continue
                    if abs(f32(f32(k["x"][i]) - x)) < r and abs(f32(f32(k["y"][i]) - y)) < r:
                        out.append(i)
        return out


def is_in_frustum(tgt, pts, cos_limit):
    """Frame::isInFrustum (F:305-368) for every point; returns flags, track (n,4), level."""
    T = np.asarray(tgt["Tcw"], np.float32).reshape(4, 4)
    O = camera_center(T)
    n = len(pts["pos"])
    flags = np.array(pts["flags"], np.int32) & ~IN_VIEW
    track = np.zeros((n, 4), np.float32)
    level = np.zeros(n, np.int32)
    for i in range(n):
        X = pts["pos"][i]
        pc = transform(T, X)
        if pc[2] < f32(0):
            continue
        invz = f32(f32(1) / pc[2])
        u = f32(f32(f32(tgt["fx"]) * pc[0]) * invz + f32(tgt["cx"]))
        v = f32(f32(f32(tgt["fy"]) * pc[1]) * invz + f32(tgt["cy"]))
        if u < f32(tgt["min_x"]) or u > f32(tgt["max_x"]) or v < f32(tgt["min_y"]) or v > f32(tgt["max_y"]):
            continue
        maxd = f32(f32(1.2) * f32(pts["max_dist"][i]))
        mind = f32(f32(0.8) * f32(pts["min_dist"][i]))
        PO = [f32(f32(X[j]) - O[j]) for j in range(3)]
        dist = norm3(PO)
        if dist < mind or dist > maxd:
            continue
        Pn = pts["normal"][i]
        vc = f32((f64(PO[0]) * f64(Pn[0]) + f64(PO[1]) * f64(Pn[1]) + f64(PO[2]) * f64(Pn[2])) / f64(dist))
        if vc < f32(cos_limit):
            continue
        flags[i] |= IN_VIEW
        track[i] = [u, v, f32(u - f32(f32(tgt["bf"]) * invz)), vc]
        level[i] = predict_scale(pts["max_dist"][i], dist, tgt)
    return flags, track, level


def _hamming(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def search_by_projection(variant, tgt, pts, th, nnratio=0.6, check_ori=True, orb_dist=50, mono=True,
                         last_Tcw=None):
    """The four SearchByProjection overloads (M:63-155, 352-470, 1506-1641,
    1661-1790).  Returns (nmatches, match) with match per target keypoint:
    point index, -1 untouched, -2 set to NULL by the rotation cull."""
    k = tgt["kps"]
    n = len(k)
    grid = Grid(tgt)
    occ = list(np.asarray(tgt["occupied"], np.uint8)) if tgt.get("occupied") is not None else [0] * n
    uR = tgt.get("u_right")
    match = [-1] * n
    hist = [[] for _ in range(HL)]
    factor = f32(f32(HL) / f32(360.0))
    T = np.asarray(tgt["Tcw"], np.float32).reshape(4, 4)
    sf = [f32(s) for s in tgt["scale_factors"]]
    nm = 0
    if variant == SIM3:  # M:357-371
        scw = norm3(T[0, :3])
        Rs = np.zeros((4, 4), np.float32)
        Rs[:3, :3] = (T[:3, :3] / scw).astype(np.float32)
        Rs[:3, 3] = (T[:3, 3] / scw).astype(np.float32)
        O = camera_center(Rs)
    elif variant in (LAST_FRAME, KEYFRAME):
        O = camera_center(T)
        if variant == LAST_FRAME:  # M:1519-1527
            L = np.asarray(last_Tcw, np.float32).reshape(4, 4)
            tlc_z = f32(dotd3(L[2, :3], O) + L[2, 3])
            forward = tlc_z > f32(tgt["b"]) and not mono
            backward = -tlc_z > f32(tgt["b"]) and not mono
    for ip in range(len(pts["flags"])):
        fl = int(pts["flags"][ip])
        if not fl & VALID:
            continue
        stereo = False
        lvl_lo, lvl_hi = -1000, 1000
        if variant == LOCAL:
            if not fl & IN_VIEW:
                continue
            lvl = int(pts["track_level"][ip])
            r = f32(2.5) if f64(pts["track"][ip][3]) > 0.998 else f32(4.0)
            if f32(th) != f32(1.0):
                r = f32(r * f32(th))
            u, v = f32(pts["track"][ip][0]), f32(pts["track"][ip][1])
            rad = f32(r * sf[lvl])
            cands = grid.area(u, v, rad, lvl - 1, lvl)
            stereo, ur, srad = True, f32(pts["track"][ip][2]), rad
        elif variant == SIM3:
            X = pts["pos"][ip]
            pc = transform(Rs, X)
            if pc[2] < f32(0.0):
                continue
            invz = f32(f32(1) / pc[2])
            u = f32(f32(f32(tgt["fx"]) * f32(pc[0] * invz)) + f32(tgt["cx"]))
            v = f32(f32(f32(tgt["fy"]) * f32(pc[1] * invz)) + f32(tgt["cy"]))
            if not (u >= f32(tgt["min_x"]) and u < f32(tgt["max_x"]) and v >= f32(tgt["min_y"]) and
                    v < f32(tgt["max_y"])):
                continue
            maxd = f32(f32(1.2) * f32(pts["max_dist"][ip]))
            mind = f32(f32(0.8) * f32(pts["min_dist"][ip]))
            PO = [f32(f32(X[j]) - O[j]) for j in range(3)]
            dist = norm3(PO)
            if dist < mind or dist > maxd:
                continue
            Pn = pts["normal"][ip]
            dot = f64(PO[0]) * f64(Pn[0]) + f64(PO[1]) * f64(Pn[1]) + f64(PO[2]) * f64(Pn[2])
            if dot < 0.5 * f64(dist):
                continue
            lvl = predict_scale(pts["max_dist"][ip], dist, tgt)
            rad = f32(f32(th) * sf[lvl])
            cands = grid.area(u, v, rad)
            lvl_lo, lvl_hi = lvl - 1, lvl
        else:
            X = pts["pos"][ip]
            pc = transform(T, X)
            invzc = f32(1.0 / f64(pc[2]))
            if variant == LAST_FRAME and invzc < 0:
                continue
            u = f32(f32(f32(tgt["fx"]) * pc[0]) * invzc + f32(tgt["cx"]))
            v = f32(f32(f32(tgt["fy"]) * pc[1]) * invzc + f32(tgt["cy"]))
            if u < f32(tgt["min_x"]) or u > f32(tgt["max_x"]) or v < f32(tgt["min_y"]) or v > f32(tgt["max_y"]):
                continue
            if variant == LAST_FRAME:
                o = int(pts["octave"][ip])
                rad = f32(f32(th) * sf[o])
                if forward:
                    cands = grid.area(u, v, rad, o)
                elif backward:
                    cands = grid.area(u, v, rad, 0, o)
                else:
                    cands = grid.area(u, v, rad, o - 1, o + 1)
                stereo, ur, srad = True, f32(u - f32(f32(tgt["bf"]) * invzc)), rad
            else:
                PO = [f32(f32(X[j]) - O[j]) for j in range(3)]
                dist = norm3(PO)
                maxd = f32(f32(1.2) * f32(pts["max_dist"][ip]))
                mind = f32(f32(0.8) * f32(pts["min_dist"][ip]))
                if dist < mind or dist > maxd:
                    continue
                lvl = predict_scale(pts["max_dist"][ip], dist, tgt)
                rad = f32(f32(th) * sf[lvl])
                cands = grid.area(u, v, rad, lvl - 1, lvl + 1)
        if not cands:
            continue
        d = pts["desc"][ip]
        best, best_i, best_l = 256, -1, -1
        best2, best_l2 = 256, -1
        for i in cands:
            if variant in (LOCAL, LAST_FRAME):
                if occ[i] == 2:
                    continue
            elif occ[i]:
                continue
            if variant == SIM3 and not (lvl_lo <= int(k["octave"][i]) <= lvl_hi):
                continue
            if stereo and uR is not None and uR[i] > 0:
                if abs(f32(ur - f32(uR[i]))) > srad:
                    continue
            dist = _hamming(d, tgt["desc"][i])
            if dist < best:
                best2, best_l2 = best, best_l
                best, best_i, best_l = dist, i, int(k["octave"][i])
            elif dist < best2:
                best2, best_l2 = dist, int(k["octave"][i])
        if variant == LOCAL:
            if not (best <= TH_HIGH):
                continue
            if best_l == best_l2 and f32(best) > f32(f32(nnratio) * f32(best2)):
                continue
        elif variant == SIM3:
            if not best <= TH_LOW:
                continue
        elif variant == LAST_FRAME:
            if not best <= TH_HIGH:
                continue
        else:
            if not best <= orb_dist:
                continue
        match[best_i] = ip
        occ[best_i] = 2 if fl & HAS_OBS else 1
        nm += 1
        if check_ori and variant in (LAST_FRAME, KEYFRAME):
            rot = f32(f32(pts["angle"][ip]) - f32(k["angle"][best_i]))
            if rot < f32(0.0):
                rot = f32(rot + f32(360.0))
            b = c_round(f32(rot * factor))
            if b == HL:
                b = 0
            hist[b].append(best_i)
    if check_ori and variant in (LAST_FRAME, KEYFRAME):
        m1 = m2 = m3 = 0
        i1 = i2 = i3 = -1
        for i in range(HL):
            s = len(hist[i])
            if s > m1:
                m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, i
            elif s > m2:
                m3, m2, i3, i2 = m2, s, i2, i
            elif s > m3:
                m3, i3 = s, i
        if m2 < f32(0.1) * f32(m1):
            i2 = i3 = -1
        elif m3 < f32(0.1) * f32(m1):
            i3 = -1
        for i in range(HL):
            if i in (i1, i2, i3):
                continue
            for slot in hist[i]:
                match[slot] = -2
                nm -= 1
    return nm, np.array(match, np.int32)


FUSE, FUSE_SIM3, SIM3_DIR = 4, 5, 6


def radius_search(variant, tgt, pts, th, last_Tcw=None):
    """The per-point searches: Fuse(pKF, vpMapPoints, th) (M:962-1115, FUSE),
    Fuse(pKF, Scw, vpPoints, th, vpReplace) (M:1119-1249, FUSE_SIM3) and one
    direction of SearchBySim3 (M:1305-1387, SIM3_DIR: last_Tcw = the points'
    own keyframe pose, tgt Tcw = [sR|t], tgt fx..cy = pKF1's).  Returns
    (count, best) with best[i] = the target keypoint of point i when its
    distance is <= TH_LOW (Fuse) / TH_HIGH (SearchBySim3), else -1."""
    k = tgt["kps"]
    grid = Grid(tgt)
    uR = tgt.get("u_right")
    T = np.asarray(tgt["Tcw"], np.float32).reshape(4, 4)
    sf = [f32(s) for s in tgt["scale_factors"]]
    isig = [f32(f32(1.0) / f32(s * s)) for s in sf]  # mvInvLevelSigma2 = 1/(s*s)
    if variant == FUSE_SIM3:  # M:1129-1133
        scw = norm3(T[0, :3])
        P = np.zeros((4, 4), np.float32)
        P[:3, :3] = (T[:3, :3] / scw).astype(np.float32)
        P[:3, 3] = (T[:3, 3] / scw).astype(np.float32)
        O = camera_center(P)
    elif variant == FUSE:
        P, O = T, camera_center(T)  # pKF->GetCameraCenter()
    else:
        L = np.asarray(last_Tcw, np.float32).reshape(4, 4)
    limit = TH_HIGH if variant == SIM3_DIR else TH_LOW
    n = len(pts["flags"])
    best_out = np.full(n, -1, np.int32)
    for ip in range(n):
        if not int(pts["flags"][ip]) & VALID:
            continue
        X = pts["pos"][ip]
        if variant == SIM3_DIR:
            pc = transform(T, transform(L, X))  # sR21*(R1w*X + t1w) + t21
        else:
            pc = transform(P, X)
        if pc[2] < f32(0.0):
            continue
        invz = f32(f32(1) / pc[2])
        u = f32(f32(f32(tgt["fx"]) * f32(pc[0] * invz)) + f32(tgt["cx"]))
        v = f32(f32(f32(tgt["fy"]) * f32(pc[1] * invz)) + f32(tgt["cy"]))
        if not (u >= f32(tgt["min_x"]) and u < f32(tgt["max_x"]) and v >= f32(tgt["min_y"]) and
                v < f32(tgt["max_y"])):  # KeyFrame::IsInImage
            continue
        ur = f32(u - f32(f32(tgt["bf"]) * invz))
        maxd = f32(f32(1.2) * f32(pts["max_dist"][ip]))
        mind = f32(f32(0.8) * f32(pts["min_dist"][ip]))
        if variant == SIM3_DIR:
            dist = norm3(pc)  # cv::norm(p3Dc2)
        else:
            PO = [f32(f32(X[j]) - O[j]) for j in range(3)]
            dist = norm3(PO)
        if dist < mind or dist > maxd:
            continue
        if variant != SIM3_DIR:  # viewing angle < 60 deg
            Pn = pts["normal"][ip]
            dot = f64(PO[0]) * f64(Pn[0]) + f64(PO[1]) * f64(Pn[1]) + f64(PO[2]) * f64(Pn[2])
            if dot < 0.5 * f64(dist):
                continue
        lvl = predict_scale(pts["max_dist"][ip], dist, tgt)
        rad = f32(f32(th) * sf[lvl])
        cands = grid.area(u, v, rad)
        best, best_i = 1 << 30, -1
        for i in cands:
            o = int(k["octave"][i])
            if o < lvl - 1 or o > lvl:
                continue
            if variant == FUSE:  # M:1053-1078
                ex = f32(u - f32(k["x"][i]))
                ey = f32(v - f32(k["y"][i]))
                e2 = f32(f32(ex * ex) + f32(ey * ey))
                if uR is not None and f32(uR[i]) >= f32(0):
                    er = f32(ur - f32(uR[i]))
                    if f64(f32(f32(e2 + f32(er * er)) * isig[o & 15])) > 7.8:
                        continue
                elif f64(f32(e2 * isig[o & 15])) > 5.99:
                    continue
            d = _hamming(pts["desc"][ip], tgt["desc"][i])
            if d < best:
                best, best_i = d, i
        if best_i >= 0 and best <= limit:
            best_out[ip] = best_i
    return int((best_out >= 0).sum()), best_out


def search_by_sim3(kf1, kf2, pts1, pts2, s12, R12, t12, th):
    """ORBmatcher::SearchBySim3 (M:1253-1491): both directions + agreement.
    pts1/pts2 one entry per keypoint of kf1/kf2, VALID = non-NULL, !isBad,
    not already matched.  Returns (nfound, match12[n1]) = KF2 keypoint or -1."""
    R12 = np.asarray(R12, np.float32).reshape(3, 3)
    t12 = np.asarray(t12, np.float32).reshape(3)
    s12 = f32(s12)
    sR12 = np.array([[f32(f64(R12[i, j]) * f64(s12)) for j in range(3)] for i in range(3)], np.float32)
    inv = 1.0 / f64(s12)
    sR21 = np.array([[f32(f64(R12[j, i]) * inv) for j in range(3)] for i in range(3)], np.float32)
    t21 = np.array([-dotd3(sR21[i], t12) for i in range(3)], np.float32)
    S21, S12 = np.eye(4, dtype=np.float32), np.eye(4, dtype=np.float32)
    S21[:3, :3], S21[:3, 3] = sR21, t21
    S12[:3, :3], S12[:3, 3] = sR12, t12
    intr = {f: kf1[f] for f in ("fx", "fy", "cx", "cy")}
    _, m1 = radius_search(SIM3_DIR, dict(kf2, Tcw=S21, **intr), pts1, th, last_Tcw=kf1["Tcw"])
    _, m2 = radius_search(SIM3_DIR, dict(kf1, Tcw=S12, **intr), pts2, th, last_Tcw=kf2["Tcw"])
    out = np.full(len(kf1["kps"]), -1, np.int32)
    for i1, i2 in enumerate(m1):
        if i2 >= 0 and m2[i2] == i1:
            out[i1] = i2
    return int((out >= 0).sum()), out
