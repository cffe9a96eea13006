"""Host-side mirror of the projection matchers over include/orbgpu_proj.h:
``is_in_frustum`` (Frame::isInFrustum), ``search_by_projection`` (the four
ORBmatcher::SearchByProjection overloads), ``radius_search`` (the per-point
searches of ORBmatcher::Fuse, both overloads, and of one SearchBySim3
direction) and ``search_by_sim3`` (ORBmatcher::SearchBySim3)."""
from __future__ import annotations

import ctypes

import numpy as np

import orbgpu

LOCAL, SIM3, LAST_FRAME, KEYFRAME = 0, 1, 2, 3
FUSE, FUSE_SIM3, SIM3_DIR = 4, 5, 6
VALID, HAS_OBS, IN_VIEW = 1, 2, 4
vp = ctypes.c_void_p


class Target(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("kps", vp), ("desc", vp), ("u_right", vp), ("occupied", vp),
                ("min_x", ctypes.c_float), ("max_x", ctypes.c_float), ("min_y", ctypes.c_float),
                ("max_y", ctypes.c_float), ("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float),
                ("cy", ctypes.c_float), ("bf", ctypes.c_float), ("b", ctypes.c_float), ("n_levels", ctypes.c_int),
                ("log_scale_factor", ctypes.c_float), ("scale_factors", ctypes.c_float * 16),
                ("Tcw", ctypes.c_float * 16)]


class Points(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("flags", vp), ("pos", vp), ("normal", vp), ("desc", vp), ("min_dist", vp),
                ("max_dist", vp), ("octave", vp), ("angle", vp), ("track", vp), ("track_level", vp)]


class Call(ctypes.Structure):
    _fields_ = [("variant", ctypes.c_int), ("check_ori", ctypes.c_int), ("nnratio", ctypes.c_float),
                ("th", ctypes.c_float), ("orb_dist", ctypes.c_int), ("mono", ctypes.c_int),
                ("last_Tcw", ctypes.c_float * 16), ("target", Target), ("points", Points)]


def _arr(a, dtype, keep):
    if a is None:
        return None
    a = np.ascontiguousarray(a, dtype)
    keep.append(a)
    return a.ctypes.data


def _target(t, keep):
    T = Target()
    k = np.ascontiguousarray(t["kps"], orbgpu.KP_DTYPE)
    keep.append(k)
    T.n = len(k)
    T.kps = k.ctypes.data
    T.desc = _arr(t["desc"], np.uint8, keep)
    T.u_right = _arr(t.get("u_right"), np.float32, keep)
    T.occupied = _arr(t.get("occupied"), np.uint8, keep)
    for f in ("min_x", "max_x", "min_y", "max_y", "fx", "fy", "cx", "cy", "bf", "b", "log_scale_factor"):
        setattr(T, f, float(t[f]))
    T.n_levels = int(t["n_levels"])
    T.scale_factors[:len(t["scale_factors"])] = [float(s) for s in t["scale_factors"]]
    T.Tcw[:] = [float(v) for v in np.asarray(t["Tcw"], np.float32).reshape(16)]
    return T


def _points(p, keep):
    P = Points()
    P.n = len(p["flags"])
    P.flags = _arr(p["flags"], np.int32, keep)
    P.pos = _arr(p.get("pos"), np.float32, keep)
    P.normal = _arr(p.get("normal"), np.float32, keep)
    P.desc = _arr(p["desc"], np.uint8, keep)
    P.min_dist = _arr(p.get("min_dist"), np.float32, keep)
    P.max_dist = _arr(p.get("max_dist"), np.float32, keep)
    P.octave = _arr(p.get("octave"), np.int32, keep)
    P.angle = _arr(p.get("angle"), np.float32, keep)
    P.track = _arr(p.get("track"), np.float32, keep)
    P.track_level = _arr(p.get("track_level"), np.int32, keep)
    return P


def search_by_projection(variant, tgt, pts, th, nnratio=0.6, check_ori=True, orb_dist=50, mono=True,
                         last_Tcw=None):
    """Returns (nmatches, match[n]) -- see orbgpu_proj.h for the encoding."""
    keep = []
    C = Call()
    C.variant, C.check_ori, C.nnratio, C.th, C.orb_dist, C.mono = variant, int(check_ori), nnratio, th, orb_dist, int(mono)
    if last_Tcw is not None:
        C.last_Tcw[:] = [float(v) for v in np.asarray(last_Tcw, np.float32).reshape(16)]
    C.target = _target(tgt, keep)
    C.points = _points(pts, keep)
    n = C.points.n if variant >= FUSE else C.target.n  # per-point variants: one entry per point
    match = np.zeros(max(n, 1), np.int32)
    nm = ctypes.c_int()
    orbgpu._check(orbgpu.lib().orbgpu_search_by_projection(ctypes.byref(C), match.ctypes.data, ctypes.byref(nm)),
                  "orbgpu_search_by_projection")
    return nm.value, match[:n]


def radius_search(variant, tgt, pts, th, last_Tcw=None):
    """FUSE / FUSE_SIM3 / SIM3_DIR: (count, best keypoint per point or -1)."""
    return search_by_projection(variant, tgt, pts, th, last_Tcw=last_Tcw)


class Sim3Search(ctypes.Structure):
    _fields_ = [("kf1", Target), ("kf2", Target), ("pts1", Points), ("pts2", Points), ("s12", ctypes.c_float),
                ("R12", ctypes.c_float * 9), ("t12", ctypes.c_float * 3), ("th", ctypes.c_float)]


def search_by_sim3(kf1, kf2, pts1, pts2, s12, R12, t12, th):
    """ORBmatcher::SearchBySim3: (nfound, match12[n1] = KF2 keypoint or -1)."""
    keep = []
    S = Sim3Search()
    S.kf1, S.kf2 = _target(kf1, keep), _target(kf2, keep)
    S.pts1, S.pts2 = _points(pts1, keep), _points(pts2, keep)
    S.s12, S.th = float(s12), float(th)
    S.R12[:] = [float(v) for v in np.asarray(R12, np.float32).reshape(9)]
    S.t12[:] = [float(v) for v in np.asarray(t12, np.float32).reshape(3)]
    n1 = S.kf1.n
    match = np.zeros(max(n1, 1), np.int32)
    nf = ctypes.c_int()
    orbgpu._check(orbgpu.lib().orbgpu_search_by_sim3(ctypes.byref(S), match.ctypes.data, ctypes.byref(nf)),
                  "orbgpu_search_by_sim3")
    return nf.value, match[:n1]


def is_in_frustum(tgt, pts, cos_limit):
    """Frame::isInFrustum on the GPU for every point: (flags, track, level)."""
    import torch
    keep = []
    T = _target(tgt, keep)
    n = len(pts["flags"])
    dev = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dt)).cuda()
    pos, nrm = dev(pts["pos"], np.float32), dev(pts["normal"], np.float32)
    mind, maxd = dev(pts["min_dist"], np.float32), dev(pts["max_dist"], np.float32)
    flags = dev(pts["flags"], np.int32)
    track = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
    level = torch.zeros(n, dtype=torch.int32, device="cuda")
    orbgpu._check(orbgpu.lib().orbgpu_is_in_frustum_device(ctypes.byref(T), n, pos.data_ptr(), nrm.data_ptr(),
                                                          mind.data_ptr(), maxd.data_ptr(), float(cos_limit),
                                                          flags.data_ptr(), track.data_ptr(), level.data_ptr(), None),
                  "orbgpu_is_in_frustum_device")
    torch.cuda.synchronize()
    return flags.cpu().numpy(), track.cpu().numpy(), level.cpu().numpy()
