"""Host-side mirror of include/orbgpu_mapping.h: LocalMapping::
CreateNewMapPoints' per-match triangulation (src/LocalMapping.cpp:369-515)."""
from __future__ import annotations

import ctypes

import numpy as np

import orbgpu

vp, f = ctypes.c_void_p, ctypes.c_float


class KF(ctypes.Structure):
    _fields_ = [("Tcw", f * 12), ("Ow", f * 3), ("fx", f), ("fy", f), ("cx", f), ("cy", f), ("invfx", f),
                ("invfy", f), ("bf", f), ("b", f), ("n", ctypes.c_int), ("kps_un", vp), ("kps", vp), ("u_right", vp),
                ("depth", vp), ("scale_factors", f * 16), ("level_sigma2", f * 16)]


class Job(ctypes.Structure):
    _fields_ = [("kf1", KF), ("kf2", KF), ("scale_factor", f), ("n", ctypes.c_int), ("pairs", vp), ("x3d", vp),
                ("ok", vp)]


def _kf(d, keep):
    K = KF()
    K.Tcw[:] = [float(x) for x in np.asarray(d["Tcw"], np.float32).reshape(12)]
    K.Ow[:] = [float(x) for x in np.asarray(d["Ow"], np.float32).reshape(3)]
    for name in ("fx", "fy", "cx", "cy", "invfx", "invfy", "bf", "b"):
        setattr(K, name, float(d[name]))
    ku = np.ascontiguousarray(d["kps_un"], orbgpu.KP_DTYPE)
    kr = np.ascontiguousarray(d["kps"], orbgpu.KP_DTYPE)
    keep += [ku, kr]
    K.n, K.kps_un, K.kps = len(ku), ku.ctypes.data, kr.ctypes.data
    for name in ("u_right", "depth"):
        if d.get(name) is not None:
            a = np.ascontiguousarray(d[name], np.float32)
            keep.append(a)
            setattr(K, name, a.ctypes.data)
    K.scale_factors[:len(d["scale_factors"])] = [float(x) for x in d["scale_factors"]]
    K.level_sigma2[:len(d["level_sigma2"])] = [float(x) for x in d["level_sigma2"]]
    return K


def triangulate_matches(kf1, kf2, pairs, scale_factor):
    """(x3d (n, 3) float32, ok (n,) bool) for the matched pairs (idx1, idx2)."""
    keep = []
    J = Job()
    J.kf1, J.kf2 = _kf(kf1, keep), _kf(kf2, keep)
    p = np.ascontiguousarray(np.asarray(pairs, np.int32).reshape(-1, 2))
    n = len(p)
    x3d = np.zeros((max(n, 1), 3), np.float32)
    ok = np.zeros(max(n, 1), np.uint8)
    J.scale_factor, J.n, J.pairs, J.x3d, J.ok = float(scale_factor), n, p.ctypes.data, x3d.ctypes.data, ok.ctypes.data
    L = orbgpu.lib()
    L.orbgpu_triangulate_matches.argtypes = [vp]
    orbgpu._check(L.orbgpu_triangulate_matches(ctypes.byref(J)), "orbgpu_triangulate_matches")
    return x3d[:n], ok[:n].astype(bool)
