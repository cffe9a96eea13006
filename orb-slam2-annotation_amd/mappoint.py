"""Host-side mirror of include/orbgpu_mappoint.h: MapPoint::
ComputeDistinctiveDescriptors (src/MapPoint.cpp:302-380) and
MapPoint::UpdateNormalAndDepth (:414-457) over batches of points, the
observations of point p being offsets[p] .. offsets[p+1]-1 in map order."""
from __future__ import annotations

import ctypes

import numpy as np

import orbgpu

vp = ctypes.c_void_p


class NormalDepthBatch(ctypes.Structure):
    _fields_ = [("n_points", ctypes.c_int), ("obs_offsets", vp), ("obs_Ow", vp), ("pos", vp), ("ref_Ow", vp),
                ("ref_level_scale", vp), ("ref_max_scale", vp), ("normal", vp), ("min_dist", vp), ("max_dist", vp)]


def _lib():
    L = orbgpu.lib()
    L.orbgpu_compute_distinctive_descriptors.argtypes = [ctypes.c_int, vp, vp, vp, vp, vp]
    L.orbgpu_update_normal_and_depth.argtypes = [vp]
    return L


def compute_distinctive_descriptors(offsets, desc, valid=None):
    """-> (best, median): per point the observation whose descriptor becomes
    mDescriptor (-1: none valid) and its median distance (-1)."""
    off = np.ascontiguousarray(offsets, np.int32)
    n = len(off) - 1
    d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    v = None if valid is None else np.ascontiguousarray(valid, np.uint8)
    best = np.zeros(max(n, 0), np.int32)
    med = np.zeros(max(n, 0), np.int32)
    orbgpu._check(_lib().orbgpu_compute_distinctive_descriptors(
        n, off.ctypes.data, d.ctypes.data if len(d) else None, None if v is None else v.ctypes.data,
        best.ctypes.data, med.ctypes.data), "orbgpu_compute_distinctive_descriptors")
    return best, med


def update_normal_and_depth(offsets, obs_Ow, pos, ref_Ow, ref_level_scale, ref_max_scale, normal=None,
                            min_dist=None, max_dist=None):
    """-> (normal (n, 3), min_dist (n,), max_dist (n,)); points without
    observations keep the values passed in (zeros by default)."""
    off = np.ascontiguousarray(offsets, np.int32)
    n = len(off) - 1
    arrs = [np.ascontiguousarray(a, np.float32) for a in (obs_Ow, pos, ref_Ow, ref_level_scale, ref_max_scale)]
    nrm = np.zeros((n, 3), np.float32) if normal is None else np.array(normal, np.float32).reshape(n, 3)
    dmin = np.zeros(n, np.float32) if min_dist is None else np.array(min_dist, np.float32)
    dmax = np.zeros(n, np.float32) if max_dist is None else np.array(max_dist, np.float32)
    b = NormalDepthBatch(n, off.ctypes.data, *(a.ctypes.data if a.size else None for a in arrs),
                         nrm.ctypes.data, dmin.ctypes.data, dmax.ctypes.data)
    orbgpu._check(_lib().orbgpu_update_normal_and_depth(ctypes.byref(b)), "orbgpu_update_normal_and_depth")
    return nrm, dmin, dmax
