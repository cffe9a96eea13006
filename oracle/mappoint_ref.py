"""CPU restatement of MapPoint::ComputeDistinctiveDescriptors
(src/MapPoint.cpp:302-380) and MapPoint::UpdateNormalAndDepth (:414-457).

TEST INFRASTRUCTURE ONLY: the parity oracle for csrc/mappoint.hip (imported by
tests/ and nothing else).  Pure Python/numpy in the reference's order: the
distance matrix, a sorted copy of each row and vDists[0.5*(N-1)], the first
strict minimum; the normal as a float32 running sum of (Pos - Ow)/norm in map
order.  OpenCV conventions (not in the reference tree, restated): cv::norm of a
float vector is sqrt of a double sum of squares; `normal + normali/norm` is
cv::scaleAdd with the float scale (float)(1/norm) (product, then sum, in
float); `normal/n` is convertTo with the float scale (float)(1/n).  No
fixture exists for these members: parity unpinned against a reference run.
"""
from __future__ import annotations

import math

import numpy as np


def descriptor_distance(a, b):
    """ORBmatcher::DescriptorDistance (src/ORBmatcher.cpp:1838-1854)."""
    return int(np.unpackbits(np.bitwise_xor(np.asarray(a, np.uint8), np.asarray(b, np.uint8))).sum())


def compute_distinctive_descriptors(desc, valid=None):
    """One point: desc (n_obs, 32) in map order, valid = not pKF->isBad().
    Returns (index in the whole list or -1, best median or -1)."""
    idx = [o for o in range(len(desc)) if valid is None or valid[o]]
    N = len(idx)
    if N == 0:
        return -1, -1
    D = [[0] * N for _ in range(N)]
    for i in range(N):
        for j in range(i + 1, N):
            d = descriptor_distance(desc[idx[i]], desc[idx[j]])
            D[i][j] = D[j][i] = d
    best_median, best = 2 ** 31 - 1, 0
    for i in range(N):
        med = sorted(D[i])[int(0.5 * (N - 1))]
        if med < best_median:
            best_median, best = med, i
    return idx[best], best_median


def _norm(v):
    return math.sqrt((float(v[0]) * float(v[0]) + float(v[1]) * float(v[1])) + float(v[2]) * float(v[2]))


def update_normal_and_depth(obs_Ow, pos, ref_Ow, level_scale, max_scale):
    """One point with at least one observation.  Returns (normal, min_dist, max_dist)."""
    f32 = np.float32
    P = np.asarray(pos, f32)
    normal = np.zeros(3, f32)
    for Ow in obs_Ow:
        ni = P - np.asarray(Ow, f32)
        s = f32(1.0 / _norm(ni))
        normal = (ni * s).astype(f32) + normal
    inv_n = f32(1.0 / len(obs_Ow))
    normal = (normal * inv_n).astype(f32)
    PC = P - np.asarray(ref_Ow, f32)
    dist = f32(_norm(PC))
    dmax = f32(dist * f32(level_scale))
    dmin = f32(dmax / f32(max_scale))
    return normal, dmin, dmax
