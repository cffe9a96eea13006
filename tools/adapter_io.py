"""Input blobs of tests/cpp/adapter_main (the drop-in C++ classes driven the
way Tracking / Frame / LoopClosing call them) and per-frame-size scenarios.

Shared by tests/test_adapter.py (parity) and bench.py's drop_in section
(latency of the class calls).  The layouts are the ones adapter_main.cpp's
read_* functions expect: fixed field order, little-endian, no headers.
Nothing here computes a result: scenarios come from synth.py, FeatureVectors
and isInFrustum flags from the caller.
"""
from __future__ import annotations

import struct

import numpy as np

F32 = np.float32
KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])


def frame_blob(tgt, sigma2=None):
    """read_frame() layout of adapter_main.cpp"""
    k = np.ascontiguousarray(tgt["kps"])
    n = len(k)
    sf = np.asarray(tgt["scale_factors"], F32)
    s2 = np.asarray(sigma2 if sigma2 is not None else sf * sf, F32)
    ur = tgt.get("u_right")
    ur = np.full(n, -1, F32) if ur is None else np.asarray(ur, F32)
    g = np.array([tgt[f] for f in ("min_x", "max_x", "min_y", "max_y", "fx", "fy", "cx", "cy", "bf", "b")], F32)
    T = np.asarray(tgt["Tcw"], F32).reshape(4, 4)
    return b"".join([struct.pack("<i", n), k.tobytes(), np.ascontiguousarray(tgt["desc"], np.uint8).tobytes(),
                     ur.tobytes(), g.tobytes(), struct.pack("<if", len(sf), float(tgt["log_scale_factor"])),
                     sf.tobytes(), s2.tobytes(), T.tobytes()])


def points_blob(p):
    n = len(p["flags"])
    z = lambda k, w: np.zeros((n, w), F32) if p.get(k) is None else np.asarray(p[k], F32).reshape(n, w)  # noqa: E731
    lvl = np.zeros(n, np.int32) if p.get("track_level") is None else np.asarray(p["track_level"], np.int32)
    return b"".join([struct.pack("<i", n), np.asarray(p["flags"], np.int32).tobytes(), z("pos", 3).tobytes(),
                     z("normal", 3).tobytes(), np.ascontiguousarray(p["desc"], np.uint8).tobytes(),
                     z("min_dist", 1).tobytes(), z("max_dist", 1).tobytes(), z("track", 4).tobytes(), lvl.tobytes()])


def proj_blob(th, kw, tgt, pts, last_Tcw):
    """run_proj input: options, LastFrame pose, target frame + occupancy, points"""
    return b"".join([struct.pack("<ffiii", th, kw.get("nnratio", 0.6), int(kw.get("check_ori", True)),
                                 int(kw.get("orb_dist", 50)), int(kw.get("mono", True))),
                     np.asarray(last_Tcw, F32).tobytes(), frame_blob(tgt),
                     np.asarray(tgt["occupied"], np.uint8).tobytes(), points_blob(pts),
                     np.asarray(pts["octave"], np.int32).tobytes(), np.asarray(pts["angle"], F32).tobytes()])


def bow_frame_blob(desc, angle, mp_state, fv):
    nodes = np.array(sorted(fv), np.int32)
    offs = np.zeros(len(nodes) + 1, np.int32)
    feats = []
    for i, k in enumerate(nodes):
        feats += list(fv[int(k)])
        offs[i + 1] = len(feats)
    return b"".join([struct.pack("<i", len(desc)), np.ascontiguousarray(desc, np.uint8).tobytes(),
                     np.asarray(angle, F32).tobytes(), np.asarray(mp_state, np.uint8).tobytes(),
                     struct.pack("<i", len(nodes)), nodes.tobytes(), offs.tobytes(),
                     np.array(feats, np.int32).tobytes()])


def bow_blob(nnratio, check_ori, A, B):
    """run_bow input: A, B = (desc, angle, mp_state, fv)"""
    return struct.pack("<fi", nnratio, int(check_ori)) + bow_frame_blob(*A) + bow_frame_blob(*B)


def pnp_frame(P, extra=25, seed=0):
    """A Frame for PnPsolver built from synth.pnp_problem P: the n
    correspondences at random slots, plus keypoints without a MapPoint (0) and
    with a bad one (2).  Returns (blob tail after the seed, slots, state)."""
    n = len(P["P2"])
    table = (F32(1.2) ** (2 * np.arange(8))).astype(F32)
    octv = np.array([int(np.nonzero(table == s)[0][0]) for s in P["sigma2"]], np.int32)
    rng = np.random.default_rng(seed)
    N = n + extra
    slots = np.sort(rng.choice(N, n, replace=False))
    state = np.zeros(N, np.uint8)
    state[slots] = 1
    rest = np.setdiff1d(np.arange(N), slots)
    state[rest[: extra // 2]] = 2
    kps = np.zeros(N, KP_DTYPE)
    kps["x"][slots], kps["y"][slots] = P["P2"][:, 0], P["P2"][:, 1]
    kps["octave"][slots] = octv
    kps["x"][rest], kps["y"][rest] = 100.0, 100.0
    pos = np.zeros((N, 3), F32)
    pos[slots] = P["P3w"]
    pos[rest] = rng.uniform(-1, 1, (len(rest), 3)).astype(F32)
    fu, fv, uc, vc = P["cam"]
    tgt = {"kps": kps, "desc": np.zeros((N, 32), np.uint8), "min_x": 0, "max_x": 640, "min_y": 0, "max_y": 480,
           "fx": fu, "fy": fv, "cx": uc, "cy": vc, "bf": 0, "b": 0, "log_scale_factor": float(np.log(F32(1.2))),
           "scale_factors": np.sqrt(table).astype(F32), "Tcw": np.eye(4, dtype=F32)}
    return frame_blob(tgt, sigma2=table) + state.tobytes() + pos.tobytes(), slots, state


def init_blob(K, kp1, kp2, m12):
    K = np.asarray(K, F32)
    return b"".join([K.tobytes(), struct.pack("<i", len(kp1)), np.asarray(kp1, F32).tobytes(),
                     struct.pack("<i", len(kp2)), np.asarray(kp2, F32).tobytes(), np.asarray(m12, np.int32).tobytes()])


K_TUM = np.array([[517.3, 0, 318.6], [0, 516.5, 255.3], [0, 0, 1]], np.float64)


def init_scene(n=1000, seed=3, outliers=0.2, noise=0.7):
    """Two views of n general 3-D points for Initializer::Initialize at the
    size Tracking::MonocularInitialization sees (>= 100 matches of a
    2x-feature initialisation extractor): keypoints of both views (with
    extra unmatched ones) and vMatches12."""
    rng = np.random.default_rng(seed)
    X = np.c_[rng.uniform(-2, 2, n), rng.uniform(-1.5, 1.5, n), rng.uniform(3, 8, n)]
    a = 0.05
    R = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]])
    t = np.array([0.3, 0.02, 0.05])
    x1 = (K_TUM @ X.T).T
    x2 = (K_TUM @ (R @ X.T + t[:, None])).T
    p1 = x1[:, :2] / x1[:, 2:] + rng.normal(scale=noise, size=(n, 2))
    p2 = x2[:, :2] / x2[:, 2:] + rng.normal(scale=noise, size=(n, 2))
    bad = rng.uniform(size=n) < outliers
    p2[bad] = rng.uniform([0, 0], [640, 480], size=(int(bad.sum()), 2))
    n1, n2 = n + 200, n + 150
    kp1 = rng.uniform([0, 0], [640, 480], size=(n1, 2)).astype(F32)
    kp2 = rng.uniform([0, 0], [640, 480], size=(n2, 2)).astype(F32)
    s1 = rng.choice(n1, n, replace=False)
    s2 = rng.choice(n2, n, replace=False)
    kp1[s1] = p1
    kp2[s2] = p2
    m12 = np.full(n1, -1, np.int32)
    m12[s1] = s2
    return kp1, kp2, m12
