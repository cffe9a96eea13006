"""Host-side mirror of the monocular Initializer's model scoring over the C
ABI in include/orbgpu_init.h (csrc/init.hip).

* ``check_homography_batch`` -- Initializer::CheckHomography
  (src/Initializer.cpp:390-495) for every RANSAC iteration's (H21, H12) at
  once: scores (nhyp,) float32 and inlier flags (nhyp, n) uint8.
* ``check_fundamental_batch`` -- Initializer::CheckFundamental (:497-594).
* ``check_both_batch`` -- both of the above in one launch.
* ``select_best`` -- FindHomography / FindFundamental's kept iteration
  (:207-212, :264-269): first strict maximum above 0, or -1.
* ``find_models`` -- Initialize up to the model choice (hypotheses + scores).
* ``reconstruct`` -- ReconstructH / ReconstructF (:596-963): motion
  hypotheses, CheckRT of each over the inliers on the GPU, the choice.

Inputs are device tensors (torch, on the GPU); the matches are
(u1, v1, u2, v2) = (mvKeys1[first].pt, mvKeys2[second].pt) rows.
"""
from __future__ import annotations

import ctypes

import numpy as np

import orbgpu

_BOUND = False


def _lib():
    global _BOUND
    L = orbgpu.lib()
    if not _BOUND:
        vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        L.orbgpu_init_check_homography_batch_device.argtypes = [vp, i, vp, vp, i, f, vp, vp, vp]
        L.orbgpu_init_check_fundamental_batch_device.argtypes = [vp, i, vp, i, f, vp, vp, vp]
        L.orbgpu_init_check_both_batch_device.argtypes = [vp, i, vp, vp, i, vp, i, f, vp, vp, vp, vp, vp]
        L.orbgpu_init_select_best.argtypes = [vp, i, ctypes.POINTER(ctypes.c_int)]
        _BOUND = True
    return L


def _stream(stream):
    return None if stream is None else getattr(stream, "cuda_stream", stream)


def _shapes(pts, mats, scores, inliers):
    import torch
    want = ((pts, torch.float32, "pts"), (mats, torch.float32, "matrices"), (scores, torch.float32, "scores"),
            (inliers, torch.uint8, "inliers"))
    for t, dt, name in want:
        if not (isinstance(t, torch.Tensor) and t.is_cuda):
            raise TypeError(f"{name} must be a torch tensor on the GPU (a host pointer would fault the kernel)")
        if t.dtype != dt:
            raise TypeError(f"{name} must be {dt}, got {t.dtype}")
        if t.device != pts.device:
            raise ValueError(f"{name} is on {t.device}, pts on {pts.device}")
    if pts.data_ptr() % 16:
        raise ValueError("pts must be 16-byte aligned (the kernel loads float4 rows)")
    n, nhyp = pts.shape[0], mats.shape[0]
    if pts.ndim != 2 or pts.shape[1] != 4 or mats.reshape(nhyp, -1).shape[1] != 9:
        raise ValueError("pts must be (n, 4) and matrices (nhyp, 3, 3)")
    if tuple(scores.shape) != (nhyp,) or tuple(inliers.shape) != (nhyp, n):
        raise ValueError("scores must be (nhyp,) and inliers (nhyp, n)")
    for t in (pts, mats, scores, inliers):
        if hasattr(t, "is_contiguous") and not t.is_contiguous():
            raise ValueError("tensors must be contiguous")
    return n, nhyp


def _same(a, ref):
    if a.dtype != ref.dtype or a.device != ref.device or not a.is_contiguous():
        raise TypeError("H12 must be a contiguous float32 GPU tensor on H21's device")


def check_homography_batch(pts, H21, H12, sigma, scores, inliers, stream=None):
    n, nhyp = _shapes(pts, H21, scores, inliers)
    if tuple(H12.shape) != tuple(H21.shape):
        raise ValueError("H12 must match H21")
    _same(H12, H21)
    orbgpu._check(_lib().orbgpu_init_check_homography_batch_device(
        orbgpu._ptr(pts), n, orbgpu._ptr(H21), orbgpu._ptr(H12), nhyp, float(sigma), orbgpu._ptr(scores),
        orbgpu._ptr(inliers), _stream(stream)), "init_check_homography_batch_device")


def check_fundamental_batch(pts, F21, sigma, scores, inliers, stream=None):
    n, nhyp = _shapes(pts, F21, scores, inliers)
    orbgpu._check(_lib().orbgpu_init_check_fundamental_batch_device(
        orbgpu._ptr(pts), n, orbgpu._ptr(F21), nhyp, float(sigma), orbgpu._ptr(scores), orbgpu._ptr(inliers),
        _stream(stream)), "init_check_fundamental_batch_device")


def check_both_batch(pts, H21, H12, F21, sigma, scores_h, inliers_h, scores_f, inliers_f, stream=None):
    """both searches' hypotheses in one launch (Initialize runs them in two
    threads, src/Initializer.cpp:133-138)"""
    n, nh = _shapes(pts, H21, scores_h, inliers_h)
    _, nf = _shapes(pts, F21, scores_f, inliers_f)
    if tuple(H12.shape) != tuple(H21.shape):
        raise ValueError("H12 must match H21")
    _same(H12, H21)
    orbgpu._check(_lib().orbgpu_init_check_both_batch_device(
        orbgpu._ptr(pts), n, orbgpu._ptr(H21), orbgpu._ptr(H12), nh, orbgpu._ptr(F21), nf, float(sigma),
        orbgpu._ptr(scores_h), orbgpu._ptr(inliers_h), orbgpu._ptr(scores_f), orbgpu._ptr(inliers_f),
        _stream(stream)), "init_check_both_batch_device")


def select_best(scores) -> int:
    s = np.ascontiguousarray(np.asarray(scores, dtype=np.float32))
    out = ctypes.c_int(-1)
    orbgpu._check(_lib().orbgpu_init_select_best(s.ctypes.data, s.shape[0], ctypes.byref(out)), "init_select_best")
    return out.value


# ---- model hypotheses (Initialize / FindHomography / FindFundamental) -----
def seed_rand_once(seed: int = 0) -> None:
    """DUtils::Random::SeedRandOnce(seed) on the orbgpu_rand stream."""
    _lib2().orbgpu_seed_rand_once(seed & 0x7FFFFFFF)


def draw_sets(n_matches: int, n_iter: int = 200) -> np.ndarray:
    """Initialize's minimal sets (Initializer.cpp:96-115) from the orbgpu_rand stream."""
    sets = np.zeros((n_iter, 8), np.int32)
    orbgpu._check(_lib2().orbgpu_init_draw_sets(n_matches, n_iter, sets.ctypes.data), "orbgpu_init_draw_sets")
    return sets


_BOUND2 = False


def _lib2():
    global _BOUND2
    L = _lib()
    if not _BOUND2:
        vp, i = ctypes.c_void_p, ctypes.c_int
        L.orbgpu_seed_rand_once.argtypes = [ctypes.c_uint]
        L.orbgpu_init_draw_sets.argtypes = [i, i, vp]
        L.orbgpu_init_workspace_bytes.argtypes = [i, i]
        L.orbgpu_init_workspace_bytes.restype = ctypes.c_size_t
        L.orbgpu_init_hypotheses_batch_device.argtypes = [vp, i, vp, i, vp, i, vp, i, vp, vp, vp, vp, vp, vp]
        _BOUND2 = True
    return L


def find_models(kp1, kp2, matches12, sigma=1.0, n_iter=200, sets=None, device="cuda", stream=None):
    """Initializer::Initialize up to the model choice (Initializer.cpp:55-140):
    mvMatches12 from matches12 (vector<int>), Normalize, the n_iter minimal
    sets (drawn from the orbgpu_rand stream unless given), every H21/H12/F21
    hypothesis and its CheckHomography / CheckFundamental score on the GPU,
    the kept iterations and RH = SH / (SH + SF).  kp1, kp2: (n, 2) keypoint
    positions (mvKeys1 / mvKeysUn of the current frame)."""
    import torch
    m12 = np.asarray(matches12)
    first = np.nonzero(m12 >= 0)[0]
    pairs = np.stack([first, m12[first]], 1).astype(np.int32)
    nm = len(pairs)
    if sets is None:
        sets = draw_sets(nm, n_iter)
    sets = np.ascontiguousarray(sets, np.int32)
    n_iter = len(sets)
    dev = torch.device(device)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dt)).to(dev)  # noqa: E731
    d_kp1, d_kp2 = t(np.asarray(kp1).reshape(-1, 2), np.float32), t(np.asarray(kp2).reshape(-1, 2), np.float32)
    d_pairs, d_sets = t(pairs, np.int32), t(sets, np.int32)
    work = torch.zeros(_lib2().orbgpu_init_workspace_bytes(len(d_kp1), len(d_kp2)), dtype=torch.uint8, device=dev)
    pts = torch.zeros((nm, 4), dtype=torch.float32, device=dev)
    h21 = torch.zeros((n_iter, 3, 3), dtype=torch.float32, device=dev)
    h12, f21 = torch.zeros_like(h21), torch.zeros_like(h21)
    orbgpu._check(_lib2().orbgpu_init_hypotheses_batch_device(
        d_kp1.data_ptr(), len(d_kp1), d_kp2.data_ptr(), len(d_kp2), d_pairs.data_ptr(), nm, d_sets.data_ptr(), n_iter,
        work.data_ptr(), pts.data_ptr(), h21.data_ptr(), h12.data_ptr(), f21.data_ptr(), _stream(stream)),
        "orbgpu_init_hypotheses_batch_device")
    sh, sf = torch.zeros(n_iter, device=dev), torch.zeros(n_iter, device=dev)
    ih = torch.zeros((n_iter, nm), dtype=torch.uint8, device=dev)
    jf = torch.zeros((n_iter, nm), dtype=torch.uint8, device=dev)
    check_both_batch(pts, h21, h12, f21, sigma, sh, ih, sf, jf, stream)
    if stream is not None:
        stream.synchronize()
    else:
        torch.cuda.synchronize(dev)
    shn, sfn = sh.cpu().numpy(), sf.cpu().numpy()
    bh, bf = select_best(shn), select_best(sfn)
    SH = np.float32(shn[bh]) if bh >= 0 else np.float32(0)
    SF = np.float32(sfn[bf]) if bf >= 0 else np.float32(0)
    return {"pairs": pairs, "sets": sets, "H21": h21.cpu().numpy(), "H12": h12.cpu().numpy(), "F21": f21.cpu().numpy(),
            "scores_h": shn, "scores_f": sfn, "best_h": bh, "best_f": bf,
            "inliers_h": ih[bh].cpu().numpy().astype(bool) if bh >= 0 else np.zeros(nm, bool),
            "inliers_f": jf[bf].cpu().numpy().astype(bool) if bf >= 0 else np.zeros(nm, bool),
            "RH": np.float32(SH / np.float32(SH + SF)) if SH + SF > 0 else np.float32(0)}


class Reconstruction(ctypes.Structure):
    _fields_ = [("ok", ctypes.c_int), ("best", ctypes.c_int), ("n_hyp", ctypes.c_int),
                ("n_good", ctypes.c_int * 8), ("parallax", ctypes.c_float * 8), ("R21", ctypes.c_float * 9),
                ("t21", ctypes.c_float * 3)]


MODEL_H, MODEL_F = 0, 1


def reconstruct(model, kp1, kp2, matches12, inliers, M21, K, sigma=1.0, min_parallax=1.0, min_triangulated=50):
    """Initializer::ReconstructH (model 0, M21 = H21) / ReconstructF (model 1,
    M21 = F21).  kp1, kp2: (n, 2) keypoint positions; matches12: vector<int>
    (mvMatches12 = the (i, m[i]) with m[i] >= 0); inliers: vbMatchesInliers
    over those pairs.  Returns a dict: ok, best, n_good, parallax, R21, t21,
    p3d (n1, 3), triangulated (n1)."""
    L = _lib()
    L.orbgpu_init_reconstruct.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float, ctypes.c_float,
                                          ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    m12 = np.asarray(matches12)
    first = np.nonzero(m12 >= 0)[0]
    pairs = np.ascontiguousarray(np.stack([first, m12[first]], 1), np.int32)
    k1 = np.ascontiguousarray(np.asarray(kp1, np.float32).reshape(-1, 2))
    k2 = np.ascontiguousarray(np.asarray(kp2, np.float32).reshape(-1, 2))
    inl = np.ascontiguousarray(np.asarray(inliers).astype(np.uint8))
    if len(inl) != len(pairs):
        raise ValueError("inliers must hold one flag per match")
    M = np.ascontiguousarray(np.asarray(M21, np.float32).reshape(9))
    Km = np.ascontiguousarray(np.asarray(K, np.float32).reshape(9))
    out = Reconstruction()
    p3d = np.zeros((max(len(k1), 1), 3), np.float32)
    tri = np.zeros(max(len(k1), 1), np.uint8)
    orbgpu._check(L.orbgpu_init_reconstruct(int(model), k1.ctypes.data, len(k1), k2.ctypes.data, len(k2),
                                            pairs.ctypes.data, len(pairs), inl.ctypes.data, M.ctypes.data,
                                            Km.ctypes.data, float(sigma), float(min_parallax),
                                            int(min_triangulated), ctypes.byref(out), p3d.ctypes.data,
                                            tri.ctypes.data), "orbgpu_init_reconstruct")
    nh = out.n_hyp
    return {"ok": bool(out.ok), "best": out.best, "n_good": list(out.n_good[:nh]),
            "parallax": np.array(out.parallax[:nh], np.float32),
            "R21": np.array(out.R21, np.float32).reshape(3, 3), "t21": np.array(out.t21, np.float32),
            "p3d": p3d[:len(k1)], "triangulated": tri[:len(k1)].astype(bool)}


def initialize(kp1, kp2, matches12, K, sigma=1.0, iterations=200):
    """Initializer(ReferenceFrame, sigma, iterations).Initialize(CurrentFrame,
    vMatches12, ...) (Initializer.cpp:55-157) in one call: draws from the
    orbgpu_rand stream after SeedRandOnce(0), hypotheses + scores + the
    reconstruction on the GPU.  Returns a dict: ok, model (0 H / 1 F), RH,
    R21, t21, p3d (n1, 3), triangulated (n1), n_good, parallax."""
    L = _lib()
    vp = ctypes.c_void_p
    L.orbgpu_init_initialize.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, vp, vp, ctypes.c_float, ctypes.c_int,
                                         vp, vp, vp, vp, vp]
    k1 = np.ascontiguousarray(np.asarray(kp1, np.float32).reshape(-1, 2))
    k2 = np.ascontiguousarray(np.asarray(kp2, np.float32).reshape(-1, 2))
    m12 = np.ascontiguousarray(np.asarray(matches12, np.int32))
    Km = np.ascontiguousarray(np.asarray(K, np.float32).reshape(9))
    out = Reconstruction()
    rh = ctypes.c_float()
    model = ctypes.c_int()
    p3d = np.zeros((max(len(k1), 1), 3), np.float32)
    tri = np.zeros(max(len(k1), 1), np.uint8)
    orbgpu._check(L.orbgpu_init_initialize(k1.ctypes.data, len(k1), k2.ctypes.data, len(k2), m12.ctypes.data,
                                           Km.ctypes.data, float(sigma), int(iterations), ctypes.byref(out),
                                           ctypes.byref(rh), ctypes.byref(model), p3d.ctypes.data, tri.ctypes.data),
                  "orbgpu_init_initialize")
    nh = out.n_hyp
    return {"ok": bool(out.ok), "model": model.value, "RH": np.float32(rh.value),
            "R21": np.array(out.R21, np.float32).reshape(3, 3), "t21": np.array(out.t21, np.float32),
            "p3d": p3d[:len(k1)], "triangulated": tri[:len(k1)].astype(bool), "n_good": list(out.n_good[:nh]),
            "parallax": np.array(out.parallax[:nh], np.float32)}
