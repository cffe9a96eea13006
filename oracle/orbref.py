"""ctypes binding of the CPU parity oracle (liborbref.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product.  Parity status: see
orbref.h (unpinned vs OpenCV 2.4; glibc sinf/cosf pinned exhaustively).
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB = None


class KeyPoint(ctypes.Structure):
    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("size", ctypes.c_float),
                ("angle", ctypes.c_float), ("response", ctypes.c_float),
                ("octave", ctypes.c_int32), ("class_id", ctypes.c_int32)]


KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        path = _HERE / "liborbref.so"
        if not path.exists():
            raise RuntimeError(f"oracle not built: {path} (run make -C oracle)")
        L = ctypes.CDLL(str(path))
        vp, i, f, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
        L.orbref_create.restype = vp
        L.orbref_create.argtypes = [i, f, i, i, i]
        L.orbref_destroy.argtypes = [vp]
        L.orbref_extract.restype = i
        L.orbref_extract.argtypes = [vp, vp, i, i, sz, vp, vp, i]
        L.orbref_level_size.argtypes = [vp, i, ctypes.POINTER(i), ctypes.POINTER(i)]
        L.orbref_level_copy.argtypes = [vp, i, vp]
        L.orbref_level_candidates.argtypes = [vp, i, vp, i]
        L.orbref_level_octree.argtypes = [vp, i, vp, i]
        L.orbref_features_per_level.argtypes = [vp, vp]
        L.orbref_scale_factors.argtypes = [vp, vp, vp, vp, vp]
        L.orbref_resize_linear_u8.argtypes = [vp, i, i, sz, vp, i, i, sz]
        L.orbref_gaussian7_u8.argtypes = [vp, i, i, sz, vp, sz]
        L.orbref_fast.argtypes = [vp, i, i, sz, i, vp, i]
        L.orbref_fast_atan2.restype = f
        L.orbref_fast_atan2.argtypes = [f, f]
        L.orbref_sinf.restype = f
        L.orbref_sinf.argtypes = [f]
        L.orbref_cosf.restype = f
        L.orbref_cosf.argtypes = [f]
        L.orbref_descriptor_distance.argtypes = [vp, vp]
        L.orbref_orb_descriptor.argtypes = [vp, sz, i, i, f, vp]
        L.orbref_ic_angle.restype = f
        L.orbref_ic_angle.argtypes = [vp, sz, i, i]
        L.orbref_sim3_ransac.argtypes = [i, vp, vp, vp, vp, vp, vp, i, i, i, i, vp, vp, vp, vp, vp, vp, vp]
        L.orbref_search_for_initialization.argtypes = [vp, vp, i, vp, vp, i, f, f, f, f, vp, i, f, i, i, vp]
        L.orbref_level_ptr.restype = vp
        L.orbref_level_ptr.argtypes = [vp, i, ctypes.POINTER(i), ctypes.POINTER(i)]
        L.orbref_stereo_matches.argtypes = [vp, vp, vp, vp, i, vp, vp, i, f, f, vp, vp]
        L.orbref_vocabulary_create.restype = vp
        L.orbref_vocabulary_create.argtypes = [i, i, i, vp, vp, vp, vp]
        L.orbref_vocabulary_destroy.argtypes = [vp]
        L.orbref_vocabulary_transform.argtypes = [vp, vp, i, i, vp, vp, vp]
        L.orbref_search_by_bow_kf_kf.argtypes = [vp, vp, vp, vp, i, vp, vp, vp, i, f, i, vp]
        L.orbref_search_by_bow_kf_f.argtypes = [vp, vp, vp, i, vp, vp, vp, vp, vp, vp, i, vp, vp, i, f, i, vp]
        L.orbref_pnp_ransac_call.argtypes = [vp, vp, vp, i, vp, i, i, vp, i, vp, vp]
        L.orbref_search_by_projection.argtypes = [i, vp, vp, i, vp, vp, vp, vp, vp, vp, i, vp, vp, vp, vp, vp, vp,
                                                  vp, vp, f, f, i, i, vp]
        L.orbref_compute_sim3_query.argtypes = [vp, i, vp, vp, vp, vp, vp, vp, vp, vp, i, vp, i, ctypes.c_uint, i,
                                                vp, vp]
        L.orbref_compute_sim3_query_ex.argtypes = [vp, i, vp, vp, vp, vp, vp, vp, vp, vp, i, vp, i, ctypes.c_uint,
                                                   i, vp, vp, vp, vp, vp, vp]
        _LIB = L
    return _LIB


def _p(a: np.ndarray) -> int:
    return a.ctypes.data


class Extractor:
    """ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)."""

    def __init__(self, nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7):
        self.nlevels = nlevels
        self.h = lib().orbref_create(nfeatures, scale_factor, nlevels, ini_th, min_th)
        if not self.h:
            raise ValueError("bad extractor parameters")

    def __del__(self):
        if getattr(self, "h", None):
            lib().orbref_destroy(self.h)
            self.h = None

    def extract(self, img: np.ndarray):
        img = np.ascontiguousarray(img, np.uint8)
        cap = 1 << 16
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = lib().orbref_extract(self.h, _p(img), img.shape[1], img.shape[0], img.strides[0],
                                 _p(kps), _p(desc), cap)
        if n < 0:
            raise RuntimeError("keypoint capacity exceeded")
        return kps[:n].copy(), desc[:n].copy()

    def level(self, l: int) -> np.ndarray:
        w, h = ctypes.c_int(), ctypes.c_int()
        if lib().orbref_level_size(self.h, l, ctypes.byref(w), ctypes.byref(h)) != 0:
            raise IndexError(l)
        out = np.zeros((h.value, w.value), np.uint8)
        lib().orbref_level_copy(self.h, l, _p(out))
        return out

    def _xys(self, fn, l: int) -> np.ndarray:
        n = fn(self.h, l, None, 0)
        out = np.zeros((max(n, 1), 3), np.int32)
        fn(self.h, l, _p(out), n)
        return out[:n]

    def candidates(self, l: int) -> np.ndarray:
        return self._xys(lib().orbref_level_candidates, l)

    def octree(self, l: int) -> np.ndarray:
        return self._xys(lib().orbref_level_octree, l)

    def features_per_level(self) -> np.ndarray:
        out = np.zeros(self.nlevels, np.int32)
        lib().orbref_features_per_level(self.h, _p(out))
        return out

    def scale_factors(self):
        arrs = [np.zeros(self.nlevels, np.float32) for _ in range(4)]
        lib().orbref_scale_factors(self.h, *[_p(a) for a in arrs])
        return arrs


def resize_linear(src: np.ndarray, dw: int, dh: int) -> np.ndarray:
    src = np.ascontiguousarray(src, np.uint8)
    dst = np.zeros((dh, dw), np.uint8)
    lib().orbref_resize_linear_u8(_p(src), src.shape[1], src.shape[0], src.strides[0], _p(dst), dw, dh, dw)
    return dst


def gaussian7(src: np.ndarray) -> np.ndarray:
    src = np.ascontiguousarray(src, np.uint8)
    dst = np.zeros_like(src)
    lib().orbref_gaussian7_u8(_p(src), src.shape[1], src.shape[0], src.strides[0], _p(dst), dst.strides[0])
    return dst


def fast(img: np.ndarray, threshold: int) -> np.ndarray:
    img = np.ascontiguousarray(img, np.uint8)
    cap = img.size
    out = np.zeros((cap, 3), np.int32)
    n = lib().orbref_fast(_p(img), img.shape[1], img.shape[0], img.strides[0], threshold, _p(out), cap)
    return out[:n]


def descriptor_distance(a: np.ndarray, b: np.ndarray) -> int:
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    return lib().orbref_descriptor_distance(_p(a), _p(b))


def search_for_initialization(kps1, desc1, kps2, desc2, img_w, img_h, prev_xy=None,
                              window=100, nnratio=0.9, check_ori=True, histo_bug=False, bounds=None):
    """Returns (nmatches, matches12, prev_xy_updated).  bounds = (minX, maxX,
    minY, maxY), default the undistorted frame [0, img_w] x [0, img_h]."""
    kps1 = np.ascontiguousarray(kps1, KP_DTYPE)
    kps2 = np.ascontiguousarray(kps2, KP_DTYPE)
    desc1 = np.ascontiguousarray(desc1, np.uint8)
    desc2 = np.ascontiguousarray(desc2, np.uint8)
    if prev_xy is None:
        prev_xy = np.stack([kps1["x"], kps1["y"]], axis=1).astype(np.float32)
    prev = np.ascontiguousarray(prev_xy, np.float32).copy()
    m12 = np.full(len(kps1), -1, np.int32)
    b = bounds if bounds is not None else (0.0, float(img_w), 0.0, float(img_h))
    n = lib().orbref_search_for_initialization(_p(kps1), _p(desc1), len(kps1), _p(kps2), _p(desc2), len(kps2),
                                               *[float(v) for v in b], _p(prev), window, nnratio, int(check_ori),
                                               int(histo_bug), _p(m12))
    return n, m12, prev


def sim3_ransac(X1, X2, maxerr1, maxerr2, K1, K2, fix_scale, min_inliers, best_inliers, samples):
    """Sim3Solver::iterate over the given triplets (see orbref.h).  Returns a
    dict: found, consumed, best_inliers, best_hyp, T12, R12, t12, s12, inliers."""
    X1 = np.ascontiguousarray(X1, np.float32)
    X2 = np.ascontiguousarray(X2, np.float32)
    e1 = np.ascontiguousarray(maxerr1, np.float32)
    e2 = np.ascontiguousarray(maxerr2, np.float32)
    k1 = np.ascontiguousarray(K1, np.float32)
    k2 = np.ascontiguousarray(K2, np.float32)
    smp = np.ascontiguousarray(samples, np.int32).reshape(-1, 3)
    n = len(X1)
    ints = np.zeros(4, np.int32)
    T = np.zeros(16, np.float32)
    R = np.zeros(9, np.float32)
    t = np.zeros(3, np.float32)
    sc = np.zeros(1, np.float32)
    inl = np.zeros(max(n, 1), np.uint8)
    lib().orbref_sim3_ransac(n, _p(X1), _p(X2), _p(e1), _p(e2), _p(k1), _p(k2), int(fix_scale), int(min_inliers),
                             int(best_inliers), len(smp), _p(smp), _p(ints), _p(T), _p(R), _p(t), _p(sc), _p(inl))
    return {"found": int(ints[0]), "consumed": int(ints[1]), "best_inliers": int(ints[2]), "best_hyp": int(ints[3]),
            "T12": T.reshape(4, 4), "R12": R.reshape(3, 3), "t12": t, "s12": float(sc[0]), "inliers": inl[:n]}


def stereo_matches(exL: Extractor, exR: Extractor, kpsL, descL, kpsR, descR, bf, min_z=0.0):
    """Frame::ComputeStereoMatches (oracle/stereo_ref.cpp) on the keypoints
    and pyramids of the two extractors' last extract() calls."""
    kpsL = np.ascontiguousarray(kpsL, KP_DTYPE)
    kpsR = np.ascontiguousarray(kpsR, KP_DTYPE)
    descL = np.ascontiguousarray(descL, np.uint8)
    descR = np.ascontiguousarray(descR, np.uint8)
    ur = np.zeros(max(len(kpsL), 1), np.float32)
    dp = np.zeros(max(len(kpsL), 1), np.float32)
    lib().orbref_stereo_matches(exL.h, exR.h, _p(kpsL), _p(descL), len(kpsL), _p(kpsR), _p(descR), len(kpsR),
                                float(bf), float(min_z), _p(ur), _p(dp))
    return ur[:len(kpsL)], dp[:len(kpsL)]


def stereo_frame(exL: Extractor, exR: Extractor, left, right, bf, min_z=0.0):
    """A stereo Frame's hot path (Frame.cpp:84-98): extract L and R with their
    own extractors, then ComputeStereoMatches.  Returns (kpsL, descL, kpsR,
    descR, uright, depth)."""
    kl, dl = exL.extract(left)
    kr, dr = exR.extract(right)
    ur, dp = stereo_matches(exL, exR, kl, dl, kr, dr, bf, min_z)
    return kl, dl, kr, dr, ur, dp


class Vocabulary:
    """DBoW2 tree from synth.synthetic_vocabulary* arrays (oracle/loop_ref.cpp)."""

    def __init__(self, k, L, parent, is_leaf, desc, weight):
        self._keep = [np.ascontiguousarray(parent, np.int32), np.ascontiguousarray(is_leaf, np.int32),
                      np.ascontiguousarray(desc, np.uint8), np.ascontiguousarray(weight, np.float64)]
        self.h = lib().orbref_vocabulary_create(k, L, len(self._keep[0]), *[_p(a) for a in self._keep])
        self._keep = None

    def __del__(self):
        if getattr(self, "h", None):
            lib().orbref_vocabulary_destroy(self.h)
            self.h = None

    def transform(self, desc, levelsup=4):
        desc = np.ascontiguousarray(desc, np.uint8)
        n = len(desc)
        words, nodes = np.zeros(n, np.int32), np.zeros(n, np.int32)
        weights = np.zeros(n, np.float64)
        lib().orbref_vocabulary_transform(self.h, _p(desc), n, levelsup, _p(words), _p(nodes), _p(weights))
        return words, nodes, weights


def search_by_bow_kf_kf(voc: Vocabulary, d1, a1, v1, d2, a2, v2, nnratio=0.75, check_ori=True):
    """SearchByBoW(KF1, KF2) with both FeatureVectors from voc (levelsup 4)."""
    arrs = [np.ascontiguousarray(d1, np.uint8), np.ascontiguousarray(a1, np.float32),
            np.ascontiguousarray(v1, np.uint8), np.ascontiguousarray(d2, np.uint8),
            np.ascontiguousarray(a2, np.float32), np.ascontiguousarray(v2, np.uint8)]
    m = np.zeros(len(arrs[0]), np.int32)
    n = lib().orbref_search_by_bow_kf_kf(voc.h, _p(arrs[0]), _p(arrs[1]), _p(arrs[2]), len(arrs[0]), _p(arrs[3]),
                                         _p(arrs[4]), _p(arrs[5]), len(arrs[3]), float(nnratio), int(check_ori),
                                         _p(m))
    return n, m


def pnp_ransac_call(P3w, P2, maxerr, cam, min_inliers, best_inliers, samples):
    """pnp_ref.ransac_call in C++ (oracle/pnp_ref.cpp): the iterate loop body
    over the given 4-tuples with Refine.  Returns dict(found, consumed,
    best_inliers, best_hyp, refined_inliers, best_R, best_t, refined_R,
    refined_t)."""
    P3 = np.ascontiguousarray(P3w, np.float32)
    P2 = np.ascontiguousarray(P2, np.float32)
    E = np.ascontiguousarray(maxerr, np.float32)
    cam = np.ascontiguousarray(np.asarray(cam, np.float64))
    smp = np.ascontiguousarray(samples, np.int32).reshape(-1, 4)
    oi = np.zeros(5, np.int32)
    op = np.zeros(24, np.float64)
    lib().orbref_pnp_ransac_call(_p(P3), _p(P2), _p(E), len(P2), _p(cam), int(min_inliers), int(best_inliers),
                                 _p(smp), len(smp), _p(oi), _p(op))
    return {"found": int(oi[0]), "consumed": int(oi[1]), "best_inliers": int(oi[2]), "best_hyp": int(oi[3]),
            "refined_inliers": int(oi[4]), "best_R": op[:9].reshape(3, 3), "best_t": op[9:12],
            "refined_R": op[12:21].reshape(3, 3), "refined_t": op[21:24]}


def _fv_csr(fv):
    nodes = np.array(sorted(fv), np.int32)
    start = np.zeros(len(nodes) + 1, np.int32)
    feats = []
    for k, nd in enumerate(nodes):
        feats.extend(fv[int(nd)])
        start[k + 1] = len(feats)
    return nodes, start, np.array(feats, np.int32)


def search_by_bow_kf_f(fvA, descA, angA, validA, fvB, descB, angB, nnratio=0.6, check_ori=True):
    """SearchByBoW(KF, F) (mode 0 of bow_ref.search_by_bow) in C++ on given
    FeatureVectors (dict node -> [features]); returns (nmatches, match[nB])."""
    na, sa, fa = _fv_csr(fvA)
    nb_, sb, fb = _fv_csr(fvB)
    arrs = [np.ascontiguousarray(descA, np.uint8), np.ascontiguousarray(angA, np.float32),
            np.ascontiguousarray(validA, np.uint8), np.ascontiguousarray(descB, np.uint8),
            np.ascontiguousarray(angB, np.float32)]
    m = np.zeros(len(arrs[3]), np.int32)
    n = lib().orbref_search_by_bow_kf_f(_p(na), _p(sa), _p(fa), len(na), _p(arrs[0]), _p(arrs[1]), _p(arrs[2]),
                                        _p(nb_), _p(sb), _p(fb), len(nb_), _p(arrs[3]), _p(arrs[4]), len(arrs[3]),
                                        float(nnratio), int(check_ori), _p(m))
    return n, m


def search_by_projection(variant, tgt, pts, th, nnratio=0.6, check_ori=True, mono=True, last_Tcw=None):
    """SearchByProjection for variant 0 (LOCAL: F, vpLocalMapPoints, th) and 2
    (LAST_FRAME: F, LastFrame, th, bMono) in C++ (proj_ref.cpp), with the
    dict layout of proj_ref.py; returns (nmatches, match)."""
    k = np.ascontiguousarray(tgt["kps"]).view(KP_DTYPE)
    n = len(k)
    f32, i32 = np.float32, np.int32
    npts = len(pts["flags"])
    A = dict(
        desc=np.ascontiguousarray(tgt["desc"], np.uint8),
        ur=None if tgt.get("u_right") is None else np.ascontiguousarray(tgt["u_right"], f32),
        occ=None if tgt.get("occupied") is None else np.ascontiguousarray(tgt["occupied"], np.uint8),
        bounds=np.array([tgt["min_x"], tgt["max_x"], tgt["min_y"], tgt["max_y"]], f32),
        cam=np.array([tgt["fx"], tgt["fy"], tgt["cx"], tgt["cy"], tgt["bf"], tgt["b"]], f32),
        sf=np.ascontiguousarray(tgt["scale_factors"], f32),
        T=np.ascontiguousarray(np.asarray(tgt["Tcw"], f32).reshape(16)),
        flags=np.ascontiguousarray(pts["flags"], i32),
        pos=np.ascontiguousarray(pts["pos"], f32),
        pdesc=np.ascontiguousarray(pts["desc"], np.uint8),
        track=np.ascontiguousarray(pts["track"], f32) if "track" in pts else np.zeros((npts, 4), f32),
        tl=np.ascontiguousarray(pts["track_level"], i32) if "track_level" in pts else np.zeros(npts, i32),
        oct=np.ascontiguousarray(pts["octave"], i32),
        ang=np.ascontiguousarray(pts["angle"], f32),
        last=np.ascontiguousarray(np.asarray(last_Tcw if last_Tcw is not None else tgt["Tcw"], f32).reshape(16)))
    m = np.zeros(n, np.int32)
    kk = np.ascontiguousarray(k)
    nm = lib().orbref_search_by_projection(
        int(variant), _p(kk), _p(A["desc"]), n, _p(A["ur"]) if A["ur"] is not None else None,
        _p(A["occ"]) if A["occ"] is not None else None, _p(A["bounds"]), _p(A["cam"]), _p(A["sf"]), _p(A["T"]),
        npts, _p(A["flags"]), _p(A["pos"]), _p(A["pdesc"]), _p(A["track"]), _p(A["tl"]), _p(A["oct"]),
        _p(A["ang"]), _p(A["last"]), float(th), float(nnratio), int(check_ori), int(mono), _p(m))
    if nm < 0:
        raise ValueError(f"variant {variant} not in the C++ oracle")
    return nm, m


_SCENE_KEYS = (("desc", np.uint8), ("angle", np.float32), ("octave", np.int32), ("valid", np.uint8),
               ("mp_world", np.float32), ("Tcw", np.float32), ("K", np.float32), ("sigma2", np.float32))


def compute_sim3_query(voc: Vocabulary, scene, cur, cands, seed, fix_scale=False):
    """One ComputeSim3 call in C++ (oracle/loop_ref.cpp) on a
    synth.loop_burst_scene.  Returns (matched, round, n_inliers, hypotheses,
    nmatches per candidate)."""
    c = scene.get("_c")
    if c is None:
        c = scene["_c"] = [np.ascontiguousarray(scene[k], t) for k, t in _SCENE_KEYS]
    cd = np.ascontiguousarray(cands, np.int32)
    out = np.zeros(4, np.int32)
    nm = np.zeros(len(cd), np.int32)
    lib().orbref_compute_sim3_query(voc.h, c[0].shape[1], *[_p(a) for a in c], int(cur), _p(cd), len(cd),
                                    int(seed) & 0xFFFFFFFF, int(fix_scale), _p(out), _p(nm))
    return int(out[0]), int(out[1]), int(out[2]), int(out[3]), nm


def compute_sim3_query_ex(voc: Vocabulary, scene, cur, cands, seed, fix_scale=False):
    """compute_sim3_query with everything a parity check compares: a dict of
    matched, round, n_inliers, hypotheses, nmatches[n_cand], m12[n_cand, n_kp]
    (vpMatches12 of SearchByBoW(KF, KF)), cand_state[n_cand, 5] (N, max_its,
    iterations, best inliers, discarded), R12/t12/s12 of the returned Sim3 and
    rand_after (the next value of the query's glibc stream after its draws)."""
    c = scene.get("_c")
    if c is None:
        c = scene["_c"] = [np.ascontiguousarray(scene[k], t) for k, t in _SCENE_KEYS]
    n_kp = c[0].shape[1]
    cd = np.ascontiguousarray(cands, np.int32)
    out = np.zeros(4, np.int32)
    nm = np.zeros(len(cd), np.int32)
    m12 = np.zeros((len(cd), n_kp), np.int32)
    pose = np.zeros(13, np.float32)
    cs = np.zeros((len(cd), 5), np.int32)
    ra = np.zeros(1, np.int32)
    lib().orbref_compute_sim3_query_ex(voc.h, n_kp, *[_p(a) for a in c], int(cur), _p(cd), len(cd),
                                       int(seed) & 0xFFFFFFFF, int(fix_scale), _p(out), _p(nm), _p(m12), _p(pose),
                                       _p(cs), _p(ra))
    return {"matched": int(out[0]), "round": int(out[1]), "n_inliers": int(out[2]), "hypotheses": int(out[3]),
            "nmatches": nm, "m12": m12, "cand_state": cs, "R12": pose[:9].reshape(3, 3), "t12": pose[9:12],
            "s12": float(pose[12]), "rand_after": int(ra[0])}
