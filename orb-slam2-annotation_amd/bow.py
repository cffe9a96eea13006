"""Host-side mirror of the bag-of-words path over include/orbgpu_bow.h:
``Vocabulary`` (DBoW2 TemplatedVocabulary: text loader, transform) and
``search_by_bow`` (ORBmatcher::SearchByBoW, both overloads)."""
from __future__ import annotations

import ctypes

import numpy as np

import orbgpu

KF_F, KF_KF = 0, 1


class VocabInfo(ctypes.Structure):
    _fields_ = [("k", ctypes.c_int), ("L", ctypes.c_int), ("scoring", ctypes.c_int), ("weighting", ctypes.c_int),
                ("n_nodes", ctypes.c_int), ("n_words", ctypes.c_int)]


class BowFrame(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("fv_n", ctypes.c_int), ("fv_nodes", ctypes.c_void_p),
                ("fv_offsets", ctypes.c_void_p), ("fv_features", ctypes.c_void_p), ("desc", ctypes.c_void_p),
                ("angle", ctypes.c_void_p), ("valid", ctypes.c_void_p)]


class Vocabulary:
    """TemplatedVocabulary<FORB::TDescriptor, FORB> in HBM."""

    def __init__(self, handle):
        self.h = handle

    @classmethod
    def load_text(cls, path: str) -> "Vocabulary":
        h = ctypes.c_void_p()
        orbgpu._check(orbgpu.lib().orbgpu_vocabulary_load_text(str(path).encode(), ctypes.byref(h)),
                      "orbgpu_vocabulary_load_text")
        return cls(h)

    @classmethod
    def load_binary(cls, path: str) -> "Vocabulary":
        """TemplatedVocabulary::loadFromBinaryFile (TemplatedVocabulary.h:1478)."""
        h = ctypes.c_void_p()
        orbgpu._check(orbgpu.lib().orbgpu_vocabulary_load_binary(str(path).encode(), ctypes.byref(h)),
                      "orbgpu_vocabulary_load_binary")
        return cls(h)

    @classmethod
    def from_arrays(cls, k, L, scoring, weighting, parent, is_leaf, desc, weight) -> "Vocabulary":
        parent = np.ascontiguousarray(parent, np.int32)
        is_leaf = np.ascontiguousarray(is_leaf, np.int32)
        desc = np.ascontiguousarray(desc, np.uint8)
        weight = np.ascontiguousarray(weight, np.float64)
        h = ctypes.c_void_p()
        orbgpu._check(orbgpu.lib().orbgpu_vocabulary_create(k, L, scoring, weighting, len(parent),
                                                            parent.ctypes.data, is_leaf.ctypes.data,
                                                            desc.ctypes.data, weight.ctypes.data, ctypes.byref(h)),
                      "orbgpu_vocabulary_create")
        return cls(h)

    def __del__(self):
        if getattr(self, "h", None):
            orbgpu.lib().orbgpu_vocabulary_destroy(self.h)
            self.h = None

    def info(self) -> VocabInfo:
        inf = VocabInfo()
        orbgpu._check(orbgpu.lib().orbgpu_vocabulary_get_info(self.h, ctypes.byref(inf)), "orbgpu_vocabulary_get_info")
        return inf

    def transform(self, desc: np.ndarray, levelsup: int = 4):
        """transform(features, BowVector, FeatureVector, levelsup); returns
        (words, nodes, weights, fv dict node -> array, bow dict word -> value)."""
        desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(desc)
        m = max(n, 1)
        word = np.zeros(m, np.int32); node = np.zeros(m, np.int32); weight = np.zeros(m, np.float64)
        fvn = np.zeros(m, np.int32); fvo = np.zeros(m + 1, np.int32); fvf = np.zeros(m, np.int32)
        bw = np.zeros(m, np.int32); bv = np.zeros(m, np.float64)
        nf = ctypes.c_int(); nb = ctypes.c_int()
        orbgpu._check(orbgpu.lib().orbgpu_bow_transform(self.h, n, desc.ctypes.data, levelsup, word.ctypes.data,
                                                        node.ctypes.data, weight.ctypes.data, fvn.ctypes.data,
                                                        fvo.ctypes.data, fvf.ctypes.data, ctypes.byref(nf),
                                                        bw.ctypes.data, bv.ctypes.data, ctypes.byref(nb)),
                      "orbgpu_bow_transform")
        fv = {int(fvn[i]): fvf[fvo[i]:fvo[i + 1]].copy() for i in range(nf.value)}
        bow = {int(bw[i]): float(bv[i]) for i in range(nb.value)}
        return word[:n], node[:n], weight[:n], fv, bow


def fv_to_csr(fv: dict):
    nodes = np.array(sorted(fv), np.int32)
    offs = np.zeros(len(nodes) + 1, np.int32)
    feats = []
    for i, k in enumerate(nodes):
        feats.extend(int(x) for x in fv[int(k)])
        offs[i + 1] = len(feats)
    return nodes, offs, np.array(feats, np.int32)


def _frame(fv, desc, angle, valid, keep):
    nodes, offs, feats = fv_to_csr(fv)
    desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    angle = np.ascontiguousarray(angle, np.float32)
    valid = np.ascontiguousarray(valid, np.uint8)
    keep.extend([nodes, offs, feats, desc, angle, valid])
    return BowFrame(len(desc), len(nodes), nodes.ctypes.data, offs.ctypes.data, feats.ctypes.data, desc.ctypes.data,
                    angle.ctypes.data, valid.ctypes.data)


def search_by_bow(mode, fvA, descA, angA, validA, fvB, descB, angB, validB, nnratio=0.6, check_ori=True):
    """ORBmatcher(nnratio, checkOri).SearchByBoW: mode KF_F (A = KF, B = F)
    or KF_KF (A = KF1, B = KF2).  Returns (nmatches, match)."""
    keep = []
    a = _frame(fvA, descA, angA, validA, keep)
    b = _frame(fvB, descB, angB, validB, keep)
    nout = b.n if mode == KF_F else a.n
    match = np.zeros(max(nout, 1), np.int32)
    nm = ctypes.c_int()
    orbgpu._check(orbgpu.lib().orbgpu_search_by_bow(mode, ctypes.byref(a), ctypes.byref(b), float(nnratio),
                                                    int(check_ori), match.ctypes.data, ctypes.byref(nm)),
                  "orbgpu_search_by_bow")
    return nm.value, match[:nout]



class TriangulationPair(ctypes.Structure):
    _fields_ = [("kf1", BowFrame), ("kf2", BowFrame), ("kps1", ctypes.c_void_p), ("kps2", ctypes.c_void_p),
                ("u_right1", ctypes.c_void_p), ("u_right2", ctypes.c_void_p), ("F12", ctypes.c_float * 9),
                ("Cw1", ctypes.c_float * 3), ("T2w", ctypes.c_float * 12), ("fx2", ctypes.c_float),
                ("fy2", ctypes.c_float), ("cx2", ctypes.c_float), ("cy2", ctypes.c_float),
                ("scale_factors2", ctypes.c_float * 16), ("level_sigma2_2", ctypes.c_float * 16),
                ("only_stereo", ctypes.c_int)]


def search_for_triangulation(fv1, fv2, P, check_ori=True, only_stereo=False):
    """ORBmatcher(0.6, checkOri).SearchForTriangulation on the GPU:
    (nmatches, match12[n1]); P in synth.triangulation_scenario's layout."""
    keep = []
    T = TriangulationPair()
    T.kf1 = _frame(fv1, P["desc1"], P["kps1"]["angle"], P["valid1"], keep)
    T.kf2 = _frame(fv2, P["desc2"], P["kps2"]["angle"], P["valid2"], keep)
    for name in ("kps1", "kps2"):
        k = np.ascontiguousarray(P[name], orbgpu.KP_DTYPE)
        keep.append(k)
        setattr(T, name, k.ctypes.data)
    for name in ("u_right1", "u_right2"):
        if P.get(name) is not None:
            a = np.ascontiguousarray(P[name], np.float32)
            keep.append(a)
            setattr(T, name, a.ctypes.data)
    T.F12[:] = [float(x) for x in np.asarray(P["F12"], np.float32).reshape(9)]
    T.Cw1[:] = [float(x) for x in np.asarray(P["Cw1"], np.float32).reshape(3)]
    T.T2w[:] = [float(x) for x in np.asarray(P["T2w"], np.float32).reshape(12)]
    T.fx2, T.fy2, T.cx2, T.cy2 = (float(P[k]) for k in ("fx2", "fy2", "cx2", "cy2"))
    T.scale_factors2[:len(P["scale_factors2"])] = [float(x) for x in P["scale_factors2"]]
    T.level_sigma2_2[:len(P["level_sigma2_2"])] = [float(x) for x in P["level_sigma2_2"]]
    T.only_stereo = int(only_stereo)
    n1 = T.kf1.n
    match = np.zeros(max(n1, 1), np.int32)
    nm = ctypes.c_int()
    L = orbgpu.lib()
    L.orbgpu_search_for_triangulation.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    orbgpu._check(L.orbgpu_search_for_triangulation(ctypes.byref(T), int(check_ori), match.ctypes.data,
                                                    ctypes.byref(nm)), "orbgpu_search_for_triangulation")
    return nm.value, match[:n1]


def bow_score(scoring, query: dict, db: list):
    """TemplatedVocabulary::score(query, kf) and the common-word count for every
    keyframe BowVector in `db` (dicts word -> value) on the GPU:
    (common (nkf,) int32, scores (nkf,) float64)."""
    qw = np.array(sorted(query), np.int32)
    qv = np.array([query[int(w)] for w in qw], np.float64)
    off = np.zeros(len(db) + 1, np.int32)
    words, vals = [], []
    for k, v in enumerate(db):
        ws = sorted(v)
        words += ws
        vals += [v[w] for w in ws]
        off[k + 1] = len(words)
    dw, dv = np.array(words, np.int32), np.array(vals, np.float64)
    common = np.zeros(max(len(db), 1), np.int32)
    scores = np.zeros(max(len(db), 1), np.float64)
    L = orbgpu.lib()
    vp = ctypes.c_void_p
    L.orbgpu_bow_score.argtypes = [ctypes.c_int, vp, vp, ctypes.c_int, ctypes.c_int, vp, vp, vp, vp, vp]
    orbgpu._check(L.orbgpu_bow_score(int(scoring), qw.ctypes.data, qv.ctypes.data, len(qw), len(db),
                                     off.ctypes.data, dw.ctypes.data if len(dw) else None,
                                     dv.ctypes.data if len(dv) else None, common.ctypes.data, scores.ctypes.data),
                  "orbgpu_bow_score")
    return common[:len(db)], scores[:len(db)]

# --------------------------------------------------------------------------
# Batched, HBM-resident forms (torch tensors on the GPU)
# --------------------------------------------------------------------------
_BATCH_BOUND = False


def _batch_lib():
    global _BATCH_BOUND
    L = orbgpu.lib()
    if not _BATCH_BOUND:
        vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        L.orbgpu_bow_transform_batch_device.argtypes = [vp, i, vp, vp, i, i, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                                        vp]
        L.orbgpu_search_by_bow_batch_device.argtypes = [i, i, vp, vp, f, i, i, vp, vp, vp]
        _BATCH_BOUND = True
    return L


def _dev(t, dtype, name):
    import torch
    if not (isinstance(t, torch.Tensor) and t.is_cuda and t.is_contiguous()):
        raise TypeError(f"{name} must be a contiguous torch tensor on the GPU")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    return t.data_ptr()


class BatchTransform:
    """Outputs of transform() for B frames of `stride` slots, in HBM:
    per-slot word/node/weight, FeatureVector CSR (fv_nodes, fv_offsets,
    fv_features, fv_n) and BowVector (bow_words, bow_values, bow_n)."""

    def __init__(self, B, stride, device):
        import torch
        i32 = dict(dtype=torch.int32, device=device)
        self.B, self.stride = B, stride
        self.word = torch.zeros((B, stride), **i32)
        self.node = torch.zeros((B, stride), **i32)
        self.weight = torch.zeros((B, stride), dtype=torch.float64, device=device)
        self.fv_nodes = torch.zeros((B, stride), **i32)
        self.fv_offsets = torch.zeros((B, stride + 1), **i32)
        self.fv_features = torch.zeros((B, stride), **i32)
        self.fv_n = torch.zeros(B, **i32)
        self.bow_words = torch.zeros((B, stride), **i32)
        self.bow_values = torch.zeros((B, stride), dtype=torch.float64, device=device)
        self.bow_n = torch.zeros(B, **i32)


def transform_batch(voc: Vocabulary, desc, counts, out: BatchTransform, levelsup=4, stream=None):
    """Frame/KeyFrame::ComputeBoW for a batch (orbgpu_bow_transform_batch_device):
    desc (B, stride, 32) uint8, counts (B,) int32, on the GPU."""
    import torch
    B, S = out.B, out.stride
    if tuple(desc.shape) != (B, S, 32) or tuple(counts.shape) != (B,):
        raise ValueError("desc must be (B, stride, 32) and counts (B,)")
    _dev(desc, torch.uint8, "desc")
    _dev(counts, torch.int32, "counts")
    orbgpu._check(_batch_lib().orbgpu_bow_transform_batch_device(
        voc.h, B, desc.data_ptr(), counts.data_ptr(), S, levelsup, out.word.data_ptr(), out.node.data_ptr(),
        out.weight.data_ptr(), out.fv_nodes.data_ptr(), out.fv_offsets.data_ptr(), out.fv_features.data_ptr(),
        out.fv_n.data_ptr(), out.bow_words.data_ptr(), out.bow_values.data_ptr(), out.bow_n.data_ptr(),
        orbgpu._stream_ptr(stream)), "orbgpu_bow_transform_batch_device")


def frame_table(tf: BatchTransform, desc, angle, valid, counts_host, rows=None):
    """orbgpu_bow_frame records (host ctypes array) pointing into HBM: frame r
    = batch row rows[r] (default all rows) of a transform output, with its
    descriptors (B, stride, 32) u8, angles (B, stride) f32 and MapPoint flags
    (B, stride) u8.  counts_host: features per row (numpy)."""
    import torch
    S = tf.stride
    _dev(desc, torch.uint8, "desc")
    _dev(angle, torch.float32, "angle")
    _dev(valid, torch.uint8, "valid")
    fv_n = tf.fv_n.cpu().numpy()
    if (fv_n < 0).any():
        raise orbgpu.OrbGpuError(orbgpu.ERR_CAPACITY, "transform_batch rejected a frame")
    rows = range(tf.B) if rows is None else rows
    rows = list(rows)
    tab = (BowFrame * max(len(rows), 1))()
    for r, b in enumerate(rows):
        tab[r] = BowFrame(int(counts_host[b]), int(fv_n[b]), tf.fv_nodes.data_ptr() + 4 * S * b,
                          tf.fv_offsets.data_ptr() + 4 * (S + 1) * b, tf.fv_features.data_ptr() + 4 * S * b,
                          desc.data_ptr() + 32 * S * b, angle.data_ptr() + 4 * S * b, valid.data_ptr() + S * b)
    return tab


def to_device_table(tab, device):
    """copy a ctypes struct array into a uint8 device tensor"""
    import torch
    raw = np.frombuffer(bytes(tab), np.uint8)
    return torch.from_numpy(raw.copy()).to(device)


def search_by_bow_batch(mode, d_frames_a, d_frames_b, batch, nnratio, check_ori, stride, match, nmatches,
                        stream=None):
    """ORBmatcher(nnratio, checkOri).SearchByBoW over `batch` pairs of device
    frame tables (orbgpu_search_by_bow_batch_device): match (batch, stride)
    int32, nmatches (batch,) int32."""
    import torch
    _dev(match, torch.int32, "match")
    _dev(nmatches, torch.int32, "nmatches")
    orbgpu._check(_batch_lib().orbgpu_search_by_bow_batch_device(
        mode, batch, d_frames_a.data_ptr(), d_frames_b.data_ptr(), float(nnratio), int(check_ori), stride,
        match.data_ptr(), nmatches.data_ptr(), orbgpu._stream_ptr(stream)), "orbgpu_search_by_bow_batch_device")
