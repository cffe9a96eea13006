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
