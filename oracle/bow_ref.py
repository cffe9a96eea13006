"""CPU restatement of the DBoW2 bag-of-words path and ORBmatcher::SearchByBoW.

TEST INFRASTRUCTURE ONLY: the parity oracle for csrc/bow.hip (imported by
tests/ and nothing else).  Citations: T = /root/reference/ORB-SLAM2/
Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h, B = .../BowVector.cpp,
FV = .../FeatureVector.cpp, M = /root/reference/ORB-SLAM2/src/ORBmatcher.cpp.
Integer/index results are compared bit-exactly; BowVector weights (double)
too -- the GPU sums them in the same order.  DBoW2 ships no vocabulary or
fixture here (ORBvoc.txt is absent): the vocabularies are synthetic, so the
vocabulary-dependent results are "parity unpinned" against the real one.
"""
from __future__ import annotations

import math

import numpy as np


class Vocabulary:
    """TemplatedVocabulary nodes: parent, children (file order), descriptor,
    weight, word_id; node 0 is the root."""

    def __init__(self, k, L, scoring, weighting):
        self.k, self.L, self.scoring, self.weighting = k, L, scoring, weighting
        self.parent = [0]
        self.children = [[]]
        self.desc = [np.zeros(32, np.uint8)]
        self.weight = [0.0]
        self.word_id = [0]
        self.n_words = 0

    def _add(self, pid, leaf, desc, weight):
        nid = len(self.parent)
        self.parent.append(pid)
        self.children.append([])
        self.children[pid].append(nid)
        self.desc.append(np.asarray(desc, np.uint8))
        self.weight.append(float(weight))
        if leaf > 0:
            self.word_id.append(self.n_words)
            self.n_words += 1
        else:
            self.word_id.append(0)

    @classmethod
    def from_arrays(cls, k, L, scoring, weighting, parent, is_leaf, desc, weight):
        v = cls(k, L, scoring, weighting)
        for i in range(len(parent)):
            v._add(int(parent[i]), int(is_leaf[i]), desc[i], weight[i])
        return v

    @classmethod
    def load_text(cls, path):
        """loadFromTextFile (T:1359-1448): the `while(!f.eof()) getline` loop
        sees one more (empty) line when the file ends with a newline."""
        text = open(path).read()
        lines = text.split("\n")
        k, L, n1, n2 = (int(x) for x in lines[0].split()[:4])
        v = cls(k, L, n1, n2)
        for line in lines[1:]:
            tok = line.split()
            pid = int(tok[0]) if len(tok) > 0 else 0
            leaf = int(tok[1]) if len(tok) > 1 else 0
            d = np.zeros(32, np.uint8)
            for j in range(32):
                if 2 + j < len(tok):
                    d[j] = int(tok[2 + j]) & 0xFF
            w = float(tok[34]) if len(tok) > 34 else 0.0
            v._add(pid, leaf, d, w)
        return v

    @classmethod
    def load_binary(cls, path):
        """loadFromBinaryFile (T:1477-1522): header u32 nb_nodes, u32 size_node,
        int k, L, scoring, weighting; records (int parent, 32 desc bytes, float
        weight, bool leaf at byte 40).  The `while(!f.eof())` loop runs once
        more after the last full record on a 0-byte read, so the persistent
        buffer's record is processed again (a short read overwrites only its
        prefix); m_nodes has nb_nodes + 1 entries, the ones no record reaches
        stay default (parent 0, unattached)."""
        data = open(path, "rb").read()
        nb_nodes, size_node = (int(x) for x in np.frombuffer(data[:8], "<u4"))
        k, L, n1, n2 = (int(x) for x in np.frombuffer(data[8:24], "<i4"))
        v = cls(k, L, n1, n2)
        buf = bytearray(size_node)
        pos = 24
        while True:
            chunk = data[pos:pos + size_node]
            pos += len(chunk)
            buf[:len(chunk)] = chunk
            pid = int(np.frombuffer(bytes(buf[0:4]), "<i4")[0])
            w = float(np.frombuffer(bytes(buf[36:40]), "<f4")[0])
            v._add(pid, 1 if buf[40] else 0, np.frombuffer(bytes(buf[4:36]), np.uint8).copy(), w)
            if len(chunk) < size_node:  # the read that hit the end of the file sets eof
                break
        assert len(v.parent) <= nb_nodes + 1, "more records than nb_nodes (undefined in the reference)"
        while len(v.parent) < nb_nodes + 1:  # default Node()s, not attached to any parent
            v.parent.append(0)
            v.children.append([])
            v.desc.append(np.zeros(32, np.uint8))
            v.weight.append(0.0)
            v.word_id.append(0)
        return v

    def transform_one(self, f, levelsup):
        """transform(feature, word, weight, nid, levelsup) (T:1242-1283)."""
        nid_level = self.L - levelsup
        nid = 0
        final = 0
        level = 0
        while True:
            level += 1
            ch = self.children[final]
            best = ch[0]
            best_d = int(np.unpackbits(np.bitwise_xor(f, self.desc[best])).sum())
            for c in ch[1:]:
                d = int(np.unpackbits(np.bitwise_xor(f, self.desc[c])).sum())
                if d < best_d:
                    best_d, best = d, c
            final = best
            if level == nid_level:
                nid = final
            if not self.children[final]:
                break
        return self.word_id[final], nid, self.weight[final]

    def transform(self, feats, levelsup):
        """transform(features, BowVector, FeatureVector, levelsup) (T:1151-1230).
        Returns (words, nodes, weights, fv: dict node -> [features],
        bow: dict word -> value)."""
        words, nodes, weights = [], [], []
        bow, fv = {}, {}
        tf = self.weighting in (0, 1)
        for i, f in enumerate(feats):
            w_id, nid, w = self.transform_one(f, levelsup)
            words.append(w_id); nodes.append(nid); weights.append(w)
            if w > 0:
                if tf:  # BowVector::addWeight (B:34-46)
                    bow[w_id] = bow[w_id] + w if w_id in bow else w
                elif w_id not in bow:  # addIfNotExist (B:50-58)
                    bow[w_id] = w
                fv.setdefault(nid, []).append(i)  # FeatureVector::addFeature (FV:31-45)
        bow = dict(sorted(bow.items()))
        must = self.scoring != 5
        if bow and not must and tf:
            nd = float(len(bow))
            bow = {k: v / nd for k, v in bow.items()}
        if must:  # BowVector::normalize (B:62-90)
            if self.scoring == 1:
                norm = 0.0
                for v in bow.values():
                    norm += v * v
                norm = math.sqrt(norm)
            else:
                norm = 0.0
                for v in bow.values():
                    norm += abs(v)
            if norm > 0.0:
                bow = {k: v / norm for k, v in bow.items()}
        return words, nodes, weights, dict(sorted(fv.items())), bow


def _dist(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def _three_maxima(hist):
    """ComputeThreeMaxima (M:1792-1833)."""
    max1 = max2 = max3 = 0
    i1 = i2 = i3 = -1
    for i, h in enumerate(hist):
        s = len(h)
        if s > max1:
            max3, max2, max1, i3, i2, i1 = max2, max1, s, i2, i1, i
        elif s > max2:
            max3, max2, i3, i2 = max2, s, i2, i
        elif s > max3:
            max3, i3 = s, i
    if max2 < np.float32(0.1) * np.float32(max1):
        i2 = i3 = -1
    elif max3 < np.float32(0.1) * np.float32(max1):
        i3 = -1
    return i1, i2, i3


def search_by_bow(mode, fvA, descA, angA, validA, fvB, descB, angB, validB, nnratio=0.6, check_ori=True):
    """SearchByBoW(KF, F) (mode 0, M:205-348) and SearchByBoW(KF1, KF2)
    (mode 1, M:604-743).  fv: dict node -> [feature indices] (ascending
    nodes).  Returns (nmatches, match) with match indexed by F (mode 0) or
    KF1 (mode 1)."""
    HL, TH_LOW = 30, 50
    factor = np.float32(HL) / np.float32(360.0)
    nout = len(descB) if mode == 0 else len(descA)
    match = [-1] * nout
    matched2 = [False] * len(descB)
    hist = [[] for _ in range(HL)]
    nm = 0
    for node in sorted(set(fvA) & set(fvB)):
        for ia in fvA[node]:
            if not validA[ia]:
                continue
            b1, b2, bidx = 256, 256, -1
            for ib in fvB[node]:
                if mode == 0:
                    if match[ib] >= 0:
                        continue
                else:
                    if matched2[ib] or not validB[ib]:
                        continue
                d = _dist(descA[ia], descB[ib])
                if d < b1:
                    b2, b1, bidx = b1, d, ib
                elif d < b2:
                    b2 = d
            ok = b1 <= TH_LOW if mode == 0 else b1 < TH_LOW
            if not ok or not (np.float32(b1) < np.float32(nnratio) * np.float32(b2)):
                continue
            if mode == 0:
                match[bidx] = ia
                out = bidx
            else:
                match[ia] = bidx
                matched2[bidx] = True
                out = ia
            if check_ori:
                rot = np.float32(np.float32(angA[ia]) - np.float32(angB[bidx]))
                if rot < 0.0:
                    rot = np.float32(rot + np.float32(360.0))
                v = float(np.float32(rot * factor))
                b = int(math.copysign(math.floor(abs(v) + 0.5), v))
                if b == HL:
                    b = 0
                hist[b].append(out)
            nm += 1
    if check_ori:
        i1, i2, i3 = _three_maxima(hist)
        for i in range(HL):
            if i in (i1, i2, i3):
                continue
            for idx in hist[i]:
                match[idx] = -1
                nm -= 1
    return nm, np.array(match, np.int32)


def search_for_triangulation(fv1, fv2, P, check_ori=True, only_stereo=False):
    """ORBmatcher::SearchForTriangulation (M:755-951) with
    CheckDistEpipolarLine (M:166-190).  fv: dict node -> [features]; P: the
    pair's arrays (synth.triangulation_scenario layout; valid = the keyframe
    has no MapPoint at that keypoint).  Returns (nmatches, match12[n1])."""
    HL, TH_LOW = 30, 50
    f32, f64 = np.float32, np.float64
    factor = f32(HL) / f32(360.0)
    k1, k2, F = P["kps1"], P["kps2"], np.asarray(P["F12"], np.float32).reshape(3, 3)
    T, Cw = np.asarray(P["T2w"], np.float32).reshape(3, 4), np.asarray(P["Cw1"], np.float32)
    C2 = [f32(f32(f64(T[r, 0]) * f64(Cw[0]) + f64(T[r, 1]) * f64(Cw[1]) + f64(T[r, 2]) * f64(Cw[2])) + T[r, 3])
          for r in range(3)]
    invz = f32(f32(1.0) / C2[2])
    ex = f32(f32(f32(f32(P["fx2"]) * C2[0]) * invz) + f32(P["cx2"]))
    ey = f32(f32(f32(f32(P["fy2"]) * C2[1]) * invz) + f32(P["cy2"]))
    uR1, uR2 = P.get("u_right1"), P.get("u_right2")
    sf, s2 = [f32(x) for x in P["scale_factors2"]], [f32(x) for x in P["level_sigma2_2"]]
    n1 = len(k1)
    match = [-1] * n1
    matched2 = [False] * len(k2)
    hist = [[] for _ in range(HL)]
    nm = 0
    for node in sorted(set(fv1) & set(fv2)):
        for i1 in fv1[node]:
            if not P["valid1"][i1]:
                continue
            st1 = uR1 is not None and f32(uR1[i1]) >= 0
            if only_stereo and not st1:
                continue
            x1, y1 = f32(k1["x"][i1]), f32(k1["y"][i1])
            a = f32(f32(f32(x1 * F[0, 0]) + f32(y1 * F[1, 0])) + F[2, 0])
            b = f32(f32(f32(x1 * F[0, 1]) + f32(y1 * F[1, 1])) + F[2, 1])
            c = f32(f32(f32(x1 * F[0, 2]) + f32(y1 * F[1, 2])) + F[2, 2])
            best, bidx = TH_LOW, -1
            for i2 in fv2[node]:
                if matched2[i2] or not P["valid2"][i2]:
                    continue
                st2 = uR2 is not None and f32(uR2[i2]) >= 0
                if only_stereo and not st2:
                    continue
                d = _dist(P["desc1"][i1], P["desc2"][i2])
                if d > TH_LOW or d > best:
                    continue
                x2, y2, o2 = f32(k2["x"][i2]), f32(k2["y"][i2]), int(k2["octave"][i2])
                if not st1 and not st2:
                    dx, dy = f32(ex - x2), f32(ey - y2)
                    if f32(f32(dx * dx) + f32(dy * dy)) < f32(f32(100) * sf[o2]):
                        continue
                num = f32(f32(f32(a * x2) + f32(b * y2)) + c)
                den = f32(f32(a * a) + f32(b * b))
                if den == f32(0):
                    continue
                dsqr = f32(f32(num * num) / den)
                if f64(dsqr) < 3.84 * f64(s2[o2]):
                    best, bidx = d, i2
            if bidx < 0:
                continue
            match[i1] = bidx
            matched2[bidx] = True
            nm += 1
            if check_ori:
                rot = f32(f32(k1["angle"][i1]) - f32(k2["angle"][bidx]))
                if rot < 0.0:
                    rot = f32(rot + f32(360.0))
                vv = float(f32(rot * factor))
                bb = int(math.copysign(math.floor(abs(vv) + 0.5), vv))
                if bb == HL:
                    bb = 0
                hist[bb].append(i1)
    if check_ori:
        i1_, i2_, i3_ = _three_maxima(hist)
        for i in range(HL):
            if i in (i1_, i2_, i3_):
                continue
            for idx in hist[i]:
                match[idx] = -1
                nm -= 1
    return nm, np.array(match, np.int32)


LOG_EPS = math.log(2.220446049250313080847e-16)  # GeneralScoring::LOG_EPS = log(DBL_EPSILON)


def bow_score(scoring, v1: dict, v2: dict):
    """TemplatedVocabulary::score(v1, v2) (ScoringObject.cpp:23-313): the merge
    walk in ascending word order, double sum in that order.  v: dict word ->
    value.  Returns (score, common words)."""
    a, b = sorted(v1.items()), sorted(v2.items())
    i = j = 0
    s, nc = 0.0, 0
    while i < len(a) and j < len(b):
        (wa, vi), (wb, wi) = a[i], b[j]
        if wa == wb:
            nc += 1
            if scoring == 0:
                s += abs(vi - wi) - abs(vi) - abs(wi)
            elif scoring in (1, 5):
                s += vi * wi
            elif scoring == 2:
                if vi + wi != 0.0:
                    s += vi * wi / (vi + wi)
            elif scoring == 3:
                if vi != 0 and wi != 0:
                    s += vi * math.log(vi / wi)
            else:
                s += math.sqrt(vi * wi)
            i += 1
            j += 1
        elif wa < wb:
            if scoring == 3:
                s += vi * (math.log(vi) - LOG_EPS)
            i += 1
        else:
            j += 1
    if scoring == 3:
        for _, vi in a[i:]:
            if vi != 0:
                s += vi * (math.log(vi) - LOG_EPS)
    if scoring == 0:
        s = -s / 2.0
    elif scoring == 1:
        s = 1.0 if s >= 1 else 1.0 - math.sqrt(1.0 - s)
    elif scoring == 2:
        s = 2.0 * s
    if scoring == 3:  # common words of the whole vectors
        nc = len(set(v1) & set(v2))
    return s, nc
