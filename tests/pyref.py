"""Second, independent restatements of small pieces of the reference in plain
Python/numpy (test infrastructure).  They are written directly from the
reference sources (file:line cited) and cross-check the C++ oracle, so a
transcription slip in oracle/orbref.cpp cannot hide behind a matching GPU
kernel written by the same hand.  Pure-Python loops: small inputs only."""
from __future__ import annotations

import math

import numpy as np

RING = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
        (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def fast(img: np.ndarray, t: int):
    """cv::FAST(img, kps, t, true), TYPE_9_16 (used at ORBextractor.cpp:818):
    a corner has 9 contiguous ring pixels all > v+t or all < v-t; score =
    max over 16 arcs of max(min d, -max d) - 1 with d = v - ring; 3x3 strict
    NMS among corners; row-major emission."""
    h, w = img.shape
    im = img.astype(np.int32)
    score = np.zeros((h, w), np.int32)
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            v = im[y, x]
            ring = [im[y + dy, x + dx] for dx, dy in RING]
            d = [v - q for q in ring]
            corner = False
            for s in range(16):
                arc = [d[(s + k) % 16] for k in range(9)]
                if min(arc) > t or max(arc) < -t:
                    corner = True
                    break
            if corner:
                best = max(max(min(d[(s + k) % 16] for k in range(9)), -max(d[(s + k) % 16] for k in range(9)))
                           for s in range(16))
                score[y, x] = best - 1
    out = []
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            s = score[y, x]
            if s == 0:
                continue
            if all(s > score[y + dy, x + dx] for dy in (-1, 0, 1) for dx in (-1, 0, 1) if dx or dy):
                out.append((x, y, int(s)))
    return out


def distribute_octree(cands, minX, maxX, minY, maxY, N):
    """ORBextractor::DistributeOctTree (ORBextractor.cpp:541-770) with a
    Python list as std::list; equal-size ties broken by creation sequence
    (documented deviation H2).  cands: list of (x, y, score); returns the
    kept candidate indices in list order."""
    import numpy as _np
    f32 = _np.float32
    nIni = int(round(float(f32(maxX - minX) / f32(maxY - minY))))
    hX = f32(maxX - minX) / f32(nIni)
    seq = [0]

    def node(x0, y0, x1, y1, keys):
        n = {"x0": x0, "y0": y0, "x1": x1, "y1": y1, "keys": keys, "nomore": len(keys) == 1, "seq": seq[0]}
        seq[0] += 1
        return n

    roots = [node(int(hX * f32(i)), 0, int(hX * f32(i + 1)), maxY - minY, []) for i in range(nIni)]
    for k, (x, y, s) in enumerate(cands):
        roots[int(f32(x) / hX)]["keys"].append(k)
    lst = []
    for r in roots:
        if r["keys"]:
            r["nomore"] = len(r["keys"]) == 1
            lst.append(r)

    def divide(p):
        hx = math.ceil((p["x1"] - p["x0"]) / 2)
        hy = math.ceil((p["y1"] - p["y0"]) / 2)
        mx, my = p["x0"] + hx, p["y0"] + hy
        parts = [[], [], [], []]
        for k in p["keys"]:
            x, y, _ = cands[k]
            q = (0 if x < mx else 1) + (0 if y < my else 2)
            parts[q].append(k)
        rects = [(p["x0"], p["y0"], mx, my), (mx, p["y0"], p["x1"], my),
                 (p["x0"], my, mx, p["y1"]), (mx, my, p["x1"], p["y1"])]
        return [(rects[q], parts[q]) for q in range(4)]

    def push_children(p, expand):
        grow = 0
        for rect, keys in divide(p):
            if keys:
                c = node(*rect, keys)
                lst.insert(0, c)
                if len(keys) > 1:
                    expand.append(c)
                    grow += 1
        return grow

    finish = False
    expand = []
    while not finish:
        prev = len(lst)
        expand = []
        n_exp = 0
        i = 0
        while i < len(lst):
            p = lst[i]
            if p["nomore"]:
                i += 1
                continue
            before = len(lst)
            n_exp += push_children(p, expand)
            i += len(lst) - before  # skip the nodes pushed in front
            lst.pop(i)
        if len(lst) >= N or len(lst) == prev:
            finish = True
        elif len(lst) + 3 * n_exp > N:
            while not finish:
                prev = len(lst)
                todo = sorted(expand, key=lambda n: (len(n["keys"]), n["seq"]))
                expand = []
                for p in reversed(todo):
                    push_children(p, expand)
                    lst.remove(p)
                    if len(lst) >= N:
                        break
                if len(lst) >= N or len(lst) == prev:
                    finish = True
    kept = []
    for n in lst:
        best = n["keys"][0]
        for k in n["keys"][1:]:
            if cands[k][2] > cands[best][2]:
                best = k
        kept.append(best)
    return kept


def resize_linear(src: np.ndarray, dw: int, dh: int) -> np.ndarray:
    """cv::resize INTER_LINEAR 8U, OpenCV 2.4 fixed point (DESIGN.md spec)."""
    sh, sw = src.shape
    f32 = np.float32
    sx_ = 1.0 / (dw / sw)
    sy_ = 1.0 / (dh / sh)

    def taps(d, scale, n):
        f = f32((d + 0.5) * scale - 0.5)
        i = math.floor(f)
        f = f32(f - f32(i))
        return i, f

    def rnd(v):
        return int(np.rint(np.float64(v)))

    xs = []
    xmax = dw
    for dx in range(dw):
        sx, fx = taps(dx, sx_, sw)
        if sx < 0:
            sx, fx = 0, f32(0)
        if sx + 1 >= sw:
            xmax = min(xmax, dx)
            if sx >= sw - 1:
                sx, fx = sw - 1, f32(0)
        xs.append((sx, rnd(f32(f32(1) - fx) * f32(2048)), rnd(fx * f32(2048))))
    w = dw
    simd_end = 0
    while simd_end <= w - 16:
        simd_end += 16
    while simd_end < w - 4:
        simd_end += 4
    out = np.zeros((dh, dw), np.uint8)
    S = src.astype(np.int64)

    def s16(v):
        return max(-32768, min(32767, v))

    for dy in range(dh):
        sy, fy = taps(dy, sy_, sh)
        b0, b1 = rnd(f32(f32(1) - fy) * f32(2048)), rnd(fy * f32(2048))
        r0, r1 = min(max(sy, 0), sh - 1), min(max(sy + 1, 0), sh - 1)
        for dx in range(dw):
            sx, a0, a1 = xs[dx]
            if dx < xmax:
                h0 = S[r0, sx] * a0 + S[r0, sx + 1] * a1
                h1 = S[r1, sx] * a0 + S[r1, sx + 1] * a1
            else:
                h0, h1 = S[r0, sx] * 2048, S[r1, sx] * 2048
            if dx < simd_end:
                v = s16(s16(((s16(h0 >> 4) * b0) >> 16) + ((s16(h1 >> 4) * b1) >> 16)) + 2) >> 2
            else:
                v = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22
            out[dy, dx] = max(0, min(255, v))
    return out


def descriptor_distance(a: np.ndarray, b: np.ndarray) -> int:
    """ORBmatcher::DescriptorDistance (ORBmatcher.cpp:1838): popcount(a^b)."""
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def search_for_initialization(k1, d1, k2, d2, bounds, prev_xy, window=100, nnratio=0.9, check_ori=True,
                              histo_factor=None):
    """ORBmatcher::SearchForInitialization (ORBmatcher.cpp:474-590) with the
    grid of Frame::AssignFeaturesToGrid / PosInGrid (Frame.cpp:241-259,
    434-443), Frame::GetFeaturesInArea (Frame.cpp:379-432) and
    ComputeThreeMaxima (ORBmatcher.cpp:1790-1835).  Float arithmetic in
    numpy float32 scalars; k1/k2 are KP_DTYPE arrays (mvKeysUn).  Returns
    (nmatches, matches12, prev_xy_updated)."""
    f32 = np.float32
    GC, GR, TH_LOW, HL = 64, 48, 50, 30
    minX, maxX, minY, maxY = (f32(v) for v in bounds)
    invW, invH = f32(GC) / f32(maxX - minX), f32(GR) / f32(maxY - minY)
    grid = [[[] for _ in range(GR)] for _ in range(GC)]
    for i in range(len(k2)):
        # C round(): half away from zero
        px = int(math.copysign(math.floor(abs(float(f32(f32(k2["x"][i]) - minX) * invW)) + 0.5),
                               float(f32(f32(k2["x"][i]) - minX) * invW)))
        py = int(math.copysign(math.floor(abs(float(f32(f32(k2["y"][i]) - minY) * invH)) + 0.5),
                               float(f32(f32(k2["y"][i]) - minY) * invH)))
        if 0 <= px < GC and 0 <= py < GR:
            grid[px][py].append(i)
    # all-pairs Hamming distances (DescriptorDistance, ORBmatcher.cpp:1838)
    dist = np.unpackbits(np.bitwise_xor(d1[:, None, :], d2[None, :, :]), axis=2).sum(axis=2).astype(int) \
        if len(k1) and len(k2) else np.zeros((len(k1), len(k2)), int)
    prev = np.array(prev_xy, np.float32, copy=True)
    m12 = [-1] * len(k1)
    m21 = [-1] * len(k2)
    mdist = [2 ** 31 - 1] * len(k2)
    hist = [[] for _ in range(HL)]
    factor = f32(HL) / f32(360.0) if histo_factor is None else f32(histo_factor)
    r = f32(window)
    nm = 0
    for i1 in range(len(k1)):
        if k1["octave"][i1] > 0:
            continue
        x, y = prev[i1, 0], prev[i1, 1]
        cx0 = max(0, int(math.floor(f32(f32(x - minX) - r) * invW)))
        cx1 = min(GC - 1, int(math.ceil(f32(f32(x - minX) + r) * invW)))
        cy0 = max(0, int(math.floor(f32(f32(y - minY) - r) * invH)))
        cy1 = min(GR - 1, int(math.ceil(f32(f32(y - minY) + r) * invH)))
        if cx0 >= GC or cx1 < 0 or cy0 >= GR or cy1 < 0:
            continue
        cand = []
        for ix in range(cx0, cx1 + 1):
            for iy in range(cy0, cy1 + 1):
                for j in grid[ix][iy]:
                    if k2["octave"][j] != 0:
                        continue
                    if abs(f32(k2["x"][j] - x)) < r and abs(f32(k2["y"][j] - y)) < r:
                        cand.append(j)
        if not cand:
            continue
        best, best2, bidx = 2 ** 31 - 1, 2 ** 31 - 1, -1
        for j in cand:
            dd = int(dist[i1, j])
            if mdist[j] <= dd:
                continue
            if dd < best:
                best2, best, bidx = best, dd, j
            elif dd < best2:
                best2 = dd
        if best <= TH_LOW and f32(best) < f32(f32(best2) * f32(nnratio)):
            if m21[bidx] >= 0:
                m12[m21[bidx]] = -1
                nm -= 1
            m12[i1], m21[bidx], mdist[bidx] = bidx, i1, best
            nm += 1
            if check_ori:
                rot = f32(f32(k1["angle"][i1]) - f32(k2["angle"][bidx]))
                if rot < 0.0:
                    rot = f32(rot + f32(360.0))
                v = float(f32(rot * factor))
                b = int(math.copysign(math.floor(abs(v) + 0.5), v))
                if b == HL:
                    b = 0
                hist[b].append(i1)
    if check_ori:
        m1 = m2 = m3 = 0
        i1_ = i2_ = i3_ = -1
        for i in range(HL):
            s = len(hist[i])
            if s > m1:
                m3, m2, m1, i3_, i2_, i1_ = m2, m1, s, i2_, i1_, i
            elif s > m2:
                m3, m2, i3_, i2_ = m2, s, i2_, i
            elif s > m3:
                m3, i3_ = s, i
        if m2 < f32(0.1) * f32(m1):
            i2_ = i3_ = -1
        elif m3 < f32(0.1) * f32(m1):
            i3_ = -1
        for i in range(HL):
            if i in (i1_, i2_, i3_):
                continue
            for a in hist[i]:
                if m12[a] >= 0:
                    m12[a] = -1
                    nm -= 1
    for i in range(len(k1)):
        if m12[i] >= 0:
            prev[i, 0], prev[i, 1] = k2["x"][m12[i]], k2["y"][m12[i]]
    return nm, np.array(m12, np.int32), prev
