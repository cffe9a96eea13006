"""CPU restatement of Frame::ComputeStereoMatches (stereo matching between the
left and right ORB features of a rectified pair).

TEST INFRASTRUCTURE ONLY: the parity oracle for csrc/stereo.hip.  Citations:
F = /root/reference/ORB-SLAM2/src/Frame.cpp.  Float arithmetic is restated in
numpy float32 scalars, in the order the reference writes it.  Bar: bit-exact
uRight / depth / -1 flags.

Spec decisions where the reference is undefined (documented in DESIGN.md):
* rows of vRowIndices outside [0, nRows) (a right keypoint within 2*scale of
  the image border, F:570-575) are skipped instead of indexing out of range;
* an 11x11 window (F:657, :676) that would leave the pyramid level (OpenCV
  asserts) makes the keypoint unmatched;
* an empty vDistIdx (no accepted match, F:735 reads element 0) skips the
  median cut.
"""
from __future__ import annotations

import math

import numpy as np

f32 = np.float32
TH_HIGH, TH_LOW = 100, 50


def hamming(a: np.ndarray, b: np.ndarray) -> int:
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def c_roundf(v) -> float:
    """std::round on a float (half away from zero), F:651-653."""
    v = float(v)
    return float(math.copysign(math.floor(abs(v) + 0.5), v))


def compute_stereo_matches(kpsL, descL, kpsR, descR, pyrL, pyrR, scale, inv_scale, bf, min_z):
    """Returns (uRight f32[N], depth f32[N]) as Frame::ComputeStereoMatches
    (F:540-748).  kps*: KP_DTYPE records; pyr*: list of u8 levels; scale /
    inv_scale: mvScaleFactors / mvInvScaleFactors (f32); bf = mbf; min_z = mb
    at call time (0 in the reference's stereo constructor, F:67/:98/:123, so
    maxD = mbf / 0 = +inf)."""
    N, Nr = len(kpsL), len(kpsR)
    uright = np.full(N, -1.0, np.float32)
    depth = np.full(N, -1.0, np.float32)
    th_orb = (TH_HIGH + TH_LOW) // 2  # F:545
    n_rows = pyrL[0].shape[0]
    rows = [[] for _ in range(n_rows)]  # F:555-576
    for iR in range(Nr):
        ky = f32(kpsR[iR]["y"])
        r = f32(f32(2.0) * f32(scale[kpsR[iR]["octave"]]))
        maxr = int(math.ceil(f32(ky + r)))
        minr = int(math.floor(f32(ky - r)))
        for yi in range(minr, maxr + 1):
            if 0 <= yi < n_rows:
                rows[yi].append(iR)
    min_d = f32(0.0)
    with np.errstate(divide="ignore"):
        max_d = f32(f32(bf) / f32(min_z))  # F:581
    dist_idx = []
    for iL in range(N):
        lvl = int(kpsL[iL]["octave"])
        vL, uL = f32(kpsL[iL]["y"]), f32(kpsL[iL]["x"])
        cand = rows[int(vL)] if int(vL) < n_rows else []
        if not cand:
            continue
        min_u = f32(uL - max_d)
        max_u = f32(uL - min_d)
        if max_u < 0:
            continue
        best, best_r = TH_HIGH, 0
        for iR in cand:  # F:618-640
            o = int(kpsR[iR]["octave"])
            if o < lvl - 1 or o > lvl + 1:
                continue
            uR = f32(kpsR[iR]["x"])
            if min_u <= uR <= max_u:
                d = hamming(descL[iL], descR[iR])
                if d < best:
                    best, best_r = d, iR
        if best >= th_orb:
            continue
        # subpixel match by correlation, F:645-729
        uR0 = f32(kpsR[best_r]["x"])
        sf = f32(inv_scale[lvl])
        su = c_roundf(f32(uL * sf))
        sv = c_roundf(f32(vL * sf))
        sr = c_roundf(f32(uR0 * sf))
        w, L = 5, 5
        IL_img, IR_img = pyrL[lvl], pyrR[lvl]
        r0, c0 = int(sv) - w, int(su) - w
        if r0 < 0 or r0 + 2 * w + 1 > IL_img.shape[0] or c0 < 0 or c0 + 2 * w + 1 > IL_img.shape[1]:
            continue
        iniu = sr + L - w
        endu = sr + L + w + 1
        if iniu < 0 or endu >= IR_img.shape[1]:  # F:668-671
            continue
        if int(sr) - L - w < 0 or r0 + 2 * w + 1 > IR_img.shape[0]:
            continue  # spec: the IR window would leave the level
        IL = IL_img[r0:r0 + 11, c0:c0 + 11].astype(np.int64)
        IL = IL - IL[w, w]
        best_sad, best_inc = 2 ** 31 - 1, 0
        dists = [0.0] * (2 * L + 1)
        for inc in range(-L, L + 1):
            cr = int(sr) + inc - w
            IR = IR_img[r0:r0 + 11, cr:cr + 11].astype(np.int64)
            IR = IR - IR[w, w]
            d = float(np.abs(IL - IR).sum())  # cv::norm(NORM_L1), exact integers
            if d < best_sad:
                best_sad, best_inc = int(d), inc
            dists[L + inc] = d
        if best_inc == -L or best_inc == L:
            continue
        d1, d2, d3 = f32(dists[L + best_inc - 1]), f32(dists[L + best_inc]), f32(dists[L + best_inc + 1])
        with np.errstate(divide="ignore", invalid="ignore"):
            delta = f32(f32(d1 - d3) / f32(f32(2.0) * f32(f32(d1 + d3) - f32(f32(2.0) * d2))))
        if delta < -1 or delta > 1:
            continue
        best_uR = f32(f32(scale[lvl]) * f32(f32(f32(sr) + f32(best_inc)) + delta))
        disp = f32(uL - best_uR)
        if disp >= min_d and disp < max_d:
            if disp <= 0:
                disp = f32(0.01)
                best_uR = f32(float(uL) - 0.01)
            depth[iL] = f32(f32(bf) / disp)
            uright[iL] = best_uR
            dist_idx.append((best_sad, iL))
    if dist_idx:  # F:734-747
        dist_idx.sort()
        median = f32(dist_idx[len(dist_idx) // 2][0])
        th = f32(f32(f32(1.5) * f32(1.4)) * median)
        for d, i in reversed(dist_idx):
            if f32(d) < th:
                break
            uright[i] = -1.0
            depth[i] = -1.0
    return uright, depth
