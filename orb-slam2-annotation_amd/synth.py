"""Seeded synthetic mono/stereo image streams.

The reference's datasets (TUM fr1_xyz, KITTI 00, EuRoC MH_01) are not in the
repository, so every benchmark and parity test runs on these streams:

* a 2048x2048 base texture: 1/f background + 8000 random rectangles and
  ellipses with uniform-random intensities (dense enough that FAST finds
  thousands of candidates per 640x480 frame, like a real indoor sequence);
* frame t = a crop of the base texture centred at (1024 + 2t, 1024 + t),
  rotated by 0.5 deg * t (bilinear), plus N(0, 2^2) noise, clamped to u8.
  Consecutive frames therefore have true correspondences for matching;
* edge fixtures: a flat image (no keypoints) and i.i.d. uniform noise
  (maximum FAST candidate count).

Everything is numpy on the host; tests hand the same bytes to the oracle and
to the HIP path.
"""
from __future__ import annotations

import functools

import numpy as np

BASE_SIZE = 2048
N_SHAPES = 8000


def _upsample(a: np.ndarray, size: int) -> np.ndarray:
    """Bilinear upsample of a small square array to size x size."""
    n = a.shape[0]
    c = np.linspace(0, n - 1, size)
    i0 = np.floor(c).astype(np.int64)
    i1 = np.minimum(i0 + 1, n - 1)
    f = c - i0
    rows = a[i0] * (1 - f)[:, None] + a[i1] * f[:, None]
    return rows[:, i0] * (1 - f)[None, :] + rows[:, i1] * f[None, :]


def base_texture(seed: int = 0x0B5E) -> np.ndarray:
    """The 2048x2048 scene (cached per seed; callers must not modify it)."""
    return _base_texture(seed)


@functools.lru_cache(maxsize=4)
def _base_texture(seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    img = np.zeros((BASE_SIZE, BASE_SIZE), np.float64)
    amp = 60.0
    for n in (8, 16, 32, 64, 128, 256, 512, 1024):  # 1/f-like background
        img += amp * _upsample(rng.standard_normal((n, n)), BASE_SIZE)
        amp *= 0.6
    img += 128.0
    yy, xx = np.mgrid[0:256, 0:256]
    for _ in range(N_SHAPES):
        w, h = rng.integers(4, 96, size=2)
        x0 = int(rng.integers(0, BASE_SIZE - w))
        y0 = int(rng.integers(0, BASE_SIZE - h))
        val = float(rng.uniform(0, 255))
        if rng.random() < 0.5:
            img[y0:y0 + h, x0:x0 + w] = val
        else:
            cy, cx = (h - 1) / 2.0, (w - 1) / 2.0
            m = ((yy[:h, :w] - cy) / max(cy, 1)) ** 2 + ((xx[:h, :w] - cx) / max(cx, 1)) ** 2 <= 1.0
            img[y0:y0 + h, x0:x0 + w][m] = val
    return img


def render_frame(base: np.ndarray, t: int, width: int, height: int, seed: int = 0,
                 baseline_px: float = 0.0, noise_sigma: float = 2.0) -> np.ndarray:
    """Frame t of the stream (u8, height x width).  baseline_px shifts the
    virtual camera horizontally (right image of a stereo pair)."""
    th = np.deg2rad(0.5 * t)
    c, s = np.cos(th), np.sin(th)
    v, u = np.mgrid[0:height, 0:width].astype(np.float64)
    u -= (width - 1) / 2.0
    v -= (height - 1) / 2.0
    u += baseline_px
    cx = BASE_SIZE / 2 + 2.0 * t
    cy = BASE_SIZE / 2 + 1.0 * t
    sx = c * u - s * v + cx
    sy = s * u + c * v + cy
    x0 = np.clip(np.floor(sx).astype(np.int64), 0, BASE_SIZE - 2)
    y0 = np.clip(np.floor(sy).astype(np.int64), 0, BASE_SIZE - 2)
    fx = np.clip(sx - x0, 0, 1)
    fy = np.clip(sy - y0, 0, 1)
    val = (base[y0, x0] * (1 - fx) * (1 - fy) + base[y0, x0 + 1] * fx * (1 - fy)
           + base[y0 + 1, x0] * (1 - fx) * fy + base[y0 + 1, x0 + 1] * fx * fy)
    rng = np.random.default_rng((seed << 20) + t)
    val += rng.normal(0.0, noise_sigma, val.shape)
    return np.clip(np.rint(val), 0, 255).astype(np.uint8)


def mono_stream(n: int, width: int = 640, height: int = 480, seed: int = 0x0B5E,
                t0: int = 0) -> np.ndarray:
    """n consecutive frames, shape (n, height, width) u8."""
    base = base_texture(seed)
    return np.stack([render_frame(base, t0 + t, width, height, seed) for t in range(n)])


def stereo_stream(n: int, width: int, height: int, seed: int, baseline_px: float = 24.0) -> np.ndarray:
    """n stereo pairs, shape (n, 2, height, width): [:,0] left, [:,1] right."""
    base = base_texture(seed)
    return np.stack([np.stack([render_frame(base, t, width, height, seed),
                               render_frame(base, t, width, height, seed + 1, baseline_px)])
                     for t in range(n)])


def flat_image(width: int = 640, height: int = 480, value: int = 128) -> np.ndarray:
    return np.full((height, width), value, np.uint8)


def noise_image(width: int = 640, height: int = 480, seed: int = 7) -> np.ndarray:
    return np.random.default_rng(seed).integers(0, 256, (height, width), dtype=np.uint8)


TRAJ_PERIOD = 512  # frames of one back-and-forth pass of the benchmark camera


def trajectory_t(frame: int) -> int:
    """Camera parameter of global frame `frame` in benchmark streams: a
    triangle wave 0..255..0 (period TRAJ_PERIOD), so arbitrarily long streams
    stay inside the base texture and consecutive frames always move by one
    step (true (t-1, t) correspondences everywhere)."""
    h = TRAJ_PERIOD // 2
    m = frame % TRAJ_PERIOD
    return m if m < h else TRAJ_PERIOD - 1 - m


def torch_stream(n: int, width: int, height: int, seed: int = 0x0B5E, device="cuda", t0: int = 0,
                 noise_sigma: float = 2.0, pitch: int | None = None, chunk: int = 64, bounded: bool = False,
                 baseline_px: float = 0.0, noise_seed: int | None = None):
    """GPU-rendered version of mono_stream for benchmark batches (same scene
    geometry; bilinear sampling and noise come from torch, so frames are not
    byte-identical to mono_stream -- parity tests use the numpy renderer).
    Frames t0 .. t0+n-1; with bounded=True global frame f is rendered at
    trajectory_t(f) (long streams).  baseline_px shifts the virtual camera
    horizontally (right images of stereo pairs); noise_seed (default seed)
    seeds the sensor noise only.  Returns a (n, height,
    pitch) uint8 tensor (pitch >= width, zero padded).  Deterministic on a
    given device type for the same arguments."""
    import torch

    pitch = pitch or width
    base = torch.from_numpy(base_texture(seed)).to(device=device, dtype=torch.float32)[None, None]
    out = torch.zeros((n, height, pitch), dtype=torch.uint8, device=device)
    gen = torch.Generator(device=device)
    gen.manual_seed((seed if noise_seed is None else noise_seed) * 7919 + t0)
    v, u = torch.meshgrid(torch.arange(height, device=device, dtype=torch.float32),
                          torch.arange(width, device=device, dtype=torch.float32), indexing="ij")
    u = u - (width - 1) / 2.0 + baseline_px
    v = v - (height - 1) / 2.0
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        t = torch.arange(t0 + s, t0 + s + m, device=device, dtype=torch.float32)
        if bounded:
            t = torch.tensor([trajectory_t(int(f)) for f in range(t0 + s, t0 + s + m)], device=device,
                             dtype=torch.float32)
        th = torch.deg2rad(0.5 * t)[:, None, None]
        c, sn = torch.cos(th), torch.sin(th)
        sx = c * u - sn * v + (BASE_SIZE / 2 + 2.0 * t)[:, None, None]
        sy = sn * u + c * v + (BASE_SIZE / 2 + 1.0 * t)[:, None, None]
        grid = torch.stack([sx / (BASE_SIZE - 1) * 2 - 1, sy / (BASE_SIZE - 1) * 2 - 1], dim=-1)
        img = torch.nn.functional.grid_sample(base.expand(m, -1, -1, -1), grid, mode="bilinear",
                                              padding_mode="border", align_corners=True)[:, 0]
        img = img + noise_sigma * torch.randn(img.shape, generator=gen, device=device)
        out[s:s + m, :, :width] = img.round().clamp(0, 255).to(torch.uint8)
    return out


def torch_stereo_stream(n_pairs: int, width: int, height: int, baseline_px: float, seed: int = 0x5E7,
                        device="cuda", t0: int = 0, pitch: int | None = None):
    """Rectified stereo pairs t0 .. t0+n_pairs-1 of a bounded camera path
    (torch_stream geometry): a (2*n_pairs, height, pitch) uint8 tensor with
    the left image of pair p at 2p and the right one (camera shifted by
    baseline_px) at 2p+1 -- the layout orbgpu_stereo_matches_batch_device
    reads.  Deterministic for the same (n_pairs, t0, seed) on a device type."""
    import torch

    pitch = pitch or width
    left = torch_stream(n_pairs, width, height, seed, device, t0, pitch=pitch, bounded=True)
    right = torch_stream(n_pairs, width, height, seed, device, t0, pitch=pitch, bounded=True,
                         baseline_px=baseline_px, noise_seed=seed + 1)
    return torch.stack([left, right], dim=1).reshape(2 * n_pairs, height, pitch).contiguous()


def sim3_problem(n: int, inlier_frac: float, seed: int, fix_scale: bool = False, noise_px: float = 0.5):
    """Correspondences of a loop-closure Sim3Solver (Sim3Solver.cpp:37-107):
    points X2 in keyframe-2 camera coordinates (depth 2..12 m, in view), X1 =
    s R X2 + t for the inliers (plus pixel-level noise), random points in view
    for the outliers.  Octaves are drawn from the 8-level pyramid (sigma^2 =
    1.2^(2 octave)).  Returns dict(X1, X2, sigma2_1, sigma2_2, K1, K2, s, R,
    t, inlier)."""
    rng = np.random.default_rng(seed)
    K = np.array([517.3, 516.5, 318.6, 255.3], np.float64)
    s = 1.0 if fix_scale else float(rng.uniform(0.7, 1.4))
    ang = rng.uniform(-0.3, 0.3, size=3)  # moderate relative rotation
    cx, cy, cz = np.cos(ang)
    sx, sy, sz = np.sin(ang)
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    R = Rz @ Ry @ Rx
    t = rng.uniform(-0.5, 0.5, size=3)

    def in_view(m):
        z = rng.uniform(2.0, 12.0, size=m)
        u = rng.uniform(20, 620, size=m)
        v = rng.uniform(20, 460, size=m)
        return np.stack([(u - K[2]) / K[0] * z, (v - K[3]) / K[1] * z, z], 1)

    X2 = in_view(n)
    X1 = (s * (R @ X2.T)).T + t
    inl = rng.uniform(size=n) < inlier_frac
    # pixel noise on inliers: perturb X1 along the image plane
    z1 = X1[:, 2:3]
    X1[:, :2] += rng.normal(scale=noise_px, size=(n, 2)) / K[:2] * z1
    out = ~inl
    X1[out] = in_view(int(out.sum()))
    oct1 = rng.integers(0, 8, size=n)
    oct2 = rng.integers(0, 8, size=n)
    sig = np.float32(1.2) ** (2 * np.arange(8))
    return {"X1": X1.astype(np.float32), "X2": X2.astype(np.float32),
            "sigma2_1": sig[oct1].astype(np.float32), "sigma2_2": sig[oct2].astype(np.float32),
            "K1": K.astype(np.float32), "K2": K.astype(np.float32), "s": s, "R": R, "t": t, "inlier": inl}


def pnp_problem(n: int, inlier_frac: float, seed: int, noise_px: float = 0.5):
    """Relocalisation correspondences of a PnPsolver (PnPsolver.cpp:104-139):
    MapPoints in world coordinates seen by a camera at a random pose; inliers
    project to their keypoint (plus pixel noise), outliers to random pixels.
    Returns dict(P3w, P2, sigma2, cam=(fu, fv, uc, vc), R, t, inlier)."""
    rng = np.random.default_rng(seed)
    fu, fv, uc, vc = 517.3, 516.5, 318.6, 255.3
    ang = rng.uniform(-0.5, 0.5, size=3)
    cx, cy, cz = np.cos(ang)
    sx, sy, sz = np.sin(ang)
    R = (np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]]) @ np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]]) @
         np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]]))
    t = rng.uniform(-1, 1, size=3)
    z = rng.uniform(1.5, 10.0, size=n)
    u = rng.uniform(10, 630, size=n)
    v = rng.uniform(10, 470, size=n)
    Xc = np.stack([(u - uc) / fu * z, (v - vc) / fv * z, z], 1)
    P3w = (Xc - t) @ R  # R^T (Xc - t)
    inl = rng.uniform(size=n) < inlier_frac
    P2 = np.stack([u, v], 1) + rng.normal(scale=noise_px, size=(n, 2))
    P2[~inl] = np.stack([rng.uniform(0, 640, size=(~inl).sum()), rng.uniform(0, 480, size=(~inl).sum())], 1)
    octave = rng.integers(0, 8, size=n)
    sig = np.float32(1.2) ** (2 * np.arange(8))
    return {"P3w": P3w.astype(np.float32), "P2": P2.astype(np.float32), "sigma2": sig[octave].astype(np.float32),
            "cam": (fu, fv, uc, vc), "R": R, "t": t, "inlier": inl}


def synthetic_vocabulary(k: int, L: int, seed: int, flip: float = 0.22):
    """A DBoW2-shaped vocabulary tree in file (BFS) order: node descriptors
    derived from their parent's by flipping each bit with probability
    `flip`, leaves at depth L with positive idf-like weights.  Returns
    (parent, is_leaf, desc[n,32], weight) without the root (node 0)."""
    rng = np.random.default_rng(seed)
    parent, is_leaf, desc, weight = [], [], [], []
    root = rng.integers(0, 256, 32, dtype=np.uint8)
    level_nodes = [(0, root)]
    for depth in range(1, L + 1):
        nxt = []
        for pid, pdesc in level_nodes:
            for _ in range(k):
                bits = np.unpackbits(pdesc)
                m = rng.uniform(size=256) < flip
                d = np.packbits(bits ^ m.astype(np.uint8))
                nid = len(parent) + 1
                parent.append(pid)
                is_leaf.append(1 if depth == L else 0)
                desc.append(d)
                weight.append(float(rng.uniform(0.5, 5.0)) if depth == L else 0.0)
                nxt.append((nid, d))
        level_nodes = nxt
    return (np.array(parent, np.int32), np.array(is_leaf, np.int32), np.array(desc, np.uint8),
            np.array(weight, np.float64))


def write_vocabulary_text(path, k, L, scoring, weighting, parent, is_leaf, desc, weight, trailing_newline=False):
    """DBoW2 text format: 'k L scoring weighting', then 'parent isLeaf d0..d31
    weight' per node (no trailing newline unless asked: the reference loader
    turns it into a spurious node)."""
    lines = [f"{k} {L} {scoring} {weighting}"]
    for i in range(len(parent)):
        lines.append(f"{parent[i]} {is_leaf[i]} " + " ".join(str(int(b)) for b in desc[i]) + " " + repr(float(weight[i])))
    with open(path, "w") as f:
        f.write("\n".join(lines) + ("\n" if trailing_newline else ""))


def write_vocabulary_binary(path, k, L, scoring, weighting, parent, is_leaf, desc, weight):
    """DBoW2 binary vocabulary as saveToBinaryFile writes it
    (TemplatedVocabulary.h:1527-1548): u32 nb_nodes (root included), u32
    size_node = 41, int k, L, scoring, weighting, then per node after the root
    int parent, 32 descriptor bytes, float weight, bool isLeaf."""
    n = len(parent)
    rec = np.zeros(n, dtype=np.dtype([("parent", "<i4"), ("desc", "u1", 32), ("weight", "<f4"), ("leaf", "u1")]))
    rec["parent"] = np.asarray(parent, np.int32)
    rec["desc"] = np.asarray(desc, np.uint8)
    rec["weight"] = np.asarray(weight, np.float64).astype(np.float32)
    rec["leaf"] = (np.asarray(is_leaf) > 0).astype(np.uint8)
    assert rec.dtype.itemsize == 41
    with open(path, "wb") as f:
        f.write(np.array([n + 1, 41], "<u4").tobytes())
        f.write(np.array([k, L, scoring, weighting], "<i4").tobytes())
        f.write(rec.tobytes())


def bow_frame_pair(voc_desc_leaves: np.ndarray, n: int, shared: float, seed: int, flip: float = 0.04):
    """Two frames' descriptors for SearchByBoW: frame-2 feature j for
    j < shared*n is frame-1 feature perm[j] with a few bits flipped (true
    correspondences), the rest are fresh; descriptors start near random
    vocabulary leaves.  Angles: frame 2 = frame 1 + 10 deg for shared ones."""
    rng = np.random.default_rng(seed)
    base = voc_desc_leaves[rng.integers(0, len(voc_desc_leaves), n)]

    def jitter(d, p):
        bits = np.unpackbits(d, axis=1)
        m = (rng.uniform(size=bits.shape) < p).astype(np.uint8)
        return np.packbits(bits ^ m, axis=1)

    d1 = jitter(base, 0.08)
    a1 = rng.uniform(0, 360, n).astype(np.float32)
    ns = int(shared * n)
    perm = rng.permutation(n)
    d2 = jitter(voc_desc_leaves[rng.integers(0, len(voc_desc_leaves), n)], 0.08)
    a2 = rng.uniform(0, 360, n).astype(np.float32)
    d2[:ns] = jitter(d1[perm[:ns]], flip)
    a2[:ns] = np.mod(a1[perm[:ns]] + 10.0, 360.0).astype(np.float32)
    return d1, a1, d2, a2


def _pose(rng, max_angle=0.3, max_t=0.5):
    ang = rng.uniform(-max_angle, max_angle, size=3)
    cx, cy, cz = np.cos(ang)
    sx, sy, sz = np.sin(ang)
    R = (np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]]) @ np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]]) @
         np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]]))
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = rng.uniform(-max_t, max_t, size=3)
    return T


def projection_scenario(n_points: int, n_distractors: int, seed: int, stereo: bool = False, scale: float = 1.0):
    """A frame observing map points, for the SearchByProjection variants:
    world points in front of the camera (Tcw), keypoints at their projections
    (pixel noise, octave = the level PredictScale gives, descriptor = the
    point's with a few bits flipped) plus distractor keypoints (random, some
    with descriptors close to points').  Returns (target dict, points dict)
    in the layouts of proj.py / proj_ref.py; `scale` != 1 makes Tcw a Sim3."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = 517.3, 516.5, 318.6, 255.3
    W, H = 640, 480
    T = _pose(rng)
    Rcw, tcw = T[:3, :3], T[:3, 3]
    z = rng.uniform(1.0, 8.0, size=n_points)
    u = rng.uniform(-20, W + 20, size=n_points)
    v = rng.uniform(-20, H + 20, size=n_points)
    Xc = np.stack([(u - cx) / fx * z, (v - cy) / fy * z, z], 1)
    Xw = (Xc - tcw) @ Rcw
    Ow = -Rcw.T @ tcw
    dist = np.linalg.norm(Xw - Ow, axis=1)
    lvl_ref = rng.integers(0, 8, size=n_points)
    sf = (np.float32(1.2) ** np.arange(8)).astype(np.float32)
    max_dist = (dist * rng.uniform(0.9, 1.1, n_points) * sf[lvl_ref]).astype(np.float32)
    min_dist = (max_dist / sf[7]).astype(np.float32)
    view = (Xw - Ow) / dist[:, None]  # MapPoint normal: mean camera-to-point direction
    normal = view + rng.normal(scale=0.15, size=view.shape)
    normal = (normal / np.linalg.norm(normal, axis=1)[:, None]).astype(np.float32)
    pdesc = rng.integers(0, 256, (n_points, 32), dtype=np.uint8)
    pangle = rng.uniform(0, 360, n_points).astype(np.float32)
    kps, kdesc = [], []
    for i in range(n_points):
        if not (0 <= u[i] < W and 0 <= v[i] < H) or rng.uniform() < 0.2:
            continue
        ratio = max_dist[i] / dist[i]
        lv = int(np.clip(np.ceil(np.log(ratio) / np.log(1.2)), 0, 7)) + int(rng.integers(-1, 2))
        lv = int(np.clip(lv, 0, 7))
        bits = np.unpackbits(pdesc[i])
        bits ^= (rng.uniform(size=256) < 0.06).astype(np.uint8)
        kps.append((u[i] + rng.normal(scale=0.8), v[i] + rng.normal(scale=0.8), 31 * sf[lv],
                    (pangle[i] + 15.0 + rng.normal(scale=2.0)) % 360.0, 0.0, lv, -1))
        kdesc.append(np.packbits(bits))
    for _ in range(n_distractors):
        j = int(rng.integers(0, n_points))
        near = rng.uniform() < 0.5
        x0 = u[j] + rng.normal(scale=6) if near else rng.uniform(0, W)
        y0 = v[j] + rng.normal(scale=6) if near else rng.uniform(0, H)
        bits = np.unpackbits(pdesc[j])
        bits ^= (rng.uniform(size=256) < (0.2 if near else 0.5)).astype(np.uint8)
        lv = int(rng.integers(0, 8))
        kps.append((np.clip(x0, 0, W - 1), np.clip(y0, 0, H - 1), 31 * sf[lv], rng.uniform(0, 360), 0.0, lv, -1))
        kdesc.append(np.packbits(bits))
    order = rng.permutation(len(kps))
    kp_arr = np.zeros(len(kps), dtype=[("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                                       ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
    for o, i in enumerate(order):
        kp_arr[o] = kps[i]
    kdesc = np.array(kdesc, np.uint8)[order]
    Tcw = T.copy()
    if scale != 1.0:
        Tcw[:3, :] *= scale
    tgt = {"kps": kp_arr, "desc": kdesc,
           "u_right": np.where(rng.uniform(size=len(kp_arr)) < 0.5, kp_arr["x"] - rng.uniform(5, 40, len(kp_arr)),
                               -1.0).astype(np.float32) if stereo else None,
           "occupied": (rng.integers(0, 3, len(kp_arr)) * (rng.uniform(size=len(kp_arr)) < 0.15)).astype(np.uint8),
           "min_x": 0.0, "max_x": float(W), "min_y": 0.0, "max_y": float(H), "fx": fx, "fy": fy, "cx": cx, "cy": cy,
           "bf": 40.0, "b": 0.08, "n_levels": 8, "log_scale_factor": float(np.log(np.float32(1.2))),
           "scale_factors": sf, "Tcw": Tcw.astype(np.float32)}
    flags = np.where(rng.uniform(size=n_points) < 0.9, 1, 0) | np.where(rng.uniform(size=n_points) < 0.9, 2, 0)
    pts = {"flags": flags.astype(np.int32), "pos": Xw.astype(np.float32),
           "normal": normal, "desc": pdesc, "min_dist": min_dist, "max_dist": max_dist,
           "octave": lvl_ref.astype(np.int32), "angle": pangle}
    return tgt, pts



def _kf_target(kps, desc, T, rng, stereo=False):
    """a keyframe dict in the layout of proj.py / proj_ref.py"""
    fx, fy, cx, cy = 517.3, 516.5, 318.6, 255.3
    sf = (np.float32(1.2) ** np.arange(8)).astype(np.float32)
    kp_arr = np.zeros(len(kps), dtype=[("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                                       ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
    for o, k in enumerate(kps):
        kp_arr[o] = k
    return {"kps": kp_arr, "desc": np.array(desc, np.uint8).reshape(-1, 32),
            "u_right": np.where(rng.uniform(size=len(kp_arr)) < 0.5, kp_arr["x"] - rng.uniform(5, 40, len(kp_arr)),
                                -1.0).astype(np.float32) if stereo else None,
            "occupied": None, "min_x": 0.0, "max_x": 640.0, "min_y": 0.0, "max_y": 480.0, "fx": fx, "fy": fy,
            "cx": cx, "cy": cy, "bf": 40.0, "b": 0.08, "n_levels": 8,
            "log_scale_factor": float(np.log(np.float32(1.2))), "scale_factors": sf,
            "Tcw": np.asarray(T, np.float32)}


def sim3_search_scenario(n_points: int, n_distractors: int, seed: int, s12: float = 1.15,
                         already: float = 0.15, bad: float = 0.05):
    """Two keyframes of a loop (ORBmatcher::SearchBySim3): world points seen by
    KF1 (map 1) and, through the similarity S12 = [s12 R12 | t12] (camera 2 ->
    camera 1), by KF2 in its own map.  Every keypoint carries a MapPoint
    entry (one per keypoint; distractor keypoints have none); `already` of
    the common points are marked as matched in both (vbAlreadyMatched1/2)
    and `bad` as isBad().  pts*["flags"] are the oracle's (VALID = non-NULL,
    good, not already matched); pts*["null"] / ["bad"] and pts1["pre"] (the
    KF2 slot already matched to each KF1 slot, or -1) describe the same state
    for the C++ class.  Returns (kf1, kf2, pts1, pts2, s12, R12, t12)."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = 517.3, 516.5, 318.6, 255.3
    sf = (np.float32(1.2) ** np.arange(8)).astype(np.float32)
    T1 = _pose(rng)
    R12 = _rot(rng, 0.2)
    t12 = rng.uniform(-0.3, 0.3, 3)
    z = rng.uniform(1.5, 8.0, n_points)
    u = rng.uniform(-20, 660, n_points)
    v = rng.uniform(-20, 500, n_points)
    pc1 = np.stack([(u - cx) / fx * z, (v - cy) / fy * z, z], 1)
    X1 = (pc1 - T1[:3, 3]) @ T1[:3, :3]
    pc2 = ((pc1 - t12) @ R12) / s12  # p3Dc1 = s12 R12 p3Dc2 + t12
    T2 = _pose(rng)
    X2 = (pc2 - T2[:3, 3]) @ T2[:3, :3]
    pdesc = rng.integers(0, 256, (n_points, 32), dtype=np.uint8)
    lvl_ref = rng.integers(0, 8, n_points)
    common = rng.uniform(size=n_points) < 0.6

    def view(pc, X, only):
        kps, desc, owner = [], [], []
        d = np.linalg.norm(pc, axis=1)
        maxd = (d * rng.uniform(0.9, 1.1, n_points) * sf[lvl_ref]).astype(np.float32)
        for i in range(n_points):
            if only is not None and not only[i]:
                continue
            if pc[i, 2] <= 0:
                continue
            uu, vv = fx * pc[i, 0] / pc[i, 2] + cx, fy * pc[i, 1] / pc[i, 2] + cy
            if not (0 <= uu < 640 and 0 <= vv < 480):
                continue
            lv = int(np.clip(np.ceil(np.log(maxd[i] / d[i]) / np.log(1.2)), 0, 7)) + int(rng.integers(-1, 2))
            lv = int(np.clip(lv, 0, 7))
            bits = np.unpackbits(pdesc[i])
            bits ^= (rng.uniform(size=256) < 0.06).astype(np.uint8)
            kps.append((uu + rng.normal(scale=0.7), vv + rng.normal(scale=0.7), 31 * sf[lv], rng.uniform(0, 360),
                        0.0, lv, -1))
            desc.append(np.packbits(bits))
            owner.append(i)
        for _ in range(n_distractors):
            j = int(rng.integers(0, n_points))
            bits = np.unpackbits(pdesc[j])
            bits ^= (rng.uniform(size=256) < 0.25).astype(np.uint8)
            lv = int(rng.integers(0, 8))
            kps.append((rng.uniform(0, 639), rng.uniform(0, 479), 31 * sf[lv], rng.uniform(0, 360), 0.0, lv, -1))
            desc.append(np.packbits(bits))
            owner.append(-1)
        order = rng.permutation(len(kps))
        kps = [kps[o] for o in order]
        desc = [desc[o] for o in order]
        owner = np.array(owner, np.int64)[order]
        n = len(kps)
        pts = {"flags": np.zeros(n, np.int32), "pos": np.zeros((n, 3), np.float32),
               "desc": np.zeros((n, 32), np.uint8), "min_dist": np.zeros(n, np.float32),
               "max_dist": np.zeros(n, np.float32), "normal": np.zeros((n, 3), np.float32)}
        pts["null"] = owner < 0
        pts["bad"] = np.zeros(n, bool)
        pts["pre"] = np.full(n, -1, np.int32)
        for k_, i in enumerate(owner):
            if i < 0:
                continue
            pts["bad"][k_] = rng.uniform() < bad
            pts["flags"][k_] = 0 if pts["bad"][k_] else 1
            pts["pos"][k_] = X[i]
            pts["desc"][k_] = pdesc[i]
            pts["max_dist"][k_] = maxd[i]
            pts["min_dist"][k_] = maxd[i] / sf[7]
        return kps, desc, owner, pts

    k1, d1, own1, pts1 = view(pc1, X1, None)
    k2, d2, own2, pts2 = view(pc2, X2, common)
    # vbAlreadyMatched1/2: some common points matched before the call (SearchByBoW)
    where2 = {int(i): k_ for k_, i in enumerate(own2) if i >= 0}
    for k_, i in enumerate(own1):
        if i >= 0 and int(i) in where2 and rng.uniform() < already:
            pts1["flags"][k_] = 0
            pts2["flags"][where2[int(i)]] = 0
            pts1["pre"][k_] = where2[int(i)]  # vpMatches12[k_] = KF2's MapPoint at that slot
    kf1 = _kf_target(k1, d1, T1, rng)
    kf2 = _kf_target(k2, d2, T2, rng)
    return kf1, kf2, pts1, pts2, np.float32(s12), R12.astype(np.float32), t12.astype(np.float32)


def triangulation_scenario(voc_desc_leaves: np.ndarray, n_points: int, seed: int, n_distractors: int = 200,
                           tracked: float = 0.3, stereo: bool = False):
    """Two neighbouring keyframes for LocalMapping::CreateNewMapPoints ->
    ORBmatcher::SearchForTriangulation: world points projected into both
    (descriptors near vocabulary leaves, so the direct-index nodes agree),
    `tracked` of the keypoints already carry a MapPoint (skipped), F12 from
    the poses as LocalMapping::ComputeF12 forms it (LocalMapping.cpp:697-713).
    Returns a dict of the pair's host arrays."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = 517.3, 516.5, 318.6, 255.3
    K = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]])
    sf = (np.float32(1.2) ** np.arange(8)).astype(np.float32)
    T1 = _pose(rng, 0.1, 0.1)
    T2 = T1.copy()
    T2[:3, :3] = _rot(rng, 0.08) @ T1[:3, :3]
    T2[:3, 3] = T1[:3, 3] + rng.uniform(-0.4, 0.4, 3)
    z = rng.uniform(2.0, 10.0, n_points)
    u = rng.uniform(0, 640, n_points)
    v = rng.uniform(0, 480, n_points)
    pc1 = np.stack([(u - cx) / fx * z, (v - cy) / fy * z, z], 1)
    Xw = (pc1 - T1[:3, 3]) @ T1[:3, :3]
    pc2 = Xw @ T2[:3, :3].T + T2[:3, 3]
    base = voc_desc_leaves[rng.integers(0, len(voc_desc_leaves), n_points)]

    def jitter(d, p):
        bits = np.unpackbits(d, axis=1)
        return np.packbits(bits ^ (rng.uniform(size=bits.shape) < p).astype(np.uint8), axis=1)

    def frame(pc, only):
        kps, desc, ang = [], [], []
        for i in range(n_points):
            if only is not None and not only[i]:
                continue
            if pc[i, 2] <= 0:
                continue
            uu, vv = fx * pc[i, 0] / pc[i, 2] + cx, fy * pc[i, 1] / pc[i, 2] + cy
            if not (0 <= uu < 640 and 0 <= vv < 480):
                continue
            lv = int(rng.integers(0, 8))
            kps.append((uu + rng.normal(scale=0.6), vv + rng.normal(scale=0.6), 31 * sf[lv], 0.0, 0.0, lv, -1))
            desc.append(jitter(base[i:i + 1], 0.03)[0])
            ang.append(float(i * 37 % 360))
        for _ in range(n_distractors):
            lv = int(rng.integers(0, 8))
            kps.append((rng.uniform(0, 639), rng.uniform(0, 479), 31 * sf[lv], 0.0, 0.0, lv, -1))
            desc.append(jitter(base[int(rng.integers(0, n_points)):][:1], 0.15)[0])
            ang.append(rng.uniform(0, 360))
        order = rng.permutation(len(kps))
        k = np.zeros(len(kps), dtype=[("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                                      ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
        for o, j in enumerate(order):
            k[o] = kps[j]
        k["angle"] = (np.array(ang)[order] + rng.normal(scale=1.0, size=len(order))) % 360.0
        return k, np.array(desc, np.uint8)[order]

    k1, d1 = frame(pc1, None)
    k2, d2 = frame(pc2, rng.uniform(size=n_points) < 0.8)
    # F12 = K1^-T [t12]x R12 K2^-1 (ComputeF12), with R12 = R1w R2w^T, t12 = -R12 t2w + t1w
    R12 = T1[:3, :3] @ T2[:3, :3].T
    t12 = -R12 @ T2[:3, 3] + T1[:3, 3]
    tx = np.array([[0, -t12[2], t12[1]], [t12[2], 0, -t12[0]], [-t12[1], t12[0], 0]])
    F12 = (np.linalg.inv(K).T @ tx @ R12 @ np.linalg.inv(K)).astype(np.float32)
    Cw1 = (-T1[:3, :3].T @ T1[:3, 3]).astype(np.float32)
    sig2 = (sf * sf).astype(np.float32)
    ur = lambda k: (np.where(rng.uniform(size=len(k)) < 0.5, k["x"] - rng.uniform(5, 40, len(k)), -1.0)  # noqa: E731
                    .astype(np.float32) if stereo else None)
    return {"kps1": k1, "kps2": k2, "desc1": d1, "desc2": d2,
            "valid1": (rng.uniform(size=len(k1)) >= tracked).astype(np.uint8),
            "valid2": (rng.uniform(size=len(k2)) >= tracked).astype(np.uint8),
            "u_right1": ur(k1), "u_right2": ur(k2), "F12": F12, "Cw1": Cw1,
            "T2w": T2[:3, :].astype(np.float32), "fx2": fx, "fy2": fy, "cx2": cx, "cy2": cy,
            "scale_factors2": sf, "level_sigma2_2": sig2}


def mapping_scenario(n_points: int, seed: int, stereo: bool = False, outliers: float = 0.15,
                     baseline: float = 0.4):
    """Two keyframes for LocalMapping::CreateNewMapPoints: world points seen
    by both (pixel noise, octaves from the distance), matched pairs (idx1,
    idx2) with `outliers` of them pointing at a wrong keypoint; stereo
    keyframes carry mvuRight / mvDepth for about half of the keypoints.
    Returns (kf1, kf2, pairs, scale_factor) in proj/mapping_ref layouts."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy, bf = 517.3, 516.5, 318.6, 255.3, 40.0
    sf = (np.float32(1.2) ** np.arange(8)).astype(np.float32)
    T1 = _pose(rng, 0.1, 0.2)
    T2 = T1.copy()
    T2[:3, :3] = _rot(rng, 0.05) @ T1[:3, :3]
    T2[:3, 3] = T1[:3, 3] + rng.uniform(-baseline, baseline, 3)
    z = rng.uniform(1.5, 12.0, n_points)
    u = rng.uniform(0, 640, n_points)
    v = rng.uniform(0, 480, n_points)
    pc1 = np.stack([(u - cx) / fx * z, (v - cy) / fy * z, z], 1)
    Xw = (pc1 - T1[:3, 3]) @ T1[:3, :3]
    pc2 = Xw @ T2[:3, :3].T + T2[:3, 3]

    def kf(T, pc):
        kp = np.zeros(n_points, dtype=[("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                                       ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
        kp["x"] = fx * pc[:, 0] / pc[:, 2] + cx + rng.normal(0, 0.6, n_points)
        kp["y"] = fy * pc[:, 1] / pc[:, 2] + cy + rng.normal(0, 0.6, n_points)
        kp["octave"] = np.clip(np.log(pc[:, 2] / 1.5) / np.log(1.2) * 0.5 + rng.integers(-1, 2, n_points), 0, 7)
        kp["size"] = 31 * sf[kp["octave"]]
        kp["class_id"] = -1
        d = {"Tcw": T[:3, :].astype(np.float32), "Ow": (-T[:3, :3].T @ T[:3, 3]).astype(np.float32),
             "fx": fx, "fy": fy, "cx": cx, "cy": cy, "invfx": float(np.float32(1) / np.float32(fx)),
             "invfy": float(np.float32(1) / np.float32(fy)), "bf": bf, "b": bf / fx, "kps_un": kp, "kps": kp,
             "u_right": None, "depth": None, "scale_factors": sf, "level_sigma2": (sf * sf).astype(np.float32)}
        if stereo:
            has = rng.uniform(size=n_points) < 0.5
            depth = np.where(has, pc[:, 2] * (1 + rng.normal(0, 0.002, n_points)), -1.0).astype(np.float32)
            d["depth"] = depth
            d["u_right"] = np.where(has, kp["x"] - bf / np.where(has, depth, 1.0), -1.0).astype(np.float32)
        return d

    k1, k2 = kf(T1, pc1), kf(T2, pc2)
    order2 = rng.permutation(n_points)  # kf2's keypoints in another order
    for key in ("kps_un", "u_right", "depth"):
        if k2[key] is not None:
            k2[key] = k2[key][order2]
    k2["kps"] = k2["kps_un"]
    inv2 = np.argsort(order2)
    idx1 = rng.permutation(n_points)[: int(0.8 * n_points)]
    idx2 = inv2[idx1]
    bad = rng.uniform(size=len(idx1)) < outliers
    idx2 = np.where(bad, rng.integers(0, n_points, len(idx1)), idx2)
    pairs = np.stack([idx1, idx2], 1).astype(np.int32)
    return k1, k2, pairs, 1.2

# --------------------------------------------------------------------------
# Loop-closure burst
# --------------------------------------------------------------------------
def synthetic_vocabulary_fast(k: int, L: int, seed: int, flip: float = 0.22):
    """synthetic_vocabulary for large trees (k=10, L=6: 1,111,110 nodes),
    vectorised per level: same BFS file order and construction (children
    are their parent's descriptor with each bit flipped with probability
    `flip`), leaf weights quantised to 1e-6 so the text form is exact.
    Returns (parent, is_leaf, desc[n,32], weight) without the root."""
    rng = np.random.default_rng(seed)
    root = rng.integers(0, 256, 32, dtype=np.uint8)
    prev_desc = root[None]
    prev_ids = np.zeros(1, np.int64)
    next_id = 1
    parents, leaves, descs, weights = [], [], [], []
    thr = int(round(flip * 65536))
    for depth in range(1, L + 1):
        n = len(prev_ids) * k
        desc = np.repeat(prev_desc, k, axis=0)
        for s in range(0, n, 1 << 17):  # bit flips in chunks (bounded memory)
            e = min(n, s + (1 << 17))
            m = rng.integers(0, 65536, (e - s, 256), dtype=np.uint16) < thr
            desc[s:e] ^= np.packbits(m, axis=1)
        parents.append(np.repeat(prev_ids, k).astype(np.int32))
        leaves.append(np.full(n, 1 if depth == L else 0, np.int32))
        descs.append(desc)
        if depth == L:
            weights.append(np.round(rng.uniform(0.5, 5.0, n), 6))
        else:
            weights.append(np.zeros(n))
        prev_desc = desc
        prev_ids = np.arange(next_id, next_id + n, dtype=np.int64)
        next_id += n
    return (np.concatenate(parents), np.concatenate(leaves), np.concatenate(descs),
            np.concatenate(weights).astype(np.float64))


def write_vocabulary_text_fast(path, k, L, scoring, weighting, parent, is_leaf, desc, weight):
    """DBoW2 text vocabulary (TemplatedVocabulary.h:1359-1448 reads it with
    stream extraction, so fixed-width space-padded fields are the same
    file to the loader): one line per node, no trailing newline.  Weights
    must be multiples of 1e-6 (written with 6 decimals, read back exactly
    as the nearest double by both loaders)."""
    n = len(parent)
    cols = []

    def digits(v, width):  # right-aligned decimal, space padded, then a space
        v = np.asarray(v, np.int64)
        out = np.full((len(v), width + 1), ord(" "), np.uint8)
        rem = v.copy()
        for c in range(width - 1, -1, -1):
            d = (rem % 10).astype(np.uint8) + ord("0")
            show = (rem > 0) | (c == width - 1)
            out[:, c] = np.where(show, d, ord(" "))
            rem //= 10
        return out

    cols.append(digits(parent, 8))
    cols.append(digits(is_leaf, 1))
    for j in range(32):
        cols.append(digits(desc[:, j], 3))
    w6 = np.round(np.asarray(weight) * 1e6).astype(np.int64)
    ip, fp = w6 // 1000000, w6 % 1000000
    wi = digits(ip, 3)[:, :3]
    dot = np.full((n, 1), ord("."), np.uint8)
    frac = np.zeros((n, 6), np.uint8)
    rem = fp.copy()
    for c in range(5, -1, -1):
        frac[:, c] = (rem % 10).astype(np.uint8) + ord("0")
        rem //= 10
    nl = np.full((n, 1), ord("\n"), np.uint8)
    rows = np.concatenate(cols + [wi, dot, frac, nl], axis=1)
    with open(path, "wb") as f:
        f.write(f"{k} {L} {scoring} {weighting}\n".encode())
        f.write(rows.tobytes()[:-1])  # no trailing newline


def _rot(rng, max_angle):
    a = rng.uniform(-max_angle, max_angle, 3)
    cx, cy, cz = np.cos(a)
    sx, sy, sz = np.sin(a)
    return (np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]]) @ np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]]) @
            np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]]))


def level_sigma2(nlevels: int = 8, scale: float = 1.2) -> np.ndarray:
    """mvLevelSigma2 of the extractor (ORBextractor.cpp:412-425, float chain)."""
    s = np.ones(nlevels, np.float32)
    for i in range(1, nlevels):
        s[i] = np.float32(s[i - 1] * np.float32(scale))
    return (s * s).astype(np.float32)


def loop_burst_scene(n_queries: int, n_cand: int, leaves: np.ndarray, n_kp: int = 1000, inlier_frac=0.4,
                     outlier_frac=0.0, mp_frac: float = 0.9, seed: int = 0x100B, fix_scale: bool = False,
                     noise_px: float = 0.4):
    """Keyframes for LoopClosing::ComputeSim3 bursts: query q has a current
    keyframe (index q) and n_cand loop candidates (index n_queries +
    q*n_cand + c).  A candidate shares round(inlier_frac * n_kp) keypoints
    with its current keyframe -- same MapPoint under a known Sim3 S12 (X1 =
    s R X2 + t in the two camera frames, plus pixel-level noise),
    descriptors a few bits apart, angles rotated by 10 deg -- and the rest
    are unrelated, except round(outlier_frac * n_kp) more that copy a
    current-keyframe descriptor (they match) but carry an unrelated MapPoint
    (geometric outliers, the "rest outliers" of the burst config).
    inlier_frac / outlier_frac are scalars or one value per candidate slot.
    Descriptors start near random vocabulary leaves (so they spread over
    the tree); keypoint octaves follow the extractor's per-level quotas;
    mp_frac of the keypoints carry a MapPoint.  Returns a dict of arrays."""
    rng = np.random.default_rng(seed)
    K = np.array([517.3, 516.5, 318.6, 255.3], np.float32)
    sig2 = level_sigma2()
    quota = np.array([217, 181, 151, 126, 105, 87, 73, 60], np.float64)
    fracs = np.broadcast_to(np.asarray(inlier_frac, np.float64), (n_cand,))
    ofracs = np.broadcast_to(np.asarray(outlier_frac, np.float64), (n_cand,))
    n_kf = n_queries * (1 + n_cand)
    desc = np.zeros((n_kf, n_kp, 32), np.uint8)
    angle = np.zeros((n_kf, n_kp), np.float32)
    octave = np.zeros((n_kf, n_kp), np.int32)
    valid = np.zeros((n_kf, n_kp), np.uint8)
    mp = np.zeros((n_kf, n_kp, 3), np.float32)
    Tcw = np.zeros((n_kf, 12), np.float32)
    truth = []

    def jitter(d, p):
        bits = np.unpackbits(d, axis=-1)
        m = (rng.random(bits.shape) < p).astype(np.uint8)
        return np.packbits(bits ^ m, axis=-1)

    def cam_points(m):
        z = rng.uniform(2.0, 12.0, m)
        u = rng.uniform(10, 630, m)
        v = rng.uniform(10, 470, m)
        return np.stack([(u - K[2]) / K[0] * z, (v - K[3]) / K[1] * z, z], 1)

    def fresh(kf):
        desc[kf] = jitter(leaves[rng.integers(0, len(leaves), n_kp)], 0.08)
        angle[kf] = rng.uniform(0, 360, n_kp).astype(np.float32)
        octave[kf] = rng.choice(8, n_kp, p=quota / quota.sum())
        valid[kf] = rng.random(n_kp) < mp_frac
        return cam_points(n_kp)

    def pose(kf, Xc):
        R, t = _rot(rng, 0.4), rng.uniform(-2, 2, 3)
        Tcw[kf, :9] = R.astype(np.float32).ravel()
        Tcw[kf, 9:] = t.astype(np.float32)
        mp[kf] = ((Xc - t) @ R).astype(np.float32)  # R^T (Xc - t)

    for q in range(n_queries):
        X1c = fresh(q)
        pose(q, X1c)
        for c in range(n_cand):
            kf = n_queries + q * n_cand + c
            X2c = fresh(kf)
            s = 1.0 if fix_scale else float(rng.uniform(0.7, 1.4))
            R12, t12 = _rot(rng, 0.3), rng.uniform(-0.5, 0.5, 3)
            cand1 = np.nonzero(valid[q])[0]
            ns = min(int(round(fracs[c] * n_kp)), len(cand1))
            no = min(int(round(ofracs[c] * n_kp)), len(cand1) - ns)
            pick = rng.choice(cand1, ns + no, replace=False)
            slots = rng.choice(n_kp, ns + no, replace=False)
            # geometric outliers: matching descriptors, unrelated MapPoints
            osrc, odst = pick[ns:], slots[ns:]
            desc[kf, odst] = jitter(desc[q, osrc], 0.03)
            angle[kf, odst] = np.mod(angle[q, osrc] - np.float32(10.0), np.float32(360.0)).astype(np.float32)
            octave[kf, odst] = octave[q, osrc]
            valid[kf, odst] = 1
            src, dst = pick[:ns], slots[:ns]
            Y = ((X1c[src] - t12) @ R12) / s  # X2 = R^T (X1 - t) / s
            Y[:, :2] += rng.normal(scale=noise_px, size=(ns, 2)) / K[:2] * Y[:, 2:3]
            ok = Y[:, 2] > 0.5
            src, dst, Y = src[ok], dst[ok], Y[ok]
            X2c[dst] = Y
            desc[kf, dst] = jitter(desc[q, src], 0.03)
            angle[kf, dst] = np.mod(angle[q, src] - np.float32(10.0), np.float32(360.0)).astype(np.float32)
            octave[kf, dst] = octave[q, src]
            valid[kf, dst] = 1
            pose(kf, X2c)
            truth.append({"s": s, "R": R12, "t": t12, "src": src, "dst": dst, "outlier_src": osrc,
                          "outlier_dst": odst})
    return {"desc": desc, "angle": angle, "octave": octave, "valid": valid, "mp_world": mp, "Tcw": Tcw, "K": K,
            "sigma2": sig2, "n_queries": n_queries, "n_cand": n_cand, "truth": truth}


def mappoint_scenario(n_points: int, seed: int, max_obs: int = 40, bad_frac: float = 0.15, flip: float = 0.06):
    """Points with CSR observations for ComputeDistinctiveDescriptors /
    UpdateNormalAndDepth: each point's descriptors are noisy copies of one
    base descriptor (a few outliers); camera centres around the point; sizes
    0, 1, 2 and up to max_obs observations; some keyframes bad."""
    rng = np.random.default_rng(seed)
    counts = rng.integers(0, max_obs + 1, n_points)
    counts[: min(n_points, 4)] = [0, 1, 2, 3][: min(n_points, 4)]
    off = np.zeros(n_points + 1, np.int32)
    off[1:] = np.cumsum(counts)
    n_obs = int(off[-1])
    base = rng.integers(0, 256, (n_points, 32), dtype=np.uint8)
    owner = np.repeat(np.arange(n_points), counts)
    bits = (rng.uniform(size=(n_obs, 256)) < flip).astype(np.uint8)
    desc = base[owner] ^ np.packbits(bits, axis=1)
    outl = rng.uniform(size=n_obs) < 0.1
    desc[outl] = rng.integers(0, 256, (int(outl.sum()), 32), dtype=np.uint8)
    valid = (rng.uniform(size=n_obs) >= bad_frac).astype(np.uint8)
    pos = rng.normal(0, 5, (n_points, 3)).astype(np.float32)
    obs_Ow = (pos[owner] + rng.normal(0, 3, (n_obs, 3))).astype(np.float32)
    ref_Ow = (pos + rng.normal(0, 3, (n_points, 3))).astype(np.float32)
    sf = (1.2 ** np.arange(8)).astype(np.float32)
    level_scale = sf[rng.integers(0, 8, n_points)]
    max_scale = np.full(n_points, sf[7], np.float32)
    return dict(offsets=off, desc=desc, valid=valid, pos=pos, obs_Ow=obs_Ow, ref_Ow=ref_Ow,
                level_scale=level_scale, max_scale=max_scale)
