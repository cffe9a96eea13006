"""CPU restatement of the Frame set-up steps between extraction and matching:
Frame::UndistortKeyPoints, Frame::ComputeImageBounds and
Frame::AssignFeaturesToGrid / PosInGrid.

TEST INFRASTRUCTURE ONLY: the parity oracle for csrc/frame.hip.  Citations:
F = /root/reference/ORB-SLAM2/src/Frame.cpp.  cv::undistortPoints is OpenCV
2.4's cvUndistortPoints (third-party, absent from the image; restated from
its published algorithm, modules/imgproc/src/undistort.cpp): the camera and
distortion matrices converted to double, (x, y) normalised with 1/fx, 1/fy,
five fixed-point iterations x = (x0 - dx) * icdist, then projected with
P = K (R = identity): parity against a real OpenCV build is unpinned.
"""
from __future__ import annotations

import math

import numpy as np

f32, f64 = np.float32, np.float64
GRID_COLS, GRID_ROWS = 64, 48  # FRAME_GRID_COLS / ROWS (include/Frame.h:36-37)


def undistort_points(pts, K, dist):
    """cvUndistortPoints(src, dst, K, dist, R=NULL, P=K) on float points.
    K = (fx, fy, cx, cy) float32, dist = (k1, k2, p1, p2[, k3]) float32."""
    fx, fy, cx, cy = (f64(f32(v)) for v in K)
    k = [0.0] * 8
    for i, v in enumerate(dist):
        k[i] = f64(f32(v))
    ifx, ify = 1.0 / fx, 1.0 / fy
    out = np.zeros((len(pts), 2), np.float32)
    for i, (px, py) in enumerate(pts):
        x = (f64(f32(px)) - cx) * ifx
        y = (f64(f32(py)) - cy) * ify
        x0, y0 = x, y
        for _ in range(5):
            r2 = x * x + y * y
            icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2)
            dx = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x)
            dy = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y
            x = (x0 - dx) * icdist
            y = (y0 - dy) * icdist
        # RR = P * I = K: xx = fx*x + 0*y + cx, yy = 0*x + fy*y + cy, ww = 1/(0*x + 0*y + 1)
        xx = fx * x + 0.0 * y + cx
        yy = 0.0 * x + fy * y + cy
        ww = 1.0 / (0.0 * x + 0.0 * y + 1.0)
        out[i, 0] = f32(xx * ww)
        out[i, 1] = f32(yy * ww)
    return out


def undistort_keypoints(kps, K, dist):
    """Frame::UndistortKeyPoints (F:462-496): mvKeysUn."""
    un = kps.copy()
    if f32(dist[0]) == 0.0:
        return un
    p = undistort_points(np.stack([kps["x"], kps["y"]], 1), K, dist)
    un["x"], un["y"] = p[:, 0], p[:, 1]
    return un


def image_bounds(K, dist, cols, rows):
    """Frame::ComputeImageBounds (F:498-530): (minX, maxX, minY, maxY)."""
    if f32(dist[0]) != 0.0:
        c = undistort_points([(0.0, 0.0), (cols, 0.0), (0.0, rows), (cols, rows)], K, dist)
        return (min(c[0, 0], c[2, 0]), max(c[1, 0], c[3, 0]), min(c[0, 1], c[1, 1]), max(c[2, 1], c[3, 1]))
    return (f32(0.0), f32(cols), f32(0.0), f32(rows))


def c_roundf(v) -> int:
    v = float(v)
    return int(math.copysign(math.floor(abs(v) + 0.5), v))


def assign_features_to_grid(kps_un, bounds):
    """Frame::AssignFeaturesToGrid / PosInGrid (F:241-259, :434-444): a list
    of keypoint indices per cell (cell = col * GRID_ROWS + row), in index
    order; out-of-grid keypoints are left out."""
    min_x, max_x, min_y, max_y = (f32(b) for b in bounds)
    inv_w = f32(f32(GRID_COLS) / f32(max_x - min_x))
    inv_h = f32(f32(GRID_ROWS) / f32(max_y - min_y))
    cells = [[] for _ in range(GRID_COLS * GRID_ROWS)]
    for i in range(len(kps_un)):
        px = c_roundf(f32(f32(f32(kps_un[i]["x"]) - min_x) * inv_w))
        py = c_roundf(f32(f32(f32(kps_un[i]["y"]) - min_y) * inv_h))
        if px < 0 or px >= GRID_COLS or py < 0 or py >= GRID_ROWS:
            continue
        cells[px * GRID_ROWS + py].append(i)
    return cells
