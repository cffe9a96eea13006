"""Frame::UndistortKeyPoints / ComputeImageBounds / AssignFeaturesToGrid
(Frame.cpp:241-259, :434-444, :462-530): the CPU restatement
(oracle/frame_ref.py) on its own and against the library (image bounds on
the host, undistortion and grid on the GPU) -- bit-exact."""
import math

import numpy as np
import pytest

import frame_ref
import orbgpu
import synth

# Examples/Monocular/TUM1.yaml
TUM1 = dict(fx=517.306408, fy=516.469215, cx=318.643040, cy=255.313989,
            dist=[0.262383, -0.953104, -0.005358, 0.002628, 1.163314])


def _distort(x, y, K, d):
    """Forward Brown-Conrady model on pixel coordinates (float64)."""
    fx, fy, cx, cy = K
    k1, k2, p1, p2, k3 = (list(d) + [0.0])[:5]
    u, v = (x - cx) / fx, (y - cy) / fy
    r2 = u * u + v * v
    rad = 1 + k1 * r2 + k2 * r2 * r2 + k3 * r2 ** 3
    ud = u * rad + 2 * p1 * u * v + p2 * (r2 + 2 * u * u)
    vd = v * rad + p1 * (r2 + 2 * v * v) + 2 * p2 * u * v
    return ud * fx + cx, vd * fy + cy


def _kps(n, w, h, seed):
    rng = np.random.default_rng(seed)
    k = np.zeros(n, orbgpu.KP_DTYPE)
    k["x"] = rng.uniform(20, w - 20, n).astype(np.float32)
    k["y"] = rng.uniform(20, h - 20, n).astype(np.float32)
    k["octave"] = rng.integers(0, 8, n)
    k["size"], k["angle"], k["response"], k["class_id"] = 31.0, 90.0, 12.0, -1
    return k


def test_oracle_undistort_inverts_the_distortion_model():
    K = (TUM1["fx"], TUM1["fy"], TUM1["cx"], TUM1["cy"])
    k = _kps(400, 640, 480, 1)
    un = frame_ref.undistort_keypoints(k, K, TUM1["dist"])
    xd, yd = _distort(un["x"].astype(np.float64), un["y"].astype(np.float64), K, TUM1["dist"])
    # five fixed-point iterations: sub-pixel, not exact, near the image corners
    assert np.median(np.hypot(xd - k["x"], yd - k["y"])) < 0.05
    np.testing.assert_array_equal(un["octave"], k["octave"])
    same = frame_ref.undistort_keypoints(k, K, [0.0, 0.1, 0, 0])  # dist[0] == 0: copy (Frame.cpp:465)
    np.testing.assert_array_equal(same, k)


def test_oracle_grid_matches_definition():
    k = _kps(900, 640, 480, 2)
    cells = frame_ref.assign_features_to_grid(k, (0.0, 640.0, 0.0, 480.0))
    flat = sorted(i for c in cells for i in c)
    assert flat == list(range(900))  # all inside for an undistorted camera
    for c, items in enumerate(cells):
        assert items == sorted(items)
        for i in items:
            px = int(math.floor(float(np.float32(k["x"][i]) * np.float32(64 / 640)) + 0.5))
            assert c // 48 == min(px, 63) or c // 48 == px


def test_image_bounds_host_vs_oracle():
    cam = orbgpu.Camera.make(TUM1["fx"], TUM1["fy"], TUM1["cx"], TUM1["cy"], TUM1["dist"])
    b = orbgpu.compute_image_bounds(cam, 640, 480)
    ref = frame_ref.image_bounds((TUM1["fx"], TUM1["fy"], TUM1["cx"], TUM1["cy"]), TUM1["dist"], 640, 480)
    got = np.array([b.min_x, b.max_x, b.min_y, b.max_y], np.float32)
    np.testing.assert_array_equal(got.view(np.uint32), np.array(ref, np.float32).view(np.uint32))
    b0 = orbgpu.compute_image_bounds(orbgpu.Camera.make(500, 500, 320, 240, [0, 0, 0, 0]), 640, 480)
    assert (b0.min_x, b0.max_x, b0.min_y, b0.max_y) == (0.0, 640.0, 0.0, 480.0)


@pytest.mark.gpu
def test_gpu_undistort_and_grid_vs_oracle():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    dev = torch.device("cuda", 0)
    K = (TUM1["fx"], TUM1["fy"], TUM1["cx"], TUM1["cy"])
    cam = orbgpu.Camera.make(*K, TUM1["dist"])
    cap, B = 1100, 3
    host = np.zeros((B, cap), orbgpu.KP_DTYPE)
    counts = np.array([1000, 0, 1097], np.int32)
    for b in range(B):
        host[b, : counts[b]] = _kps(int(counts[b]), 640, 480, 10 + b)
    kps = torch.from_numpy(host.view(np.float32).reshape(B, cap, 7)).to(dev)
    cnt = torch.from_numpy(counts).to(dev)
    un = torch.zeros_like(kps)
    orbgpu.undistort_keypoints_batch(cam, kps, cnt, un)
    bounds = orbgpu.compute_image_bounds(cam, 640, 480)
    starts = torch.zeros((B, 64 * 48 + 1), dtype=torch.int32, device=dev)
    items = torch.zeros((B, cap), dtype=torch.int32, device=dev)
    orbgpu.assign_features_to_grid_batch(bounds, un, cnt, starts, items)
    torch.cuda.synchronize()
    un_h = un.cpu().numpy().reshape(B, cap * 7).view(orbgpu.KP_DTYPE).reshape(B, cap)
    st, it = starts.cpu().numpy(), items.cpu().numpy()
    bref = (bounds.min_x, bounds.max_x, bounds.min_y, bounds.max_y)
    for b in range(B):
        n = counts[b]
        ref = frame_ref.undistort_keypoints(host[b, :n], K, TUM1["dist"])
        assert un_h[b, :n].tobytes() == ref.tobytes(), f"frame {b}: mvKeysUn differs"
        cells = frame_ref.assign_features_to_grid(ref, bref)
        for c in range(64 * 48):
            got = list(it[b, st[b, c]:st[b, c + 1]])
            assert got == cells[c], (b, c, got, cells[c])
