"""Frame::ComputeStereoMatches (Frame.cpp:540-748): the CPU restatement
(oracle/stereo_ref.py) on its own, and the HIP kernel (csrc/stereo.hip,
through the C ABI) against it on the same keypoints, descriptors and pyramid
levels -- bit-exact uRight / depth (and the same -1 set)."""
import numpy as np
import pytest

import orbref
import stereo_ref
import synth


def _stereo_pair(w, h, baseline, seed=0x51E0, t=3):
    base = synth.base_texture(seed)
    left = synth.render_frame(base, t, w, h, seed)
    right = synth.render_frame(base, t, w, h, seed + 1, baseline)
    return left, right


def _oracle(ex, left, right, bf, min_z=0.0):
    kl, dl = ex.extract(left)
    pl = [ex.level(l) for l in range(ex.nlevels)]
    kr, dr = ex.extract(right)
    pr = [ex.level(l) for l in range(ex.nlevels)]
    s, inv, _, _ = ex.scale_factors()
    ur, dp = stereo_ref.compute_stereo_matches(kl, dl, kr, dr, pl, pr, s, inv, bf, min_z)
    return kl, ur, dp


def test_oracle_recovers_baseline_disparity():
    """A right view rendered 24 px to the side: accepted matches have
    disparity ~24 px and depth = bf / disparity."""
    ex = orbref.Extractor(nfeatures=600)
    left, right = _stereo_pair(480, 360, 24.0)
    bf = 40.0
    kl, ur, dp = _oracle(ex, left, right, bf)
    ok = ur >= 0
    assert ok.sum() > 100, ok.sum()
    disp = kl["x"][ok] - ur[ok]
    assert np.median(np.abs(disp - 24.0)) < 1.0
    np.testing.assert_array_equal(dp[ok], (np.float32(bf) / disp.astype(np.float32)).astype(np.float32))
    # the median cut leaves no accepted match at or above 2.1 x the median SAD: checked indirectly by
    # rerunning with a finite max disparity smaller than the baseline -> nothing accepted
    _, ur2, _ = _oracle(ex, left, right, bf, min_z=bf / 10.0)
    assert (ur2 >= 0).sum() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,nf,baseline,bf", [(640, 480, 1000, 24.0, 40.0),
                                                (1241, 376, 2000, 30.0, 0.54 * 718.856),  # KITTI00-02.yaml Camera.bf
                                                (752, 480, 1200, 18.0, 47.90639384423901)])  # EuRoC.yaml Camera.bf
def test_gpu_stereo_matches_vs_oracle(w, h, nf, baseline, bf):
    torch = pytest.importorskip("torch")
    import orbgpu
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    pairs = [_stereo_pair(w, h, baseline, seed=0x51E0 + i, t=i) for i in range(2)]
    B = 2 * len(pairs)
    ex = orbgpu.Extractor(nfeatures=nf, width=w, height=h, max_batch=B)
    pitch = (w + 15) // 16 * 16
    host = np.zeros((B, h, pitch), np.uint8)
    for p, (l, r) in enumerate(pairs):
        host[2 * p, :, :w] = l
        host[2 * p + 1, :, :w] = r
    dev = torch.device("cuda", 0)
    imgs = torch.from_numpy(host).to(dev)
    cap = ex.max_keypoints
    kps = torch.zeros((B, cap, 7), dtype=torch.float32, device=dev)
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
    counts = torch.zeros(B, dtype=torch.int32, device=dev)
    ur = torch.full((len(pairs), cap), -7.0, dtype=torch.float32, device=dev)
    dp = torch.full((len(pairs), cap), -7.0, dtype=torch.float32, device=dev)
    ex.extract_batch(imgs, kps, desc, counts)
    orbgpu.stereo_matches_batch(ex, imgs, len(pairs), kps, desc, counts, bf, 0.0, ur, dp)
    ex.sync()
    kps_h = kps.cpu().numpy()
    desc_h = desc.cpu().numpy()
    n = counts.cpu().numpy()
    ur_h, dp_h = ur.cpu().numpy(), dp.cpu().numpy()
    s, inv, _, _ = ex.scale_factors()
    for p in range(len(pairs)):
        fl, fr = 2 * p, 2 * p + 1
        kl = orbgpu.keypoints_from_raw(kps_h[fl, : n[fl]])
        kr = orbgpu.keypoints_from_raw(kps_h[fr, : n[fr]])
        pl = [ex.level(l, fl) for l in range(ex.nlevels)]
        pr = [ex.level(l, fr) for l in range(ex.nlevels)]
        ur_ref, dp_ref = stereo_ref.compute_stereo_matches(kl, desc_h[fl, : n[fl]], kr, desc_h[fr, : n[fr]],
                                                           pl, pr, s, inv, bf, 0.0)
        g_ur, g_dp = ur_h[p, : n[fl]], dp_h[p, : n[fl]]
        assert (ur_ref >= 0).sum() > 50
        bad = np.nonzero(g_ur.view(np.uint32) != ur_ref.view(np.uint32))[0]
        assert len(bad) == 0, f"pair {p}: uRight differs at {len(bad)} kps, first {bad[:5]} gpu={g_ur[bad[:5]]} ref={ur_ref[bad[:5]]}"
        bad = np.nonzero(g_dp.view(np.uint32) != dp_ref.view(np.uint32))[0]
        assert len(bad) == 0, f"pair {p}: depth differs at {len(bad)} kps"


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["euroc_stereo", "kitti_stereo"])
def test_gpu_stereo_matches_bench_batch_vs_oracle(config):
    """The bench's stereo legs at their timed size: 128 pairs per launch, so
    csrc/stereo.hip deals each pair to S = ceil(2 * CUs / 128) blocks (4 on
    MI355X's 256 CUs) instead of the 32 a one- or two-pair launch uses.
    Every pair's uRight / depth against stereo_ref on the GPU's own keypoints
    and pyramid levels (bit-exact, the same -1 set), and the first and last
    pairs' extraction against the C++ oracle's stereo Frame."""
    torch = pytest.importorskip("torch")
    import orbgpu
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    W, H, NF, bf, base_px = {"euroc_stereo": (752, 480, 1200, 47.90639384423901, 18.0),
                             "kitti_stereo": (1241, 376, 2000, 0.54 * 718.856, 30.0)}[config]
    P = 128
    dev = torch.device("cuda", 0)
    pitch = (W + 15) // 16 * 16
    imgs = synth.torch_stereo_stream(P, W, H, base_px, device=dev, pitch=pitch, t0=P)
    ex = orbgpu.Extractor(nfeatures=NF, width=W, height=H, max_batch=2 * P)
    cap = ex.max_keypoints
    kps = torch.zeros((2 * P, cap, 7), dtype=torch.float32, device=dev)
    desc = torch.zeros((2 * P, cap, 32), dtype=torch.uint8, device=dev)
    counts = torch.zeros(2 * P, dtype=torch.int32, device=dev)
    ur = torch.full((P, cap), -7.0, dtype=torch.float32, device=dev)
    dp = torch.full((P, cap), -7.0, dtype=torch.float32, device=dev)
    ex.extract_batch(imgs, kps, desc, counts, row_step=pitch, frame_step=pitch * H)
    orbgpu.stereo_matches_batch(ex, imgs, P, kps, desc, counts, bf, 0.0, ur, dp, row_step=pitch,
                                frame_step=pitch * H)
    ex.sync()
    kps_h, desc_h, n = kps.cpu().numpy(), desc.cpu().numpy(), counts.cpu().numpy()
    ur_h, dp_h = ur.cpu().numpy(), dp.cpu().numpy()
    s, inv, _, _ = ex.scale_factors()
    with_depth = 0
    for p in range(P):
        fl, fr = 2 * p, 2 * p + 1
        kl = orbgpu.keypoints_from_raw(kps_h[fl, : n[fl]])
        kr = orbgpu.keypoints_from_raw(kps_h[fr, : n[fr]])
        pl = [ex.level(l, fl) for l in range(ex.nlevels)]
        pr = [ex.level(l, fr) for l in range(ex.nlevels)]
        ur_ref, dp_ref = stereo_ref.compute_stereo_matches(kl, desc_h[fl, : n[fl]], kr, desc_h[fr, : n[fr]],
                                                           pl, pr, s, inv, bf, 0.0)
        g_ur, g_dp = ur_h[p, : n[fl]], dp_h[p, : n[fl]]
        bad = np.nonzero(g_ur.view(np.uint32) != ur_ref.view(np.uint32))[0]
        assert len(bad) == 0, f"pair {p}: uRight differs at {len(bad)} kps, first {bad[:5]}"
        bad = np.nonzero(g_dp.view(np.uint32) != dp_ref.view(np.uint32))[0]
        assert len(bad) == 0, f"pair {p}: depth differs at {len(bad)} kps"
        with_depth += int((ur_ref >= 0).sum())
    assert with_depth > 100 * P
    exL, exR = orbref.Extractor(nfeatures=NF), orbref.Extractor(nfeatures=NF)
    for p in (0, P - 1):
        left = np.ascontiguousarray(imgs[2 * p, :, :W].cpu().numpy())
        right = np.ascontiguousarray(imgs[2 * p + 1, :, :W].cpu().numpy())
        kl, dl, kr, dr, ur_r, dp_r = orbref.stereo_frame(exL, exR, left, right, bf)
        assert orbgpu.keypoints_from_raw(kps_h[2 * p, : n[2 * p]]).tobytes() == kl.tobytes()
        assert orbgpu.keypoints_from_raw(kps_h[2 * p + 1, : n[2 * p + 1]]).tobytes() == kr.tobytes()
        np.testing.assert_array_equal(desc_h[2 * p, : n[2 * p]], dl)
        np.testing.assert_array_equal(desc_h[2 * p + 1, : n[2 * p + 1]], dr)
        assert ur_h[p, : n[2 * p]].view(np.uint32).tobytes() == ur_r.view(np.uint32).tobytes()
        assert dp_h[p, : n[2 * p]].view(np.uint32).tobytes() == dp_r.view(np.uint32).tobytes()
