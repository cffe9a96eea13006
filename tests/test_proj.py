"""Projection-matcher rows: Frame::isInFrustum and the
four ORBmatcher::SearchByProjection overloads, GPU vs the Python oracle
(oracle/proj_ref.py).  Bar: bit-exact matches (point index per keypoint,
-1 untouched, -2 culled) and counts; the frustum test's flags, levels and
float track fields exactly."""
import numpy as np
import pytest

import proj_ref
import synth


def _local_inputs(seed, stereo=False):
    tgt, pts = synth.projection_scenario(600, 300, seed, stereo=stereo)
    fl, tr, lv = proj_ref.is_in_frustum(tgt, pts, 0.5)
    pts = dict(pts, flags=fl, track=tr, track_level=lv)
    return tgt, pts


def test_oracle_frustum_and_local_search_find_true_points():
    tgt, pts = _local_inputs(1)
    assert (pts["flags"] & proj_ref.IN_VIEW).sum() > 200
    nm, m = proj_ref.search_by_projection(proj_ref.LOCAL, tgt, pts, th=1.0, nnratio=0.8)
    assert nm == (m >= 0).sum() > 150
    # a matched keypoint carries the point's (flipped) descriptor
    ok = [np.unpackbits(tgt["desc"][k] ^ pts["desc"][m[k]]).sum() < 40 for k in np.nonzero(m >= 0)[0]]
    assert np.mean(ok) > 0.95


def test_oracle_last_frame_rotation_cull():
    tgt, pts = synth.projection_scenario(500, 300, 3)
    last = tgt["Tcw"].copy()
    nm, m = proj_ref.search_by_projection(proj_ref.LAST_FRAME, tgt, pts, th=15.0, check_ori=True, mono=True,
                                          last_Tcw=last)
    assert nm == (m >= 0).sum() > 100


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_is_in_frustum_exact(seed):
    import proj
    tgt, pts = synth.projection_scenario(800, 0, seed)
    for cos_limit in (0.5, 0.8):
        fr, tr, lr = proj_ref.is_in_frustum(tgt, pts, cos_limit)
        fg, tg, lg = proj.is_in_frustum(tgt, pts, cos_limit)
        np.testing.assert_array_equal(fg, fr)
        inv = (fr & proj_ref.IN_VIEW) != 0
        np.testing.assert_array_equal(lg[inv], lr[inv])
        np.testing.assert_array_equal(tg[inv].view(np.uint32), tr[inv].view(np.uint32))


CASES = [  # variant, th, kwargs, stereo, scale
    (0, 1.0, dict(nnratio=0.8), False, 1.0),
    (0, 3.0, dict(nnratio=0.6), True, 1.0),
    (1, 10.0, dict(), False, 1.7),
    (1, 4.0, dict(), False, 1.0),
    (2, 15.0, dict(check_ori=True, mono=True), False, 1.0),
    (2, 7.0, dict(check_ori=False, mono=False), True, 1.0),
    (3, 10.0, dict(check_ori=True, orb_dist=100), False, 1.0),
    (3, 3.0, dict(check_ori=False, orb_dist=64), False, 1.0),
]


@pytest.mark.gpu
@pytest.mark.parametrize("variant,th,kw,stereo,scale", CASES)
def test_gpu_search_by_projection_exact(variant, th, kw, stereo, scale):
    import proj
    for seed in (10, 11, 12):
        tgt, pts = synth.projection_scenario(700, 400, seed + variant * 7, stereo=stereo, scale=scale)
        if variant == 0:
            fl, tr, lv = proj_ref.is_in_frustum(tgt, pts, 0.5)
            pts = dict(pts, flags=fl, track=tr, track_level=lv)
        if variant == 2:
            rng = np.random.default_rng(seed)
            last = tgt["Tcw"].copy()
            last[:3, 3] += rng.uniform(-0.2, 0.2, 3).astype(np.float32)
            kw = dict(kw, last_Tcw=last)
        nm_r, m_r = proj_ref.search_by_projection(variant, tgt, pts, th, **kw)
        nm_g, m_g = proj.search_by_projection(variant, tgt, pts, th, **kw)
        assert nm_g == nm_r, f"seed {seed}"
        np.testing.assert_array_equal(m_g, m_r)
        assert nm_r > 20


def _run_both(variant, tgt, pts, th, kw, seed):
    import proj
    if variant == 0:
        fl, tr, lv = proj_ref.is_in_frustum(tgt, pts, 0.5)
        pts = dict(pts, flags=fl, track=tr, track_level=lv)
    if variant == 2:
        rng = np.random.default_rng(seed)
        last = tgt["Tcw"].copy()
        last[:3, 3] += rng.uniform(-0.2, 0.2, 3).astype(np.float32)
        kw = dict(kw, last_Tcw=last)
    nm_r, m_r = proj_ref.search_by_projection(variant, tgt, pts, th, **kw)
    nm_g, m_g = proj.search_by_projection(variant, tgt, pts, th, **kw)
    assert nm_g == nm_r
    np.testing.assert_array_equal(m_g, m_r)
    return nm_r


@pytest.mark.gpu
@pytest.mark.parametrize("variant,th,kw", [(0, 1.0, dict(nnratio=0.8)), (1, 10.0, dict()),
                                           (2, 15.0, dict(check_ori=True, mono=True)),
                                           (3, 10.0, dict(check_ori=True, orb_dist=100))])
def test_gpu_search_by_projection_large_target_exact(variant, th, kw):
    """A target above the kernel's LDS descriptor budget (2048 keypoints):
    descriptors are read from HBM instead; same bar."""
    tgt, pts = synth.projection_scenario(1500, 1200, 40 + variant, stereo=variant in (0, 2))
    assert len(tgt["kps"]) > 2048
    assert _run_both(variant, tgt, pts, th, kw, 40) > 100


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1, 2, 3])
def test_gpu_search_by_projection_crowded_exact(variant):
    """Many points onto few keypoints: most points compete for the same
    slots, so the in-order walk's hiding decides nearly every match."""
    tgt, pts = synth.projection_scenario(900, 40, 60 + variant)
    keep = np.random.default_rng(7).permutation(len(tgt["kps"]))[:60]
    tgt = dict(tgt, kps=tgt["kps"][keep], desc=tgt["desc"][keep])
    for key in ("u_right", "occupied"):
        if tgt.get(key) is not None:
            tgt[key] = tgt[key][keep]
    th = 30.0 if variant else 3.0
    kw = {1: dict(), 2: dict(check_ori=True, mono=True), 3: dict(check_ori=True, orb_dist=100),
          0: dict(nnratio=0.9)}[variant]
    _run_both(variant, tgt, pts, th, kw, 60)


@pytest.mark.gpu
def test_gpu_search_by_projection_empty_inputs():
    import proj
    tgt, pts = synth.projection_scenario(200, 50, 9)
    none = {k: (v[:0] if isinstance(v, np.ndarray) and v.ndim and len(v) == len(pts["flags"]) else v)
            for k, v in pts.items()}
    for variant, th, kw in [(1, 10.0, dict()), (3, 10.0, dict(check_ori=True, orb_dist=100))]:
        nm_r, m_r = proj_ref.search_by_projection(variant, tgt, none, th, **kw)
        nm_g, m_g = proj.search_by_projection(variant, tgt, none, th, **kw)
        assert nm_g == nm_r == 0
        np.testing.assert_array_equal(m_g, m_r)
