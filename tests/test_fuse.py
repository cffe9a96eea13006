"""Per-point projection searches (SURVEY.md 8b callers LocalMapping.cpp:619-663,
LoopClosing.cpp:386/729): ORBmatcher::Fuse (both overloads) and
ORBmatcher::SearchBySim3, GPU vs the Python oracle (oracle/proj_ref.py).
Bar: bit-exact best keypoint per point, counts and SearchBySim3's
agreed matches."""
import numpy as np
import pytest

import proj_ref
import synth


def _truth_ok(tgt, pts, best):
    """a found keypoint carries the point's (lightly flipped) descriptor"""
    hit = np.nonzero(best >= 0)[0]
    return np.mean([np.unpackbits(tgt["desc"][best[i]] ^ pts["desc"][i]).sum() < 40 for i in hit])


def test_oracle_fuse_finds_true_keypoints():
    tgt, pts = synth.projection_scenario(600, 300, 5, stereo=True)
    n, best = proj_ref.radius_search(proj_ref.FUSE, tgt, pts, 3.0)
    assert n == (best >= 0).sum() > 150 and _truth_ok(tgt, pts, best) > 0.95
    n2, best2 = proj_ref.radius_search(proj_ref.FUSE, dict(tgt, u_right=None), pts, 3.0)
    assert n2 > 150  # monocular: the 5.99 chi-square test only


def test_oracle_fuse_sim3_and_sim3_search():
    tgt, pts = synth.projection_scenario(600, 300, 6, scale=1.7)
    n, best = proj_ref.radius_search(proj_ref.FUSE_SIM3, tgt, pts, 4.0)
    assert n > 150 and _truth_ok(tgt, pts, best) > 0.95
    kf1, kf2, p1, p2, s, R, t = synth.sim3_search_scenario(500, 200, 7, s12=1.05)
    nf, m12 = proj_ref.search_by_sim3(kf1, kf2, p1, p2, s, R, t, 7.5)
    assert nf == (m12 >= 0).sum() > 40
    # agreed matches never touch an already-matched / NULL / bad entry
    assert all(p1["flags"][i] & 1 for i in np.nonzero(m12 >= 0)[0])
    assert all(p2["flags"][m12[i]] & 1 for i in np.nonzero(m12 >= 0)[0])


FUSE_CASES = [  # variant, th, stereo, scale, n_points, n_distractors
    (proj_ref.FUSE, 3.0, False, 1.0, 700, 400),
    (proj_ref.FUSE, 3.0, True, 1.0, 700, 400),
    (proj_ref.FUSE, 10.0, True, 1.0, 300, 900),
    (proj_ref.FUSE_SIM3, 4.0, False, 1.7, 700, 400),
    (proj_ref.FUSE_SIM3, 4.0, False, 1.0, 1500, 1200),  # > 2048 keypoints: descriptors from HBM
]


@pytest.mark.gpu
@pytest.mark.parametrize("variant,th,stereo,scale,npts,ndis", FUSE_CASES)
def test_gpu_fuse_exact(variant, th, stereo, scale, npts, ndis):
    import proj
    for seed in (20, 21):
        tgt, pts = synth.projection_scenario(npts, ndis, seed + variant, stereo=stereo, scale=scale)
        n_r, b_r = proj_ref.radius_search(variant, tgt, pts, th)
        n_g, b_g = proj.radius_search(variant, tgt, pts, th)
        np.testing.assert_array_equal(b_g, b_r)
        assert n_g == n_r > 50


@pytest.mark.gpu
def test_gpu_fuse_many_points_few_keypoints():
    """3000 points over 80 keypoints: most windows are empty or hold another
    point's keypoint; per-point results stay independent (Fuse's
    Replace/AddObservation order is the caller's replay)"""
    import proj
    tgt, pts = synth.projection_scenario(3000, 30, 31)
    keep = np.random.default_rng(3).permutation(len(tgt["kps"]))[:80]
    tgt = dict(tgt, kps=tgt["kps"][keep], desc=tgt["desc"][keep], occupied=None)
    n_r, b_r = proj_ref.radius_search(proj_ref.FUSE, tgt, pts, 20.0)
    n_g, b_g = proj.radius_search(proj_ref.FUSE, tgt, pts, 20.0)
    np.testing.assert_array_equal(b_g, b_r)
    assert n_g == n_r > 30


@pytest.mark.gpu
def test_gpu_fuse_empty_inputs():
    import proj
    tgt, pts = synth.projection_scenario(200, 50, 9)
    none = {k: (v[:0] if isinstance(v, np.ndarray) and v.ndim and len(v) == len(pts["flags"]) else v)
            for k, v in pts.items()}
    assert proj.radius_search(proj_ref.FUSE, tgt, none, 3.0)[0] == 0
    empty_tgt = dict(tgt, kps=tgt["kps"][:0], desc=tgt["desc"][:0], occupied=None)
    n_g, b_g = proj.radius_search(proj_ref.FUSE, empty_tgt, pts, 3.0)
    assert n_g == 0 and (b_g == -1).all() and len(b_g) == len(pts["flags"])


@pytest.mark.gpu
@pytest.mark.parametrize("seed,s12,th", [(40, 1.0, 7.5), (41, 1.15, 7.5), (42, 0.9, 10.0)])
def test_gpu_search_by_sim3_exact(seed, s12, th):
    import proj
    kf1, kf2, p1, p2, s, R, t = synth.sim3_search_scenario(600, 250, seed, s12=s12)
    n_r, m_r = proj_ref.search_by_sim3(kf1, kf2, p1, p2, s, R, t, th)
    n_g, m_g = proj.search_by_sim3(kf1, kf2, p1, p2, s, R, t, th)
    np.testing.assert_array_equal(m_g, m_r)
    assert n_g == n_r > 20
