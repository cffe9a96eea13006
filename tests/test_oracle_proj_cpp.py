"""The C++ restatement of the two per-frame SearchByProjection overloads
(oracle/proj_ref.cpp: LOCAL -- Tracking::SearchLocalPoints, LAST_FRAME --
Tracking::TrackWithMotionModel) against the Python oracle (oracle/proj_ref.py)
on the same scenarios: matches and counts bit-exact.  The C++ form exists so
bench.py's drop-in table times compiled code on the CPU side; this test pins
it to the oracle the GPU kernels are checked against (CPU only)."""
import numpy as np
import pytest

import orbref
import proj_ref
import synth


@pytest.mark.parametrize("seed,stereo,th", [(1, False, 1.0), (2, True, 1.0), (3, True, 3.0), (4, False, 5.0)])
def test_cpp_local_equals_python(seed, stereo, th):
    tgt, pts = synth.projection_scenario(500, 250, seed, stereo=stereo)
    fl, tr, lv = proj_ref.is_in_frustum(tgt, pts, 0.5)
    pts = dict(pts, flags=fl, track=tr, track_level=lv)
    n_p, m_p = proj_ref.search_by_projection(proj_ref.LOCAL, tgt, pts, th, nnratio=0.8)
    n_c, m_c = orbref.search_by_projection(proj_ref.LOCAL, tgt, pts, th, nnratio=0.8)
    assert n_p > 50
    assert n_c == n_p
    np.testing.assert_array_equal(m_c, np.asarray(m_p, np.int32))


@pytest.mark.parametrize("seed,stereo,mono,dz", [(5, False, True, 0.05), (6, True, False, 0.3), (7, True, False, -0.3),
                                                 (8, True, False, 0.0)])
def test_cpp_last_frame_equals_python(seed, stereo, mono, dz):
    tgt, pts = synth.projection_scenario(400, 250, seed, stereo=stereo)
    last = np.asarray(tgt["Tcw"], np.float32).copy()
    last[2, 3] += np.float32(dz)  # forward / backward motion selects the level window (bMono false)
    for ori in (True, False):
        n_p, m_p = proj_ref.search_by_projection(proj_ref.LAST_FRAME, tgt, pts, 15.0, check_ori=ori, mono=mono,
                                                 last_Tcw=last)
        n_c, m_c = orbref.search_by_projection(proj_ref.LAST_FRAME, tgt, pts, 15.0, check_ori=ori, mono=mono,
                                               last_Tcw=last)
        assert n_p > 30
        assert n_c == n_p
        np.testing.assert_array_equal(m_c, np.asarray(m_p, np.int32))


@pytest.mark.parametrize("nnratio,check_ori,invalid", [(0.7, True, 0.0), (0.6, True, 0.3), (0.75, False, 0.1)])
def test_cpp_search_by_bow_kf_f_equals_python(nnratio, check_ori, invalid):
    """SearchByBoW(KF, F) (Tracking::TrackReferenceKeyFrame) in C++
    (oracle/loop_ref.cpp) vs bow_ref.search_by_bow mode 0."""
    import bow_ref
    par, leaf, desc, w = synth.synthetic_vocabulary(8, 4, 5)
    ref = bow_ref.Vocabulary.from_arrays(8, 4, 0, 0, par, leaf, desc, w)
    rng = np.random.default_rng(23)
    for trial in range(3):
        n1 = int(rng.integers(200, 1100))
        d1, a1, d2, a2 = synth.bow_frame_pair(desc[leaf == 1], n1, 0.6, seed=200 + trial)
        fv1 = ref.transform(d1, 2)[3]
        fv2 = ref.transform(d2, 2)[3]
        v1 = rng.uniform(size=n1) >= invalid
        nm_p, m_p = bow_ref.search_by_bow(0, fv1, d1, a1, v1, fv2, d2, a2, np.ones(len(d2), bool), nnratio, check_ori)
        nm_c, m_c = orbref.search_by_bow_kf_f(fv1, d1, a1, v1, fv2, d2, a2, nnratio, check_ori)
        assert nm_p > 20
        assert nm_c == nm_p
        np.testing.assert_array_equal(m_c, m_p)


@pytest.mark.parametrize("n,inl,min_inl,seed", [(120, 0.6, 40, 1), (300, 0.5, 100, 2), (60, 0.6, 15, 3),
                                                (200, 0.9, 150, 4)])
def test_cpp_pnp_ransac_call_equals_numpy(n, inl, min_inl, seed):
    """PnPsolver::iterate's loop body with Refine in C++ (oracle/pnp_ref.cpp)
    vs the numpy oracle: integer outcomes equal, poses to 1e-6."""
    import pnp_ref
    P = synth.pnp_problem(n, inl, seed)
    maxerr = (P["sigma2"] * np.float32(5.991)).astype(np.float32)
    rng = np.random.default_rng(seed)
    samples = np.array([rng.choice(n, 4, replace=False) for _ in range(30)], np.int32)
    o_p = pnp_ref.ransac_call(P["P3w"], P["P2"], maxerr, P["cam"], min_inl, 0, np.zeros(n, bool), samples)
    o_c = orbref.pnp_ransac_call(P["P3w"], P["P2"], maxerr, P["cam"], min_inl, 0, samples)
    for key in ("found", "consumed", "best_inliers", "best_hyp", "refined_inliers"):
        assert o_c[key] == o_p[key], key
    assert o_p["best_hyp"] >= 0
    np.testing.assert_allclose(o_c["best_R"], o_p["best_R"], atol=1e-6)
    np.testing.assert_allclose(o_c["best_t"], o_p["best_t"], atol=1e-6 * (1 + np.abs(o_p["best_t"]).max()))
    if o_p["found"]:
        np.testing.assert_allclose(o_c["refined_R"], o_p["refined_R"], atol=1e-6)
        np.testing.assert_allclose(o_c["refined_t"], o_p["refined_t"], atol=1e-6 * (1 + np.abs(o_p["refined_t"]).max()))
