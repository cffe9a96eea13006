"""ORBmatcher::SearchForTriangulation (LocalMapping::CreateNewMapPoints,
LocalMapping.cpp:355-360; ORBmatcher.cpp:755-951 with CheckDistEpipolarLine
:166-190), GPU vs the Python oracle (oracle/bow_ref.py).  Bar: bit-exact
match12 and count.  Vocabularies are synthetic (ORBvoc.txt is absent)."""
import numpy as np
import pytest

import bow_ref
import synth


def _scene(seed, **kw):
    par, leaf, desc, w = synth.synthetic_vocabulary(6, 4, 30 + seed)
    voc = bow_ref.Vocabulary.from_arrays(6, 4, 0, 0, par, leaf, desc, w)
    P = synth.triangulation_scenario(desc[leaf == 1], 500, seed, **kw)
    fv1 = voc.transform(P["desc1"], 2)[3]
    fv2 = voc.transform(P["desc2"], 2)[3]
    return fv1, fv2, P


def test_oracle_triangulation_matches_are_epipolar_and_unique():
    fv1, fv2, P = _scene(1)
    nm, m = bow_ref.search_for_triangulation(fv1, fv2, P, check_ori=False)
    assert nm == (m >= 0).sum() > 40
    got = m[m >= 0]
    assert len(set(got.tolist())) == len(got)             # vbMatched2
    assert all(P["valid1"][i] for i in np.nonzero(m >= 0)[0]) and all(P["valid2"][j] for j in got)
    F = P["F12"].astype(np.float64)
    for i in np.nonzero(m >= 0)[0]:
        x1 = np.array([P["kps1"]["x"][i], P["kps1"]["y"][i], 1.0])
        j = m[i]
        x2 = np.array([P["kps2"]["x"][j], P["kps2"]["y"][j], 1.0])
        l = x1 @ F
        assert (x2 @ l) ** 2 / (l[0] ** 2 + l[1] ** 2) < 3.84 * P["level_sigma2_2"][P["kps2"]["octave"][j]] * 1.001
    nm2, _ = bow_ref.search_for_triangulation(fv1, fv2, P, check_ori=True)
    assert nm2 <= nm


@pytest.mark.gpu
@pytest.mark.parametrize("seed,check_ori,stereo,only_stereo", [(1, False, False, False), (2, True, False, False),
                                                               (3, True, True, False), (4, False, True, True)])
def test_gpu_search_for_triangulation_exact(seed, check_ori, stereo, only_stereo):
    import bow
    fv1, fv2, P = _scene(seed, stereo=stereo)
    n_r, m_r = bow_ref.search_for_triangulation(fv1, fv2, P, check_ori, only_stereo)
    n_g, m_g = bow.search_for_triangulation(fv1, fv2, P, check_ori, only_stereo)
    np.testing.assert_array_equal(m_g, m_r)
    assert n_g == n_r > 10


@pytest.mark.gpu
def test_gpu_search_for_triangulation_empty_and_all_tracked():
    import bow
    fv1, fv2, P = _scene(5)
    P0 = dict(P, valid1=np.zeros_like(P["valid1"]))
    assert bow.search_for_triangulation(fv1, fv2, P0)[0] == 0
    assert bow.search_for_triangulation({}, fv2, P)[0] == 0
