"""Bag-of-words rows: DBoW2 vocabulary loading,
TemplatedVocabulary::transform (words, direct-index nodes, BowVector,
FeatureVector) and ORBmatcher::SearchByBoW, GPU vs the Python oracle.

Bar: bit-exact -- word/node ids, FeatureVector, match indices and counts,
and the BowVector's double weights (summed in the reference's order).  The
vocabularies are synthetic (ORBvoc.txt is not in the reference tree):
parity against the real vocabulary is unpinned."""
import numpy as np
import pytest

import bow_ref
import synth


def _voc_arrays(k, L, seed):
    return synth.synthetic_vocabulary(k, L, seed)


def test_oracle_loader_roundtrip_and_trailing_newline(tmp_path):
    par, leaf, desc, w = _voc_arrays(3, 3, 1)
    p = tmp_path / "voc.txt"
    synth.write_vocabulary_text(p, 3, 3, 0, 0, par, leaf, desc, w)
    v = bow_ref.Vocabulary.load_text(p)
    ref = bow_ref.Vocabulary.from_arrays(3, 3, 0, 0, par, leaf, desc, w)
    assert v.parent == ref.parent and v.children == ref.children and v.weight == ref.weight
    assert all(np.array_equal(a, b) for a, b in zip(v.desc, ref.desc)) and v.n_words == 27
    p2 = tmp_path / "voc_nl.txt"
    synth.write_vocabulary_text(p2, 3, 3, 0, 0, par, leaf, desc, w, trailing_newline=True)
    v2 = bow_ref.Vocabulary.load_text(p2)
    assert len(v2.parent) == len(v.parent) + 1
    assert v2.parent[-1] == 0 and v2.children[0][-1] == len(v2.parent) - 1
    assert v2.weight[-1] == 0.0 and not v2.desc[-1].any() and v2.n_words == v.n_words


def test_oracle_binary_loader_last_record_twice(tmp_path):
    """loadFromBinaryFile (TemplatedVocabulary.h:1477-1522): the eof loop
    processes the last record a second time; weights are the file's floats."""
    par, leaf, desc, w = _voc_arrays(3, 3, 1)
    p = tmp_path / "voc.bin"
    synth.write_vocabulary_binary(p, 3, 3, 2, 1, par, leaf, desc, w)
    v = bow_ref.Vocabulary.load_binary(p)
    ref = bow_ref.Vocabulary.from_arrays(3, 3, 2, 1, par, leaf, desc, np.float32(w).astype(np.float64))
    n = len(ref.parent)
    assert (v.k, v.L, v.scoring, v.weighting) == (3, 3, 2, 1)
    assert len(v.parent) == n + 1 and v.parent[:n] == ref.parent and v.weight[:n] == ref.weight
    assert v.parent[n] == ref.parent[n - 1] and v.children[ref.parent[n - 1]][-2:] == [n - 1, n]
    assert np.array_equal(v.desc[n], ref.desc[n - 1]) and v.n_words == ref.n_words + 1 == 28
    # the duplicate never wins the strict minimum: words of the text-format tree
    feats = np.random.default_rng(3).integers(0, 256, (200, 32), dtype=np.uint8)
    feats[:50] = desc[len(par) - 1]
    assert v.transform(feats, 1)[:3] == ref.transform(feats, 1)[:3]
    # a file cut inside the last record: its prefix overwrites the previous record's
    raw = open(p, "rb").read()
    p2 = tmp_path / "cut.bin"
    open(p2, "wb").write(raw[:-20])
    v2 = bow_ref.Vocabulary.load_binary(p2)
    # 21 bytes of the last record: parent + 17 descriptor bytes, the rest from the one before
    assert len(v2.parent) == n + 1 and v2.parent[n - 1] == ref.parent[n - 1]
    assert np.array_equal(v2.desc[n - 1][:17], ref.desc[n - 1][:17])
    assert np.array_equal(v2.desc[n - 1][17:], ref.desc[n - 2][17:]) and v2.weight[n - 1] == ref.weight[n - 2]
    assert v2.parent[n] == 0 and all(n not in c for c in v2.children)  # m_nodes[nb_nodes]: default, unattached


def test_oracle_transform_structure():
    par, leaf, desc, w = _voc_arrays(5, 4, 2)
    v = bow_ref.Vocabulary.from_arrays(5, 4, 0, 0, par, leaf, desc, w)
    rng = np.random.default_rng(0)
    feats = desc[leaf == 1][rng.integers(0, 625, 200)]
    words, nodes, weights, fv, bowv = v.transform(feats, levelsup=2)
    assert all(0 <= x < v.n_words for x in words)
    depth2 = set(range(1 + 5, 1 + 5 + 25))  # node ids of level 2 in BFS order
    assert set(nodes) <= depth2
    assert sorted(i for lst in fv.values() for i in lst) == list(range(200))
    assert abs(sum(bowv.values()) - 1.0) < 1e-12


def test_oracle_search_by_bow_finds_true_correspondences():
    par, leaf, desc, w = _voc_arrays(6, 4, 3)
    v = bow_ref.Vocabulary.from_arrays(6, 4, 0, 0, par, leaf, desc, w)
    d1, a1, d2, a2 = synth.bow_frame_pair(desc[leaf == 1], 300, 0.5, seed=4)
    fv1 = v.transform(d1, 2)[3]
    fv2 = v.transform(d2, 2)[3]
    nm, m = bow_ref.search_by_bow(0, fv1, d1, a1, np.ones(300, bool), fv2, d2, a2, np.ones(300, bool), 0.75, True)
    assert nm == (m >= 0).sum() >= 60
    valid = m[m >= 0]
    assert len(set(valid.tolist())) == len(valid)


VOCAB_CASES = [(10, 3, 0, 0, 1), (5, 4, 1, 1, 2), (5, 4, 2, 2, 0), (4, 5, 3, 3, 3), (6, 4, 5, 0, 4), (6, 4, 5, 1, 2)]


@pytest.mark.gpu
@pytest.mark.parametrize("k,L,scoring,weighting,levelsup", VOCAB_CASES)
def test_gpu_transform_bit_exact(k, L, scoring, weighting, levelsup):
    import bow
    par, leaf, desc, w = _voc_arrays(k, L, 10 + k + L)
    ref = bow_ref.Vocabulary.from_arrays(k, L, scoring, weighting, par, leaf, desc, w)
    gv = bow.Vocabulary.from_arrays(k, L, scoring, weighting, par, leaf, desc, w)
    assert gv.info().n_words == ref.n_words and gv.info().n_nodes == len(ref.parent)
    rng = np.random.default_rng(k * 100 + L)
    feats = rng.integers(0, 256, (700, 32), dtype=np.uint8)
    feats[:300] = desc[leaf == 1][rng.integers(0, int(leaf.sum()), 300)]
    words, nodes, weights, fv, bowv = gv.transform(feats, levelsup)
    rw, rn, rwt, rfv, rbow = ref.transform(feats, levelsup)
    np.testing.assert_array_equal(words, rw)
    np.testing.assert_array_equal(nodes, rn)
    np.testing.assert_array_equal(weights, np.array(rwt))
    assert list(fv) == list(rfv) and all(np.array_equal(fv[n_], rfv[n_]) for n_ in fv)
    assert list(bowv) == list(rbow)
    np.testing.assert_array_equal(np.array(list(bowv.values())), np.array(list(rbow.values())))


@pytest.mark.gpu
def test_gpu_vocabulary_text_loader(tmp_path):
    import bow
    par, leaf, desc, w = _voc_arrays(4, 3, 7)
    for nl in (False, True):
        p = tmp_path / f"v{int(nl)}.txt"
        synth.write_vocabulary_text(p, 4, 3, 0, 0, par, leaf, desc, w, trailing_newline=nl)
        gv = bow.Vocabulary.load_text(p)
        ref = bow_ref.Vocabulary.load_text(p)
        assert gv.info().n_nodes == len(ref.parent) and gv.info().n_words == ref.n_words
        feats = np.random.default_rng(1).integers(0, 256, (300, 32), dtype=np.uint8)
        gw, gn, gwt = gv.transform(feats, 1)[:3]
        rw, rn, rwt = ref.transform(feats, 1)[:3]
        np.testing.assert_array_equal(gw, rw)
        np.testing.assert_array_equal(gn, rn)
        np.testing.assert_array_equal(gwt, np.array(rwt))


@pytest.mark.gpu
def test_gpu_vocabulary_binary_loader(tmp_path):
    import bow
    import orbgpu
    par, leaf, desc, w = _voc_arrays(5, 4, 9)
    for scoring, weighting in ((0, 0), (1, 3), (5, 1)):
        p = tmp_path / f"v{scoring}{weighting}.bin"
        synth.write_vocabulary_binary(p, 5, 4, scoring, weighting, par, leaf, desc, w)
        gv = bow.Vocabulary.load_binary(p)
        ref = bow_ref.Vocabulary.load_binary(p)
        info = gv.info()
        assert (info.k, info.L, info.scoring, info.weighting) == (5, 4, scoring, weighting)
        assert info.n_nodes == len(ref.parent) == len(par) + 2 and info.n_words == ref.n_words
        feats = np.random.default_rng(scoring).integers(0, 256, (500, 32), dtype=np.uint8)
        feats[:200] = desc[leaf == 1][np.random.default_rng(1).integers(0, int(leaf.sum()), 200)]
        feats[200:230] = desc[len(par) - 1]  # the twice-read last leaf
        words, nodes, weights, fv, bowv = gv.transform(feats, 2)
        rw, rn, rwt, rfv, rbow = ref.transform(feats, 2)
        np.testing.assert_array_equal(words, rw)
        np.testing.assert_array_equal(nodes, rn)
        np.testing.assert_array_equal(weights, np.array(rwt))
        assert list(fv) == list(rfv) and all(np.array_equal(fv[n_], rfv[n_]) for n_ in fv)
        assert list(bowv) == list(rbow)
        np.testing.assert_array_equal(np.array(list(bowv.values())), np.array(list(rbow.values())))
    # malformed files fail loudly (the reference reads garbage there)
    raw = open(tmp_path / "v00.bin", "rb").read()
    bad = {"short": raw[:20], "ksize": raw[:8] + np.array([25, 4, 0, 0], "<i4").tobytes() + raw[24:],
           "recsize": raw[:4] + np.array([40], "<u4").tobytes() + raw[8:],
           "count": np.array([5], "<u4").tobytes() + raw[4:]}
    for name, data in bad.items():
        q = tmp_path / f"bad_{name}.bin"
        open(q, "wb").write(data)
        with pytest.raises(orbgpu.OrbGpuError):
            bow.Vocabulary.load_binary(q)


@pytest.mark.gpu
@pytest.mark.parametrize("mode,nnratio,check_ori,invalid", [(0, 0.7, True, 0.0), (0, 0.75, False, 0.0),
                                                            (1, 0.75, True, 0.2), (1, 0.6, False, 0.0),
                                                            (0, 0.6, True, 0.3)])
def test_gpu_search_by_bow_bit_exact(mode, nnratio, check_ori, invalid):
    import bow
    par, leaf, desc, w = _voc_arrays(8, 4, 5)
    ref = bow_ref.Vocabulary.from_arrays(8, 4, 0, 0, par, leaf, desc, w)
    rng = np.random.default_rng(17)
    for trial in range(4):
        n1, n2 = int(rng.integers(50, 1200)), 0
        d1, a1, d2, a2 = synth.bow_frame_pair(desc[leaf == 1], n1, 0.6, seed=100 + trial)
        fv1 = ref.transform(d1, 2)[3]
        fv2 = ref.transform(d2, 2)[3]
        v1 = rng.uniform(size=n1) >= invalid
        v2 = rng.uniform(size=n1) >= invalid if mode == 1 else np.ones(n1, bool)
        nm_r, m_r = bow_ref.search_by_bow(mode, fv1, d1, a1, v1, fv2, d2, a2, v2, nnratio, check_ori)
        nm_g, m_g = bow.search_by_bow(mode, fv1, d1, a1, v1, fv2, d2, a2, v2, nnratio, check_ori)
        assert nm_g == nm_r
        np.testing.assert_array_equal(m_g, m_r)
        assert nm_r > 20


# ---- keyframe database scoring (KeyFrameDatabase::Detect*Candidates) ------
def _bow_db(scoring, weighting, n_kf, seed):
    par, leaf, desc, w = synth.synthetic_vocabulary(6, 4, 60 + seed)
    voc = bow_ref.Vocabulary.from_arrays(6, 4, scoring, weighting, par, leaf, desc, w)
    rng = np.random.default_rng(seed)
    leaves = desc[leaf == 1]
    base = leaves[rng.integers(0, len(leaves), 400)]
    db = []
    for k in range(n_kf):  # keyframes re-observe a drifting subset of a common scene
        pick = rng.choice(400, 250, replace=False) if k % 3 else rng.choice(400, 150, replace=False)
        d = base[pick] ^ (rng.uniform(size=(len(pick), 32)) < 0.02).astype(np.uint8) * np.uint8(1)
        db.append(voc.transform(d, 2)[4])
    q = voc.transform(base[rng.choice(400, 300, replace=False)], 2)[4]
    return q, db


@pytest.mark.parametrize("scoring", [0, 1, 2, 3, 4, 5])
def test_oracle_bow_score_properties(scoring):
    q, db = _bow_db(scoring, 0, 3, 1)
    s_self, nc_self = bow_ref.bow_score(scoring, q, q)
    assert nc_self == len(q)
    if scoring in (0, 1, 4):  # normalised scores: identical vectors score 1
        assert abs(s_self - 1.0) < 1e-7  # L2: 1 - sqrt(1 - s) amplifies the rounding of s
    s, nc = bow_ref.bow_score(scoring, q, db[0])
    assert 0 < nc < len(q)


@pytest.mark.gpu
@pytest.mark.parametrize("scoring,weighting", [(0, 0), (1, 0), (2, 1), (3, 0), (4, 2), (5, 3)])
def test_gpu_bow_score_vs_oracle(scoring, weighting):
    """scores bit-exact (KL: the device log, to 1e-12 relative), common-word counts exact"""
    import bow
    q, db = _bow_db(scoring, weighting, 300, 2)
    db += [{}, dict(q)]  # an empty keyframe and the query itself
    common, scores = bow.bow_score(scoring, q, db)
    ref = [bow_ref.bow_score(scoring, q, v) for v in db]
    np.testing.assert_array_equal(common, [r[1] for r in ref])
    if scoring == 3:
        np.testing.assert_allclose(scores, [r[0] for r in ref], rtol=1e-12, atol=1e-12)
    else:
        np.testing.assert_array_equal(scores.view(np.uint64), np.array([r[0] for r in ref]).view(np.uint64))
