"""LoopClosing::ComputeSim3 hot loop (the
loop-closure burst): SearchByBoW(KF, KF) with ORBmatcher(0.75, true) over a
k=10, L=6 DBoW2 vocabulary, the Sim3Solver set-up, and the round-robin
iterate(5) RANSAC (src/LoopClosing.cpp:273-356).

CPU: the oracle pieces (oracle/loop_ref.py) against the independent
restatements they must agree with (bow_ref on small trees, the text
vocabulary round trip) and on a scene with a known Sim3.
GPU: csrc/loop.hip + csrc/bow.hip on a 50-pair slice at full size (1000
keypoints per keyframe, the 1.1 M-node vocabulary loaded from DBoW2 text)
against the oracle -- FeatureVectors, SearchByBoW matches and the Sim3Solver
set-up bit-exact; ComputeSim3's integer outcomes (matched candidate, round,
iterations per solver, inlier counts, rand() draws) equal; the returned pose
within the tolerance of tests/test_ransac.py.  The random stream is the
host glibc's (srand(seed) per query) on the oracle side."""
import ctypes

import numpy as np
import pytest

import bow_ref
import loop_ref
import synth


def _small_vocab(k=6, L=3, seed=3):
    p, l, d, w = synth.synthetic_vocabulary_fast(k, L, seed)
    return k, L, p, l, d, w


def test_array_vocabulary_matches_bow_ref():
    k, L, p, l, d, w = _small_vocab()
    ref = bow_ref.Vocabulary.from_arrays(k, L, 0, 0, p, l, d, w)
    arr = loop_ref.ArrayVocabulary(k, L, 0, 0, p, l, d, w)
    rng = np.random.default_rng(1)
    D = rng.integers(0, 256, (300, 32), dtype=np.uint8)
    for levelsup in (0, 1, 2, 4):
        words, nodes, weights, fv, _ = ref.transform(D, levelsup)
        w2, n2, wt2, fv2 = arr.transform(D, levelsup)
        np.testing.assert_array_equal(w2, words)
        np.testing.assert_array_equal(n2, nodes)
        np.testing.assert_array_equal(wt2, weights)
        assert {a: list(b) for a, b in fv.items()} == fv2


def test_fast_vocabulary_text_roundtrip(tmp_path):
    k, L, p, l, d, w = _small_vocab(5, 3, 9)
    path = tmp_path / "voc.txt"
    synth.write_vocabulary_text_fast(path, k, L, 0, 0, p, l, d, w)
    assert not path.read_bytes().endswith(b"\n")  # no spurious trailing node
    v = bow_ref.Vocabulary.load_text(str(path))
    assert len(v.parent) == len(p) + 1
    np.testing.assert_array_equal(np.array(v.parent[1:]), p)
    np.testing.assert_array_equal(np.stack(v.desc[1:]), d)
    np.testing.assert_array_equal(np.array(v.weight[1:]), w)


def _oracle_pipeline(scene, avoc, queries, seeds, fix_scale=False):
    """FeatureVectors, SearchByBoW(KF1, KF2), Sim3Solver set-up and
    ComputeSim3 per query, all on the CPU oracle."""
    fvs = {}

    def fv(kf):
        if kf not in fvs:
            fvs[kf] = avoc.transform(scene["desc"][kf], 4)[3]
        return fvs[kf]

    out = []
    for (cur, cands), seed in zip(queries, seeds):
        solvers, per = [], []
        for c in cands:
            nm, m12 = bow_ref.search_by_bow(1, fv(cur), scene["desc"][cur], scene["angle"][cur], scene["valid"][cur],
                                            fv(c), scene["desc"][c], scene["angle"][c], scene["valid"][c],
                                            nnratio=0.75, check_ori=True)
            corr = loop_ref.sim3_setup(m12, scene["valid"][cur], scene["valid"][c], scene["mp_world"][cur],
                                       scene["mp_world"][c], scene["Tcw"][cur], scene["Tcw"][c],
                                       scene["octave"][cur], scene["octave"][c], scene["sigma2"])
            per.append((nm, m12, corr))
            solvers.append(loop_ref.Sim3SolverRef(corr, scene["K"], scene["K"], fix_scale) if nm >= 20 else None)
        res = loop_ref.compute_sim3(solvers, seed)
        res["after"] = loop_ref.libc().rand()  # the next value of the stream after the query
        out.append((per, solvers, res))
    return out


def test_oracle_compute_sim3_recovers_the_loop():
    k, L, p, l, d, w = 10, 4, *synth.synthetic_vocabulary_fast(10, 4, 5)
    avoc = loop_ref.ArrayVocabulary(k, L, 0, 0, p, l, d, w)
    scene = synth.loop_burst_scene(2, 3, d[l == 1], n_kp=500, inlier_frac=[0.0, 0.4, 0.4], seed=21)
    queries = [(q, [2 + 3 * q + c for c in range(3)]) for q in range(2)]
    res = _oracle_pipeline(scene, avoc, queries, [7, 8])
    for q, (per, solvers, r) in enumerate(res):
        assert per[0][0] < 20  # unrelated candidate: discarded before RANSAC
        assert r["matched"] in (1, 2)
        tr = scene["truth"][q * 3 + r["matched"]]
        pose = solvers[r["matched"]].best_pose
        assert abs(pose["s12"] - tr["s"]) < 0.05
        assert np.abs(pose["R12"] - tr["R"]).max() < 0.05


# ---- GPU: the burst on a 50-pair slice at full size ------------------------

def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def big_vocab(tmp_path_factory):
    p, l, d, w = synth.synthetic_vocabulary_fast(10, 6, 0x70C)
    path = tmp_path_factory.mktemp("voc") / "voc_k10_L6.txt"
    synth.write_vocabulary_text_fast(path, 10, 6, 0, 0, p, l, d, w)
    return path, (p, l, d, w)


@pytest.mark.gpu
@pytest.mark.parametrize("fracs,ofracs,fix_scale", [
    # unrelated / false loop / weak / two true loops with 50 % geometric outliers: several rounds
    ([0.0, 0.0, 0.03, 0.4, 0.4], [0.0, 0.08, 0.05, 0.5, 0.5], False),
    # the bench's configuration (40 % true, the rest outliers), stereo (fixed scale)
    (0.4, 0.6, True),
    # false loops only: every solver runs to mRansacMaxIts, no Sim3 returned
    (0.0, [0.0, 0.06, 0.08, 0.1, 0.05], False)])
def test_gpu_loop_burst_slice_vs_oracle(big_vocab, fracs, ofracs, fix_scale):
    torch = _gpu()
    import bow
    import loop
    import orbgpu
    path, (p, l, d, w) = big_vocab
    voc = bow.Vocabulary.load_text(str(path))
    info = voc.info()
    assert (info.k, info.L, info.n_nodes) == (10, 6, len(p) + 1)
    avoc = loop_ref.ArrayVocabulary(10, 6, 0, 0, p, l, d, w)
    nq, nc = 10, 5
    scene = synth.loop_burst_scene(nq, nc, d[l == 1], n_kp=1000, inlier_frac=fracs, outlier_frac=ofracs,
                                   seed=33 + fix_scale, fix_scale=fix_scale)
    kfs = loop.Keyframes(scene["desc"], scene["angle"], scene["octave"], scene["valid"], scene["mp_world"],
                         scene["Tcw"], scene["K"], scene["sigma2"])
    kfs.compute_bow(voc)
    queries = [(q, [nq + q * nc + c for c in range(nc)]) for q in range(nq)]
    seeds = [1000 + q for q in range(nq)]
    lb = loop.LoopBurst(kfs, [(a, b, s) for (a, b), s in zip(queries, seeds)], fix_scale=fix_scale)
    lb.step()
    torch.cuda.synchronize()
    ref = _oracle_pipeline(scene, avoc, queries, seeds, fix_scale)
    # FeatureVectors of the keyframes (transform on the GPU vs the oracle)
    for kf in (0, nq, nq + 1):
        fv = avoc.transform(scene["desc"][kf], 4)[3]
        n = int(kfs.tf.fv_n[kf])
        nodes = kfs.tf.fv_nodes[kf, :n].cpu().numpy()
        offs = kfs.tf.fv_offsets[kf, :n + 1].cpu().numpy()
        feats = kfs.tf.fv_features[kf].cpu().numpy()
        assert list(nodes) == list(fv)
        for i, nd in enumerate(nodes):
            assert list(feats[offs[i]:offs[i + 1]]) == fv[int(nd)]
    match, nm, ncorr = lb.match.cpu().numpy(), lb.nmatches.cpu().numpy(), lb.n_corr.cpu().numpy()
    results, states = lb.query_results(), lb.candidate_states()
    n_hyp = 0
    for q, (per, solvers, r) in enumerate(ref):
        for c in range(nc):
            pc = q * nc + c
            nm_r, m12_r, corr = per[c]
            assert nm[pc] == nm_r, (q, c)
            np.testing.assert_array_equal(match[pc, :1000], m12_r)
            if nm_r < 20:
                assert ncorr[pc] == -1
                continue
            assert ncorr[pc] == len(corr[0])
            np.testing.assert_array_equal(lb.corr_kf1_slots(pc), corr[4])
            st = states[pc]
            s = solvers[c]
            assert (st.n, st.max_iterations, st.iterations, st.best_inliers) == \
                (s.N, s.max_its, s.iterations, s.best), (q, c)
        g = results[q]
        assert (g.matched, g.round, g.n_inliers, g.hypotheses) == \
            (r["matched"], r["round"], r["n_inliers"], r["hypotheses"]), q
        assert g.draws == 3 * r["hypotheses"]
        after = g.rng_after  # the GPU's stream state after the query's draws
        assert orbgpu.lib().orbgpu_rand_r(ctypes.byref(after)) == r["after"]
        n_hyp += g.hypotheses
        if g.matched >= 0:
            pose = solvers[g.matched].best_pose
            np.testing.assert_allclose(np.array(g.R12).reshape(3, 3), pose["R12"], atol=2e-4)
            assert abs(g.s12 - pose["s12"]) < 2e-4
            t = np.array(g.t12)
            np.testing.assert_allclose(t, pose["t12"], atol=2e-4 * (1 + np.abs(pose["t12"]).max()))
            vb = lb.vb_inliers(q, results)
            want = np.zeros(1000, bool)
            want[solvers[g.matched].idx[solvers[g.matched].best_mask]] = True
            np.testing.assert_array_equal(vb, want)
    assert n_hyp > 0
    if np.ndim(fracs) and fracs[0] == 0.0:  # the unrelated first candidate never reaches 20 matches
        assert all(ncorr[q * nc] == -1 for q in range(nq))
    if np.ndim(fracs) == 0 and fracs == 0.0:
        assert all(r.matched == -1 for r in results[:nq])
        assert all(st.discarded for st in states[:nq * nc])


def test_cpp_query_ex_matches_python_pipeline():
    """orbref.compute_sim3_query_ex (oracle/loop_ref.cpp: what bench.py's
    loop-burst parity and the 100 x 5 GPU test compare against) equals the
    Python oracle pipeline: matches, solver states, outcome, pose and the
    stream after the query's draws."""
    import orbref
    k, L, p, l, d, w = 10, 4, *synth.synthetic_vocabulary_fast(10, 4, 5)
    avoc = loop_ref.ArrayVocabulary(k, L, 0, 0, p, l, d, w)
    cvoc = orbref.Vocabulary(k, L, p, l, d, w)
    nq, nc = 3, 4
    scene = synth.loop_burst_scene(nq, nc, d[l == 1], n_kp=500, inlier_frac=[0.0, 0.05, 0.4, 0.4],
                                   outlier_frac=[0.0, 0.1, 0.5, 0.5], seed=23)
    queries = [(q, [nq + q * nc + c for c in range(nc)]) for q in range(nq)]
    seeds = [41 + q for q in range(nq)]
    ref = _oracle_pipeline(scene, avoc, queries, seeds)
    matched = 0
    for (cur, cands), seed, (per, solvers, r) in zip(queries, seeds, ref):
        got = orbref.compute_sim3_query_ex(cvoc, scene, cur, cands, seed)
        for c in range(nc):
            assert got["nmatches"][c] == per[c][0]
            np.testing.assert_array_equal(got["m12"][c], per[c][1])
            if solvers[c] is not None:
                s = solvers[c]
                assert tuple(got["cand_state"][c][:4]) == (s.N, s.max_its, s.iterations, s.best)
        assert (got["matched"], got["round"], got["n_inliers"], got["hypotheses"]) == \
            (r["matched"], r["round"], r["n_inliers"], r["hypotheses"])
        assert got["rand_after"] == r["after"]
        if r["matched"] >= 0:
            matched += 1
            pose = solvers[r["matched"]].best_pose
            np.testing.assert_allclose(got["R12"], pose["R12"], atol=1e-6)
            np.testing.assert_allclose(got["t12"], pose["t12"], atol=1e-6 * (1 + np.abs(pose["t12"]).max()))
            assert abs(got["s12"] - pose["s12"]) < 1e-6
    assert matched > 0


@pytest.mark.gpu
def test_gpu_loop_burst_bench_size_vs_oracle(big_vocab):
    """bench.py's loop_burst leg at its timed size: 100 ComputeSim3 queries x 5
    candidates in one burst (the bench mix: 40 % true correspondences), every
    query against the C++ oracle (oracle/loop_ref.cpp, per-query random_r
    stream): SearchByBoW match counts and vpMatches12, solver states, the
    outcome (candidate, round, inliers, hypotheses, draws), the stream after
    the draws and the returned Sim3 within tests/test_ransac.py's tolerance."""
    torch = _gpu()
    from concurrent.futures import ThreadPoolExecutor

    import bow
    import loop
    import orbgpu
    import orbref
    import ransac
    path, (p, l, d, w) = big_vocab
    voc = bow.Vocabulary.load_text(str(path))
    nq, nc = 100, 5
    scene = synth.loop_burst_scene(nq, nc, d[l == 1], n_kp=1000, inlier_frac=0.4, outlier_frac=0.6, seed=55,
                                   fix_scale=False)
    kfs = loop.Keyframes(scene["desc"], scene["angle"], scene["octave"], scene["valid"], scene["mp_world"],
                         scene["Tcw"], scene["K"], scene["sigma2"])
    kfs.compute_bow(voc)
    queries = [(q, [nq + q * nc + c for c in range(nc)], 1000 + q) for q in range(nq)]
    lb = loop.LoopBurst(kfs, queries, fix_scale=False)
    lb.step()
    torch.cuda.synchronize()
    cvoc = orbref.Vocabulary(10, 6, p, l, d, w)
    scene["_c"] = None
    orbref.compute_sim3_query_ex(cvoc, scene, 0, queries[0][1], 1000)  # lays out the scene arrays once
    with ThreadPoolExecutor(8) as pool:  # ctypes releases the GIL; each query has its own random_r state
        refs = list(pool.map(lambda qc: orbref.compute_sim3_query_ex(cvoc, scene, qc[0], qc[1], qc[2]), queries))
    match, nm = lb.match.cpu().numpy(), lb.nmatches.cpu().numpy()
    results, states = lb.query_results(), lb.candidate_states()
    n_matched = 0
    for q, r in enumerate(refs):
        for c in range(nc):
            pc = q * nc + c
            assert nm[pc] == r["nmatches"][c], (q, c)
            np.testing.assert_array_equal(match[pc, :1000], r["m12"][c])
            if r["nmatches"][c] >= 20:
                st = states[pc]
                assert (st.n, st.max_iterations, st.iterations, st.best_inliers) == \
                    tuple(int(v) for v in r["cand_state"][c][:4]), (q, c)
        g = results[q]
        assert (g.matched, g.round, g.n_inliers, g.hypotheses) == \
            (r["matched"], r["round"], r["n_inliers"], r["hypotheses"]), q
        assert g.draws == 3 * r["hypotheses"]
        after = ransac.RandState.from_buffer_copy(bytes(g.rng_after))
        assert orbgpu.lib().orbgpu_rand_r(ctypes.byref(after)) == r["rand_after"], q
        if r["matched"] >= 0:
            n_matched += 1
            np.testing.assert_allclose(np.array(g.R12).reshape(3, 3), r["R12"], atol=2e-4)
            assert abs(g.s12 - r["s12"]) < 2e-4
            np.testing.assert_allclose(np.array(g.t12), r["t12"], atol=2e-4 * (1 + np.abs(r["t12"]).max()))
    assert n_matched >= 50
