"""RANSAC rows: the glibc-compatible random stream,
the Sim3Solver oracle, and the GPU Sim3 RANSAC against the oracle.

Tolerance (floating point): the hypotheses' Sim3 (T12, R12, t12, s12) match
the oracle to atol 2e-4 (rotation, scale) / 2e-4 * (1 + |t|) (translation);
integer outcomes (found, iterations consumed, best inlier count, best
hypothesis, inlier masks) must be identical."""
import ctypes
import math
import subprocess
import sys

import numpy as np
import pytest

import orbref
import synth

LIBC = ctypes.CDLL("libc.so.6")


def _ransac():
    import ransac
    return ransac


@pytest.mark.parametrize("seed", [0, 1, 2, 12345, 2 ** 31 + 5, 0xFFFFFFFF])
def test_rand_matches_glibc(seed):
    """orbgpu_srand_r/orbgpu_rand_r == glibc srand/rand (pinned by the host libc)."""
    ransac = _ransac()
    import orbgpu
    st = ransac.RandState()
    orbgpu.lib().orbgpu_srand_r(ctypes.byref(st), seed)
    LIBC.srand(ctypes.c_uint(seed))
    ours = [orbgpu.lib().orbgpu_rand_r(ctypes.byref(st)) for _ in range(2000)]
    ref = [LIBC.rand() for _ in range(2000)]
    assert ours == ref


def test_default_stream_is_srand1():
    """Without srand, glibc's stream equals srand(1); a fresh process checks it."""
    out = subprocess.run([sys.executable, "-c",
                          "import ctypes; l=ctypes.CDLL('libc.so.6'); print(*[l.rand() for _ in range(8)])"],
                         capture_output=True, text=True, check=True).stdout.split()
    ransac = _ransac()
    import orbgpu
    st = ransac.RandState()
    orbgpu.lib().orbgpu_srand_r(ctypes.byref(st), 1)
    assert [int(v) for v in out] == [orbgpu.lib().orbgpu_rand_r(ctypes.byref(st)) for _ in range(8)]


def test_random_int_and_triplet_draws_match_reference_formula():
    """RandomInt (Random.cpp:47-50) and the swap-remove draw (Sim3Solver.cpp:172-183)."""
    ransac = _ransac()
    ransac.srand(0)
    LIBC.srand(0)
    for lo, hi in [(0, 0), (0, 9), (3, 17), (0, 999)]:
        for _ in range(50):
            ref = int((LIBC.rand() / (2147483647 + 1.0)) * (hi - lo + 1)) + lo
            assert ransac.random_int(lo, hi) == ref
    st = ransac.get_state()
    tri = ransac.draw_triplets(57, 40)
    ransac.set_state(st)
    again = ransac.draw_triplets(57, 40)
    assert np.array_equal(tri, again)
    assert all(len(set(r)) == 3 for r in tri.tolist()) and tri.min() >= 0 and tri.max() < 57


def test_set_ransac_parameters_iterations():
    """nIterations = ceil(log(1-p)/log(1-eps^3)) capped (Sim3Solver.cpp:111-141)."""
    ransac = _ransac()
    P = synth.sim3_problem(200, 0.5, seed=3)
    s = ransac.Sim3Solver(P["X1"], P["X2"], P["sigma2_1"], P["sigma2_2"], P["K1"], P["K2"])
    s.set_ransac_parameters(0.99, 20, 300)
    eps = np.float32(20) / np.float32(200)
    assert s.max_its == min(300, math.ceil(math.log(0.01) / math.log(1 - float(eps) ** 3)))
    s.set_ransac_parameters(0.99, 200, 300)   # minInliers == N
    assert s.max_its == 1
    s.set_ransac_parameters(0.99, 150, 300)   # eps = 0.75
    assert s.max_its == math.ceil(math.log(0.01) / math.log(1 - 0.75 ** 3))
    s.set_ransac_parameters(0.99, 400, 300)   # eps > 1: NaN -> 1
    assert s.max_its == 1


def _run_oracle(P, samples, min_inl, fix_scale, best=0):
    ransac = _ransac()
    return orbref.sim3_ransac(P["X1"], P["X2"], ransac.max_error(P["sigma2_1"]), ransac.max_error(P["sigma2_2"]),
                              P["K1"], P["K2"], fix_scale, min_inl, best, samples)


@pytest.mark.parametrize("fix_scale", [False, True])
def test_sim3_oracle_recovers_ground_truth(fix_scale):
    P = synth.sim3_problem(300, 0.6, seed=11, fix_scale=fix_scale)
    rng = np.random.default_rng(5)
    samples = np.stack([rng.choice(300, 3, replace=False) for _ in range(300)]).astype(np.int32)
    r = _run_oracle(P, samples, 20, fix_scale)
    assert r["found"] == 1 and r["best_inliers"] > 20
    np.testing.assert_allclose(r["R12"], P["R"], atol=2e-2)
    assert abs(r["s12"] - P["s"]) < 2e-2
    inl = r["inliers"].astype(bool)
    assert (inl & P["inlier"]).sum() >= 0.9 * inl.sum()


def _problems(count=24, seed=100):
    """a mixed batch: sizes, inlier ratios (incl. none), scale fixed or not"""
    rng = np.random.default_rng(seed)
    out = []
    for b in range(count):
        n = int(rng.integers(3, 400))
        frac = [0.0, 0.1, 0.3, 0.6, 0.9][b % 5]
        fix = bool(b % 2)
        P = synth.sim3_problem(n, frac, seed=seed + b, fix_scale=fix)
        n_hyp = int(rng.integers(0, 300)) if b % 7 else 300
        samples = np.stack([rng.choice(n, 3, replace=False) for _ in range(n_hyp)]).astype(np.int32) \
            if n_hyp else np.zeros((0, 3), np.int32)
        min_inl = int(rng.integers(3, 40))
        best = int(rng.integers(0, 10)) if b % 3 == 0 else 0
        out.append((P, samples, min_inl, fix, best))
    return out


@pytest.mark.gpu
def test_sim3_gpu_batch_vs_oracle():
    ransac = _ransac()
    probs = _problems()
    B = len(probs)
    arr = (ransac.Sim3Problem * B)()
    X1s, X2s, E1, E2, S = [], [], [], [], []
    off = soff = 0
    for b, (P, samples, min_inl, fix, best) in enumerate(probs):
        p = arr[b]
        p.n, p.offset, p.fix_scale, p.min_inliers, p.best_inliers = len(P["X1"]), off, int(fix), min_inl, best
        p.n_hyp, p.sample_offset = len(samples), soff
        p.K1[:] = [float(v) for v in P["K1"]]
        p.K2[:] = [float(v) for v in P["K2"]]
        X1s.append(P["X1"]); X2s.append(P["X2"])
        E1.append(ransac.max_error(P["sigma2_1"])); E2.append(ransac.max_error(P["sigma2_2"]))
        S.append(samples)
        off += len(P["X1"]); soff += len(samples)
    inl = np.full(off, 7, np.uint8)
    res = ransac.sim3_ransac_batch(arr, np.concatenate(X1s), np.concatenate(X2s), np.concatenate(E1),
                                   np.concatenate(E2), np.concatenate(S), inl)
    nfound = 0
    for b, (P, samples, min_inl, fix, best) in enumerate(probs):
        g, r = res[b], _run_oracle(P, samples, min_inl, fix, best)
        assert (g.found, g.consumed, g.best_inliers, g.best_hyp) == \
            (r["found"], r["consumed"], r["best_inliers"], r["best_hyp"]), f"problem {b}"
        o, n = arr[b].offset, arr[b].n
        if r["best_hyp"] >= 0:
            np.testing.assert_array_equal(inl[o:o + n], r["inliers"], err_msg=f"problem {b}")
            np.testing.assert_allclose(np.array(g.R12).reshape(3, 3), r["R12"], atol=2e-4)
            assert abs(g.s12 - r["s12"]) <= 2e-4 * max(1.0, abs(r["s12"]))
            t = r["t12"]
            np.testing.assert_allclose(np.array(g.t12), t, atol=2e-4 * (1 + np.abs(t).max()))
        else:
            assert (inl[o:o + n] == 7).all()
        nfound += g.found
    assert nfound >= 5


@pytest.mark.gpu
def test_sim3_solver_iterate_consumes_the_reference_stream():
    """Sim3Solver.iterate(5) round-robin like LoopClosing (LoopClosing.cpp:339-411):
    outputs and the random stream position equal a sequential replay with the
    oracle (one hypothesis at a time, draws from glibc itself)."""
    ransac = _ransac()
    probs = [synth.sim3_problem(n, f, seed=40 + i) for i, (n, f) in enumerate([(150, 0.2), (60, 0.5), (300, 0.05)])]
    ransac.srand(0)
    solvers = [ransac.Sim3Solver(P["X1"], P["X2"], P["sigma2_1"], P["sigma2_2"], P["K1"], P["K2"], fix_scale=False)
               for P in probs]
    for s in solvers:
        s.set_ransac_parameters(0.99, 20, 300)
    # reference replay
    LIBC.srand(0)
    state = [{"it": 0, "best": 0} for _ in probs]

    def ref_iterate(i, n_it):
        P, st, s = probs[i], state[i], solvers[i]
        N = len(P["X1"])
        cur = 0
        while st["it"] < s.max_its and cur < n_it:
            cur += 1
            st["it"] += 1
            avail = list(range(N))
            tri = []
            for _ in range(3):
                r = int((LIBC.rand() / (2147483647 + 1.0)) * len(avail))
                tri.append(avail[r]); avail[r] = avail[-1]; avail.pop()
            o = _run_oracle(P, np.array([tri], np.int32), 20, False, st["best"])
            st["best"] = o["best_inliers"]
            if o["found"]:
                return True, o
        return False, None

    done = [False] * len(probs)
    for _round in range(80):
        for i, s in enumerate(solvers):
            if done[i]:
                continue
            T, no_more, inl, n = s.iterate(5)
            ok, o = ref_iterate(i, 5)
            assert (T is not None) == ok
            assert s.best_inliers == state[i]["best"] and s.iterations == state[i]["it"]
            if ok:
                assert n == o["best_inliers"]
                np.testing.assert_array_equal(inl, o["inliers"].astype(bool))
                done[i] = True
            elif no_more:
                done[i] = True
        if all(done):
            break
    # both streams are at the same position
    assert [ransac.rand() for _ in range(5)] == [LIBC.rand() for _ in range(5)]
