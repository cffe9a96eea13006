"""PnPsolver row: EPnP + RANSAC on the GPU against the
numpy oracle (oracle/pnp_ref.py).

Tolerance (floating point, the north star's "PnP pose within a stated float
tolerance"): the refined pose Tcw of the GPU and of the oracle agree to
|dR|_max <= 1e-3 and |dt|_max <= 1e-3 * (1 + |t|_max); integer outcomes
(found, iterations consumed, best inlier count) must be identical, and the
inlier masks may differ in at most 1 % of the correspondences (points whose
reprojection error sits on the 5.991 sigma^2 threshold)."""
import ctypes
import math

import numpy as np
import pytest

import pnp_ref
import synth

LIBC = ctypes.CDLL("libc.so.6")


def _ransac():
    import ransac
    return ransac


def test_qr_solve_restatement_is_least_squares():
    rng = np.random.default_rng(0)
    for _ in range(20):
        A = rng.normal(size=(6, 4))
        b = rng.normal(size=6)
        np.testing.assert_allclose(pnp_ref._qr_solve(A, b), np.linalg.lstsq(A, b, rcond=None)[0], atol=1e-9)


def test_epnp_minimal_sets_mostly_accurate():
    """EPnP on 4 noise-free points is approximate (three beta linearisations +
    5 Gauss-Newton steps); with the canonical null-space basis most minimal
    sets land within a few pixels, as RANSAC needs."""
    errs = []
    for trial in range(100):
        P = synth.pnp_problem(4, 1.0, seed=500 + trial, noise_px=0.0)
        errs.append(pnp_ref.compute_pose(P["P3w"].astype(np.float64), P["P2"].astype(np.float64), P["cam"])[2])
    assert np.mean(np.array(errs) < 5.0) >= 0.6


@pytest.mark.parametrize("n", [6, 50])
def test_epnp_oracle_exact_on_noise_free_points(n):
    P = synth.pnp_problem(n, 1.0, seed=n, noise_px=0.0)
    R, t, err = pnp_ref.compute_pose(P["P3w"].astype(np.float64), P["P2"].astype(np.float64), P["cam"])
    assert err < 1e-3
    np.testing.assert_allclose(R, P["R"], atol=1e-5)
    np.testing.assert_allclose(t, P["t"], atol=1e-4)


def test_set_ransac_parameters_like_tracking():
    """SetRansacParameters(0.99,10,300,4,0.5,5.991) (Tracking.cpp:1796; PnPsolver.cpp:159-195)."""
    ransac = _ransac()
    for n, expect_min in [(30, 15), (15, 10), (9, 10), (201, 100)]:
        P = synth.pnp_problem(n, 0.5, seed=1)
        s = ransac.PnPsolver(P["P3w"], P["P2"], P["sigma2"], *P["cam"])
        s.set_ransac_parameters(0.99, 10, 300, 4, 0.5, 5.991)
        assert s.min_inliers == max(int(np.float32(n) * np.float32(0.5)), 10, 4) == expect_min
        eps = max(np.float32(0.5), np.float32(s.min_inliers) / np.float32(n))
        if s.min_inliers == n:
            assert s.max_its == 1
        elif eps < 1:
            assert s.max_its == max(1, min(300, math.ceil(math.log(0.01) / math.log(1 - float(eps) ** 3))))
        np.testing.assert_array_equal(s.maxerr, P["sigma2"] * np.float32(5.991))


def test_oracle_ransac_finds_pose():
    P = synth.pnp_problem(120, 0.5, seed=7)
    rng = np.random.default_rng(3)
    samples = np.stack([rng.choice(120, 4, replace=False) for _ in range(300)])
    maxerr = P["sigma2"] * np.float32(5.991)
    r = pnp_ref.ransac_call(P["P3w"], P["P2"], maxerr, P["cam"], 40, 0, np.zeros(120, bool), samples)
    assert r["found"] == 1
    np.testing.assert_allclose(r["refined_R"], P["R"], atol=5e-3)
    assert (r["refined_mask"] & P["inlier"]).sum() >= 0.95 * P["inlier"].sum()


def _pose_close(Tg, R, t):
    Tg = np.asarray(Tg, np.float64).reshape(4, 4)
    assert np.abs(Tg[:3, :3] - R).max() <= 1e-3
    assert np.abs(Tg[:3, 3] - t).max() <= 1e-3 * (1 + np.abs(t).max())


@pytest.mark.gpu
def test_pnp_gpu_batch_vs_oracle():
    ransac = _ransac()
    rng = np.random.default_rng(9)
    cases = []
    for b in range(16):
        n = int(rng.integers(12, 300))
        frac = [0.0, 0.3, 0.5, 0.8, 1.0][b % 5]
        P = synth.pnp_problem(n, frac, seed=200 + b)
        n_hyp = int(rng.integers(1, 200))
        samples = np.stack([rng.choice(n, 4, replace=False) for _ in range(n_hyp)]).astype(np.int32)
        min_inl = max(int(np.float32(n) * np.float32(0.5)), 10)
        cases.append((P, samples, min_inl))
    arr = (ransac.PnPProblem * len(cases))()
    P3, P2, E, S = [], [], [], []
    off = soff = 0
    for b, (P, samples, min_inl) in enumerate(cases):
        p = arr[b]
        n = len(P["P3w"])
        p.n, p.offset, p.min_inliers, p.best_inliers, p.n_hyp, p.sample_offset = n, off, min_inl, 0, len(samples), soff
        p.fu, p.fv, p.uc, p.vc = P["cam"]
        P3.append(P["P3w"]); P2.append(P["P2"]); E.append(P["sigma2"] * np.float32(5.991)); S.append(samples)
        off += n; soff += len(samples)
    bm = np.zeros(off, np.uint8)
    rm = np.zeros(off, np.uint8)
    res = ransac.pnp_ransac_batch(arr, np.concatenate(P3), np.concatenate(P2), np.concatenate(E),
                                  np.concatenate(S), bm, rm)
    nfound = 0
    for b, (P, samples, min_inl) in enumerate(cases):
        g = res[b]
        n = len(P["P3w"])
        o = pnp_ref.ransac_call(P["P3w"], P["P2"], P["sigma2"] * np.float32(5.991), P["cam"], min_inl, 0,
                                np.zeros(n, bool), samples)
        assert (g.found, g.consumed, g.best_inliers) == (o["found"], o["consumed"], o["best_inliers"]), f"case {b}"
        off_b = arr[b].offset
        if o["found"]:
            nfound += 1
            _pose_close(g.refined_Tcw, o["refined_R"], o["refined_t"])
            diff = (rm[off_b:off_b + n].astype(bool) != o["refined_mask"]).sum()
            assert diff <= max(1, n // 100), f"case {b}: {diff} refined-mask differences"
            assert abs(g.refined_inliers - int(o["refined_mask"].sum())) <= max(1, n // 100)
    assert nfound >= 6


@pytest.mark.gpu
def test_pnp_solver_iterate_consumes_the_reference_stream():
    """PnPsolver.iterate(5) like Tracking::Relocalization (Tracking.cpp:1815-1830):
    outcome and random-stream position equal a sequential replay with the
    oracle drawing from glibc itself."""
    ransac = _ransac()
    P = synth.pnp_problem(80, 0.6, seed=77)
    ransac.srand(0)
    s = ransac.PnPsolver(P["P3w"], P["P2"], P["sigma2"], *P["cam"])
    s.set_ransac_parameters(0.99, 10, 300, 4, 0.5, 5.991)
    T, no_more, inl, n = s.iterate(5)
    # replay: the `||` loop runs max(maxIts - 0, 5) iterations unless Refine succeeds
    LIBC.srand(0)
    N = len(P["P3w"])
    samples = []
    for _ in range(max(s.max_its, 5)):
        avail = list(range(N))
        tri = []
        for _ in range(4):
            r = int((LIBC.rand() / (2147483647 + 1.0)) * len(avail))
            tri.append(avail[r]); avail[r] = avail[-1]; avail.pop()
        samples.append(tri)
    o = pnp_ref.ransac_call(P["P3w"], P["P2"], s.maxerr, P["cam"], s.min_inliers, 0, np.zeros(N, bool),
                            np.array(samples))
    assert o["found"] == 1 and T is not None
    assert s.iterations == o["consumed"]
    _pose_close(T, o["refined_R"], o["refined_t"])
    # rewind glibc to the position the reference would be at
    LIBC.srand(0)
    for _ in range(4 * o["consumed"]):
        LIBC.rand()
    assert [ransac.rand() for _ in range(5)] == [LIBC.rand() for _ in range(5)]
