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


def _qr_cases():
    """6 x 4 systems whose LAST row holds a column's largest magnitude: the
    reference's eta scan (PnPsolver.cpp:975-980) never reads the last row, so
    eta -- and the rounding of every later step -- differs from a scan over
    all rows; plus a system the reference calls singular (rows k .. nr-2 of
    column 0 zero, the last row not): it returns with X untouched."""
    rng = np.random.default_rng(7)
    cases = []
    for t in range(32):
        A = rng.normal(size=(6, 4))
        A[5, t % 4] = 40.0 * (1 + rng.random())  # last row: the column maximum
        cases.append((A, rng.normal(size=6)))
    A = rng.normal(size=(6, 4))
    A[:5, 0] = 0.0
    cases.append((A, rng.normal(size=6)))
    return cases


def _qr_all_rows(A, b):
    """the same Householder QR with eta over ALL rows and a division (the
    pre-round-4 restatement): what the letter-faithful scan must differ from"""
    A = A.copy()
    b = b.copy()
    nr, nc = A.shape
    A1, A2 = np.zeros(nc), np.zeros(nc)
    for k in range(nc):
        eta = np.abs(A[k:, k]).max()
        A[k:, k] /= eta
        sigma = np.sqrt((A[k:, k] ** 2).sum())
        sigma = -sigma if A[k, k] < 0 else sigma
        A[k, k] += sigma
        A1[k], A2[k] = sigma * A[k, k], -eta * sigma
        for j in range(k + 1, nc):
            tau = (A[k:, k] * A[k:, j]).sum() / A1[k]
            A[k:, j] -= tau * A[k:, k]
    for j in range(nc):
        b[j:] -= (A[j:, j] * b[j:]).sum() / A1[j] * A[j:, j]
    X = np.zeros(nc)
    X[nc - 1] = b[nc - 1] / A2[nc - 1]
    for i in range(nc - 2, -1, -1):
        X[i] = (b[i] - (A[i, i + 1:] * X[i + 1:]).sum()) / A2[i]
    return X


def _qr_cpp(A, b, X0):
    import ctypes
    import orbref
    L = orbref.lib()
    f = L.orbref_qr_solve_6x4
    f.argtypes = [ctypes.c_void_p] * 3
    A = np.ascontiguousarray(A, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    X = np.array(X0, np.float64)
    f(A.ctypes.data, b.ctypes.data, X.ctypes.data)
    return X


def test_qr_solve_eta_scan_is_the_references():
    """oracle/pnp_ref.py == oracle/pnp_ref.cpp bit for bit on the eta-scan
    cases; the last-row-maximum systems differ in rounding from an all-rows
    scan on some systems (the scan is observable), and the singular case
    leaves X as it was."""
    cases = _qr_cases()
    X0 = np.array([0.25, -1.5, 3.0, 7.0])
    differ = 0
    for A, b in cases[:-1]:
        xp = pnp_ref._qr_solve(A, b, X0)
        xc = _qr_cpp(A, b, X0)
        assert xp.tobytes() == xc.tobytes()
        np.testing.assert_allclose(xp, np.linalg.lstsq(A, b, rcond=None)[0], rtol=1e-9, atol=1e-9)
        differ += xp.tobytes() != _qr_all_rows(A, b).tobytes()
    assert differ > 0
    A, b = cases[-1]
    assert pnp_ref._qr_solve(A, b, X0).tobytes() == X0.tobytes()
    assert _qr_cpp(A, b, X0).tobytes() == X0.tobytes()


@pytest.mark.gpu
def test_gpu_qr_solve_eta_scan_equals_oracle():
    """csrc/epnp.h qr_solve_6x4 (the EPnP Gauss-Newton solve on the GPU) on
    the same cases, through orbgpu_debug_qr_solve_6x4_device: bit-identical
    to the oracle, the singular case leaving X untouched"""
    import ctypes
    import orbgpu
    import torch
    cases = _qr_cases()
    X0 = np.array([0.25, -1.5, 3.0, 7.0])
    A = torch.tensor(np.stack([a.reshape(-1) for a, _ in cases]), dtype=torch.float64, device="cuda")
    b = torch.tensor(np.stack([bb for _, bb in cases]), dtype=torch.float64, device="cuda")
    X = torch.tensor(np.tile(X0, (len(cases), 1)), dtype=torch.float64, device="cuda")
    f = orbgpu.lib().orbgpu_debug_qr_solve_6x4_device
    f.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_void_p]
    assert f(A.data_ptr(), b.data_ptr(), X.data_ptr(), len(cases), None) == 0
    torch.cuda.synchronize()
    got = X.cpu().numpy()
    for i, (a, bb) in enumerate(cases):
        assert got[i].tobytes() == pnp_ref._qr_solve(a, bb, X0).tobytes(), i


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
