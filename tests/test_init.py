"""Initializer::CheckHomography / CheckFundamental and the kept-iteration
choice of FindHomography / FindFundamental (src/Initializer.cpp:160-290,
:390-594): the CPU restatement (oracle/init_ref.py) on known answers, and the
batched GPU scorer (csrc/init.hip) against it -- scores and inlier flags
bit-exact.  Parity of the restatement against the reference itself is
unpinned (the reference needs OpenCV; no fixtures exist), see DESIGN.md §6."""
import numpy as np
import pytest

import init_ref

F = np.float32
K = np.array([[517.3, 0, 318.6], [0, 516.5, 255.3], [0, 0, 1]])


def _scene(n, planar, seed, outliers=0.2, noise=0.7):
    """two views of n points (planar or not) -> ((n,4) float32 matches, H21 or F21)"""
    rng = np.random.default_rng(seed)
    if planar:
        X = np.c_[rng.uniform(-2, 2, n), rng.uniform(-1.5, 1.5, n), np.full(n, 5.0)]
    else:
        X = np.c_[rng.uniform(-2, 2, n), rng.uniform(-1.5, 1.5, n), rng.uniform(3, 8, n)]
    a = 0.05
    R = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]])
    t = np.array([0.3, 0.02, 0.05])
    x1 = (K @ X.T).T
    x2 = (K @ (R @ X.T + t[:, None])).T
    p1, p2 = x1[:, :2] / x1[:, 2:], x2[:, :2] / x2[:, 2:]
    p2 = p2 + rng.normal(0, noise, p2.shape)
    m = rng.random(n) < outliers
    p2[m] = rng.uniform([0, 0], [640, 480], (m.sum(), 2))
    pts = np.c_[p1, p2].astype(F)
    Ki = np.linalg.inv(K)
    if planar:  # plane z = 5: H = K (R + t n^T / d) K^-1
        M = K @ (R + np.outer(t, [0, 0, 1]) / 5.0) @ Ki
    else:
        tx = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])
        M = Ki.T @ tx @ R @ Ki
    return pts, M / M[2, 2] if planar else M / np.linalg.norm(M)


def _hyps(M, nhyp, seed, scale=2e-3):
    """RANSAC-like hypotheses: the true model perturbed, plus degenerate ones"""
    rng = np.random.default_rng(seed)
    H = M[None] * (1 + rng.normal(0, scale, (nhyp, 3, 3)))
    H[0] = M
    if nhyp > 3:
        H[1] = 0.0                 # all-zero: 0/0 -> NaN chi-squares
        H[2] = np.diag([1.0, 1, 0])  # w = 0 on every point -> inf
    return H.astype(F)


def _inv(H):
    out = np.empty_like(H)
    for k in range(H.shape[0]):
        try:
            out[k] = np.linalg.inv(H[k].astype(np.float64)).astype(F)
        except np.linalg.LinAlgError:
            out[k] = 0.0
    return out


# ---- CPU: the restatement on known answers --------------------------------

def test_oracle_exact_homography_scores_every_match():
    pts, H = _scene(300, True, 1, outliers=0.0, noise=0.0)
    H = H.astype(F)
    s, inl = init_ref.check_homography(pts, H, np.linalg.inv(H).astype(F))
    assert inl.all()
    assert 2 * 300 * 5.991 * 0.999 < s <= 2 * 300 * 5.991


def test_oracle_outliers_are_flagged():
    pts, H = _scene(400, True, 2, outliers=0.3, noise=0.0)
    H = H.astype(F)
    _, inl = init_ref.check_homography(pts, H, np.linalg.inv(H).astype(F))
    assert 0.6 < inl.mean() < 0.8
    pts, Fm = _scene(400, False, 3, outliers=0.3, noise=0.0)
    _, inl = init_ref.check_fundamental(pts, Fm.astype(F))
    assert 0.6 < inl.mean() < 0.8


def test_oracle_sequential_float_sum():
    # two terms per match added in loop order, in float32 (:447-478)
    pts = np.array([[10, 10, 10, 10], [20, 20, 20.5, 20]], F)
    I = np.eye(3, dtype=F)
    s, inl = init_ref.check_homography(pts, I, I, sigma=1.0)
    t = F(5.991) - F(0.25)
    want = F(F(F(F(0) + F(5.991)) + F(5.991)) + t)
    want = F(want + t)
    assert s == want and inl.tolist() == [True, True]


def test_oracle_select_best_first_strict_max():
    assert init_ref.select_best([0.0, -1.0]) == -1
    assert init_ref.select_best([1.0, 3.0, 3.0, 2.0]) == 1
    assert init_ref.select_best([]) == -1


def test_select_best_abi_matches_oracle():
    import initializer
    rng = np.random.default_rng(5)
    for _ in range(20):
        s = rng.integers(-2, 5, 50).astype(F)
        assert initializer.select_best(s) == init_ref.select_best(s)
    assert initializer.select_best(np.zeros(0, F)) == -1


# ---- GPU: batched scorer vs the restatement, bit-exact --------------------

def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.mark.gpu
@pytest.mark.parametrize("n,nhyp,seed", [(0, 4, 0), (1, 3, 1), (255, 16, 2), (700, 200, 3), (2049, 64, 4),
                                          (9001, 8, 5)])  # 9001: two full 4096-match chunks + a tail
def test_gpu_check_homography_bit_exact(n, nhyp, seed):
    torch = _gpu()
    import initializer
    pts, H = _scene(max(n, 1), True, seed)
    pts = pts[:n]
    H21 = _hyps(H, nhyp, seed + 10)
    H12 = _inv(H21)
    dev = torch.device("cuda", 0)
    scores = torch.full((nhyp,), -7.0, device=dev)
    inl = torch.full((nhyp, n), 9, dtype=torch.uint8, device=dev)
    initializer.check_homography_batch(torch.from_numpy(pts).to(dev), torch.from_numpy(H21).to(dev),
                                       torch.from_numpy(H12).to(dev), 1.0, scores, inl)
    torch.cuda.synchronize()
    s, f = scores.cpu().numpy(), inl.cpu().numpy()
    for h in range(nhyp):
        ws, wi = init_ref.check_homography(pts, H21[h], H12[h], 1.0)
        np.testing.assert_array_equal(s[h], ws, err_msg=f"hyp {h}")
        np.testing.assert_array_equal(f[h].astype(bool), wi, err_msg=f"hyp {h}")
    assert initializer.select_best(s) == init_ref.select_best(s)


@pytest.mark.gpu
@pytest.mark.parametrize("n,nhyp,seed,sigma", [(0, 2, 0, 1.0), (3, 5, 1, 1.0), (700, 200, 2, 1.0),
                                               (1500, 32, 3, 1.6), (9001, 6, 4, 1.0)])
def test_gpu_check_fundamental_bit_exact(n, nhyp, seed, sigma):
    torch = _gpu()
    import initializer
    pts, M = _scene(max(n, 1), False, seed)
    pts = pts[:n]
    F21 = _hyps(M, nhyp, seed + 20, scale=5e-3)
    dev = torch.device("cuda", 0)
    scores = torch.zeros(nhyp, device=dev)
    inl = torch.zeros((nhyp, n), dtype=torch.uint8, device=dev)
    initializer.check_fundamental_batch(torch.from_numpy(pts).to(dev), torch.from_numpy(F21).to(dev), sigma,
                                        scores, inl)
    torch.cuda.synchronize()
    s, f = scores.cpu().numpy(), inl.cpu().numpy()
    for h in range(nhyp):
        ws, wi = init_ref.check_fundamental(pts, F21[h], sigma)
        np.testing.assert_array_equal(s[h], ws, err_msg=f"hyp {h}")
        np.testing.assert_array_equal(f[h].astype(bool), wi, err_msg=f"hyp {h}")
    assert initializer.select_best(s) == init_ref.select_best(s)


@pytest.mark.gpu
def test_gpu_check_both_matches_separate_launches():
    torch = _gpu()
    import initializer
    n = 900
    pts, H = _scene(n, True, 7)
    _, M = _scene(n, False, 8)
    H21, F21 = _hyps(H, 200, 9), _hyps(M, 150, 10, scale=5e-3)
    H12 = _inv(H21)
    dev = torch.device("cuda", 0)
    d = {k: torch.from_numpy(v).to(dev) for k, v in dict(p=pts, h=H21, g=H12, f=F21).items()}
    sh, sf = torch.zeros(200, device=dev), torch.zeros(150, device=dev)
    ih, jf = torch.zeros((200, n), dtype=torch.uint8, device=dev), torch.zeros((150, n), dtype=torch.uint8, device=dev)
    initializer.check_both_batch(d["p"], d["h"], d["g"], d["f"], 1.0, sh, ih, sf, jf)
    torch.cuda.synchronize()
    s_h, i_h, s_f, i_f = sh.cpu().numpy(), ih.cpu().numpy(), sf.cpu().numpy(), jf.cpu().numpy()
    for h in range(200):
        ws, wi = init_ref.check_homography(pts, H21[h], H12[h], 1.0)
        np.testing.assert_array_equal(s_h[h], ws)
        np.testing.assert_array_equal(i_h[h].astype(bool), wi)
    for h in range(150):
        ws, wi = init_ref.check_fundamental(pts, F21[h], 1.0)
        np.testing.assert_array_equal(s_f[h], ws)
        np.testing.assert_array_equal(i_f[h].astype(bool), wi)


@pytest.mark.gpu
def test_gpu_check_both_multi_chunk():
    """n = 9001 crosses two 4096-match chunk boundaries of init.hip's score
    loop (the serial sum carried across chunks) and leaves a partial tail."""
    torch = _gpu()
    import initializer
    n = 9001
    pts, H = _scene(n, True, 17)
    _, M = _scene(n, False, 18)
    H21, F21 = _hyps(H, 5, 19), _hyps(M, 4, 20, scale=5e-3)
    H12 = _inv(H21)
    dev = torch.device("cuda", 0)
    d = {k: torch.from_numpy(v).to(dev) for k, v in dict(p=pts, h=H21, g=H12, f=F21).items()}
    sh, sf = torch.zeros(5, device=dev), torch.zeros(4, device=dev)
    ih = torch.zeros((5, n), dtype=torch.uint8, device=dev)
    jf = torch.zeros((4, n), dtype=torch.uint8, device=dev)
    initializer.check_both_batch(d["p"], d["h"], d["g"], d["f"], 1.0, sh, ih, sf, jf)
    torch.cuda.synchronize()
    for h in range(5):
        ws, wi = init_ref.check_homography(pts, H21[h], H12[h], 1.0)
        np.testing.assert_array_equal(sh[h].cpu().numpy(), ws)
        np.testing.assert_array_equal(ih[h].cpu().numpy().astype(bool), wi)
    for h in range(4):
        ws, wi = init_ref.check_fundamental(pts, F21[h], 1.0)
        np.testing.assert_array_equal(sf[h].cpu().numpy(), ws)
        np.testing.assert_array_equal(jf[h].cpu().numpy().astype(bool), wi)


def test_binding_rejects_host_and_wrong_dtype():
    """A host array or a float64 matrix must never reach the kernel."""
    torch = pytest.importorskip("torch")
    import initializer
    pts = np.zeros((4, 4), F)
    H = np.zeros((2, 3, 3), F)
    with pytest.raises(TypeError):  # numpy (host) arrays
        initializer.check_fundamental_batch(pts, H, 1.0, np.zeros(2, F), np.zeros((2, 4), np.uint8))
    tp = torch.zeros((4, 4), dtype=torch.float32)
    with pytest.raises(TypeError):  # CPU tensors
        initializer.check_fundamental_batch(tp, torch.zeros((2, 3, 3)), 1.0, torch.zeros(2),
                                            torch.zeros((2, 4), dtype=torch.uint8))


# ---- model hypotheses: Normalize + ComputeH21 / ComputeF21 ----------------

def _sets_from_glibc(nm, n_iter=200, seed=0):
    """Initialize's draws (Initializer.cpp:96-115) with the host glibc rand()"""
    import ctypes
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(seed)
    out = np.zeros((n_iter, 8), np.int32)
    for it in range(n_iter):
        avail = list(range(nm))
        for j in range(8):
            r = int((libc.rand() / (2147483647 + 1.0)) * len(avail))
            out[it, j] = avail[r]
            avail[r] = avail[-1]
            avail.pop()
    return out


def _frames(n, planar, seed, extra=40):
    """keypoints of two frames (with unmatched extras) and vMatches12"""
    pts, M = _scene(n, planar, seed)
    rng = np.random.default_rng(seed)
    kp1 = np.vstack([pts[:, :2], rng.uniform([0, 0], [640, 480], (extra, 2))]).astype(F)
    kp2 = np.vstack([rng.uniform([0, 0], [640, 480], (extra, 2)), pts[:, 2:]]).astype(F)
    m12 = np.full(len(kp1), -1, np.int32)
    m12[:n] = np.arange(n) + extra
    return kp1, kp2, m12, M


def test_draw_sets_match_glibc():
    import initializer
    import ransac
    ransac.srand(0)
    np.testing.assert_array_equal(initializer.draw_sets(150, 200), _sets_from_glibc(150))


def test_oracle_normalize_and_models():
    kp1, kp2, m12, M = _frames(300, True, 31)
    pn, T = init_ref.normalize(kp1)
    assert abs(float(np.abs(pn[:, 0]).mean()) - 1.0) < 1e-4 and abs(float(pn[:, 1].mean())) < 1e-4
    np.testing.assert_allclose((T @ np.c_[kp1, np.ones(len(kp1))].T).T[:, :2], pn, atol=1e-4)
    first = np.nonzero(m12 >= 0)[0]
    pairs = np.stack([first, m12[first]], 1)
    r = init_ref.find_models(kp1, kp2, pairs, _sets_from_glibc(len(pairs), 50))
    H = r["H21"][r["best_h"]].astype(np.float64)
    H = H / H[2, 2]
    assert np.abs(H - M).max() < 0.05 * np.abs(M).max()
    assert r["RH"] > 0.4  # planar scene: the homography wins (Initializer.cpp:140)


@pytest.mark.gpu
@pytest.mark.parametrize("n,planar,seed", [(300, True, 41), (1000, False, 42), (600, True, 43), (120, False, 44)])
def test_gpu_find_models_vs_oracle(n, planar, seed):
    """Normalize + the 200 H/F hypotheses on the GPU (init_models.hip) + the
    bit-exact scorers, against init_ref.find_models: the kept iterations are
    equal, H/F of every iteration agree to 1e-3 (up to sign: the SVD's null
    vector sign is arbitrary and both scores are sign invariant), scores to
    1e-4 relative."""
    _gpu()
    import initializer
    kp1, kp2, m12, _ = _frames(n, planar, seed)
    first = np.nonzero(m12 >= 0)[0]
    pairs = np.stack([first, m12[first]], 1)
    sets = _sets_from_glibc(len(pairs))
    g = initializer.find_models(kp1, kp2, m12, sets=sets)
    r = init_ref.find_models(kp1, kp2, pairs, sets)
    assert g["best_h"] == r["best_h"] and g["best_f"] == r["best_f"]

    def close(a, b, tol):
        a, b = a.astype(np.float64).reshape(-1, 9), b.astype(np.float64).reshape(-1, 9)
        sc = np.abs(b).max(1, keepdims=True)
        return np.minimum(np.abs(a - b), np.abs(a + b)).max(1) / sc[:, 0] < tol

    assert close(g["H21"], r["H21"], 1e-3).mean() > 0.97
    assert close(g["F21"], r["F21"], 1e-3).mean() > 0.97
    for k in ("scores_h", "scores_f"):
        np.testing.assert_allclose(g[k], r[k], rtol=1e-4, atol=1e-3)
    assert abs(float(g["RH"]) - float(r["RH"])) < 1e-4
    bh = r["best_h"]
    ref_inl = init_ref.check_homography(r["pts"], r["H21"][bh], r["H12"][bh])[1]
    assert (g["inliers_h"] != ref_inl).sum() <= max(1, n // 200)


# ---- ReconstructH / ReconstructF (Initializer.cpp:596-963) ----------------
_A = 0.05
_R_TRUE = np.array([[np.cos(_A), 0, np.sin(_A)], [0, 1, 0], [-np.sin(_A), 0, np.cos(_A)]])


def _recon_scene(kind, n, seed):
    """two views with the exact model and its inliers: "ground" (plane y = 1.5
    seen with a lateral move: ReconstructH accepts), "tilted" (a tilted plane:
    the classic two-fold homography ambiguity, ReconstructH refuses), "general"
    (3-D points, ReconstructF accepts).  Returns kp1, kp2, m12, pairs, M, inl, t."""
    rng = np.random.default_rng(seed)
    if kind == "ground":
        X = np.c_[rng.uniform(-4, 4, n), np.full(n, 1.5), rng.uniform(2, 20, n)]
        t, nrm, d = np.array([0.6, 0.0, 0.0]), np.array([0, 1.0, 0]), 1.5
    elif kind == "tilted":
        x = rng.uniform(-2, 2, n)
        X = np.c_[x, rng.uniform(-1.5, 1.5, n), 5.0 + 0.4 * x]
        t, nrm, d = np.array([0.5, 0.05, 0.1]), np.array([-0.4, 0, 1.0]), 5.0
    else:
        X = np.c_[rng.uniform(-2, 2, n), rng.uniform(-1.5, 1.5, n), rng.uniform(3, 8, n)]
        t = np.array([0.5, 0.05, 0.1])
    x1, x2 = (K @ X.T).T, (K @ (_R_TRUE @ X.T + t[:, None])).T
    p1 = (x1[:, :2] / x1[:, 2:]).astype(F)
    p2 = (x2[:, :2] / x2[:, 2:] + rng.normal(0, 0.5, (n, 2))).astype(F)
    keep = np.all((p1 >= 0) & (p1 < [640, 480]) & (p2 >= 0) & (p2 < [640, 480]), 1)
    p1, p2 = p1[keep], p2[keep]
    m = len(p1)
    Ki = np.linalg.inv(K)
    if kind == "general":
        tx = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])
        M = Ki.T @ tx @ _R_TRUE @ Ki
        M = (M / np.linalg.norm(M)).astype(F)
        inl = init_ref.check_fundamental(np.c_[p1, p2], M)[1]
    else:
        M = K @ (_R_TRUE + np.outer(t, nrm) / d) @ Ki
        M = (M / M[2, 2]).astype(F)
        inl = init_ref.check_homography(np.c_[p1, p2], M, init_ref.inv3(M))[1]
    # frame 2's keypoints in another order, plus unmatched extras in both frames
    perm = rng.permutation(m)
    kp1 = np.vstack([p1, rng.uniform([0, 0], [640, 480], (30, 2))]).astype(F)
    kp2 = np.vstack([rng.uniform([0, 0], [640, 480], (30, 2)), p2[perm]]).astype(F)
    m12 = np.full(len(kp1), -1, np.int32)
    m12[perm] = np.arange(m) + 30
    first = np.nonzero(m12 >= 0)[0]
    pairs = np.stack([first, m12[first]], 1)
    return kp1, kp2, m12, pairs, M, np.asarray(inl, bool), t


def _rot_angle(Ra, Rb):
    c = (np.trace(np.asarray(Ra, np.float64) @ np.asarray(Rb, np.float64).T) - 1) / 2
    return np.degrees(np.arccos(np.clip(c, -1, 1)))


@pytest.mark.parametrize("kind", ["ground", "general"])
def test_oracle_reconstruct_recovers_motion(kind):
    kp1, kp2, m12, pairs, M, inl, t = _recon_scene(kind, 500, 71)
    r = init_ref.reconstruct(0 if kind == "ground" else 1, kp1, kp2, pairs, inl, M, K.astype(F))
    assert r["ok"]
    assert _rot_angle(r["R21"], _R_TRUE) < 0.5
    assert np.dot(r["t21"], t / np.linalg.norm(t)) > 0.99
    assert r["triangulated"].sum() > 0.5 * inl.sum()
    k1, k2, _, pr, Mt, it, _ = _recon_scene("tilted", 500, 71)
    assert not init_ref.reconstruct(0, k1, k2, pr, it, Mt, K.astype(F))["ok"]  # two hypotheses explain every inlier


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n,seed", [("ground", 500, 71), ("general", 500, 72), ("general", 1500, 73),
                                         ("tilted", 500, 74), ("ground", 1200, 75)])
def test_gpu_reconstruct_vs_oracle(kind, n, seed):
    """ReconstructH / ReconstructF: hypotheses on the host, CheckRT on the GPU.
    Tolerance (the SVDs are Jacobi in double on both sides, OpenCV's float
    Jacobi is not reproducible): same decision and kept motion (R21, t21 to
    1e-4), per-hypothesis nGood as multisets within 0.5 % + 2, the kept
    hypothesis's parallax to 1e-3 relative, triangulated flags >= 99 % equal
    and the 3-D points to 1e-3 relative where both triangulate."""
    _gpu()
    import initializer
    kp1, kp2, m12, pairs, M, inl, _ = _recon_scene(kind, n, seed)
    model = 0 if kind != "general" else 1
    r = init_ref.reconstruct(model, kp1, kp2, pairs, inl, M, K.astype(F))
    g = initializer.reconstruct(model, kp1, kp2, m12, inl, M, K.astype(F))
    assert g["ok"] == r["ok"] == (kind != "tilted")
    for a, b in zip(sorted(g["n_good"]), sorted(r["n_good"])):
        assert abs(a - b) <= 2 + 0.005 * b
    if r["ok"]:
        np.testing.assert_allclose(g["R21"], r["R21"], atol=1e-4)
        np.testing.assert_allclose(g["t21"], r["t21"], atol=1e-4)
        pg, pr = float(g["parallax"][g["best"]]), float(r["parallax"][r["best"]])
        assert abs(pg - pr) <= 1e-3 * pr
        assert (g["triangulated"] == r["triangulated"]).mean() >= 0.99
        both = g["triangulated"] & r["triangulated"]
        assert both.sum() > 100
        np.testing.assert_allclose(g["p3d"][both], r["p3d"][both], rtol=1e-3, atol=1e-4)


@pytest.mark.gpu
def test_gpu_reconstruct_degenerate():
    """no inliers: CheckRT counts nothing, both models refuse"""
    _gpu()
    import initializer
    kp1, kp2, m12, pairs, M, inl, _ = _recon_scene("general", 300, 76)
    none = np.zeros_like(inl)
    Mh = _recon_scene("ground", 300, 76)[4]
    for model, Mm in ((0, Mh), (1, M)):
        r = init_ref.reconstruct(model, kp1, kp2, pairs, none, Mm, K.astype(F))
        g = initializer.reconstruct(model, kp1, kp2, m12, none, Mm, K.astype(F))
        assert g["ok"] is False and r["ok"] is False
        assert all(x == 0 for x in g["n_good"]) and g["n_good"] == r["n_good"]


# ---- Initializer::Initialize end to end (Initializer.cpp:55-157) ------------
def _oracle_initialize(kp1, kp2, m12, K_, iterations=200):
    first = np.nonzero(m12 >= 0)[0]
    pairs = np.stack([first, m12[first]], 1)
    r = init_ref.find_models(kp1, kp2, pairs, _sets_from_glibc(len(pairs), iterations))
    useH = float(r["RH"]) > 0.40
    if useH:
        M = r["H21"][r["best_h"]]
        inl = init_ref.check_homography(r["pts"], M, r["H12"][r["best_h"]])[1]
    else:
        M = r["F21"][r["best_f"]]
        inl = init_ref.check_fundamental(r["pts"], M)[1]
    rec = init_ref.reconstruct(0 if useH else 1, kp1, kp2, pairs, np.asarray(inl, bool), M, K_)
    return dict(rec, model=0 if useH else 1, RH=r["RH"])


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n,seed", [("ground", 600, 81), ("general", 600, 82)])
def test_gpu_initialize_vs_oracle(kind, n, seed):
    """the whole Initialize: the kept model and decision equal, R21 / t21 to
    2e-3 (the hypotheses are Jacobi vs LAPACK SVDs of the same DLT: section 5d)"""
    _gpu()
    import initializer
    import ransac
    kp1, kp2, m12, pairs, M, inl, _ = _recon_scene(kind, n, seed)
    ransac.srand(0)  # the process stream as SeedRandOnce(0) leaves it
    g = initializer.initialize(kp1, kp2, m12, K.astype(F))
    r = _oracle_initialize(kp1, kp2, m12, K.astype(F))
    assert g["model"] == r["model"] == (0 if kind == "ground" else 1)
    assert abs(float(g["RH"]) - float(r["RH"])) < 1e-3
    assert g["ok"] == r["ok"] is True
    np.testing.assert_allclose(g["R21"], r["R21"], atol=2e-3)
    np.testing.assert_allclose(g["t21"], r["t21"], atol=2e-3)
    assert (g["triangulated"] == r["triangulated"]).mean() > 0.98
