"""The header-only C++ drop-in (include/orbslam2_amd/ORBextractor.h,
ORBmatcher.h) used the way ORB-SLAM2's Frame / Initializer use the
reference classes, driven by tests/cpp/adapter_main.cpp."""
import os
import struct
import subprocess
from pathlib import Path

import numpy as np
import pytest
import torch

import orbref
import synth

ROOT = Path(__file__).resolve().parent.parent
CPP = ROOT / "tests" / "cpp"
EXE = CPP / "adapter_main"


@pytest.fixture(scope="module")
def exe():
    subprocess.run(["make", "-s", "-C", str(CPP)], check=True)
    return str(EXE)


@pytest.mark.parametrize("nf,scale,nl", [(1000, 1.2, 8), (2000, 1.2, 8), (500, 1.5, 5)])
def test_adapter_scale_tables_match_oracle(exe, nf, scale, nl):
    """GetScaleFactors & co. (ORBextractor.cpp:419-434) before any frame."""
    out = subprocess.run([exe, "scales", str(nf), str(scale), str(nl)], check=True, capture_output=True,
                         text=True).stdout.split("\n")
    levels, sf = out[0].split()
    assert int(levels) == nl and np.float32(float(sf)) == np.float32(scale)
    got = np.array([[float.fromhex(v) for v in line.split()] for line in out[1:1 + nl]], np.float32)
    ex = orbref.Extractor(nfeatures=nf, scale_factor=scale, nlevels=nl)
    ref = np.stack(ex.scale_factors(), 1).astype(np.float32)
    np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_adapter_empty_image_returns_untouched(exe):
    """ORBextractor.cpp:1056: `if(_image.empty()) return;` -- no device needed."""
    r = subprocess.run([exe, "empty"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure path")
def test_adapter_without_device_throws(exe):
    r = subprocess.run([exe, "nodevice"], capture_output=True, text=True)
    assert r.returncode == 0 and "threw" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
def test_adapter_device_argument(exe):
    """ORBextractor(..., device): the handle is created on that GPU; an
    ordinal outside the visible devices throws (runtime_error carrying the
    library's message) instead of running elsewhere."""
    r = subprocess.run([exe, "device", "0"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "0", r.stdout + r.stderr
    r = subprocess.run([exe, "device", "99"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 3 and "ordinal 99" in r.stderr, r.stdout + r.stderr


@pytest.mark.gpu
def test_adapter_device_guard_restores_thread_device(exe):
    """Device.h: a member call of an object placed on GPU k runs on
    k and restores the thread's device afterwards, so a default object used
    next on the same thread stays on the thread's device; both matchers give
    the same SearchForInitialization result."""
    r = subprocess.run([exe, "devguard"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("ok "), (r.returncode, r.stdout + r.stderr)


def _read_frame(buf, off):
    n, = struct.unpack_from("<i", buf, off)
    off += 4
    kps = np.frombuffer(buf, orbref.KP_DTYPE, n, off)
    off += 28 * n
    desc = np.frombuffer(buf, np.uint8, 32 * n, off).reshape(n, 32)
    return kps, desc, off + 32 * n


@pytest.mark.gpu
@pytest.mark.parametrize("copy_engine,device", [(False, None), (True, None), (False, 0)])
def test_adapter_extract_and_match_vs_oracle(exe, tmp_path, copy_engine, device):
    """ORBextractor (with the host pyramid copy) + SearchForInitialization
    through the C++ classes; transfers by copy kernels (default) and, with
    ORBGPU_SINGLE_ZEROCOPY=0 ORBGPU_HOST_ZEROCOPY=0, by the copy engine; and
    with both objects placed on device 0 through their `device` constructor
    argument (include/orbslam2_amd/Device.h)."""
    w, h, nf = 640, 480, 1000
    frames = synth.mono_stream(2, w, h, seed=0x0B5E)
    for i, f in enumerate(frames):
        (tmp_path / f"f{i}.raw").write_bytes(f.tobytes())
    out = tmp_path / "out.bin"
    env = dict(os.environ)
    if copy_engine:
        env.update(ORBGPU_SINGLE_ZEROCOPY="0", ORBGPU_HOST_ZEROCOPY="0")
    if device is not None:
        env["ADAPTER_DEVICE"] = str(device)
    r = subprocess.run([exe, "extract", str(w), str(h), str(nf), str(tmp_path / "f0.raw"),
                        str(tmp_path / "f1.raw"), str(out)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    buf = out.read_bytes()
    k0, d0, off = _read_frame(buf, 0)
    k1, d1, off = _read_frame(buf, off)
    nm, = struct.unpack_from("<i", buf, off)
    m12 = np.frombuffer(buf, np.int32, len(k0), off + 4)
    off += 4 + 4 * len(k0)
    lw, lh = struct.unpack_from("<ii", buf, off)
    lvl1 = np.frombuffer(buf, np.uint8, lw * lh, off + 8).reshape(lh, lw)

    ex = orbref.Extractor(nfeatures=nf)
    kr0, dr0 = ex.extract(frames[0])
    kr1, dr1 = ex.extract(frames[1])
    assert k0.tobytes() == kr0.tobytes() and np.array_equal(d0, dr0)
    assert k1.tobytes() == kr1.tobytes() and np.array_equal(d1, dr1)
    np.testing.assert_array_equal(lvl1, ex.level(1))
    n_r, m_r, _ = orbref.search_for_initialization(kr0, dr0, kr1, dr1, w, h)
    assert nm == n_r
    np.testing.assert_array_equal(m12, m_r)


# ---- ORBmatcher / PnPsolver / Sim3Solver class surfaces (C++) --------------
# adapter_main drives the header-only classes with mini Frame / KeyFrame /
# MapPoint types carrying the reference's member names; the outputs are
# compared with the CPU oracle (proj_ref, bow_ref, pnp_ref, loop_ref) on the
# same scenario.

F32 = np.float32


from tools.adapter_io import bow_frame_blob as _bow_frame_blob  # noqa: E402
from tools.adapter_io import frame_blob as _frame_blob  # noqa: E402
from tools.adapter_io import points_blob as _points_blob  # noqa: E402


def _run(exe, tmp_path, mode, blob, *args):
    inp, out = tmp_path / f"{mode}.in", tmp_path / f"{mode}.out"
    inp.write_bytes(blob)
    r = subprocess.run([exe, mode, *map(str, args), str(inp), str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return out.read_bytes()


PROJ_CASES = [  # variant, th, kwargs, stereo, scale (as tests/test_proj.py)
    (0, 1.0, dict(nnratio=0.8), False, 1.0),
    (0, 3.0, dict(nnratio=0.6), True, 1.0),
    (1, 10.0, dict(), False, 1.7),
    (2, 15.0, dict(check_ori=True, mono=True), False, 1.0),
    (2, 7.0, dict(check_ori=False, mono=False), True, 1.0),
    (3, 10.0, dict(check_ori=True, orb_dist=100), False, 1.0),
]


@pytest.mark.gpu
@pytest.mark.parametrize("variant,th,kw,stereo,scale", PROJ_CASES)
def test_adapter_orbmatcher_search_by_projection(exe, tmp_path, variant, th, kw, stereo, scale):
    """ORB_SLAM2::ORBmatcher::SearchByProjection (all four overloads) vs oracle/proj_ref.py"""
    import proj_ref
    tgt, pts = synth.projection_scenario(700, 400, 20 + variant * 7, stereo=stereo, scale=scale)
    if variant == 0:
        fl, tr, lv = proj_ref.is_in_frustum(tgt, pts, 0.5)
        pts = dict(pts, flags=fl, track=tr, track_level=lv)
    last = np.asarray(tgt["Tcw"], F32).copy()
    if variant == 2:
        last[:3, 3] += np.random.default_rng(3).uniform(-0.2, 0.2, 3).astype(F32)
        kw = dict(kw, last_Tcw=last)
    nm_r, m_r = proj_ref.search_by_projection(variant, tgt, pts, th, **kw)
    blob = b"".join([struct.pack("<ffiii", th, kw.get("nnratio", 0.6), int(kw.get("check_ori", True)),
                                 int(kw.get("orb_dist", 50)), int(kw.get("mono", True))), last.tobytes(),
                     _frame_blob(tgt), np.asarray(tgt["occupied"], np.uint8).tobytes(), _points_blob(pts),
                     np.asarray(pts["octave"], np.int32).tobytes(), np.asarray(pts["angle"], F32).tobytes()])
    buf = _run(exe, tmp_path, "proj", blob, variant)
    nm, = struct.unpack_from("<i", buf, 0)
    got = np.frombuffer(buf, np.int32, len(tgt["kps"]), 4)
    occ = np.asarray(tgt["occupied"])
    want = np.where(m_r >= 0, m_r, np.where(m_r == -2, -1, np.where(occ > 0, -3, -1)))
    assert nm == nm_r
    np.testing.assert_array_equal(got, want)
    assert nm_r > 30


@pytest.mark.gpu
@pytest.mark.parametrize("nnratio,check_ori", [(0.75, True), (0.6, False)])
def test_adapter_orbmatcher_search_by_bow(exe, tmp_path, nnratio, check_ori):
    """ORB_SLAM2::ORBmatcher::SearchByBoW(KF, F) and (KF1, KF2) vs oracle/bow_ref.py"""
    import bow_ref
    par, leaf, desc, w = synth.synthetic_vocabulary(8, 4, 5)
    voc = bow_ref.Vocabulary.from_arrays(8, 4, 0, 0, par, leaf, desc, w)
    rng = np.random.default_rng(23)
    n = 900
    d1, a1, d2, a2 = synth.bow_frame_pair(desc[leaf == 1], n, 0.6, seed=41)
    fv1, fv2 = voc.transform(d1, 2)[3], voc.transform(d2, 2)[3]
    s1 = rng.choice([0, 1, 1, 1, 1, 1, 1, 2], n).astype(np.uint8)  # none / good / bad MapPoint
    s2 = rng.choice([0, 1, 1, 1, 1, 1, 1, 2], n).astype(np.uint8)
    blob = struct.pack("<fi", nnratio, int(check_ori)) + _bow_frame_blob(d1, a1, s1, fv1) + \
        _bow_frame_blob(d2, a2, s2, fv2)
    buf = _run(exe, tmp_path, "bow", blob)
    n1, = struct.unpack_from("<i", buf, 0)
    m1 = np.frombuffer(buf, np.int32, n, 4)
    n2, = struct.unpack_from("<i", buf, 4 + 4 * n)
    m2 = np.frombuffer(buf, np.int32, n, 8 + 4 * n)
    r1, mr1 = bow_ref.search_by_bow(0, fv1, d1, a1, s1 == 1, fv2, d2, a2, np.ones(n, bool), nnratio, check_ori)
    r2, mr2 = bow_ref.search_by_bow(1, fv1, d1, a1, s1 == 1, fv2, d2, a2, s2 == 1, nnratio, check_ori)
    assert (n1, n2) == (r1, r2) and r1 > 50 and r2 > 50
    np.testing.assert_array_equal(m1, mr1)  # per F slot: the KF slot whose MapPoint it got
    np.testing.assert_array_equal(m2, mr2)  # per KF1 slot: the KF2 slot


LIBC = None


def _libc():
    global LIBC
    if LIBC is None:
        import ctypes
        LIBC = ctypes.CDLL("libc.so.6")
    return LIBC


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n,frac", [(0, 80, 0.6), (5, 200, 0.5)])
def test_adapter_pnpsolver_relocalization(exe, tmp_path, seed, n, frac):
    """ORB_SLAM2::PnPsolver driven as Tracking::Relocalization does, vs a
    sequential oracle replay (oracle/pnp_ref.py) drawing from glibc itself."""
    import pnp_ref
    P = synth.pnp_problem(n, frac, seed=77 + seed)
    table = (F32(1.2) ** (2 * np.arange(8))).astype(F32)
    octv = np.array([int(np.nonzero(table == s)[0][0]) for s in P["sigma2"]], np.int32)
    # interleave keypoints without a MapPoint (0) and with a bad one (2)
    rng = np.random.default_rng(seed)
    extra = 25
    N = n + extra
    slots = np.sort(rng.choice(N, n, replace=False))
    state = np.zeros(N, np.uint8)
    state[slots] = 1
    rest = np.setdiff1d(np.arange(N), slots)
    state[rest[: extra // 2]] = 2
    kps = np.zeros(N, orbref.KP_DTYPE)
    kps["x"][slots], kps["y"][slots] = P["P2"][:, 0], P["P2"][:, 1]
    kps["octave"][slots] = octv
    kps["x"][rest], kps["y"][rest] = 100.0, 100.0
    pos = np.zeros((N, 3), F32)
    pos[slots] = P["P3w"]
    pos[rest] = rng.uniform(-1, 1, (len(rest), 3)).astype(F32)
    fu, fv, uc, vc = P["cam"]
    tgt = {"kps": kps, "desc": np.zeros((N, 32), np.uint8), "min_x": 0, "max_x": 640, "min_y": 0, "max_y": 480,
           "fx": fu, "fy": fv, "cx": uc, "cy": vc, "bf": 0, "b": 0, "log_scale_factor": float(np.log(F32(1.2))),
           "scale_factors": np.sqrt(table).astype(F32), "Tcw": np.eye(4, dtype=F32)}
    blob = struct.pack("<I", 0) + _frame_blob(tgt, sigma2=table) + state.tobytes() + pos.tobytes()
    buf = _run(exe, tmp_path, "pnp", blob)
    found, n_inl, its, best, min_inl, max_its = struct.unpack_from("<6i", buf, 0)
    T = np.frombuffer(buf, F32, 16, 24).reshape(4, 4)
    vb = np.frombuffer(buf, np.uint8, N, 88).astype(bool)
    nxt = list(np.frombuffer(buf, np.int32, 5, 88 + N))
    # oracle replay (Tracking.cpp:1786-1822 with one solver): the `||` loop
    L = _libc()
    L.srand(0)
    samples = []
    for _ in range(max(max_its, 5)):
        avail = list(range(n))
        tri = []
        for _ in range(4):
            r = int((L.rand() / (2147483647 + 1.0)) * len(avail))
            tri.append(avail[r]); avail[r] = avail[-1]; avail.pop()
        samples.append(tri)
    maxerr = (P["sigma2"] * F32(5.991)).astype(F32)
    o = pnp_ref.ransac_call(P["P3w"], P["P2"], maxerr, P["cam"], min_inl, 0, np.zeros(n, bool), np.array(samples))
    assert found == o["found"] == 1
    assert its == o["consumed"]
    assert np.abs(T[:3, :3] - o["refined_R"]).max() <= 1e-3
    assert np.abs(T[:3, 3] - o["refined_t"]).max() <= 1e-3 * (1 + np.abs(o["refined_t"]).max())
    want = np.zeros(N, bool)
    want[slots[o["refined_mask"]]] = True
    assert (vb != want).sum() <= max(1, n // 100)
    assert abs(n_inl - int(o["refined_mask"].sum())) <= max(1, n // 100)
    assert not vb[rest].any()
    L.srand(0)
    for _ in range(4 * o["consumed"]):
        L.rand()
    assert nxt == [L.rand() for _ in range(5)]


def _sim3_kf_blob(Tcw, K, sig2, state, pos, octv):
    return b"".join([struct.pack("<i", len(state)), np.asarray(Tcw, F32).tobytes(), np.asarray(K, F32).tobytes(),
                     np.asarray(sig2, F32).tobytes(), np.asarray(state, np.uint8).tobytes(),
                     np.asarray(pos, F32).tobytes(), np.asarray(octv, np.int32).tobytes()])


@pytest.mark.gpu
@pytest.mark.parametrize("fix_scale", [False, True])
def test_adapter_sim3solver_compute_sim3(exe, tmp_path, fix_scale):
    """ORB_SLAM2::Sim3Solver driven as LoopClosing::ComputeSim3 does (round-robin
    iterate(5) over the candidates) vs oracle/loop_ref.py with glibc draws."""
    import loop_ref
    p, l, d, w = synth.synthetic_vocabulary_fast(10, 3, 4)
    nc = 4
    sc = synth.loop_burst_scene(1, nc, d[l == 1], n_kp=400, inlier_frac=[0.0, 0.02, 0.3, 0.3],
                                outlier_frac=[0.0, 0.15, 0.3, 0.3], seed=9 + fix_scale, fix_scale=fix_scale)
    rng = np.random.default_rng(2)
    state = np.where(sc["valid"] > 0, np.where(rng.random(sc["valid"].shape) < 0.05, 2, 1), 0).astype(np.uint8)
    blob = struct.pack("<Iii", 0, int(fix_scale), nc)
    blob += _sim3_kf_blob(sc["Tcw"][0], sc["K"], sc["sigma2"], state[0], sc["mp_world"][0], sc["octave"][0])
    m12s, solvers = [], []
    for c in range(nc):
        kf = 1 + c
        tr = sc["truth"][c]
        m12 = np.full(400, -1, np.int32)
        m12[np.r_[tr["src"], tr["outlier_src"]]] = np.r_[tr["dst"], tr["outlier_dst"]]
        m12s.append(m12)
        blob += _sim3_kf_blob(sc["Tcw"][kf], sc["K"], sc["sigma2"], state[kf], sc["mp_world"][kf],
                              sc["octave"][kf]) + m12.tobytes()
        nm = int(((m12 >= 0) & (state[kf][np.maximum(m12, 0)] > 0)).sum())
        corr = loop_ref.sim3_setup(m12, state[0] == 1, state[kf] == 1, sc["mp_world"][0], sc["mp_world"][kf],
                                   sc["Tcw"][0], sc["Tcw"][kf], sc["octave"][0], sc["octave"][kf], sc["sigma2"])
        solvers.append(loop_ref.Sim3SolverRef(corr, sc["K"], sc["K"], fix_scale) if nm >= 20 else None)
    buf = _run(exe, tmp_path, "sim3", blob)
    matched, rnd, n_inl = struct.unpack_from("<3i", buf, 0)
    per = np.frombuffer(buf, np.int32, 3 * nc, 12).reshape(nc, 3)
    off = 12 + 12 * nc
    R = np.frombuffer(buf, F32, 9, off).reshape(3, 3)
    t = np.frombuffer(buf, F32, 3, off + 36)
    s, = struct.unpack_from("<f", buf, off + 48)
    vb = np.frombuffer(buf, np.uint8, 400, off + 52).astype(bool)
    nxt = list(np.frombuffer(buf, np.int32, 5, off + 52 + 400))
    ref = loop_ref.compute_sim3(solvers, 0)
    after = [loop_ref.libc().rand() for _ in range(5)]
    assert (matched, rnd, n_inl) == (ref["matched"], ref["round"], ref["n_inliers"])
    for c in range(nc):
        sv = solvers[c]
        assert tuple(per[c]) == ((sv.iterations, sv.best, sv.N) if sv is not None else (-1, -1, -1)), c
    assert nxt == after
    assert matched >= 0
    pose = solvers[matched].best_pose
    assert np.abs(R - pose["R12"]).max() < 2e-4 and abs(s - pose["s12"]) < 2e-4
    assert np.abs(t - pose["t12"]).max() < 2e-4 * (1 + np.abs(pose["t12"]).max())
    want = np.zeros(400, bool)
    want[solvers[matched].idx[solvers[matched].best_mask]] = True
    np.testing.assert_array_equal(vb, want)


# ---- Fuse / SearchBySim3 / SearchForTriangulation (LocalMapping, LoopClosing)
def _fuse_replay(variant, best, slot_state, slot_obs, bad0, pobs, inkf):
    """The reference's MapPoint updates after the per-point searches
    (ORBmatcher.cpp:1091-1111, :1228-1245) over the adapter test's map model
    (MapPoint::Replace moves the keyframe observation and marks the old point
    bad).  Labels: point i, slot dummy 100000 + k, -1 NULL."""
    n_kp, n_pts = len(slot_state), len(best)
    owner = [100000 + k if slot_state[k] else -1 for k in range(n_kp)]
    bad = {i: bool(bad0[i]) for i in range(n_pts)}
    bad.update({100000 + k: slot_state[k] == 2 for k in range(n_kp)})
    nobs = {i: int(pobs[i]) for i in range(n_pts)}
    nobs.update({100000 + k: int(slot_obs[k]) for k in range(n_kp)})
    where = {100000 + k: k for k in range(n_kp) if slot_state[k]}  # the keyframe slot of a point in it
    in_kf = {i for i in range(n_pts) if inkf[i]}
    found = {owner[k] for k in range(n_kp) if owner[k] != -1 and not bad[owner[k]]}
    repl = [-1] * n_pts

    def add(p, k):
        if p in where or p in in_kf:
            return
        where[p] = k
        nobs[p] += 1

    def replace(a, b):  # a->Replace(b)
        if a == b:
            return
        if a in where:
            k = where.pop(a)
            if b not in where and b not in in_kf:
                owner[k] = b
                add(b, k)
            else:
                owner[k] = -1
        bad[a] = True
        nobs[a] = 0

    nf = 0
    for i in range(n_pts):
        if variant == 4:
            if bad[i] or i in where or i in in_kf or best[i] < 0:
                continue
        elif bad[i] or i in found or best[i] < 0:
            continue
        pin = owner[best[i]]
        if pin != -1:
            if not bad[pin]:
                if variant == 5:
                    repl[i] = pin
                elif nobs[pin] > nobs[i]:
                    replace(i, pin)
                else:
                    replace(pin, i)
        else:
            add(i, best[i])
            owner[best[i]] = i
        nf += 1
    return nf, owner, [int(bad[i]) for i in range(n_pts)], repl


@pytest.mark.gpu
@pytest.mark.parametrize("variant,th,stereo,scale", [(4, 3.0, True, 1.0), (4, 6.0, False, 1.0), (5, 4.0, False, 1.7)])
def test_adapter_orbmatcher_fuse(exe, tmp_path, variant, th, stereo, scale):
    """ORB_SLAM2::ORBmatcher::Fuse (both overloads): GPU searches + the host
    replay of the reference's updates, vs oracle/proj_ref.py + the replay"""
    import proj_ref
    tgt, pts = synth.projection_scenario(700, 400, 50 + variant, stereo=stereo, scale=scale)
    rng = np.random.default_rng(variant)
    n_kp, n_pts = len(tgt["kps"]), len(pts["flags"])
    slot_state = np.where(rng.uniform(size=n_kp) < 0.3, rng.choice([1, 1, 1, 2], n_kp), 0).astype(np.uint8)
    slot_obs = rng.integers(1, 6, n_kp).astype(np.int32)
    pobs = rng.integers(1, 6, n_pts).astype(np.int32)
    inkf = (rng.uniform(size=n_pts) < (0.05 if variant == 4 else 0.0)).astype(np.uint8)
    bad0 = (np.asarray(pts["flags"]) & 1) == 0
    pose = np.asarray(tgt["Tcw"], F32)
    if variant == 5:  # Scw = the scenario's Sim3; the keyframe's own pose is not read
        kf_tgt, Scw = dict(tgt, Tcw=np.eye(4, dtype=F32)), pose
        oracle_pts = dict(pts, flags=(~bad0).astype(np.int32))
    else:
        kf_tgt, Scw = tgt, np.eye(4, dtype=F32)
        oracle_pts = dict(pts, flags=((~bad0) & (inkf == 0)).astype(np.int32))
    _, best = proj_ref.radius_search(variant, tgt, oracle_pts, th)
    nf_r, owner_r, bad_r, repl_r = _fuse_replay(variant, best, slot_state, slot_obs, bad0, pobs, inkf)
    blob = b"".join([struct.pack("<f", th), _frame_blob(kf_tgt), Scw.tobytes(), slot_state.tobytes(),
                     slot_obs.tobytes(), _points_blob(dict(pts, flags=np.where(bad0, 0, 1))), pobs.tobytes(),
                     inkf.tobytes()])
    buf = _run(exe, tmp_path, "fuse", blob, variant)
    got = np.frombuffer(buf, np.int32)
    assert got[0] == nf_r > 50
    np.testing.assert_array_equal(got[1:1 + n_kp], owner_r)
    np.testing.assert_array_equal(got[1 + n_kp:1 + n_kp + n_pts], bad_r)
    np.testing.assert_array_equal(got[1 + n_kp + n_pts:], repl_r)
    assert any(o != -1 and o < 100000 for o in owner_r)  # some AddMapPoint happened
    if variant == 4:
        assert sum(bad_r) > bad0.sum()  # and some Replace


@pytest.mark.gpu
@pytest.mark.parametrize("seed,s12", [(60, 1.0), (61, 1.1)])
def test_adapter_orbmatcher_search_by_sim3(exe, tmp_path, seed, s12):
    """ORB_SLAM2::ORBmatcher::SearchBySim3 vs oracle/proj_ref.py"""
    import proj_ref
    kf1, kf2, p1, p2, s, R, t = synth.sim3_search_scenario(600, 250, seed, s12=s12)
    nf_r, m_r = proj_ref.search_by_sim3(kf1, kf2, p1, p2, s, R, t, 7.5)

    def cpp_pts(p):  # exists-and-good flags for the class (already-matched entries are ordinary MapPoints)
        return dict(p, flags=((~p["null"]) & (~p["bad"])).astype(np.int32))
    blob = b"".join([struct.pack("<ff", 7.5, float(s)), np.asarray(R, F32).tobytes(), np.asarray(t, F32).tobytes(),
                     _frame_blob(kf1), _frame_blob(kf2), _points_blob(cpp_pts(p1)), _points_blob(cpp_pts(p2)),
                     p1["null"].astype(np.int32).tobytes(), p2["null"].astype(np.int32).tobytes(),
                     p1["pre"].astype(np.int32).tobytes()])
    buf = _run(exe, tmp_path, "sim3search", blob)
    got = np.frombuffer(buf, np.int32)
    want = np.where(p1["pre"] >= 0, p1["pre"], m_r)
    assert got[0] == nf_r > 20
    np.testing.assert_array_equal(got[1:], want)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,check_ori,stereo", [(2, True, False), (3, False, True)])
def test_adapter_orbmatcher_search_for_triangulation(exe, tmp_path, seed, check_ori, stereo):
    """ORB_SLAM2::ORBmatcher::SearchForTriangulation vs oracle/bow_ref.py"""
    import bow_ref
    par, leaf, desc, w = synth.synthetic_vocabulary(6, 4, 30 + seed)
    voc = bow_ref.Vocabulary.from_arrays(6, 4, 0, 0, par, leaf, desc, w)
    P = synth.triangulation_scenario(desc[leaf == 1], 500, seed, stereo=stereo)
    fv1, fv2 = voc.transform(P["desc1"], 2)[3], voc.transform(P["desc2"], 2)[3]
    nm_r, m_r = bow_ref.search_for_triangulation(fv1, fv2, P, check_ori, False)
    sf, s2 = P["scale_factors2"], P["level_sigma2_2"]
    T2 = np.eye(4, dtype=F32)
    T2[:3, :] = P["T2w"]

    def kf(i, T):
        g = {"min_x": 0.0, "max_x": 640.0, "min_y": 0.0, "max_y": 480.0, "fx": P["fx2"], "fy": P["fy2"],
             "cx": P["cx2"], "cy": P["cy2"], "bf": 0.0, "b": 0.0, "log_scale_factor": float(np.log(F32(1.2)))}
        t = dict(g, kps=P[f"kps{i}"], desc=P[f"desc{i}"], u_right=P[f"u_right{i}"], scale_factors=sf, Tcw=T)
        nodes = np.array(sorted((fv1, fv2)[i - 1]), np.int32)
        offs = np.zeros(len(nodes) + 1, np.int32)
        feats = []
        for j, k in enumerate(nodes):
            feats += list((fv1, fv2)[i - 1][int(k)])
            offs[j + 1] = len(feats)
        return b"".join([_frame_blob(t, s2), (1 - P[f"valid{i}"]).astype(np.uint8).tobytes(),
                         struct.pack("<i", len(nodes)), nodes.tobytes(), offs.tobytes(),
                         np.array(feats, np.int32).tobytes()])
    blob = b"".join([struct.pack("<ii", int(check_ori), 0), np.asarray(P["F12"], F32).tobytes(),
                     np.asarray(P["Cw1"], F32).tobytes(), kf(1, np.eye(4, dtype=F32)), kf(2, T2)])
    buf = _run(exe, tmp_path, "tri", blob)
    got = np.frombuffer(buf, np.int32)
    pairs = [(i, int(m_r[i])) for i in range(len(m_r)) if m_r[i] >= 0]
    assert got[0] == nm_r > 30 and got[1] == len(pairs)
    np.testing.assert_array_equal(got[2:].reshape(-1, 2), np.array(pairs, np.int32).reshape(-1, 2))


@pytest.mark.gpu
def test_adapter_initializer_monocular_initialization(exe, tmp_path):
    """ORB_SLAM2::Initializer(F1, 1.0, 200).Initialize(F2, ...) in a fresh
    process (SeedRandOnce(0) seeds the stream) vs the oracle pipeline"""
    import test_init as ti
    kp1, kp2, m12, pairs, M, inl, _ = ti._recon_scene("general", 600, 82)
    K = ti.K.astype(F32)
    blob = b"".join([K.tobytes(), struct.pack("<i", len(kp1)), np.asarray(kp1, F32).tobytes(),
                     struct.pack("<i", len(kp2)), np.asarray(kp2, F32).tobytes(), np.asarray(m12, np.int32).tobytes()])
    buf = _run(exe, tmp_path, "init", blob)
    ok, model = struct.unpack_from("<ii", buf, 0)
    rh, = struct.unpack_from("<f", buf, 8)
    R = np.frombuffer(buf, F32, 9, 12).reshape(3, 3)
    t = np.frombuffer(buf, F32, 3, 48)
    r = ti._oracle_initialize(kp1, kp2, m12, K)
    assert ok == int(r["ok"]) == 1 and model == r["model"] == 1
    assert abs(rh - float(r["RH"])) < 1e-3
    np.testing.assert_allclose(R, r["R21"], atol=2e-3)
    np.testing.assert_allclose(t, r["t21"], atol=2e-3)


def _kfdb_scene(scoring=0, n_kf=120, seed=5):
    """keyframes along a looping path over 1200 landmarks (keyframe k sees
    landmarks [10k, 10k + 250) mod 1200), BowVectors from a synthetic
    vocabulary; covisibility = path neighbours"""
    import bow_ref
    par, leaf, desc, w = synth.synthetic_vocabulary(6, 4, 77)
    voc = bow_ref.Vocabulary.from_arrays(6, 4, scoring, 0, par, leaf, desc, w)
    rng = np.random.default_rng(seed)
    leaves = desc[leaf == 1]
    lm = leaves[rng.integers(0, len(leaves), 1200)]

    def observe(ids):
        d = lm[ids] ^ (rng.uniform(size=(len(ids), 32)) < 0.03).astype(np.uint8)
        return voc.transform(d, 2)[4]
    kfs = []
    for k in range(n_kf):
        ids = (10 * k + np.arange(250)) % 1200
        ids = ids[rng.uniform(size=250) < 0.85]
        near = [j for j in sorted(range(max(0, k - 6), min(n_kf, k + 7)), key=lambda j: (abs(j - k), j)) if j != k]
        kfs.append({"id": k + 1, "bow": observe(ids), "connected": set(near),
                    "best_covis": near[:10], "loop_query": 0, "loop_words": 0, "loop_score": np.float32(0),
                    "reloc_query": 0, "reloc_words": 0, "reloc_score": np.float32(0)})
    frame_bow = observe((500 + np.arange(250)) % 1200)
    return voc, kfs, frame_bow


def _bow_blob(bow):
    ws = np.array(sorted(bow), np.int32)
    return struct.pack("<i", len(ws)) + ws.tobytes() + np.array([bow[int(x)] for x in ws], np.float64).tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("scoring", [0, 1])
def test_adapter_keyframe_database(exe, tmp_path, scoring):
    """orbslam2_amd::KeyFrameDatabaseT (GPU scores) vs oracle/kfdb_ref.py:
    DetectLoopCandidates for two query keyframes, DetectRelocalizationCandidates
    for one frame -- candidate lists equal, in order"""
    import kfdb_ref
    voc, kfs, fbow = _kfdb_scene(scoring)
    db = kfdb_ref.KeyFrameDatabase(voc.n_words, scoring)
    for i in range(len(kfs)):
        db.add(kfs, i)
    queries = [(0, 118, 0.01), (0, 60, 0.02), (1, 1000, fbow)]
    want = []
    for kind, a, b in queries:
        if kind == 0:  # the query keyframe is not in the database yet (LoopClosing::DetectLoop)
            db.erase(kfs, a)
            want.append(db.detect_loop(kfs, a, b))
            db.inv = [lst for lst in db.inv]
            for w in sorted(kfs[a]["bow"]):
                db.inv[w].append(a)
        else:
            want.append(db.detect_reloc(kfs, b, a))
    parts = [struct.pack("<iii", scoring, voc.n_words + 1, len(kfs))]
    for k in kfs:
        conn = np.array(sorted(k["connected"]), np.int32)
        cov = np.array(k["best_covis"], np.int32)
        parts += [struct.pack("<I", k["id"]), _bow_blob(k["bow"]), struct.pack("<i", len(conn)), conn.tobytes(),
                  struct.pack("<i", len(cov)), cov.tobytes()]
    parts.append(struct.pack("<i", len(queries)))
    for kind, a, b in queries:
        parts.append(struct.pack("<iif", 0, a, b) if kind == 0 else struct.pack("<iI", 1, a) + _bow_blob(b))
    buf = _run(exe, tmp_path, "kfdb", b"".join(parts))
    got, o = [], 0
    for _ in queries:
        n, = struct.unpack_from("<i", buf, o)
        got.append(list(np.frombuffer(buf, np.int32, n, o + 4)))
        o += 4 + 4 * n
    assert got == want
    assert len(want[0]) >= 1 and min(want[0]) < 10  # the loop back to the first keyframes is found
    assert len(want[2]) >= 1


@pytest.mark.gpu
@pytest.mark.parametrize("scoring,weighting,fmt", [(0, 0, "txt"), (1, 1, "txt"), (2, 0, "bin")])
def test_adapter_orb_vocabulary(exe, tmp_path, scoring, weighting, fmt):
    """orbslam2_amd::ORBVocabulary: loadFromTextFile / loadFromBinaryFile,
    transform (Frame::ComputeBoW, levelsup 4) and score vs oracle/bow_ref.py -- bit-exact"""
    import bow_ref
    par, leaf, desc, w = synth.synthetic_vocabulary(6, 5, 91)
    vp = tmp_path / f"voc.{fmt}"
    if fmt == "bin":
        synth.write_vocabulary_binary(vp, 6, 5, scoring, weighting, par, leaf, desc, w)
        ref = bow_ref.Vocabulary.load_binary(vp)
    else:
        synth.write_vocabulary_text(vp, 6, 5, scoring, weighting, par, leaf, desc, w)
        ref = bow_ref.Vocabulary.load_text(vp)
    rng = np.random.default_rng(4)
    leaves = desc[leaf == 1]
    d1 = leaves[rng.integers(0, len(leaves), 500)] ^ (rng.uniform(size=(500, 32)) < 0.04).astype(np.uint8)
    d2 = np.vstack([d1[:300], rng.integers(0, 256, (200, 32), dtype=np.uint8)])
    blob = struct.pack("<ii", 4, len(d1)) + d1.tobytes() + struct.pack("<i", len(d2)) + d2.tobytes()
    inp, out = tmp_path / "voc.in", tmp_path / "voc.out"
    inp.write_bytes(blob)
    r = subprocess.run([exe, "voc", str(vp), str(inp), str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    buf = out.read_bytes()
    size, sc = struct.unpack_from("<ii", buf, 0)
    assert size == ref.n_words and sc == scoring
    o = 8
    bows = []
    for d in (d1, d2):
        _, _, _, rfv, rbow = ref.transform(d, 4)
        nb, = struct.unpack_from("<i", buf, o)
        o += 4
        got = {}
        for _ in range(nb):
            wd, = struct.unpack_from("<i", buf, o)
            val, = struct.unpack_from("<d", buf, o + 4)
            got[wd] = val
            o += 12
        assert got == rbow  # ids and double weights bit-exact
        nf, = struct.unpack_from("<i", buf, o)
        o += 4
        gfv = {}
        for _ in range(nf):
            node, cnt = struct.unpack_from("<ii", buf, o)
            gfv[node] = list(np.frombuffer(buf, np.int32, cnt, o + 8))
            o += 8 + 4 * cnt
        assert gfv == {k: list(v) for k, v in rfv.items()}
        bows.append(rbow)
    s, = struct.unpack_from("<d", buf, o)
    assert s == bow_ref.bow_score(scoring, bows[0], bows[1])[0]


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,nf,bf,base", [(752, 480, 1200, 47.90639384423901, 18.0),
                                            (1241, 376, 2000, 0.54 * 718.856, 30.0)])
def test_adapter_stereo_frame_vs_oracle(exe, tmp_path, w, h, nf, bf, base):
    """The stereo Frame through the drop-in classes: two ORBextractor objects
    on two threads, then ComputeStereoMatchesGPU on their HBM pyramids
    (StereoMatcher.h, orbgpu_stereo_matches_pair) vs the oracle stereo Frame
    (two oracle extractors + oracle/stereo_ref.cpp), bit-exact; and the same
    Frame with both extractions issued from one thread (ExtractPair)"""
    pair = synth.stereo_stream(1, w, h, 0x5E7, base)[0]
    (tmp_path / "l.raw").write_bytes(pair[0].tobytes())
    (tmp_path / "r.raw").write_bytes(pair[1].tobytes())
    out = tmp_path / "st.bin"
    r = subprocess.run([exe, "stereo", str(w), str(h), str(nf), repr(float(np.float32(bf))), str(tmp_path / "l.raw"),
                        str(tmp_path / "r.raw"), str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    buf = out.read_bytes()
    kl, dl, off = _read_frame(buf, 0)
    kr, dr, off = _read_frame(buf, off)
    ur = np.frombuffer(buf, np.float32, len(kl), off)
    dp = np.frombuffer(buf, np.float32, len(kl), off + 4 * len(kl))
    exL, exR = orbref.Extractor(nf), orbref.Extractor(nf)
    rk = orbref.stereo_frame(exL, exR, pair[0], pair[1], np.float32(bf))
    assert kl.tobytes() == rk[0].tobytes() and np.array_equal(dl, rk[1])
    assert kr.tobytes() == rk[2].tobytes() and np.array_equal(dr, rk[3])
    assert ur.tobytes() == rk[4].tobytes() and dp.tobytes() == rk[5].tobytes()
    assert (ur >= 0).mean() > 0.3
    # an unmodified stereo Frame.cpp reads mvImagePyramid (Frame.cpp:547-676):
    # no copy was made for the GPU stereo path, the first read copies the
    # levels once per extractor, and they are the oracle's pyramid bit for bit
    off += 8 * len(kl)
    c0 = np.frombuffer(buf, np.int64, 2, off)
    n_rows, = struct.unpack_from("<i", buf, off + 16)
    off += 20
    assert list(c0) == [0, 0] and n_rows == h
    for ex in (exL, exR):
        nlev, = struct.unpack_from("<i", buf, off)
        off += 4
        assert nlev == 8
        for lv in range(nlev):
            lw, lh = struct.unpack_from("<ii", buf, off)
            got = np.frombuffer(buf, np.uint8, lw * lh, off + 8).reshape(lh, lw)
            off += 8 + lw * lh
            np.testing.assert_array_equal(got, ex.level(lv))
    assert list(np.frombuffer(buf, np.int64, 2, off)) == [1, 1]
    # the same Frame with both extractions issued from one thread
    # (ORBextractor::ExtractPair, orbgpu_extract_pair): the oracle's results too
    off += 16
    kl2, dl2, off = _read_frame(buf, off)
    kr2, dr2, off = _read_frame(buf, off)
    ur2 = np.frombuffer(buf, np.float32, len(kl2), off)
    dp2 = np.frombuffer(buf, np.float32, len(kl2), off + 4 * len(kl2))
    assert off + 8 * len(kl2) == len(buf)
    assert kl2.tobytes() == rk[0].tobytes() and np.array_equal(dl2, rk[1])
    assert kr2.tobytes() == rk[2].tobytes() and np.array_equal(dr2, rk[3])
    assert ur2.tobytes() == rk[4].tobytes() and dp2.tobytes() == rk[5].tobytes()


def test_adapter_initializer_fewer_than_8_matches_returns_false(exe, tmp_path):
    """Initialize with < 8 matches returns false (no throw out of Tracking's
    thread; the reference's draws would index an empty vector).  Needs no GPU:
    the check runs before any device call."""
    kp = np.random.default_rng(0).uniform(0, 400, (20, 2)).astype(F32)
    m12 = np.full(20, -1, np.int32)
    m12[:7] = np.arange(7)
    blob = b"".join([np.eye(3, dtype=F32).tobytes(), struct.pack("<i", 20), kp.tobytes(), struct.pack("<i", 20),
                     kp.tobytes(), m12.tobytes()])
    buf = _run(exe, tmp_path, "init", blob)
    ok, = struct.unpack_from("<i", buf, 0)
    assert ok == 0
