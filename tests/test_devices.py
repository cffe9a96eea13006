"""Device placement of the host-form calls (VERDICT r5 "next" #4):
the launchers that set a kernel attribute or read a device property once
(SearchByProjection's and SearchByBoW's dynamic-LDS limit, the stereo
kernel's growing LDS limit and CU count) keep that state per device ordinal
(csrc/device_state.h), so a thread that calls on device 0 and then on device
1 -- or a second device reached first from another thread -- runs correctly
on both.  The reference's hosts call these from several threads
(src/Frame.cpp:84-87, src/Tracking.cpp:141-149, LoopClosing beside
Tracking).  Every result is compared with the oracle bit for bit.

Needs a GPU (-m gpu); the multi-device test skips with fewer than 2 visible
devices (the gpurun box has one)."""
import threading

import numpy as np
import pytest

import bow_ref
import proj_ref
import stereo_ref
import synth


def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _proj_case(seed):
    tgt, pts = synth.projection_scenario(700, 400, seed)
    fl, tr, lv = proj_ref.is_in_frustum(tgt, pts, 0.5)
    pts = dict(pts, flags=fl, track=tr, track_level=lv)
    return tgt, pts, proj_ref.search_by_projection(proj_ref.LOCAL, tgt, pts, 1.0, nnratio=0.8)


def _bow_case(seed):
    par, leaf, desc, w = synth.synthetic_vocabulary(8, 4, 5)
    ref = bow_ref.Vocabulary.from_arrays(8, 4, 0, 0, par, leaf, desc, w)
    d1, a1, d2, a2 = synth.bow_frame_pair(desc[leaf == 1], 900, 0.6, seed=seed)
    fv1, fv2 = ref.transform(d1, 2)[3], ref.transform(d2, 2)[3]
    v1 = np.ones(len(d1), bool)
    v2 = np.ones(len(d2), bool)
    args = (fv1, d1, a1, v1, fv2, d2, a2, v2, 0.75, True)
    return args, bow_ref.search_by_bow(1, *args)


def _stereo_on(torch, device, seed):
    """ComputeStereoMatches (batch form) for one synthetic pair on an
    extractor placed on `device`, against stereo_ref on the GPU's own
    keypoints and levels."""
    import orbgpu
    w, h, nf, bf = 640, 480, 1000, 40.0
    base = synth.base_texture(seed)
    left = synth.render_frame(base, 3, w, h, seed)
    right = synth.render_frame(base, 3, w, h, seed + 1, 24.0)
    ex = orbgpu.Extractor(nfeatures=nf, width=w, height=h, max_batch=2, device=device)
    dev = torch.device("cuda", device)
    host = np.zeros((2, h, w), np.uint8)
    host[0], host[1] = left, right
    imgs = torch.from_numpy(host).to(dev)
    cap = ex.max_keypoints
    kps = torch.zeros((2, cap, 7), dtype=torch.float32, device=dev)
    desc = torch.zeros((2, cap, 32), dtype=torch.uint8, device=dev)
    counts = torch.zeros(2, dtype=torch.int32, device=dev)
    ur = torch.full((1, cap), -7.0, dtype=torch.float32, device=dev)
    dp = torch.full((1, cap), -7.0, dtype=torch.float32, device=dev)
    ex.extract_batch(imgs, kps, desc, counts)
    orbgpu.stereo_matches_batch(ex, imgs, 1, kps, desc, counts, bf, 0.0, ur, dp)
    ex.sync()
    n = counts.cpu().numpy()
    kh, dh = kps.cpu().numpy(), desc.cpu().numpy()
    kl, kr = orbgpu.keypoints_from_raw(kh[0, :n[0]]), orbgpu.keypoints_from_raw(kh[1, :n[1]])
    s, inv, _, _ = ex.scale_factors()
    pl = [ex.level(l, 0) for l in range(ex.nlevels)]
    pr = [ex.level(l, 1) for l in range(ex.nlevels)]
    ur_r, dp_r = stereo_ref.compute_stereo_matches(kl, dh[0, :n[0]], kr, dh[1, :n[1]], pl, pr, s, inv, bf, 0.0)
    assert (ur_r >= 0).sum() > 50
    assert ur[0, :n[0]].cpu().numpy().view(np.uint32).tobytes() == ur_r.view(np.uint32).tobytes()
    assert dp[0, :n[0]].cpu().numpy().view(np.uint32).tobytes() == dp_r.view(np.uint32).tobytes()


def _calls_on(torch, device, seed, cases):
    """SearchByProjection, SearchByBoW and ComputeStereoMatches on `device`
    from the calling thread, each against the oracle."""
    import bow
    import orbgpu
    import proj
    orbgpu.set_thread_device(device)
    assert orbgpu.get_thread_device() == device
    tgt, pts, (nm_r, m_r) = cases["proj"]
    nm_g, m_g = proj.search_by_projection(proj_ref.LOCAL, tgt, pts, 1.0, nnratio=0.8)
    assert nm_g == nm_r and nm_r > 20
    np.testing.assert_array_equal(m_g, m_r)
    args, (nb_r, mb_r) = cases["bow"]
    nb_g, mb_g = bow.search_by_bow(1, *args)
    assert nb_g == nb_r and nb_r > 20
    np.testing.assert_array_equal(mb_g, mb_r)
    _stereo_on(torch, device, seed)
    assert orbgpu.get_thread_device() == device


def _in_threads(fns):
    errs = []

    def wrap(f):
        try:
            f()
        except BaseException as e:  # noqa: BLE001 -- re-raised on the main thread
            errs.append(e)

    ts = [threading.Thread(target=wrap, args=(f,)) for f in fns]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]


@pytest.mark.gpu
def test_first_call_on_a_fresh_thread_after_set_thread_device_0():
    """A thread that never touched HIP: orbgpu_set_thread_device(0), then the
    first SearchByProjection / SearchByBoW / ComputeStereoMatches of that
    thread succeed and equal the oracle."""
    torch = _gpu()
    cases = {"proj": _proj_case(31), "bow": _bow_case(32)}
    _in_threads([lambda: _calls_on(torch, 0, 0x51E0, cases)])


@pytest.mark.gpu
def test_two_threads_on_every_visible_device():
    """Two threads per visible device, each on its device, then one thread
    walking every device in turn (the case a per-process "attribute set"
    flag got wrong): every call equals the oracle."""
    torch = _gpu()
    import orbgpu
    n = orbgpu.device_count()
    if n < 2:
        pytest.skip(f"{n} visible device(s): the per-device state needs >= 2 to be exercised across devices")
    cases = {"proj": _proj_case(41), "bow": _bow_case(42)}
    fns = [(lambda d=d, k=k: _calls_on(torch, d, 0x51E0 + k, cases)) for d in range(n) for k in range(2)]
    _in_threads(fns)

    def walk():
        for d in reversed(range(n)):
            _calls_on(torch, d, 0x5200 + d, cases)
    _in_threads([walk])
