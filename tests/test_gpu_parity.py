"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on
the same seeded inputs.  Bit-exact for every integer/byte output and for the
float keypoint fields (they are computed with identical IEEE operations)."""
from pathlib import Path

import numpy as np
import pytest

import orbref
import synth

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _gpu():
    import orbgpu
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return orbgpu


def _assert_same_kps(kg, dg, kr, dr):
    assert len(kg) == len(kr), (len(kg), len(kr))
    for f in ("x", "y", "size", "angle", "response", "octave", "class_id"):
        a, b = kg[f], kr[f]
        bad = np.nonzero(a.view(np.uint32) != b.view(np.uint32))[0] if a.dtype.kind == "f" else np.nonzero(a != b)[0]
        assert len(bad) == 0, f"field {f}: {len(bad)} mismatches, first {bad[:5]} gpu={a[bad[:5]]} ref={b[bad[:5]]}"
    bad = np.nonzero((dg != dr).any(axis=1))[0]
    assert len(bad) == 0, f"descriptors differ at {len(bad)} keypoints, first {bad[:5]}"


def test_device_is_gfx950():
    og = _gpu()
    assert og.device_arch().startswith("gfx950")


@pytest.mark.parametrize("frame", [0, 3])
def test_pyramid_levels(mono_frames, frame):
    og = _gpu()
    ex = og.Extractor()
    ref = orbref.Extractor()
    img = mono_frames[frame]
    ex.extract(img)
    ref.extract(img)
    for l in range(8):
        a, b = ex.level(l), ref.level(l)
        assert a.shape == b.shape
        d = np.nonzero(a != b)
        assert len(d[0]) == 0, f"level {l}: {len(d[0])} pixels differ, first {list(zip(*d))[:5]}"


@pytest.mark.parametrize("w,h,nf,kind", [(640, 480, 1000, "stream"), (640, 480, 1000, "noise"),
                                         (1241, 376, 2000, "stream"), (752, 480, 1200, "noise")])
def test_blurred_levels(w, h, nf, kind):
    """GaussianBlur(7x7, sigma 2, REFLECT_101) of every level, bit-exact
    (incl. the half-to-even / half-up column rounding split at 4*floor(w/4))."""
    og = _gpu()
    ex = og.Extractor(nfeatures=nf, width=w, height=h)
    img = synth.mono_stream(1, w, h, seed=11)[0] if kind == "stream" else synth.noise_image(w, h)
    ex.extract(img)
    for l in range(8):
        a, b = ex.blurred(l), orbref.gaussian7(ex.level(l))
        d = np.nonzero(a != b)
        assert len(d[0]) == 0, f"level {l}: {len(d[0])} pixels differ, first {list(zip(*d))[:5]}"


@pytest.mark.parametrize("frame", [0, 1, 2, 5])
def test_extract_mono_640x480(mono_frames, frame):
    og = _gpu()
    ex = og.Extractor()
    ref = orbref.Extractor()
    kg, dg = ex.extract(mono_frames[frame])
    kr, dr = ref.extract(mono_frames[frame])
    _assert_same_kps(kg, dg, kr, dr)


def test_extract_noise_and_flat():
    og = _gpu()
    ex = og.Extractor()
    ref = orbref.Extractor()
    for img in (synth.noise_image(), synth.flat_image()):
        kg, dg = ex.extract(img)
        kr, dr = ref.extract(img)
        _assert_same_kps(kg, dg, kr, dr)


def test_empty_image_untouched():
    og = _gpu()
    ex = og.Extractor()
    assert ex.extract(np.zeros((0, 0), np.uint8)) is None


@pytest.mark.parametrize("w,h,nf", [(1241, 376, 2000), (752, 480, 1200)])
def test_extract_stereo_geometries(w, h, nf):
    og = _gpu()
    ex = og.Extractor(nfeatures=nf, width=w, height=h)
    ref = orbref.Extractor(nfeatures=nf)
    frames = synth.stereo_stream(1, w, h, seed=11)
    for img in frames[0]:
        kg, dg = ex.extract(img)
        kr, dr = ref.extract(img)
        _assert_same_kps(kg, dg, kr, dr)


@pytest.mark.parametrize("w,h,nf", [(1241, 376, 4000), (640, 480, 2500)])
def test_extract_many_features(w, h, nf):
    """Large feature budgets (the KITTI initialisation extractor uses 2 x
    nFeatures, Tracking.cpp:149): the octree's inner pass orders several
    hundred level-0 nodes (rank sort up to 512, bitonic above) and the
    level-0 candidate lists approach the in-LDS key capacity."""
    og = _gpu()
    ex = og.Extractor(nfeatures=nf, width=w, height=h)
    ref = orbref.Extractor(nfeatures=nf)
    for img in synth.mono_stream(2, w, h, seed=0x0B5E + nf):
        kg, dg = ex.extract(img)
        kr, dr = ref.extract(img)
        _assert_same_kps(kg, dg, kr, dr)


@pytest.mark.parametrize("w,h,nf", [(640, 480, 1000), (1241, 376, 2000), (752, 480, 1200)])
def test_pyramid_paths_agree(w, h, nf):
    """The two device pyramid passes: batches up to 8 frames take the banded
    single-launch kernel (row bands with every level in LDS, halo rows
    recomputed), larger batches the tick pipeline.  Both equal the oracle's
    levels on every frame, also from a caller buffer with a padded row
    step."""
    og = _gpu()
    frames = synth.mono_stream(12, w, h, seed=23)
    ref = orbref.Extractor(nfeatures=nf)
    want = []
    for img in frames[:3]:
        ref.extract(img)
        want.append([ref.level(l) for l in range(8)])
    p16 = (w + 15) // 16 * 16
    for B, pitch in ((3, p16), (12, p16), (2, p16 + 48)):
        ex = og.Extractor(nfeatures=nf, width=w, height=h, max_batch=B)
        buf = np.zeros((B, h, pitch), np.uint8)
        buf[:, :, :w] = frames[:B]
        imgs = torch.from_numpy(buf).cuda()
        cap = ex.max_keypoints
        kps = torch.zeros((B, cap, 7), dtype=torch.float32, device="cuda")
        desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
        counts = torch.zeros(B, dtype=torch.int32, device="cuda")
        ex.extract_batch(imgs, kps, desc, counts)
        ex.sync()
        for f in range(min(B, 3)):
            for l in range(1, 8):
                a = ex.level(l, frame=f)
                d = np.nonzero(a != want[f][l])
                assert len(d[0]) == 0, f"B={B} pitch={pitch} frame {f} level {l}: {len(d[0])} pixels differ"


@pytest.mark.parametrize("w,h,nf", [(640, 480, 1000), (1241, 376, 2000), (752, 480, 1200), (640, 224, 500)])
def test_single_frame_host_path_levels_and_keypoints(w, h, nf):
    """The single-frame host path (orbgpu_extract: pinned staging, copy kernel,
    band pyramid with 64 bands -- 48 at 640x224, whose level 7 has 63 rows).
    Every level, level 0 included, and the keypoints and descriptors equal the
    oracle's, over consecutive calls of one extractor (a call must not see the
    previous frame's rows)."""
    og = _gpu()
    frames = synth.mono_stream(3, w, h, seed=29)
    ref = orbref.Extractor(nfeatures=nf)
    ex = og.Extractor(nfeatures=nf, width=w, height=h, max_batch=1)
    for img in frames:
        kg, dg = ex.extract(img)
        kr, dr = ref.extract(img)
        for l in range(8):
            a = ex.level(l)
            d = np.nonzero(a != ref.level(l))
            assert len(d[0]) == 0, f"{w}x{h} level {l}: {len(d[0])} pixels differ"
        _assert_same_kps(kg, dg, kr, dr)


def test_single_frame_repeated_calls_read_complete_results():
    """The single-frame call returns when its completion flag (written after
    the extraction by a one-wave kernel into coherent pinned memory) arrives,
    not after a stream synchronisation: 120 calls alternating two frames on
    two extractors (the stereo pair's pattern) must each return exactly that
    frame's keypoints and descriptors -- a result read before all of the
    call's output stores landed would differ."""
    og = _gpu()
    frames = synth.mono_stream(2, 640, 480, seed=31)
    ref = orbref.Extractor(nfeatures=1000)
    exs = [og.Extractor(nfeatures=1000, width=640, height=480, max_batch=1) for _ in range(2)]
    want = []
    for f in frames:
        kg, dg = exs[0].extract(f)
        _assert_same_kps(kg, dg, *ref.extract(f))
        want.append((kg.tobytes(), dg.tobytes()))
    for it in range(120):
        j = (it // 2) % 2 if it % 3 else it % 2
        kg, dg = exs[it % 2].extract(frames[j])
        assert (kg.tobytes(), dg.tobytes()) == want[j], f"call {it} (frame {j}, extractor {it % 2}) differs"


def test_batch_device_matches_single(mono_frames):
    og = _gpu()
    B = len(mono_frames)
    ex = og.Extractor(max_batch=B)
    imgs = torch.from_numpy(mono_frames).cuda()
    cap = ex.max_keypoints
    kps = torch.zeros((B, cap, 7), dtype=torch.float32, device="cuda")
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(B, dtype=torch.int32, device="cuda")
    ex.extract_batch(imgs, kps, desc, counts)
    ex.sync()
    ref = orbref.Extractor()
    kk, dd, cc = kps.cpu().numpy(), desc.cpu().numpy(), counts.cpu().numpy()
    for b in range(B):
        kr, dr = ref.extract(mono_frames[b])
        kg = og.keypoints_from_raw(kk[b, :cc[b]])
        _assert_same_kps(kg, dd[b, :cc[b]], kr, dr)


@pytest.mark.parametrize("chunks", [2, 4])
def test_batch_octree_describe_chunks_match_oracle(monkeypatch, chunks):
    """ORBGPU_OD_CHUNKS: the octree of chunk c+1 on the batch stream beside the
    describe of chunk c on a second stream (run_batch); every frame of a
    64-frame batch equals the oracle, the chunk boundaries included."""
    og = _gpu()
    monkeypatch.setenv("ORBGPU_OD_CHUNKS", str(chunks))
    B = 64
    frames = synth.mono_stream(B, 640, 480, seed=91)
    ex = og.Extractor(max_batch=B)
    imgs = torch.from_numpy(np.ascontiguousarray(frames)).cuda()
    cap = ex.max_keypoints
    kps = torch.zeros((B, cap, 7), dtype=torch.float32, device="cuda")
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(B, dtype=torch.int32, device="cuda")
    ex.extract_batch(imgs, kps, desc, counts)
    ex.sync()
    ref = orbref.Extractor()
    kk, dd, cc = kps.cpu().numpy(), desc.cpu().numpy(), counts.cpu().numpy()
    step = B // chunks
    for b in sorted({0, 1, step - 1, step, step + 1, B - 1, B // 2 + 3}):
        kr, dr = ref.extract(frames[b])
        kg = og.keypoints_from_raw(kk[b, :cc[b]])
        _assert_same_kps(kg, dd[b, :cc[b]], kr, dr)


@pytest.mark.parametrize("B", [1, 16])
def test_octree_key_scratch_path_matches_oracle(monkeypatch, B):
    """ORBGPU_OCT_KCAP_A=256 leaves levels 0-1 a 192-key LDS capacity, so
    every level-0/1 octree runs on the HBM-scratch key store with u32
    quadrant counters (the in-LDS path keeps u16 counters), in 1024-thread
    (B=1) and 256-thread (B=16) workgroups; every frame equals the oracle."""
    og = _gpu()
    monkeypatch.setenv("ORBGPU_OCT_KCAP_A", "256")
    frames = synth.mono_stream(B, 640, 480, seed=57)
    ex = og.Extractor(max_batch=B)
    imgs = torch.from_numpy(np.ascontiguousarray(frames)).cuda()
    cap = ex.max_keypoints
    kps = torch.zeros((B, cap, 7), dtype=torch.float32, device="cuda")
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(B, dtype=torch.int32, device="cuda")
    ex.extract_batch(imgs, kps, desc, counts)
    ex.sync()
    ref = orbref.Extractor()
    kk, dd, cc = kps.cpu().numpy(), desc.cpu().numpy(), counts.cpu().numpy()
    for b in sorted({0, B // 2, B - 1}):
        kr, dr = ref.extract(frames[b])
        kg = og.keypoints_from_raw(kk[b, :cc[b]])
        _assert_same_kps(kg, dd[b, :cc[b]], kr, dr)


def test_timed_headline_batch_512_vs_oracle():
    """The configuration bench.py times, checked at full size:
    two consecutive 512-frame batches of the bench's bounded 640x480 stream at
    the bench's pitch, one extractor with max_batch 512 (the tick pyramid, the
    octree's 256-thread level groups, the XCD-swizzled describe grid), then the
    stream-form SearchForInitialization over the second batch (512 pairs:
    256-thread pair blocks, the extractor's level-0 bound), whose pair 0 reads
    the first batch's last frame in place (src/Tracking.cpp:768-769).  Frames
    across the batch -- both ends, the 64-frame and 256-frame boundaries --
    and the pairs between them equal the oracle bit for bit."""
    og = _gpu()
    B, W, H, NF = 512, 640, 480, 1000
    pitch = (W + 15) // 16 * 16
    ex = og.Extractor(nfeatures=NF, width=W, height=H, max_batch=B)
    cap = ex.max_keypoints
    sets = []
    for t0 in (0, B):
        imgs = synth.torch_stream(B, W, H, device="cuda", pitch=pitch, bounded=True, t0=t0)
        kps = torch.zeros((B, cap, 7), dtype=torch.float32, device="cuda")
        desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
        counts = torch.zeros(B, dtype=torch.int32, device="cuda")
        ex.extract_batch(imgs, kps, desc, counts, row_step=pitch, frame_step=pitch * H)
        ex.sync()
        sets.append((imgs, kps, desc, counts))
    (ia, ka, da, ca), (ib, kb, db, cb) = sets
    m12 = torch.full((B, cap), -7, dtype=torch.int32, device="cuda")
    nm = torch.zeros(B, dtype=torch.int32, device="cuda")
    og.search_for_initialization_stream(W, H, kb, db, cb, ka[B - 1], da[B - 1], ca[B - 1:B], m12, nm,
                                        max_level0=ex.level_capacity[0])
    torch.cuda.synchronize()
    assert int(cb.min()) > 900 and int(nm.min()) >= 0
    ref = orbref.Extractor(nfeatures=NF)

    def host(t, b):
        return np.ascontiguousarray(t[b, :, :W].cpu().numpy())

    kk, dd, cc = kb.cpu().numpy(), db.cpu().numpy(), cb.cpu().numpy()
    mm, nn = m12.cpu().numpy(), nm.cpu().numpy()
    R = {}
    for b in (0, 1, 63, 64, 65, 255, 256, 257, 510, 511):
        R[b] = ref.extract(host(ib, b))
        _assert_same_kps(og.keypoints_from_raw(kk[b, :cc[b]]), dd[b, :cc[b]], *R[b])
    R[-1] = ref.extract(host(ia, B - 1))
    n = int(ca[B - 1])
    _assert_same_kps(og.keypoints_from_raw(ka[B - 1, :n].cpu().numpy()), da[B - 1, :n].cpu().numpy(), *R[-1])
    for b in (0, 1, 64, 65, 256, 257, 511):
        f1 = R[b - 1]
        n_r, m_r, _ = orbref.search_for_initialization(f1[0], f1[1], R[b][0], R[b][1], W, H)
        assert int(nn[b]) == n_r, (b, int(nn[b]), n_r)
        np.testing.assert_array_equal(mm[b, :len(f1[0])], m_r)
        assert n_r > 50  # consecutive frames of the stream really match


@pytest.mark.parametrize("check_ori,annotated", [(True, False), (False, False), (True, True)])
def test_search_for_initialization(mono_frames, check_ori, annotated):
    og = _gpu()
    ref = orbref.Extractor()
    k1, d1 = ref.extract(mono_frames[0])
    k2, d2 = ref.extract(mono_frames[1])
    n_r, m_r, p_r = orbref.search_for_initialization(k1, d1, k2, d2, 640, 480, check_ori=check_ori,
                                                     histo_bug=annotated)
    n_g, m_g, p_g = og.search_for_initialization(k1, d1, k2, d2, 640, 480, check_ori=check_ori,
                                                 annotated_histo=annotated)
    assert n_g == n_r
    np.testing.assert_array_equal(m_g, m_r)
    np.testing.assert_array_equal(p_g.view(np.uint32), p_r.view(np.uint32))


def _conflict_frames(seed, n=420, protos=24, flips=3):
    """Level-0 keypoints whose descriptors are noisy copies of a few
    prototypes: most queries see many candidates at equal or near distances,
    so matches are stolen and candidates skipped (vMatchedDistance) -- the
    paths where the GPU's per-query top-k list runs out and re-scans."""
    import orbgpu
    rng = np.random.default_rng(seed)
    P = rng.integers(0, 256, (protos, 32), dtype=np.uint8)

    def frame():
        k = np.zeros(n, orbgpu.KP_DTYPE)
        k["x"] = rng.uniform(20, 620, n).astype(np.float32)
        k["y"] = rng.uniform(20, 460, n).astype(np.float32)
        k["size"] = 31.0
        k["angle"] = rng.uniform(0, 360, n).astype(np.float32)
        k["octave"] = 0
        k["class_id"] = -1
        d = P[rng.integers(0, protos, n)].copy()
        for i in range(n):
            for _ in range(int(rng.integers(0, flips + 1))):
                b = int(rng.integers(0, 256))
                d[i, b >> 3] ^= np.uint8(1 << (b & 7))
        return k, d
    return frame() + frame()


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("check_ori", [True, False])
def test_search_for_initialization_conflicts(seed, check_ori):
    og = _gpu()
    k1, d1, k2, d2 = _conflict_frames(seed)
    n_r, m_r, p_r = orbref.search_for_initialization(k1, d1, k2, d2, 640, 480, check_ori=check_ori)
    n_g, m_g, p_g = og.search_for_initialization(k1, d1, k2, d2, 640, 480, check_ori=check_ori)
    assert n_r > 20
    assert n_g == n_r
    np.testing.assert_array_equal(m_g, m_r)
    np.testing.assert_array_equal(p_g.view(np.uint32), p_r.view(np.uint32))


def test_search_for_initialization_distorted_bounds(mono_frames):
    """Undistorted keypoints (mvKeysUn) with Frame bounds other than
    [0,W]x[0,H]: some keypoints fall outside the grid (PosInGrid rejects
    them, Frame.cpp:434-443)."""
    og = _gpu()
    ref = orbref.Extractor()
    k1, d1 = ref.extract(mono_frames[0])
    k2, d2 = ref.extract(mono_frames[1])
    for k in (k1, k2):  # a radial-ish warp standing in for cv::undistortPoints
        dx, dy = k["x"] - 320.0, k["y"] - 240.0
        r2 = (dx * dx + dy * dy).astype(np.float32) * np.float32(2e-7)
        k["x"] = (np.float32(320.0) + dx * (np.float32(1.0) + r2)).astype(np.float32)
        k["y"] = (np.float32(240.0) + dy * (np.float32(1.0) + r2)).astype(np.float32)
    bounds = (-7.25, 631.5, -3.0, 470.75)
    n_r, m_r, p_r = orbref.search_for_initialization(k1, d1, k2, d2, 640, 480, bounds=bounds)
    n_g, m_g, p_g = og.search_for_initialization(k1, d1, k2, d2, 640, 480, bounds=og.GridBounds(*bounds))
    assert n_r > 100
    assert n_g == n_r
    np.testing.assert_array_equal(m_g, m_r)
    np.testing.assert_array_equal(p_g.view(np.uint32), p_r.view(np.uint32))


@pytest.mark.parametrize("w,h,nf", [(640, 480, 1000), (1241, 376, 2000), (752, 480, 1200)])
def test_stages_candidates_and_octree(w, h, nf):
    """Stage-level parity: FAST candidates and octree output per level."""
    og = _gpu()
    ex = og.Extractor(nfeatures=nf, width=w, height=h)
    ref = orbref.Extractor(nfeatures=nf)
    img = synth.mono_stream(1, w, h, seed=5)[0]
    ex.extract(img)
    ref.extract(img)
    for l in range(8):
        np.testing.assert_array_equal(ex.level(l), ref.level(l), err_msg=f"pyramid level {l}")
        cg, cr = ex.candidates(l), ref.candidates(l)
        assert cg.shape == cr.shape, f"level {l}: {len(cg)} vs {len(cr)} candidates"
        np.testing.assert_array_equal(cg, cr, err_msg=f"candidates level {l}")
        og_, or_ = ex.octree(l), ref.octree(l)
        assert og_.shape == or_.shape, f"level {l}: octree {len(og_)} vs {len(or_)}"
        np.testing.assert_array_equal(og_, or_, err_msg=f"octree level {l}")


@pytest.mark.parametrize("name,w,h,nf,seed,n", [("mono640_f0", 640, 480, 1000, 0x0B5E, 2),
                                                ("kitti_f0", 1241, 376, 2000, 21, 1),
                                                ("euroc_f0", 752, 480, 1200, 22, 1)])
def test_gpu_against_golden_fixtures(name, w, h, nf, seed, n):
    """HIP path vs the committed oracle fixtures (tests/golden, see make_golden.py)."""
    og = _gpu()
    g = np.load(Path(__file__).resolve().parent / "golden" / f"{name}.npz")
    frames = synth.mono_stream(n, w, h, seed=seed)
    ex = og.Extractor(nfeatures=nf, width=w, height=h)
    k, d = ex.extract(frames[0])
    assert k.view(np.uint8).reshape(-1, 28).tobytes() == g["kps"].tobytes()
    assert np.array_equal(d, g["desc"])
    if n > 1:
        k1, d1 = ex.extract(frames[1])
        nm, m12, _ = og.search_for_initialization(k, d, k1, d1, w, h)
        assert nm == int(g["nmatches"]) and np.array_equal(m12, g["matches12"])


def test_batch_matcher_device_path(mono_frames):
    """search_for_initialization_batch over consecutive pairs == host form."""
    og = _gpu()
    B = 4
    ex = og.Extractor(max_batch=B)
    imgs = torch.from_numpy(mono_frames[:B]).cuda()
    cap = ex.max_keypoints
    kps = torch.zeros((B, cap, 7), dtype=torch.float32, device="cuda")
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(B, dtype=torch.int32, device="cuda")
    ex.extract_batch(imgs, kps, desc, counts)
    m12 = torch.full((B - 1, cap), -7, dtype=torch.int32, device="cuda")
    nm = torch.zeros(B - 1, dtype=torch.int32, device="cuda")
    og.search_for_initialization_batch(640, 480, kps[:-1], desc[:-1], counts[:-1], kps[1:], desc[1:], counts[1:],
                                       m12, nm)
    ex.sync()
    kk, dd, cc = kps.cpu().numpy(), desc.cpu().numpy(), counts.cpu().numpy()
    for b in range(B - 1):
        k1 = og.keypoints_from_raw(kk[b, :cc[b]])
        k2 = og.keypoints_from_raw(kk[b + 1, :cc[b + 1]])
        n_r, m_r, _ = orbref.search_for_initialization(k1, dd[b, :cc[b]], k2, dd[b + 1, :cc[b + 1]], 640, 480)
        assert int(nm[b]) == n_r
        np.testing.assert_array_equal(m12[b, :cc[b]].cpu().numpy(), m_r)
