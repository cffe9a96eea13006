"""SearchForInitialization capacity: the 2x-features
initialisation extractor (Tracking.cpp:149: mpIniORBextractor with
2*nFeatures) puts ~870 keypoints on level 0 of a KITTI 1241x376 frame, above
the 512 the small LDS variant holds.  Such pairs run in the 1024 variant
(above that: the 2048 variant, F2's descriptors from HBM) and stay bit-exact
against the oracle; above 2048 the status is per pair (nmatches = -1), never
a process-global flag.  Also: DescriptorDistance over
HBM pairs (orbgpu_hamming_pairs_device) against numpy popcounts."""
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


def _kitti_init_pair():
    frames = synth.mono_stream(2, 1241, 376, seed=0x0B5E + 3)
    ref = orbref.Extractor(nfeatures=4000)
    (k1, d1), (k2, d2) = (ref.extract(f) for f in frames)
    return k1, d1, k2, d2


def test_kitti_init_extractor_pair_bit_exact():
    og = _gpu()
    k1, d1, k2, d2 = _kitti_init_pair()
    n0 = int((k1["octave"] == 0).sum())
    assert n0 > 512, n0  # exercises the large variant
    n_r, m_r, p_r = orbref.search_for_initialization(k1, d1, k2, d2, 1241, 376)
    n_g, m_g, p_g = og.search_for_initialization(k1, d1, k2, d2, 1241, 376)
    assert n_r > 50
    assert n_g == n_r
    np.testing.assert_array_equal(m_g, m_r)
    np.testing.assert_array_equal(p_g.view(np.uint32), p_r.view(np.uint32))


def _pack(frames, cap):
    B = len(frames)
    kps = np.zeros((B, cap, 7), np.float32)
    desc = np.zeros((B, cap, 32), np.uint8)
    counts = np.zeros(B, np.int32)
    for b, (k, d) in enumerate(frames):
        kps[b, :len(k)] = k.view(np.float32).reshape(-1, 7)
        desc[b, :len(k)] = d
        counts[b] = len(k)
    return (torch.from_numpy(kps).cuda(), torch.from_numpy(desc).cuda(), torch.from_numpy(counts).cuda())


def _crowded(n, seed):
    import orbgpu
    rng = np.random.default_rng(seed)
    k = np.zeros(n, orbgpu.KP_DTYPE)
    k["x"] = rng.uniform(10, 630, n).astype(np.float32)
    k["y"] = rng.uniform(10, 470, n).astype(np.float32)
    k["size"], k["octave"], k["class_id"] = 31.0, 0, -1
    k["angle"] = rng.uniform(0, 360, n).astype(np.float32)
    return k, rng.integers(0, 256, (n, 32), dtype=np.uint8)


def test_batch_mixed_capacity_is_per_pair(mono_frames):
    """pair 0 normal, pair 1 in the 1024 variant, pair 2 in the 2048 variant,
    pair 3 over capacity: each gets its own status; a single-pair call
    afterwards is unaffected."""
    og = _gpu()
    ref = orbref.Extractor()
    f0, f1 = ref.extract(mono_frames[0]), ref.extract(mono_frames[1])
    mid1, mid2 = _crowded(800, 1), _crowded(800, 2)
    big1, big2 = _crowded(1900, 3), _crowded(2040, 4)
    # big2 re-observes big1: jittered positions, a few flipped descriptor bits
    rng = np.random.default_rng(7)
    big2[0][:1900]["x"] = big1[0]["x"] + rng.uniform(-3, 3, 1900).astype(np.float32)
    big2[0][:1900]["y"] = big1[0]["y"] + rng.uniform(-3, 3, 1900).astype(np.float32)
    big2[1][:1900] = big1[1] ^ (rng.random((1900, 32)) < 0.03).astype(np.uint8) << rng.integers(0, 8, (1900, 32)).astype(np.uint8)
    over1, over2 = _crowded(2100, 5), _crowded(900, 6)
    cap = 2100
    K1, D1, N1 = _pack([f0, mid1, big1, over1], cap)
    K2, D2, N2 = _pack([f1, mid2, big2, over2], cap)
    m12 = torch.full((4, cap), -7, dtype=torch.int32, device="cuda")
    nm = torch.full((4,), 99, dtype=torch.int32, device="cuda")
    og.search_for_initialization_batch(640, 480, K1, D1, N1, K2, D2, N2, m12, nm)
    torch.cuda.synchronize()
    nm, m12 = nm.cpu().numpy(), m12.cpu().numpy()
    for b, (a, c) in enumerate([(f0, f1), (mid1, mid2), (big1, big2)]):
        n_r, m_r, _ = orbref.search_for_initialization(a[0], a[1], c[0], c[1], 640, 480)
        assert nm[b] == n_r, b
        np.testing.assert_array_equal(m12[b, :len(a[0])], m_r)
    assert nm[2] > 0
    assert nm[3] == -1
    assert (m12[3, :2100] == -1).all()
    # the next single-pair calls see no stale error; the host form takes the 2048 variant too
    n_r, m_r, _ = orbref.search_for_initialization(f0[0], f0[1], f1[0], f1[1], 640, 480)
    n_g, m_g, _ = og.search_for_initialization(f0[0], f0[1], f1[0], f1[1], 640, 480)
    assert n_g == n_r and np.array_equal(m_g, m_r)
    n_r, m_r, p_r = orbref.search_for_initialization(big1[0], big1[1], big2[0], big2[1], 640, 480)
    n_g, m_g, p_g = og.search_for_initialization(big1[0], big1[1], big2[0], big2[1], 640, 480)
    assert n_g == n_r and np.array_equal(m_g, m_r)
    np.testing.assert_array_equal(p_g.view(np.uint32), p_r.view(np.uint32))
    with pytest.raises(og.OrbGpuError) as ei:
        og.search_for_initialization(over1[0], over1[1], over2[0], over2[1], 640, 480)
    assert ei.value.code == og.ERR_CAPACITY


@pytest.mark.parametrize("n", [0, 1, 255, 256, 10007])
def test_hamming_pairs_device(n):
    og = _gpu()
    rng = np.random.default_rng(n)
    a = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    b = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    if n > 2:
        b[0] = a[0]          # distance 0
        b[1] = ~a[1]         # distance 256
    out = torch.full((max(n, 1),), -1, dtype=torch.int32, device="cuda")
    og.hamming_pairs(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda(), out)
    torch.cuda.synchronize()
    want = np.unpackbits(a ^ b, axis=1).sum(1).astype(np.int32)
    np.testing.assert_array_equal(out.cpu().numpy()[:n], want)
    for i in range(min(n, 50)):
        assert want[i] == orbref.descriptor_distance(a[i], b[i])


@pytest.mark.gpu
def test_pack_rows_device_equals_host_unpack():
    """orbgpu_pack_rows_device (the delivery of a batch's trimmed outputs):
    frame b's first counts[b] rows of each tensor at the exclusive prefix sum
    of the counts, for keypoint (28 B), descriptor (32 B) and match (4 B) rows,
    ragged counts including empty frames and full-capacity frames."""
    import torch
    import orbgpu
    import shard
    rng = np.random.default_rng(5)
    B, cap = 37, 130
    counts = rng.integers(0, cap + 1, B).astype(np.int32)
    counts[[0, 7, 8]] = 0
    counts[[3, 36]] = cap
    kps = torch.tensor(rng.standard_normal((B, cap, 7)).astype(np.float32), device="cuda")
    desc = torch.tensor(rng.integers(0, 256, (B, cap, 32)).astype(np.uint8), device="cuda")
    m12 = torch.tensor(rng.integers(-2, 500, (B, cap)).astype(np.int32), device="cuda")
    c = torch.tensor(counts, device="cuda")
    c2 = torch.tensor(counts[::-1].copy(), device="cuda")
    pk = torch.zeros((B * cap, 7), dtype=torch.float32, device="cuda")
    pd = torch.zeros((B * cap, 32), dtype=torch.uint8, device="cuda")
    pm = torch.zeros(B * cap, dtype=torch.int32, device="cuda")
    orbgpu.pack_rows(B, cap, [(kps, pk, c), (desc, pd, c), (m12, pm, c2)])
    torch.cuda.synchronize()
    for rows, packed, cnt in ((kps, pk, counts), (desc, pd, counts), (m12, pm, counts[::-1])):
        n = int(cnt.sum())
        back = shard.unpack_rows(packed[:n].cpu().numpy(), cnt, cap)
        ref = rows.cpu().numpy().copy()
        for b in range(B):
            ref[b, cnt[b]:] = 0
        assert np.array_equal(back, ref)
        assert not packed[n:].cpu().numpy().any()  # nothing written past the used rows


@pytest.mark.parametrize("threads", ["256", "512", "1024"])
def test_batch_block_sizes_and_level0_bound(mono_frames, monkeypatch, threads):
    """A batch that fills the chip (>= 256 pairs) runs the small variant with
    ORBGPU_MATCH_THREADS threads per pair: every block size equals the
    oracle.  With max_level0 (the extractor's level-0 capacity) the larger
    variants are launched only when the bound needs them; a pair above the
    last variant launched reports -1."""
    og = _gpu()
    monkeypatch.setenv("ORBGPU_MATCH_THREADS", threads)
    ref = orbref.Extractor()
    f0, f1 = ref.extract(mono_frames[0]), ref.extract(mono_frames[1])
    mid1, mid2 = _crowded(800, 11), _crowded(800, 12)
    big1, big2 = _crowded(1900, 13), _crowded(1500, 14)
    kinds = [(f0, f1), (mid1, mid2), (big1, big2)]
    want = [orbref.search_for_initialization(a[0], a[1], c[0], c[1], 640, 480)[:2] for a, c in kinds]
    B, cap = 258, 1900
    order = [b % 3 if b % 8 == 0 else 0 for b in range(B)]  # mostly normal pairs, as a stream has
    K1, D1, N1 = _pack([kinds[k][0] for k in order], cap)
    K2, D2, N2 = _pack([kinds[k][1] for k in order], cap)
    for bound, ok in ((0, (True, True, True)), (600, (True, True, False)), (300, (True, False, False))):
        m12 = torch.full((B, cap), -7, dtype=torch.int32, device="cuda")
        nm = torch.full((B,), 99, dtype=torch.int32, device="cuda")
        og.search_for_initialization_batch(640, 480, K1, D1, N1, K2, D2, N2, m12, nm, max_level0=bound)
        torch.cuda.synchronize()
        nm_h, m12_h = nm.cpu().numpy(), m12.cpu().numpy()
        for b, k in enumerate(order):
            n1 = len(kinds[k][0][0])
            if ok[k]:
                assert nm_h[b] == want[k][0], (bound, b, k)
                np.testing.assert_array_equal(m12_h[b, :n1], want[k][1])
            else:
                assert nm_h[b] == -1, (bound, b, k)
                assert (m12_h[b, :n1] == -1).all()
