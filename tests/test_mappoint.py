"""MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cpp:302-380) and
MapPoint::UpdateNormalAndDepth (:414-457) over batches of points: GPU
(csrc/mappoint.hip through include/orbgpu_mappoint.h) vs oracle/mappoint_ref.py.

Bar: bit-exact -- the chosen observation and its median (integer work), and
the float normal / distance bounds (the oracle follows the same expression
order; the OpenCV conventions it restates are documented there and in
DESIGN.md §5, parity unpinned against a reference run)."""
import numpy as np
import pytest

import mappoint_ref
import synth


def _oracle_distinctive(sc):
    off, desc, valid = sc["offsets"], sc["desc"], sc["valid"]
    out = [mappoint_ref.compute_distinctive_descriptors(desc[off[p]:off[p + 1]], valid[off[p]:off[p + 1]])
           for p in range(len(off) - 1)]
    return np.array([o[0] for o in out], np.int32), np.array([o[1] for o in out], np.int32)


def test_oracle_distinctive_known_answers():
    rng = np.random.default_rng(0)
    d = rng.integers(0, 256, (1, 32), dtype=np.uint8)
    assert mappoint_ref.compute_distinctive_descriptors(d) == (0, 0)  # N = 1: median of [0]
    two = rng.integers(0, 256, (2, 32), dtype=np.uint8)
    assert mappoint_ref.compute_distinctive_descriptors(two) == (0, 0)  # rows [0, d]: element 0
    assert mappoint_ref.compute_distinctive_descriptors(two, [0, 1]) == (1, 0)  # bad keyframe skipped
    assert mappoint_ref.compute_distinctive_descriptors(two, [0, 0]) == (-1, -1)
    a = np.zeros(32, np.uint8)
    b = a.copy(); b[:2] = 0xFF    # 16 bits from a
    c = a.copy(); c[:4] = 0xFF    # 32 bits from a, 16 from b
    # three: element 1 of every sorted row is 16; the first row wins
    assert mappoint_ref.compute_distinctive_descriptors(np.stack([a, c, b])) == (0, 16)
    # the repeated descriptor has median 0 (rows [240, 0, 0, 0, 16] sorted: element 2)
    far = np.full(32, 0xFF, np.uint8)
    assert mappoint_ref.compute_distinctive_descriptors(np.stack([far, b, b, b, a])) == (1, 0)
    # equal medians: the first one wins
    assert mappoint_ref.compute_distinctive_descriptors(np.stack([a, a, b, b]))[0] == 0


def test_oracle_normal_depth_known_answer():
    n, dmin, dmax = mappoint_ref.update_normal_and_depth([[0, 0, 0], [2, 0, 0]], [1, 0, 0], [0, 0, 0], 1.44, 3.5831808)
    np.testing.assert_array_equal(n, np.zeros(3, np.float32))  # opposite directions cancel
    assert dmax == np.float32(1.44) and dmin == np.float32(np.float32(1.44) / np.float32(3.5831808))
    n, _, _ = mappoint_ref.update_normal_and_depth([[0, 0, 0]], [0, 3, 4], [0, 0, 0], 1.0, 1.0)
    np.testing.assert_array_equal(n, np.array([0, 0.6, 0.8], np.float32))


@pytest.mark.gpu
@pytest.mark.parametrize("n_points,max_obs,seed", [(1, 5, 1), (37, 12, 2), (600, 40, 3), (40, 200, 4)])
def test_gpu_distinctive_descriptors_bit_exact(n_points, max_obs, seed):
    import mappoint
    sc = synth.mappoint_scenario(n_points, seed, max_obs=max_obs)
    rb, rm = _oracle_distinctive(sc)
    gb, gm = mappoint.compute_distinctive_descriptors(sc["offsets"], sc["desc"], sc["valid"])
    np.testing.assert_array_equal(gb, rb)
    np.testing.assert_array_equal(gm, rm)
    # all keyframes good (valid = NULL)
    rb2 = np.array([mappoint_ref.compute_distinctive_descriptors(sc["desc"][a:b])[0]
                    for a, b in zip(sc["offsets"][:-1], sc["offsets"][1:])], np.int32)
    gb2, _ = mappoint.compute_distinctive_descriptors(sc["offsets"], sc["desc"])
    np.testing.assert_array_equal(gb2, rb2)


@pytest.mark.gpu
def test_gpu_distinctive_descriptors_ties_and_empty():
    import mappoint
    a = np.zeros(32, np.uint8)
    b = a.copy(); b[:2] = 0xFF
    c = a.copy(); c[:4] = 0xFF
    groups = [np.stack([a, a, b, b]), np.stack([a, c, b]), np.zeros((0, 32), np.uint8), np.stack([c] * 70 + [a] * 71),
              np.stack([b])]
    off = np.cumsum([0] + [len(g) for g in groups]).astype(np.int32)
    desc = np.concatenate(groups)
    gb, gm = mappoint.compute_distinctive_descriptors(off, desc)
    want = [mappoint_ref.compute_distinctive_descriptors(g) for g in groups]
    assert gb.tolist() == [w[0] for w in want] and gm.tolist() == [w[1] for w in want]
    empty = mappoint.compute_distinctive_descriptors(np.zeros(1, np.int32), np.zeros((0, 32), np.uint8))
    assert len(empty[0]) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("n_points,max_obs,seed", [(1, 3, 5), (700, 30, 6), (50, 150, 7)])
def test_gpu_normal_and_depth_bit_exact(n_points, max_obs, seed):
    import mappoint
    sc = synth.mappoint_scenario(n_points, seed, max_obs=max_obs)
    off = sc["offsets"]
    init = np.full((n_points, 3), 7.0, np.float32)
    gn, gmin, gmax = mappoint.update_normal_and_depth(off, sc["obs_Ow"], sc["pos"], sc["ref_Ow"], sc["level_scale"],
                                                      sc["max_scale"], normal=init, min_dist=np.full(n_points, 7.0),
                                                      max_dist=np.full(n_points, 7.0))
    for p in range(n_points):
        if off[p + 1] == off[p]:  # no observation: outputs untouched
            assert (gn[p] == 7.0).all() and gmin[p] == 7.0 and gmax[p] == 7.0
            continue
        rn, rmin, rmax = mappoint_ref.update_normal_and_depth(sc["obs_Ow"][off[p]:off[p + 1]], sc["pos"][p],
                                                              sc["ref_Ow"][p], sc["level_scale"][p],
                                                              sc["max_scale"][p])
        np.testing.assert_array_equal(gn[p], rn)
        assert gmin[p] == rmin and gmax[p] == rmax
