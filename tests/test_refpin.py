"""Parity pinned to the REFERENCE ITSELF where its code compiles here.

oracle/ref.mk compiles the reference's DUtils/Random.cpp, Timestamp.cpp,
DBoW2/BowVector.cpp and FeatureVector.cpp unmodified (from /root/reference)
into oracle/_ref/libdbow2ref.so, with the C entry points of
oracle/ref_shim.cpp.  Against that binary:

* the random stream: DUtils::Random::SeedRandOnce(0) +
  RandomInt(min, max) vs orbgpu_seed_rand_once / orbgpu_random_int (the
  stream every RANSAC of the build draws from), over the ranges the
  Initializer, PnPsolver and Sim3Solver use;
* BowVector / FeatureVector: BowVector::addWeight /
  addIfNotExist / normalize(L1 | L2) and FeatureVector::addFeature fed the
  per-feature (word, node, weight) of a transform, vs the GPU library's
  BowVector / FeatureVector (-m gpu) and the oracle's (CPU), for every
  weighting (TF_IDF, TF, IDF, BINARY) and the L1 / L2 / DOT_PRODUCT scorings.

The GPU test library is loaded without a device for the RNG (host code).
When oracle/_ref is absent (a box without /root/reference that was not given
the prebuilt .so) the tests skip.
"""
import ctypes
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
REFLIB = ROOT / "oracle" / "_ref" / "libdbow2ref.so"


@pytest.fixture(scope="module")
def ref():
    if not REFLIB.exists():
        pytest.skip("oracle/_ref/libdbow2ref.so not built (make -C oracle -f ref.mk)")
    L = ctypes.CDLL(str(REFLIB))
    vp, i = ctypes.c_void_p, ctypes.c_int
    L.ref_seed_rand_once.argtypes = [i]
    L.ref_seed_rand.argtypes = [i]
    L.ref_random_int.argtypes = [i, i]
    L.ref_random_int.restype = i
    L.ref_bow_vectors.argtypes = [i, vp, vp, vp, i, i, vp, vp, vp, vp, vp, vp, vp]
    return L


def _ranges(seed=0, n=6000):
    """(min, max) pairs as the solvers draw them: shrinking index sets"""
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        N = int(rng.choice([8, 20, 37, 100, 300, 1000, 4000]))
        k = int(rng.choice([3, 4, 8]))
        out += [(0, N - 1 - j) for j in range(k)]
    return out[:n]


def test_random_int_stream_equals_reference_dutils(ref):
    """Initializer.cpp:102 SeedRandOnce(0), then RandomInt over the draws of
    the minimal-set loops; glibc seeds 0 and 1 give the same stream."""
    import orbgpu
    lib = orbgpu.lib()
    lib.orbgpu_seed_rand_once.argtypes = [ctypes.c_uint]
    lib.orbgpu_random_int.restype = ctypes.c_int
    ref.ref_seed_rand_once(0)
    lib.orbgpu_srand(7)  # a different state first: SeedRandOnce(0) must reset it
    lib.orbgpu_seed_rand_once(0)
    rs = _ranges()
    want = [ref.ref_random_int(a, b) for a, b in rs]
    got = [lib.orbgpu_random_int(a, b) for a, b in rs]
    assert got == want
    # SeedRandOnce is once per process in the reference: a second call keeps the stream going
    ref.ref_seed_rand_once(123)
    lib.orbgpu_seed_rand_once(123)
    assert [lib.orbgpu_random_int(0, 99) for _ in range(500)] == [ref.ref_random_int(0, 99) for _ in range(500)]


@pytest.mark.parametrize("seed", [0, 1, 2, 12345, 2 ** 31 - 1])
def test_seeded_stream_equals_reference_dutils(ref, seed):
    """DUtils::Random::SeedRand(seed) (= srand) vs orbgpu_srand(seed)"""
    import orbgpu
    lib = orbgpu.lib()
    lib.orbgpu_random_int.restype = ctypes.c_int
    ref.ref_seed_rand(seed)
    lib.orbgpu_srand(seed & 0xFFFFFFFF)
    rs = _ranges(seed, 2000)
    assert [lib.orbgpu_random_int(a, b) for a, b in rs] == [ref.ref_random_int(a, b) for a, b in rs]


def _ref_vectors(ref, words, nodes, weights, weighting, scoring):
    n = len(words)
    m = max(n, 1)
    w = np.ascontiguousarray(words, np.int32)
    nd = np.ascontiguousarray(nodes, np.int32)
    wt = np.ascontiguousarray(weights, np.float64)
    bw, bv = np.zeros(m, np.int32), np.zeros(m, np.float64)
    fn, fo, ff = np.zeros(m, np.int32), np.zeros(m + 1, np.int32), np.zeros(m, np.int32)
    bn, fvn = ctypes.c_int(), ctypes.c_int()
    ref.ref_bow_vectors(n, w.ctypes.data, nd.ctypes.data, wt.ctypes.data, weighting, scoring, bw.ctypes.data,
                        bv.ctypes.data, ctypes.byref(bn), fn.ctypes.data, fo.ctypes.data, ff.ctypes.data,
                        ctypes.byref(fvn))
    bow = {int(bw[i]): float(bv[i]) for i in range(bn.value)}
    fv = {int(fn[i]): list(ff[fo[i]:fo[i + 1]]) for i in range(fvn.value)}
    return bow, fv


def _bits(d):
    return {k: np.float64(v).view(np.uint64) for k, v in d.items()}


CASES = [(wgt, sc) for wgt in (0, 1, 2, 3) for sc in (0, 1, 5)]


@pytest.mark.parametrize("weighting,scoring", CASES)
def test_oracle_bow_vectors_equal_reference_dbow2(ref, weighting, scoring):
    """oracle/bow_ref.py's BowVector / FeatureVector vs the reference's
    compiled BowVector / FeatureVector fed the oracle's (word, node, weight)"""
    import bow_ref
    import synth
    par, leaf, desc, w = synth.synthetic_vocabulary(8, 4, 5)
    voc = bow_ref.Vocabulary.from_arrays(8, 4, scoring, weighting, par, leaf, desc, w)
    D = synth.bow_frame_pair(desc[leaf == 1], 700, 0.5, seed=3)[0]
    words, nodes, weights, fv, bow = voc.transform(D, 2)
    rb, rf = _ref_vectors(ref, words, nodes, weights, weighting, scoring)
    assert {k: list(v) for k, v in fv.items()} == rf
    assert _bits(bow) == _bits(rb)


@pytest.mark.gpu
@pytest.mark.parametrize("weighting,scoring", CASES)
def test_gpu_bow_vectors_equal_reference_dbow2(ref, weighting, scoring):
    """csrc/bow.hip's BowVector / FeatureVector (orbgpu_bow_transform) vs the
    reference's compiled BowVector / FeatureVector fed the GPU's own
    (word, node, weight) per feature, bit for bit"""
    import bow
    import synth
    par, leaf, desc, w = synth.synthetic_vocabulary_fast(10, 4, 9)
    voc = bow.Vocabulary.from_arrays(10, 4, scoring, weighting, par, leaf, desc, w)
    for seed in (1, 2):
        D = synth.bow_frame_pair(desc[leaf == 1], 1000, 0.5, seed=seed)[0]
        words, nodes, weights, fv, bw = voc.transform(D, 4)
        rb, rf = _ref_vectors(ref, words, nodes, weights, weighting, scoring)
        assert {k: list(v) for k, v in fv.items()} == rf
        assert _bits(bw) == _bits(rb)
        assert len(rb) > 100
