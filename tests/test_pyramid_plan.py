"""The fused pyramid kernel's plan (csrc/pyramid_plan.cpp), executed on the
CPU by orbgpu_debug_pyramid_emulate with the kernel's own LDS ring slots, row
records, per-lane column entries and fixed-point arithmetic, reproduces the
oracle's level-by-level ComputePyramid (ORBextractor.cpp:1123-1148) bit for
bit.  The emulation also checks the schedule itself: every read finds its
source row in its slot, no write of a tick lands in a slot read during it.
No GPU needed; the GPU kernel is checked against the oracle by
tests/test_gpu_parity.py::test_pyramid_levels."""
import numpy as np
import pytest

import orbgpu
import orbref
import synth


def _check(img, nfeatures=1000, scale_factor=1.2, nlevels=8):
    levels, info = orbgpu.pyramid_plan_emulate(img, nfeatures, scale_factor, nlevels)
    ref = orbref.Extractor(nfeatures=nfeatures, scale_factor=scale_factor, nlevels=nlevels)
    ref.extract(np.ascontiguousarray(img))
    for l in range(1, nlevels):
        b = ref.level(l)
        a = levels[l - 1]
        assert a.shape == b.shape, (l, a.shape, b.shape)
        d = np.nonzero(a != b)
        assert len(d[0]) == 0, f"level {l}: {len(d[0])} pixels differ, first {list(zip(*d))[:5]}"
    return info


@pytest.mark.parametrize("w,h,nf", [(640, 480, 1000), (1241, 376, 2000), (752, 480, 1200)])
@pytest.mark.parametrize("kind", ["stream", "noise"])
def test_plan_emulation_matches_oracle(w, h, nf, kind):
    img = synth.mono_stream(1, w, h, seed=7)[0] if kind == "stream" else synth.noise_image(w, h)
    info = _check(img, nf)
    assert info["lds_bytes"] <= 160 * 1024
    assert info["compute_waves"] + info["producer_waves"] <= 16


@pytest.mark.parametrize("w,h,sf,nl", [(320, 240, 1.2, 5), (1280, 720, 1.2, 8), (641, 479, 1.2, 8),
                                       (800, 600, 1.5, 5), (900, 700, 2.0, 4), (700, 500, 1.1, 12)])
def test_plan_emulation_other_geometries(w, h, sf, nl):
    """odd sizes, other scale factors and level counts (the tick schedule,
    ring sizes and tail quads change with each)"""
    rng = np.random.default_rng(w * h)
    img = (rng.random((h, w)) * 255).astype(np.uint8)
    _check(img, 1000, sf, nl)


def test_plan_figures_640x480():
    """the headline geometry's plan: one 11-wave block per frame,
    LDS small enough for two blocks per CU"""
    _, info = orbgpu.pyramid_plan_emulate(np.zeros((480, 640), np.uint8))
    assert info["rows_per_chunk"] == 8
    assert info["compute_waves"] + info["producer_waves"] <= 16 and info["entries_per_lane"] == 1
    assert info["lds_bytes"] <= 80 * 1024
