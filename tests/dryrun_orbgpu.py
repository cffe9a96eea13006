"""CPU stand-in for the orbgpu surface bench.py uses, for
`bench.py --cpu-dry-run tests/dryrun_orbgpu.py` (TESTS ONLY).

It lets tests/test_bench_launch.py run bench.py's own launcher (--gpus N ->
torchrun child), rank logic, sharding, boundary exchange and gather over
gloo on the CPU.  Every compute call goes to the CPU oracle (oracle/), which
is what the test compares the gathered outputs with -- so the test checks
the multi-rank plumbing, not the kernels (the kernels' parity is the -m gpu
suite's job).  The product never imports this module.
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import torch

_ROOT = Path(__file__).resolve().parents[1]
for _p in (_ROOT / "oracle", _ROOT / "orb-slam2-annotation_amd"):
    if str(_p) not in sys.path:
        sys.path.insert(0, str(_p))

import orbref  # noqa: E402

MATCH_CHECK_ORI = 1
MATCH_ANNOTATED_HISTO = 2


def _round_half_even(v: float) -> int:
    return int(np.rint(np.float32(v)))


class Extractor:
    """ORBextractor on the CPU oracle; batch tensors on the CPU."""

    def __init__(self, nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7, width=640, height=480,
                 max_batch=1):
        self.nfeatures, self.width, self.height, self.max_batch = nfeatures, width, height, max_batch
        self.ex = orbref.Extractor(nfeatures, scale_factor, nlevels, ini_th, min_th)
        self.args = (nfeatures, scale_factor, nlevels, ini_th, min_th)
        self.max_keypoints = nfeatures + 3 * nlevels + 64
        self.level_capacity = [self.max_keypoints] * nlevels
        _, inv, _, _ = self.ex.scale_factors()
        self.level_sizes = [(_round_half_even(width * inv[l]), _round_half_even(height * inv[l]))
                            for l in range(nlevels)]

    def extract_batch(self, images, kps, desc, counts, stream=None, row_step=None, frame_step=None):
        W = self.width
        for b in range(images.shape[0]):
            k, d = self.ex.extract(images[b, :, :W].numpy())
            n = len(k)
            assert n <= kps.shape[1]
            kps[b, :n] = torch.from_numpy(k.view(np.float32).reshape(n, 7).copy())
            desc[b, :n] = torch.from_numpy(d.copy())
            counts[b] = n

    def sync(self, stream=None):
        pass

    def profile(self, enable=True):
        pass

    def set_stage_event(self, stage, event=None):
        pass

    def stage_times(self, reset=True):
        return {"pyramid": 0.0, "fast_cells": 0.0, "octree": 0.0, "describe": 0.0}, 1


def _kp(t, n):
    return t[:n].numpy().copy().view(orbref.KP_DTYPE).reshape(n)


def search_for_initialization_batch(img_w, img_h, kps1, desc1, n1, kps2, desc2, n2, matches12, nmatches,
                                    prev_xy=None, window=100, nnratio=0.9, flags=MATCH_CHECK_ORI, stream=None,
                                    bounds=None, max_level0=0):
    for b in range(n2.shape[0]):
        a, c = int(n1[b]), int(n2[b])
        matches12[b] = -1
        if a == 0 or c == 0:
            nmatches[b] = 0
            continue
        nm, m12, _ = orbref.search_for_initialization(
            _kp(kps1[b], a), desc1[b, :a].numpy(), _kp(kps2[b], c), desc2[b, :c].numpy(), img_w, img_h,
            window=window, nnratio=nnratio, check_ori=bool(flags & MATCH_CHECK_ORI),
            histo_bug=bool(flags & MATCH_ANNOTATED_HISTO))
        matches12[b, :a] = torch.from_numpy(m12)
        nmatches[b] = nm


def search_for_initialization_stream(img_w, img_h, kps, desc, n, prev_kps, prev_desc, prev_n, matches12, nmatches,
                                     prev_xy=None, window=100, nnratio=0.9, flags=MATCH_CHECK_ORI, stream=None,
                                     bounds=None, max_level0=0):
    """the stream form: pair b matches frame b-1 (pair 0: the prev frame) against frame b"""
    B = n.shape[0]
    k1 = torch.cat([prev_kps[None], kps[:B - 1]])
    d1 = torch.cat([prev_desc[None], desc[:B - 1]])
    n1 = torch.cat([prev_n.reshape(1), n[:B - 1]])
    search_for_initialization_batch(img_w, img_h, k1, d1, n1, kps, desc, n, matches12, nmatches, prev_xy, window,
                                    nnratio, flags, stream, bounds, max_level0)


def stereo_matches_batch(ex: Extractor, images, npairs, kps, desc, counts, bf, min_z, uright, depth, stream=None,
                         row_step=None, frame_step=None):
    """Frame::ComputeStereoMatches of pairs (2p, 2p+1): the oracle stereo
    Frame (two extractors, Frame.cpp:84-98) re-run on the pair; its
    keypoints must be the ones extract_batch wrote."""
    W = ex.width
    exL, exR = orbref.Extractor(*ex.args), orbref.Extractor(*ex.args)
    for p in range(npairs):
        kl, dl, kr, dr, ur, dp = orbref.stereo_frame(exL, exR, images[2 * p, :, :W].numpy(),
                                                     images[2 * p + 1, :, :W].numpy(), bf, min_z)
        n = len(kl)
        assert n == int(counts[2 * p]) and kps[2 * p, :n].numpy().tobytes() == kl.tobytes()
        uright[p] = -1.0
        depth[p] = -1.0
        uright[p, :n] = torch.from_numpy(ur)
        depth[p, :n] = torch.from_numpy(dp)
