"""Stereo front-end throughput on one MI355X:
per step, B rectified pairs (2B frames, left/right interleaved) are extracted
in one batch and matched by Frame::ComputeStereoMatches (csrc/stereo.hip).
Prints one JSON line: pairs/s of extract(L,R) + stereo matching, the stereo
kernel's own time per step, and the fraction of left keypoints with depth.

Synthetic data: synth.render_frame left views and right views rendered with a
horizontal camera shift (baseline in px), 16 distinct pairs tiled to B.

usage: python tools/bench_stereo.py --config kitti|euroc [--pairs 128] [--steps 10] [--warmup 2]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT / "orb-slam2-annotation_amd", ROOT / "oracle"):
    sys.path.insert(0, str(p))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import orbgpu  # noqa: E402
import synth  # noqa: E402

CONFIGS = {  # width, height, nfeatures, Camera.bf, baseline px of the synthetic right view
    "kitti": (1241, 376, 2000, 0.54 * 718.856, 30.0),   # Examples/Stereo/KITTI00-02.yaml
    "euroc": (752, 480, 1200, 47.90639384423901, 18.0),  # Examples/Stereo/EuRoC.yaml
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="kitti", choices=sorted(CONFIGS))
    ap.add_argument("--pairs", type=int, default=128)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    W, H, NF, BF, BASE = CONFIGS[a.config]
    P = a.pairs
    dev = torch.device("cuda", 0)
    pitch = (W + 15) // 16 * 16
    base = synth.base_texture(0x5E7)
    distinct = 16
    host = np.zeros((2 * distinct, H, pitch), np.uint8)
    for i in range(distinct):
        host[2 * i, :, :W] = synth.render_frame(base, i, W, H, 11)
        host[2 * i + 1, :, :W] = synth.render_frame(base, i, W, H, 12, BASE)
    reps = (P + distinct - 1) // distinct
    imgs = torch.from_numpy(np.concatenate([host] * reps)[: 2 * P]).to(dev).contiguous()
    ex = orbgpu.Extractor(nfeatures=NF, width=W, height=H, max_batch=2 * P)
    cap = ex.max_keypoints
    kps = torch.zeros((2 * P, cap, 7), dtype=torch.float32, device=dev)
    desc = torch.zeros((2 * P, cap, 32), dtype=torch.uint8, device=dev)
    counts = torch.zeros(2 * P, dtype=torch.int32, device=dev)
    ur = torch.zeros((P, cap), dtype=torch.float32, device=dev)
    dp = torch.zeros((P, cap), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step(ev=None):
        ex.extract_batch(imgs, kps, desc, counts, stream=stream)
        if ev is not None:
            ev[0].record(stream)
        orbgpu.stereo_matches_batch(ex, imgs, P, kps, desc, counts, BF, 0.0, ur, dp, stream=stream)
        if ev is not None:
            ev[1].record(stream)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    ex.sync(stream)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(evs[i])
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    ex.sync(stream)
    st_ms = sum(x.elapsed_time(y) for x, y in evs) / a.steps
    n = counts.cpu().numpy()
    urh = ur.cpu().numpy()
    with_depth = float(np.mean([(urh[p, : n[2 * p]] >= 0).mean() for p in range(P)]))
    print(json.dumps({
        "metric": "stereo pairs/s: extract L+R + ComputeStereoMatches", "value": round(P * a.steps / el, 1),
        "unit": "pairs/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(el / a.steps * 1e3, 3), "stereo_kernel_ms_per_step": round(st_ms, 4),
        "stereo_kernel_us_per_pair": round(st_ms * 1e3 / P, 3),
        "keypoints_per_frame": round(float(n.mean()), 1), "left_keypoints_with_depth": round(with_depth, 3),
        "config": {"workload": a.config, "width": W, "height": H, "nfeatures": NF, "pairs_per_step": P,
                   "bf": BF, "synthetic_baseline_px": BASE},
        "data": "synthetic"}))


if __name__ == "__main__":
    main()
