"""Extraction throughput of one 512-frame step split over S extractors on S
streams (S = 1, 2, 4): do kernels of different stages overlapping on the
chip (a FAST pass beside an octree pass, ...) raise throughput?
usage: python tools/split_stream_probe.py [steps]"""
import json
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "orb-slam2-annotation_amd")]
import orbgpu  # noqa: E402
import synth  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
W, H, B = 640, 480, 512
torch.cuda.set_device(0)
pitch = 640
frames = synth.torch_stream(B, W, H, device="cuda", pitch=pitch, bounded=True)
out = {}
for S in (1, 2, 4):
    b = B // S
    exs = [orbgpu.Extractor(nfeatures=1000, width=W, height=H, max_batch=b) for _ in range(S)]
    sts = [torch.cuda.Stream() for _ in range(S)]
    cap = exs[0].max_keypoints
    kps = torch.zeros((B, cap, 7), dtype=torch.float32, device="cuda")
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(B, dtype=torch.int32, device="cuda")

    def step():
        for k in range(S):
            exs[k].extract_batch(frames[k * b:(k + 1) * b], kps[k * b:(k + 1) * b], desc[k * b:(k + 1) * b],
                                 counts[k * b:(k + 1) * b], stream=sts[k], row_step=pitch, frame_step=pitch * H)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    out[f"streams_{S}"] = {"ms_per_step": round(dt * 1e3, 4), "frames_per_s": round(B / dt, 1)}
    del exs
print(json.dumps(out))
