"""Extraction alone (no matcher beside it): a 512-frame 640x480 batch
extracted N times back to back on one stream -- for per-kernel durations under
rocprofv3 --kernel-trace --stats without the bench's concurrent matcher.
  ORBGPU_LIBRARY=... python tools/extract_iso.py [B] [N]"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "orb-slam2-annotation_amd")]
import orbgpu  # noqa: E402
import synth  # noqa: E402

W, H = 640, 480
B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
frames = synth.torch_stream(B, W, H, device="cuda", pitch=640, bounded=True)
ex = orbgpu.Extractor(nfeatures=1000, width=W, height=H, max_batch=B)
cap = ex.max_keypoints
kps = torch.zeros((B, cap, 7), dtype=torch.float32, device="cuda")
desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
for _ in range(N):
    ex.extract_batch(frames, kps, desc, cnt, row_step=640, frame_step=640 * H)
torch.cuda.synchronize()
print("done", int(cnt.sum()))
