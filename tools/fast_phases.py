"""Diagnostic: FAST cell-kernel phase cycle totals from a FAST_PROBE build
(FILES=fast.hip tools/pyr_variants.sh fastp:-DFAST_PROBE=1)."""
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "orb-slam2-annotation_amd"))
import orbgpu  # noqa: E402
import synth  # noqa: E402

W, H, B = 640, 480, 512
dev = torch.device("cuda", 0)
pitch = (W + 15) // 16 * 16
ex = orbgpu.Extractor(nfeatures=1000, width=W, height=H, max_batch=B)
cap = ex.max_keypoints
frames = synth.torch_stream(B, W, H, seed=7, device=dev, pitch=pitch)
kps = torch.zeros((B, cap, 7), dtype=torch.float32, device=dev)
desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
counts = torch.zeros(B, dtype=torch.int32, device=dev)
stream = torch.cuda.current_stream(dev)
ex.extract_batch(frames, kps, desc, counts, stream=stream, row_step=pitch, frame_step=pitch * H)
torch.cuda.synchronize()
fn = orbgpu.lib().orbgpu_debug_fast_phases
fn.argtypes = [ctypes.c_void_p]
ph = np.zeros(16, np.uint64)
assert fn(ph.ctypes.data) == 0
n, nr = int(ph[4]), int(ph[6])
print(f"cells {n}, retried {nr} ({100 * nr / max(n, 1):.1f} %)")
for i, name in enumerate(["stage window", "zero score tile", "corners t=20", "nms+emit t=20"]):
    print(f"  {name:16s} {ph[i] / max(n, 1):8.0f} cyc/cell")
print(f"  {'retry t=7':16s} {ph[5] / max(nr, 1):8.0f} cyc/retried cell")
if ph[8]:
    c = ph[8]
    print(f"fast_corners calls {c}: per call compass iters {ph[9]/c:.1f}, contig batches {ph[10]/c:.2f}, "
          f"arc batches {ph[11]/c:.2f}, survivors {ph[12]/c:.1f}, corners {ph[13]/c:.1f}, pixels {ph[14]/c:.1f}")
