"""Diagnostic: per-block phase shares of pyramid_kernel from a stamp build
(tools/pyr_variants.sh stamps:-DPYR_PROBE=8).  Run on the GPU box with
ORBGPU_LIBRARY pointing at that build.  Reads only the stamp buffer."""
import ctypes
import os
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
for _ in range(3):
    ex.extract_batch(frames, kps, desc, counts, stream=stream, row_step=pitch, frame_step=pitch * H)
torch.cuda.synchronize()
L = orbgpu.lib()
fn = L.orbgpu_debug_pyr_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
nb = int(os.environ.get("NBLOCKS", "4608"))
st = np.zeros((nb, 10), np.uint64)
assert fn(st.ctypes.data, nb) == 0
st = st.astype(np.int64)
d = np.diff(st[:, :9], axis=1)
names = ["stage+rec"] + [f"level {l}" for l in range(1, 8)]
tot = st[:, 8] - st[:, 0]
print(f"blocks {nb}: block lifetime mean {tot.mean():.0f} cyc  p10 {np.percentile(tot,10):.0f}  p90 {np.percentile(tot,90):.0f}")
for i, n in enumerate(names):
    print(f"  {n:10s} mean {d[:, i].mean():8.0f} cyc  share {100 * d[:, i].mean() / tot.mean():5.1f} %  p90 {np.percentile(d[:, i], 90):8.0f}")
fw = L.orbgpu_debug_pyr_waves
fw.argtypes = [ctypes.c_void_p, ctypes.c_int]
wv = np.zeros((nb, 8, 16), np.uint64)
assert fw(wv.ctypes.data, nb) == 0
wv = wv.astype(np.int64)
for lv in range(1, 8):
    rel = wv[:, lv, :] - st[:, lv][:, None]
    print(f"level {lv} wave done (cyc after level start), mean per wave:", " ".join(f"{x:.0f}" for x in rel.mean(0)))
