"""Per-tick timeline of pyramid_tick_kernel from a diagnostic build
(make BUILD=build_stamps LIB=liborbgpu_stamps.so EXTRA=-DPYR_STAMPS=1).
Run on the GPU box:  ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_stamps.so python tools/pyr_ticks.py
Prints, for blocks 0..63 of a 512-frame batch: block span, compute time per
tick of wave 0, its barrier wait, the producer's wait for its chunk."""
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "orb-slam2-annotation_amd")]
import orbgpu  # noqa: E402
import synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
W, H = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (640, 480)
torch.cuda.set_device(0)
frames = synth.torch_stream(B, W, H, bounded=True)
ex = orbgpu.Extractor(width=W, height=H, max_batch=B, nfeatures=1000 if W == 640 else 2000)
cap = ex.max_keypoints
kps = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
counts = torch.zeros(B, dtype=torch.int32, device="cuda")
for _ in range(3):
    ex.extract_batch(frames, kps, desc, counts)
torch.cuda.synchronize()
lib = orbgpu.lib()
st = np.zeros(64 * 160 * 16, np.uint64)
bl = np.zeros(1024 * 6, np.uint64)
lib.orbgpu_debug_pyr_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
assert lib.orbgpu_debug_pyr_stamps(st.ctypes.data, bl.ctypes.data) == 0
bl = bl.reshape(1024, 6)[:B].astype(np.int64)
rt0 = bl[:, 0].min()
life_us = (bl[:, 1] - bl[:, 0]) / 100.0
print("block lifetime us: mean %.1f min %.1f max %.1f; kernel span (first start..last end) %.1f us" %
      (life_us.mean(), life_us.min(), life_us.max(), (bl[:, 1].max() - rt0) / 100.0))
clk = (bl[:, 3] - bl[:, 2]) / np.maximum(1, bl[:, 1] - bl[:, 0]) * 100.0
print("in-kernel clock MHz: median %.0f" % np.median(clk))
starts = np.sort((bl[:, 0] - rt0) / 100.0)
print("block start times us (every 32nd):", [round(x, 1) for x in starts[::32]])
cu = (bl[:, 5] & 0xF) * 1000 + ((bl[:, 4] >> 13) & 0x7) * 100 + ((bl[:, 4] >> 8) & 0xF) + ((bl[:, 4] >> 12) & 1) * 16
u, c = np.unique(cu, return_counts=True)
print("distinct CUs used:", len(u), "blocks per CU histogram:", np.bincount(c).tolist())
st = st.reshape(64, 160, 16).astype(np.int64)
_, info = orbgpu.pyramid_plan_emulate(np.zeros((H, W), np.uint8), 1000, 1.2, 8)
K = info["ticks"]
nw = info["compute_waves"]
print("plan", info)
start = st[:, :K, 15]
span = st[:, K - 1, :nw].max(1) - st[:, 0, 15]
print("block span cycles: mean %.0f min %d max %d" % (span.mean(), span.min(), span.max()))
done = st[:, :K, :nw] - start[:, :, None]  # each compute wave's finish, relative to wave 0's tick start
prod = st[:, :K, 14] - start
print("per compute wave: mean finish within the tick (cycles), over ticks 4..K-8")
for w in range(nw):
    print(f"  wave {w:2d}: {done[:, 4:K - 8, w].mean():7.0f}  (max {done[:, 4:K - 8, w].max():6d})")
print(f"  producer ready: {prod[:, 4:K - 8].mean():7.0f}")
tick = st[:, 1:K, 15] - st[:, :K - 1, 15]
print("tick length mean %.0f" % tick[:, 4:K - 8].mean())
# per-XCD block lifetime and clock (all blocks of the batch)
xcc = bl[:, 5] & 0xF
for x in np.unique(xcc):
    m = xcc == x
    print("xcc %d: blocks %3d lifetime us mean %.1f min %.1f max %.1f  clock MHz mean %.0f min %.0f max %.0f" %
          (x, m.sum(), life_us[m].mean(), life_us[m].min(), life_us[m].max(), clk[m].mean(), clk[m].min(), clk[m].max()))
cyc = bl[:, 3] - bl[:, 2]
print("block cycles (all blocks): mean %.0f min %d max %d" % (cyc.mean(), cyc.min(), cyc.max()))
