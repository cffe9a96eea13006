"""Octree pass trace of frame 0 of a 640x480 batch (debug API): per level the
passes, inner-loop flag, list size, children pushed, survivors, nodes still to
expand, sort size bound and key count.  usage: python tools/octree_trace.py"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "orb-slam2-annotation_amd")]
import orbgpu  # noqa: E402
import synth  # noqa: E402

W, H = 640, 480
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
frames = synth.torch_stream(B, W, H, device="cuda", pitch=640, bounded=True)
ex = orbgpu.Extractor(nfeatures=1000, width=W, height=H, max_batch=B)
ex.enable_octree_trace()
cap = ex.max_keypoints
kps = torch.zeros((B, cap, 7), dtype=torch.float32, device="cuda")
desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
ex.extract_batch(frames, kps, desc, cnt, row_step=640, frame_step=640 * H)
torch.cuda.synchronize()
raw = np.zeros(16 * 512, np.int32)
orbgpu._check(orbgpu.lib().orbgpu_debug_octree_trace(ex.h, 0, raw.ctypes.data, raw.size), "octree_trace")
for l, rows in enumerate(ex.octree_trace()):
    print(f"level {l}: {len(rows)} passes (inner, nL, C, S, nexp, kstop, nk, N)")
    for r in rows:
        print("   ", [int(v) for v in r])
    # phase stamps (OCT_STAMPS build): 0 start, 60 cell offsets, 61 key->cell map, 1 keys, 2 roots,
    # 3+4p hist, 4+4p order, 5+4p nodes, 6+4p remap, 63 end
    st = raw[l * 512 + 384: l * 512 + 512].view(np.uint32).astype(np.uint64)
    t = st[0::2] | (st[1::2] << np.uint64(32))
    if t[0]:
        rel = [(k, int(t[k] - t[0])) for k in range(64) if t[k]]
        print("    stamps (index, cycles since start):", rel)
