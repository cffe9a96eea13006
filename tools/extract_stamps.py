"""Per-wave phase cycles of the FAST and describe kernels from a diagnostic
build (make BUILD=build_xs LIB=liborbgpu_xs.so EXTRA="-DFAST_STAMPS
-DDESC_STAMPS"): a 512-frame 640x480 batch extracted a few times, sampled
waves' phase durations (s_memtime, shader clock) averaged.  Run on the GPU box:
  ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_xs.so python tools/extract_stamps.py"""
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "orb-slam2-annotation_amd")]
import orbgpu  # noqa: E402
import synth  # noqa: E402

W, H, B = 640, 480, int(sys.argv[1]) if len(sys.argv) > 1 else 512
frames = synth.torch_stream(B, W, H, device="cuda", pitch=640, bounded=True)
ex = orbgpu.Extractor(nfeatures=1000, width=W, height=H, max_batch=B)
cap = ex.max_keypoints
kps = torch.zeros((B, cap, 7), dtype=torch.float32, device="cuda")
desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
lib = orbgpu.lib()
out = {}
for name in ("fast", "desc"):
    fn = getattr(lib, f"orbgpu_debug_{name}_stamps")
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
for it in range(4):
    for name in ("fast", "desc"):
        st = np.zeros(16, np.uint64)
        getattr(lib, f"orbgpu_debug_{name}_stamps")(st.ctypes.data, 1)
    ex.extract_batch(frames, kps, desc, cnt, row_step=640, frame_step=640 * H)
    torch.cuda.synchronize()
st = np.zeros(16, np.uint64)
lib.orbgpu_debug_fast_stamps(st.ctypes.data, 0)
n = max(int(st[15]), 1)
out["fast"] = {"sampled_waves": n, "staging_cycles": float(st[5]) / n,
               "compass_t20_cycles": float(st[6]) / n, "arc_t20_cycles": float(st[1] - st[6]) / n,
               "nms_t20_cycles": float(st[2]) / n, "retry_t7_cycles": float(st[3]) / n,
               "entry_to_staged_cycles": float(st[0]) / n, "empty_window_cycles": float(st[4]) / n,
               "survivors_t20": float(st[8]) / n, "corners_t20": float(st[9]) / n, "retry_frac": float(st[10]) / n}
st = np.zeros(16, np.uint64)
lib.orbgpu_debug_desc_stamps(st.ctypes.data, 0)
n = max(int(st[15]), 1)
out["describe"] = {"sampled_waves": n, "key_ref_cycles": float(st[0]) / n,
                   "stage_moments_blur_cycles": float(st[1]) / n, "orientation_cycles": float(st[2]) / n,
                   "tests_store_cycles": float(st[3]) / n,
                   "raw_phase_means": [round(float(st[k]) / n, 1) for k in range(8)]}
print(json.dumps(out, indent=1))
