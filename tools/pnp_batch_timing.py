"""PnP RANSAC batch timing: 16 solvers as Tracking::
Relocalization builds them (one per candidate keyframe), each with n
correspondences and the 300 hypotheses of a first iterate(5) call
(mRansacMaxIts = 300), through orbgpu_pnp_ransac_batch_device on
HBM-resident inputs; HIP events around the launch pair, median of reps.
Run under rocprofv3 --kernel-trace --stats for the per-kernel split.
usage: python tools/pnp_batch_timing.py [batch] [n] [n_hyp] [reps]"""
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "orb-slam2-annotation_amd")]
import orbgpu  # noqa: E402
import ransac  # noqa: E402
import synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
n = int(sys.argv[2]) if len(sys.argv) > 2 else 300
H = int(sys.argv[3]) if len(sys.argv) > 3 else 300
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
torch.cuda.set_device(0)
L = orbgpu.lib()
rng = np.random.default_rng(5)
probs = (ransac.PnPProblem * B)()
P3, P2, E, S = [], [], [], []
for b in range(B):
    P = synth.pnp_problem(n, 0.5, seed=300 + b)
    p = probs[b]
    p.n, p.offset, p.min_inliers, p.best_inliers, p.n_hyp, p.sample_offset = n, b * n, 10, 0, H, b * H
    p.fu, p.fv, p.uc, p.vc = P["cam"]
    P3.append(P["P3w"]); P2.append(P["P2"]); E.append(P["sigma2"] * np.float32(5.991))
    S.append(np.stack([rng.choice(n, 4, replace=False) for _ in range(H)]).astype(np.int32))
dev = lambda a, dt: torch.from_numpy(np.ascontiguousarray(np.concatenate(a), dt)).cuda()
d3, d2, de, ds = dev(P3, np.float32), dev(P2, np.float32), dev(E, np.float32), dev(S, np.int32)
dp = torch.from_numpy(np.frombuffer(bytes(probs), np.uint8).copy()).cuda()
ws = torch.zeros(int(L.orbgpu_pnp_workspace_bytes(B * n, B * H)), dtype=torch.uint8, device="cuda")
res = torch.zeros(B * ctypes.sizeof(ransac.PnPResult), dtype=torch.uint8, device="cuda")
bm = torch.zeros(B * n, dtype=torch.uint8, device="cuda")
rm = torch.zeros(B * n, dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream()
ptr = lambda t: ctypes.c_void_p(t.data_ptr())


def call():
    rc = L.orbgpu_pnp_ransac_batch_device(B, ptr(dp), H, B * n, B * H, ptr(d3), ptr(d2), ptr(de), ptr(ds), ptr(ws),
                                          ptr(res), ptr(bm), ptr(rm), ctypes.c_void_p(s.cuda_stream))
    assert rc == 0, orbgpu.last_error()


for _ in range(3):
    call()
torch.cuda.synchronize()
ts = []
for _ in range(reps):
    a, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    call()
    b_.record(s)
    b_.synchronize()
    ts.append(a.elapsed_time(b_))
rr = (ransac.PnPResult * B).from_buffer_copy(res.cpu().numpy().tobytes())
print(json.dumps({"batch": B, "n": n, "n_hyp": H, "median_ms": round(float(np.median(ts)), 4),
                  "min_ms": round(float(np.min(ts)), 4), "found": sum(r.found for r in rr),
                  "consumed": [r.consumed for r in rr][:8]}))
