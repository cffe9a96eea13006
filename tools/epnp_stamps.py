"""Phase timeline of the PnP RANSAC kernels from a diagnostic build
(make BUILD=build_stamps LIB=liborbgpu_stamps.so EXTRA=-DEPNP_STAMPS=1).
Run on the GPU box:
  ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_stamps.so python tools/epnp_stamps.py [n] [n_hyp]
Prints the s_memtime deltas (shader clock cycles) between the phase marks of
epnp_wave.h's compute_pose_group for one minimal-set hypothesis (G = 16) and
for the first Refine (G = 64), and pnp_score_kernel's phases."""
import ctypes
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "orb-slam2-annotation_amd")]
import orbgpu  # noqa: E402
import ransac  # noqa: E402
import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
n_hyp = int(sys.argv[2]) if len(sys.argv) > 2 else 300
P = synth.pnp_problem(n, 0.5, seed=7)
rng = np.random.default_rng(1)
samples = np.stack([rng.choice(n, 4, replace=False) for _ in range(n_hyp)]).astype(np.int32)
arr = (ransac.PnPProblem * 1)()
p = arr[0]
p.n, p.offset, p.min_inliers, p.best_inliers, p.n_hyp, p.sample_offset = n, 0, 10, 0, n_hyp, 0
p.fu, p.fv, p.uc, p.vc = P["cam"]
E = (P["sigma2"] * np.float32(5.991)).astype(np.float32)
for _ in range(3):
    bm = np.zeros(n, np.uint8)
    rm = np.zeros(n, np.uint8)
    res = ransac.pnp_ransac_batch(arr, P["P3w"], P["P2"], E, samples, bm, rm)
print("found", res[0].found, "consumed", res[0].consumed, "best", res[0].best_inliers, "refined", res[0].refined_inliers)
L = orbgpu.lib()
L.orbgpu_debug_epnp_stamps.argtypes = [ctypes.c_void_p]
st = np.zeros((3, 32), np.uint64)
assert L.orbgpu_debug_epnp_stamps(st.ctypes.data) == 0
st = st.astype(np.int64)
names = ["start", "control pts", "pinv(CC)", "M^T M", "Jacobi 12x12", "canonical null", "L 6x10",
         "svd_solve 6x4", "gauss-newton 1", "r_and_t 1", "svd_solve 6x3", "gauss-newton 2", "r_and_t 2",
         "svd_solve 6x5", "gauss-newton 3", "r_and_t 3 / end"]
for row, title in ((0, "hypothesis (G=16, n=4)"), (1, "Refine (G=64)")):
    s = st[row]
    print(f"== {title}: total {s[15] - s[0]} cycles, Jacobi sweeps {s[16]}")
    for k in range(1, 16):
        if s[k] and s[k - 1]:
            print(f"  {names[k]:18s} {s[k] - s[k - 1]:8d}")
s = st[2]
print("== pnp_score_kernel (solver 0)")
for k, nm in ((1, "to first best mask"), (2, "inlier list"), (3, "Refine"), (4, "to end")):
    if s[k] and s[k - 1]:
        print(f"  {nm:18s} {s[k] - s[k - 1]:8d}")
print(f"  total {s[4] - s[0]}")
