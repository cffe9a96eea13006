"""Cost model of the fused pyramid plan (no GPU): per tick, each compute
wave's work is its busiest lane's rows (a tail wave's rows weighted by
TAIL_W); a tick lasts its slowest wave.  Prints the plan's useful lane-rows,
the executed wave-rows, the sum over ticks of the slowest wave, and the
per-wave mean rows per tick.  usage: pyr_plan_cost.py [W H NFEAT]"""
import ctypes
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "orb-slam2-annotation_amd"))
import orbgpu  # noqa: E402

W, H, NF = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (640, 480, 1000)
TAIL_W = 1.5
lib = orbgpu.lib()
f = lib.orbgpu_debug_pyramid_plan_rows
f.argtypes = [ctypes.c_int, ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
              ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
dims = np.zeros(4, np.int32)
assert f(NF, 1.2, 8, W, H, None, 0, None, 0, dims.ctypes.data) == 0
K, n, cw, E = (int(x) for x in dims)
rows = np.zeros(K * n, np.int32)
info = np.zeros(n, np.int32)
assert f(NF, 1.2, 8, W, H, rows.ctypes.data, rows.size, info.ctypes.data, info.size, dims.ctypes.data) == 0
rows = rows.reshape(K, n).astype(float)
lvl, tail = info & 0xFF, (info >> 8) & 1
rows[:, lvl == 0] = 0
w = np.where(tail == 1, TAIL_W, 1.0)
cost = rows * w
CL = n // E
per_lane = cost[:, :CL] + (cost[:, CL:] if E > 1 else 0)
waves = per_lane.reshape(K, CL // 64, 64).max(2)
print(f"{W}x{H}: ticks {K}, compute waves {cw}, entries/lane {E}")
print(f"useful lane-rows {cost.sum():.0f}, executed wave-rows x64 {waves.sum() * 64:.0f} "
      f"(efficiency {cost.sum() / (waves.sum() * 64):.3f})")
print(f"sum over ticks of the slowest wave {waves.max(1).sum():.0f} rows; mean wave {waves.mean(1).sum():.0f}; "
      f"balance {waves.mean(1).sum() / waves.max(1).sum():.3f}")
print("per wave mean rows per tick:", np.round(waves.mean(0), 2).tolist())
print("levels per wave:", [sorted(set(lvl[64 * i:64 * i + 64].tolist())) for i in range(CL // 64)])
# per level: its lanes' rows per tick (max over the level's lanes) and lane count
for l in range(1, 8):
    m = (lvl == l) & (tail == 0)
    if m.any():
        r = rows[:, m].max(1)
        print(f"level {l}: lanes {m.sum():3d}  rows/tick max {r.max():.0f} mean {r.mean():.2f}  ticks>0 {int((r > 0).sum())}")
mt = tail == 1
if mt.any():
    r = rows[:, mt].max(1)
    print(f"tail : lanes {mt.sum():3d}  rows/tick max {r.max():.0f} mean {r.mean():.2f}")
