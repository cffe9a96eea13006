"""Timing of the MapPoint batch updates (csrc/mappoint.hip): 20,000 points,
up to 40 observations each (mean ~20), device-resident inputs; ms per batch
from HIP events, plus the scalar oracle's time for 500 of the points."""
import json, sys, time
sys.path.insert(0, "orb-slam2-annotation_amd")
sys.path.insert(0, "oracle")
import ctypes
import numpy as np
import torch
import orbgpu, mappoint, synth, mappoint_ref

dev = torch.device("cuda:0")
NP = 20000
sc = synth.mappoint_scenario(NP, 11, max_obs=40)
t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dt)).to(dev)
off, desc, valid = t(sc["offsets"], np.int32), t(sc["desc"], np.uint8), t(sc["valid"], np.uint8)
best = torch.zeros(NP, dtype=torch.int32, device=dev)
med = torch.zeros(NP, dtype=torch.int32, device=dev)
L = orbgpu.lib()
vp = ctypes.c_void_p
L.orbgpu_compute_distinctive_descriptors_batch_device.argtypes = [ctypes.c_int, vp, vp, vp, vp, vp, vp]
L.orbgpu_update_normal_and_depth_batch_device.argtypes = [vp, vp]
s = torch.cuda.current_stream().cuda_stream
obs_Ow, pos, ref_Ow = t(sc["obs_Ow"], np.float32), t(sc["pos"], np.float32), t(sc["ref_Ow"], np.float32)
ls, ms = t(sc["level_scale"], np.float32), t(sc["max_scale"], np.float32)
nrm = torch.zeros((NP, 3), dtype=torch.float32, device=dev)
dmin = torch.zeros(NP, dtype=torch.float32, device=dev)
dmax = torch.zeros(NP, dtype=torch.float32, device=dev)
B = mappoint.NormalDepthBatch(NP, off.data_ptr(), obs_Ow.data_ptr(), pos.data_ptr(), ref_Ow.data_ptr(), ls.data_ptr(),
                              ms.data_ptr(), nrm.data_ptr(), dmin.data_ptr(), dmax.data_ptr())


def dd():
    orbgpu._check(L.orbgpu_compute_distinctive_descriptors_batch_device(NP, off.data_ptr(), desc.data_ptr(),
                                                                        valid.data_ptr(), best.data_ptr(),
                                                                        med.data_ptr(), s), "dd")


def nd():
    orbgpu._check(L.orbgpu_update_normal_and_depth_batch_device(ctypes.byref(B), s), "nd")


res = {"points": NP, "observations": int(sc["offsets"][-1])}
for name, fn in (("distinctive_ms", dd), ("normal_depth_ms", nd)):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    res[name] = e0.elapsed_time(e1) / 20
o = sc["offsets"]
t0 = time.perf_counter()
for p in range(500):
    mappoint_ref.compute_distinctive_descriptors(sc["desc"][o[p]:o[p + 1]], sc["valid"][o[p]:o[p + 1]])
res["oracle_distinctive_ms_per_point_1thread"] = (time.perf_counter() - t0) / 500 * 1e3
gb = best.cpu().numpy()
res["check_first_500"] = bool(all(gb[p] == mappoint_ref.compute_distinctive_descriptors(
    sc["desc"][o[p]:o[p + 1]], sc["valid"][o[p]:o[p + 1]])[0] for p in range(0, 500, 25)))
print(json.dumps(res))
