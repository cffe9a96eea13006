"""orbgpu_extract (the drop-in single-frame path) latency: median of 200 calls."""
import sys, time
sys.path.insert(0, "orb-slam2-annotation_amd")
import numpy as np
import orbgpu, synth

img = synth.mono_stream(1, 640, 480, seed=3)[0]
ex = orbgpu.Extractor(nfeatures=1000, width=640, height=480, max_batch=1)
for _ in range(20):
    ex.extract(img)
ts = []
for _ in range(200):
    t0 = time.perf_counter()
    ex.extract(img)
    ts.append(time.perf_counter() - t0)
print(f"median {np.median(ts) * 1e3:.4f} ms  p10 {np.percentile(ts, 10) * 1e3:.4f}", flush=True)
