"""Phase timeline of one SearchByBoW(KF, F) call (search_by_bow_kernel, block 0)
from a diagnostic build (make BUILD=build_stamps LIB=liborbgpu_stamps.so
EXTRA=-DBOW_STAMPS=1).  Run on the GPU box:
  ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_stamps.so python tools/bow_stamps.py
Scenario: the drop-in table's (1000-feature frames, k=10 L=6 vocabulary,
levelsup 4).  Prints shader-clock cycles since kernel start per phase."""
import ctypes
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "orb-slam2-annotation_amd"), str(ROOT / "oracle")]
import bow  # noqa: E402
import orbgpu  # noqa: E402
import synth  # noqa: E402

par, leaf, vdesc, w = synth.synthetic_vocabulary_fast(10, 6, 7)
voc = bow.Vocabulary.from_arrays(10, 6, 0, 0, par, leaf, vdesc, w)
d1, a1, d2, a2 = synth.bow_frame_pair(vdesc[leaf == 1], 1000, 0.6, seed=41)
fv1, fv2 = voc.transform(d1, 4)[3], voc.transform(d2, 4)[3]
rng = np.random.default_rng(23)
s1 = rng.choice([0, 1, 1, 1, 1, 1, 1, 2], 1000).astype(np.uint8)
lib = orbgpu.lib()
lib.orbgpu_debug_bow_stamps.argtypes = [ctypes.c_void_p]
for rep in range(3):
    nm, _ = bow.search_by_bow(bow.KF_F, fv1, d1, a1, s1 == 1, fv2, d2, a2, np.ones(1000, bool), 0.7, True)
st = np.zeros(32, np.uint64)
assert lib.orbgpu_debug_bow_stamps(st.ctypes.data) == 0
st = st.astype(np.int64)
t0 = st[0]
names = {1: "staged (descriptors, lists, flags, angles)", 2: "common nodes", 3: "node walk done (block)",
         30: "end"}
print("matches", nm)
for k in (1, 2, 3, 30):
    print(f"  {names[k]:45s} {st[k] - t0:8d}")
walk = st[8:24] - t0
print("  waves' walk ends:", walk[walk > 0].tolist())
