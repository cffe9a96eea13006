"""The C-ABI library loads and exports every function the public headers
declare; without a gfx950 device it fails loudly (no CPU fallback)."""
import ctypes
import re
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parent.parent
HEADERS = sorted((ROOT / "include").glob("orbgpu*.h"))


def declared_functions():
    names = []
    for h in HEADERS:
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        names += re.findall(r"\b(orbgpu_\w+)\s*\(", text)
    return sorted(set(names))


def test_library_exports_every_declared_symbol():
    import orbgpu
    lib = orbgpu.lib()
    names = declared_functions()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_keypoint_struct_matches_cv_keypoint_layout():
    import orbgpu
    assert orbgpu.KP_DTYPE.itemsize == 28
    assert [orbgpu.KP_DTYPE.fields[f][1] for f in ("x", "y", "size", "angle", "response", "octave", "class_id")] == \
        [0, 4, 8, 12, 16, 20, 24]


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure path")
def test_no_device_fails_loudly():
    import orbgpu
    with pytest.raises(orbgpu.OrbGpuError) as e:
        orbgpu.Extractor()
    assert e.value.code in (orbgpu.ERR_NO_DEVICE, orbgpu.ERR_HIP)
    with pytest.raises(orbgpu.OrbGpuError):
        orbgpu.search_for_initialization(np.zeros(0, orbgpu.KP_DTYPE), np.zeros((0, 32), np.uint8),
                                         np.zeros(0, orbgpu.KP_DTYPE), np.zeros((0, 32), np.uint8), 640, 480)
