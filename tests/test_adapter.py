"""The header-only C++ drop-in (include/orbslam2_amd/ORBextractor.h,
ORBmatcher.h) used the way ORB-SLAM2's Frame / Initializer use the
reference classes, driven by tests/cpp/adapter_main.cpp."""
import struct
import subprocess
from pathlib import Path

import numpy as np
import pytest
import torch

import orbref
import synth

ROOT = Path(__file__).resolve().parent.parent
CPP = ROOT / "tests" / "cpp"
EXE = CPP / "adapter_main"


@pytest.fixture(scope="module")
def exe():
    subprocess.run(["make", "-s", "-C", str(CPP)], check=True)
    return str(EXE)


@pytest.mark.parametrize("nf,scale,nl", [(1000, 1.2, 8), (2000, 1.2, 8), (500, 1.5, 5)])
def test_adapter_scale_tables_match_oracle(exe, nf, scale, nl):
    """GetScaleFactors & co. (ORBextractor.cpp:419-434) before any frame."""
    out = subprocess.run([exe, "scales", str(nf), str(scale), str(nl)], check=True, capture_output=True,
                         text=True).stdout.split("\n")
    levels, sf = out[0].split()
    assert int(levels) == nl and np.float32(float(sf)) == np.float32(scale)
    got = np.array([[float.fromhex(v) for v in line.split()] for line in out[1:1 + nl]], np.float32)
    ex = orbref.Extractor(nfeatures=nf, scale_factor=scale, nlevels=nl)
    ref = np.stack(ex.scale_factors(), 1).astype(np.float32)
    np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_adapter_empty_image_returns_untouched(exe):
    """ORBextractor.cpp:1056: `if(_image.empty()) return;` -- no device needed."""
    r = subprocess.run([exe, "empty"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure path")
def test_adapter_without_device_throws(exe):
    r = subprocess.run([exe, "nodevice"], capture_output=True, text=True)
    assert r.returncode == 0 and "threw" in r.stdout, r.stdout + r.stderr


def _read_frame(buf, off):
    n, = struct.unpack_from("<i", buf, off)
    off += 4
    kps = np.frombuffer(buf, orbref.KP_DTYPE, n, off)
    off += 28 * n
    desc = np.frombuffer(buf, np.uint8, 32 * n, off).reshape(n, 32)
    return kps, desc, off + 32 * n


@pytest.mark.gpu
def test_adapter_extract_and_match_vs_oracle(exe, tmp_path):
    w, h, nf = 640, 480, 1000
    frames = synth.mono_stream(2, w, h, seed=0x0B5E)
    for i, f in enumerate(frames):
        (tmp_path / f"f{i}.raw").write_bytes(f.tobytes())
    out = tmp_path / "out.bin"
    r = subprocess.run([exe, "extract", str(w), str(h), str(nf), str(tmp_path / "f0.raw"),
                        str(tmp_path / "f1.raw"), str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    buf = out.read_bytes()
    k0, d0, off = _read_frame(buf, 0)
    k1, d1, off = _read_frame(buf, off)
    nm, = struct.unpack_from("<i", buf, off)
    m12 = np.frombuffer(buf, np.int32, len(k0), off + 4)
    off += 4 + 4 * len(k0)
    lw, lh = struct.unpack_from("<ii", buf, off)
    lvl1 = np.frombuffer(buf, np.uint8, lw * lh, off + 8).reshape(lh, lw)

    ex = orbref.Extractor(nfeatures=nf)
    kr0, dr0 = ex.extract(frames[0])
    kr1, dr1 = ex.extract(frames[1])
    assert k0.tobytes() == kr0.tobytes() and np.array_equal(d0, dr0)
    assert k1.tobytes() == kr1.tobytes() and np.array_equal(d1, dr1)
    np.testing.assert_array_equal(lvl1, ex.level(1))
    n_r, m_r, _ = orbref.search_for_initialization(kr0, dr0, kr1, dr1, w, h)
    assert nm == n_r
    np.testing.assert_array_equal(m12, m_r)
