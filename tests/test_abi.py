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


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure path")
def test_device_placement_validation_without_device():
    """ordinals are validated before any device is touched
    (negative -> ORBGPU_ERR_ARG), and without a device every placement call
    fails loudly (ORBGPU_ERR_NO_DEVICE); the count is 0."""
    import orbgpu
    L = orbgpu.lib()
    assert orbgpu.device_count() == 0
    assert L.orbgpu_set_thread_device(-1) == orbgpu.ERR_ARG
    assert "ordinal" in orbgpu.last_error()
    assert L.orbgpu_set_thread_device(0) == orbgpu.ERR_NO_DEVICE
    h = ctypes.c_void_p(12345)
    assert L.orbgpu_extractor_create_on_device(-2, 1000, 1.2, 8, 20, 7, 640, 480, 1, ctypes.byref(h)) == orbgpu.ERR_ARG
    assert h.value is None  # *out cleared on failure
    assert L.orbgpu_extractor_create_on_device(0, 1000, 1.2, 8, 20, 7, 640, 480, 1,
                                               ctypes.byref(h)) == orbgpu.ERR_NO_DEVICE
    d = ctypes.c_int(7)
    assert L.orbgpu_get_thread_device(ctypes.byref(d)) == orbgpu.ERR_NO_DEVICE and d.value == -1
    with pytest.raises(orbgpu.OrbGpuError):
        orbgpu.Extractor(device=0)


@pytest.mark.gpu
def test_device_placement_on_gpu():
    """An extractor placed on device 0 reports it, works from a thread whose
    current device was never set, and equals the oracle; ordinals outside the
    visible devices are refused; the thread device round-trips."""
    import threading
    import orbgpu
    import orbref
    import synth
    n = orbgpu.device_count()
    assert n >= 1
    orbgpu.set_thread_device(0)
    assert orbgpu.get_thread_device() == 0
    with pytest.raises(orbgpu.OrbGpuError) as e:
        orbgpu.set_thread_device(n)
    assert e.value.code == orbgpu.ERR_ARG
    with pytest.raises(orbgpu.OrbGpuError) as e:
        orbgpu.Extractor(device=n)
    assert e.value.code == orbgpu.ERR_ARG
    ex = orbgpu.Extractor(device=0)
    assert ex.device == 0
    img = synth.mono_stream(1)[0]
    out = {}
    t = threading.Thread(target=lambda: out.update(r=ex.extract(img)))
    t.start()
    t.join()
    kr, dr = orbref.Extractor().extract(img)
    kg, dg = out["r"]
    assert kg.tobytes() == kr.tobytes() and np.array_equal(dg, dr)


def test_abi_version_matches_header():
    """ORBGPU_ABI_VERSION of include/orbgpu.h equals what the loaded library
    reports (no device needed): a host built against another header can tell."""
    import re
    import orbgpu
    hdr = (Path(__file__).resolve().parents[1] / "include" / "orbgpu.h").read_text()
    v = int(re.search(r"#define ORBGPU_ABI_VERSION (\d+)", hdr).group(1))
    assert orbgpu.lib().orbgpu_abi_version() == v


@pytest.mark.gpu
def test_get_info_sized_writes_no_more_than_the_callers_struct():
    """A caller built against the round-4 header (orbgpu_extractor_info
    without the trailing `device`) passes its own size: the library fills
    its fields and leaves the bytes past them untouched."""
    import orbgpu
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ex = orbgpu.Extractor()
    L = orbgpu.lib()
    full = ctypes.sizeof(orbgpu._Info)
    old = full - 4  # the struct before the device field
    buf = (ctypes.c_uint8 * (full + 16))(*([0xAB] * (full + 16)))
    assert L.orbgpu_extractor_get_info_sized(ex.h, ctypes.cast(buf, ctypes.c_void_p),
                                             ctypes.c_size_t(old)) == 0
    raw = bytes(buf)
    assert raw[old:] == b"\xAB" * (full + 16 - old)
    info = orbgpu._Info.from_buffer_copy(raw[:old] + b"\0" * 4)
    assert (info.nlevels, info.width, info.height) == (8, 640, 480)
    assert L.orbgpu_extractor_get_info_sized(ex.h, ctypes.cast(buf, ctypes.c_void_p),
                                             ctypes.c_size_t(0)) == orbgpu.ERR_ARG


@pytest.mark.gpu
def test_device_event_orders_two_streams():
    """orbgpu.DeviceEvent (orbgpu_device_event_*: no system-scope fence) orders
    a second stream behind a batch extraction on the first: the counts the
    second stream copies after waiting on the event are the extraction's, and
    the extractor's stage hook takes the event too."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import orbgpu
    import synth
    B = 16
    frames = torch.from_numpy(np.ascontiguousarray(synth.mono_stream(B, 640, 480, seed=77))).cuda()
    ex = orbgpu.Extractor(max_batch=B)
    cap = ex.max_keypoints
    kps = torch.zeros((B, cap, 7), dtype=torch.float32, device="cuda")
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(B, dtype=torch.int32, device="cuda")
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    ev, ev_fast = orbgpu.DeviceEvent(), orbgpu.DeviceEvent()
    ex.set_stage_event("fast_cells", ev_fast)
    out = torch.full((B,), -1, dtype=torch.int32, device="cuda")
    ref = []
    for rep in range(3):
        torch.cuda.synchronize()
        counts.fill_(-5)
        torch.cuda.synchronize()
        ex.extract_batch(frames, kps, desc, counts, stream=a)
        ev.record(a)
        b.wait_event(ev)  # torch streams call event.wait(stream)
        with torch.cuda.stream(b):
            out.copy_(counts)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        assert (got > 0).all(), got
        if rep == 0:
            ref = got.copy()
        assert (got == ref).all()
    ex.set_stage_event("fast_cells", None)
