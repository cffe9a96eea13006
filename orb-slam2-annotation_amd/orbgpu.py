"""Python binding of liborbgpu.so (the MI355X ORB front-end) via ctypes.

This is a thin host-side mirror of the reference's class surface for tests
and the benchmark:

* ``Extractor``  ~ ORB_SLAM2::ORBextractor  (ORBextractor.h:47-111):
  ``extract(img)`` is ``operator()`` for one host image; ``extract_batch``
  runs B HBM-resident frames in one launch sequence.
* ``search_for_initialization`` / ``search_for_initialization_batch`` ~
  ORBmatcher::SearchForInitialization (ORBmatcher.cpp:474-590).

No CPU fallback exists: if the shared library is missing, or the process has
no gfx950 device, every call raises.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
# ORBGPU_LIBRARY selects another build of the same library (e.g. a tuning variant)
LIB_PATH = Path(os.environ.get("ORBGPU_LIBRARY", str(_HERE / "liborbgpu.so")))
_LIB = None

OK, ERR_ARG, ERR_HIP, ERR_CAPACITY, ERR_UNSUPPORTED, ERR_NO_DEVICE = 0, -1, -2, -3, -4, -5
MATCH_CHECK_ORI = 1
MATCH_ANNOTATED_HISTO = 2

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])


class OrbGpuError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"{what} failed ({code}): {last_error()}")
        self.code = code


class GridBounds(ctypes.Structure):
    """Frame::mnMinX, mnMaxX, mnMinY, mnMaxY (Frame.cpp:505-530)."""
    _fields_ = [("min_x", ctypes.c_float), ("max_x", ctypes.c_float),
                ("min_y", ctypes.c_float), ("max_y", ctypes.c_float)]


class PackDesc(ctypes.Structure):
    """orbgpu_pack_desc (include/orbgpu.h)"""
    _fields_ = [("rows", ctypes.c_void_p), ("packed", ctypes.c_void_p), ("counts", ctypes.c_void_p),
                ("row_bytes", ctypes.c_int)]


class Camera(ctypes.Structure):
    """orbgpu_camera: mK (fx, fy, cx, cy) and mDistCoef (k1, k2, p1, p2[, k3])."""
    _fields_ = [("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float),
                ("dist", ctypes.c_float * 5), ("ndist", ctypes.c_int)]

    @classmethod
    def make(cls, fx, fy, cx, cy, dist):
        c = cls(fx, fy, cx, cy)
        for i, v in enumerate(dist):
            c.dist[i] = v
        c.ndist = len(dist)
        return c


GRID_COLS, GRID_ROWS = 64, 48


def bounds_for(img_w, img_h) -> GridBounds:
    """Grid bounds of an undistorted frame: [0, cols] x [0, rows]."""
    return GridBounds(0.0, float(img_w), 0.0, float(img_h))


class _Info(ctypes.Structure):
    _fields_ = [("nlevels", ctypes.c_int), ("width", ctypes.c_int), ("height", ctypes.c_int),
                ("max_batch", ctypes.c_int), ("max_keypoints", ctypes.c_int),
                ("level_width", ctypes.c_int * 32), ("level_height", ctypes.c_int * 32),
                ("features_per_level", ctypes.c_int * 32), ("level_capacity", ctypes.c_int * 32),
                ("device", ctypes.c_int)]


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            raise RuntimeError(f"HIP extension not built: {LIB_PATH} (run __graft_entry__.build())")
        # One HIP runtime per process: when PyTorch is present, load the
        # libamdhip64 it ships first, so liborbgpu's dependency resolves to the
        # same runtime (a second runtime loaded before it cannot see the device
        # once torch has opened it).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(str(LIB_PATH))
        vp, i, f, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
        L.orbgpu_last_error.restype = ctypes.c_char_p
        L.orbgpu_device_arch.argtypes = [ctypes.c_char_p, i]
        L.orbgpu_extractor_create.argtypes = [i, f, i, i, i, i, i, i, ctypes.POINTER(vp)]
        L.orbgpu_extractor_create_on_device.argtypes = [i, i, f, i, i, i, i, i, i, ctypes.POINTER(vp)]
        L.orbgpu_extractor_destroy.argtypes = [vp]
        L.orbgpu_device_event_create.argtypes = [ctypes.POINTER(vp)]
        L.orbgpu_device_event_destroy.argtypes = [vp]
        L.orbgpu_device_event_record.argtypes = [vp, vp]
        L.orbgpu_stream_wait_device_event.argtypes = [vp, vp]
        L.orbgpu_device_count.argtypes = [ctypes.POINTER(i)]
        L.orbgpu_set_thread_device.argtypes = [i]
        L.orbgpu_get_thread_device.argtypes = [ctypes.POINTER(i)]
        L.orbgpu_extractor_get_info.argtypes = [vp, ctypes.POINTER(_Info)]
        L.orbgpu_extractor_get_scales.argtypes = [vp, vp, vp, vp, vp]
        L.orbgpu_extract.argtypes = [vp, vp, i, i, sz, vp, vp, i, ctypes.POINTER(i)]
        L.orbgpu_extract_batch_device.argtypes = [vp, vp, i, sz, sz, vp, vp, vp, i, vp]
        L.orbgpu_extractor_sync.argtypes = [vp, vp]
        L.orbgpu_extractor_profile.argtypes = [vp, i]
        L.orbgpu_extractor_stage_times.argtypes = [vp, vp, ctypes.POINTER(i), i]
        L.orbgpu_extractor_set_stage_event.argtypes = [vp, i, vp]
        L.orbgpu_extractor_copy_level.argtypes = [vp, i, i, vp, sz]
        L.orbgpu_hamming_pairs_device.argtypes = [vp, vp, i, vp, vp]
        L.orbgpu_pack_rows_device.argtypes = [i, i, i, ctypes.POINTER(PackDesc), vp]
        L.orbgpu_search_for_initialization_batch_device.argtypes = [
            i, GridBounds, vp, vp, vp, sz, vp, vp, vp, sz, vp, i, f, i, vp, vp, vp]
        L.orbgpu_search_for_initialization_batch_device_bounded.argtypes = [
            i, GridBounds, vp, vp, vp, sz, vp, vp, vp, sz, vp, i, f, i, i, vp, vp, vp]
        L.orbgpu_search_for_initialization_stream_device.argtypes = [
            i, GridBounds, vp, vp, vp, sz, vp, vp, vp, vp, i, f, i, i, vp, vp, vp]
        L.orbgpu_debug_level_candidates.argtypes = [vp, i, i, vp, i]
        L.orbgpu_debug_level_blur.argtypes = [vp, i, i, vp, sz]
        L.orbgpu_debug_level_octree.argtypes = [vp, i, i, vp, i]
        L.orbgpu_debug_octree_trace.argtypes = [vp, i, vp, i]
        L.orbgpu_debug_pyramid_emulate.argtypes = [i, f, i, i, i, vp, sz, vp, sz, vp]
        L.orbgpu_search_for_initialization.argtypes = [GridBounds, vp, vp, i, vp, vp, i, vp, i, f, i, vp,
                                                       ctypes.POINTER(i)]
        # orbgpu_frame.h
        L.orbgpu_compute_image_bounds.argtypes = [ctypes.POINTER(Camera), i, i, ctypes.POINTER(GridBounds)]
        L.orbgpu_undistort_keypoints_batch_device.argtypes = [ctypes.POINTER(Camera), i, vp, vp, i, vp, vp]
        L.orbgpu_assign_features_to_grid_batch_device.argtypes = [i, GridBounds, vp, vp, i, vp, vp, vp]
        # orbgpu_stereo.h
        L.orbgpu_stereo_matches_batch_device.argtypes = [vp, vp, sz, sz, i, vp, vp, vp, i, f, f, vp, vp, vp]
        # orbgpu_ransac.h
        L.orbgpu_srand.argtypes = [ctypes.c_uint]
        L.orbgpu_srand.restype = None
        L.orbgpu_rand.restype = i
        L.orbgpu_random_int.argtypes = [i, i]
        L.orbgpu_rand_get_state.argtypes = [vp]
        L.orbgpu_rand_get_state.restype = None
        L.orbgpu_rand_set_state.argtypes = [vp]
        L.orbgpu_rand_set_state.restype = None
        L.orbgpu_srand_r.argtypes = [vp, ctypes.c_uint]
        L.orbgpu_srand_r.restype = None
        L.orbgpu_rand_r.argtypes = [vp]
        L.orbgpu_sim3_workspace_bytes.argtypes = [i]
        L.orbgpu_sim3_workspace_bytes.restype = sz
        L.orbgpu_sim3_ransac_batch_device.argtypes = [i, vp, i, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.orbgpu_sim3_ransac_batch.argtypes = [i, vp, i, vp, vp, vp, vp, i, vp, vp, vp]
        L.orbgpu_pnp_workspace_bytes.argtypes = [i, i]
        L.orbgpu_pnp_workspace_bytes.restype = sz
        L.orbgpu_pnp_ransac_batch_device.argtypes = [i, vp, i, i, i, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.orbgpu_pnp_ransac_batch.argtypes = [i, vp, i, vp, vp, vp, i, vp, vp, vp, vp]
        # orbgpu_bow.h
        L.orbgpu_vocabulary_load_text.argtypes = [ctypes.c_char_p, ctypes.POINTER(vp)]
        L.orbgpu_vocabulary_load_binary.argtypes = [ctypes.c_char_p, ctypes.POINTER(vp)]
        L.orbgpu_vocabulary_create.argtypes = [i, i, i, i, i, vp, vp, vp, vp, ctypes.POINTER(vp)]
        L.orbgpu_vocabulary_destroy.argtypes = [vp]
        L.orbgpu_vocabulary_get_info.argtypes = [vp, vp]
        L.orbgpu_bow_transform_batch_device.argtypes = [vp, i, vp, vp, i, i, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                                        vp]
        L.orbgpu_bow_transform.argtypes = [vp, i, vp, i, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.orbgpu_search_by_bow_batch_device.argtypes = [i, i, vp, vp, f, i, i, vp, vp, vp]
        L.orbgpu_search_by_bow.argtypes = [i, vp, vp, f, i, vp, vp]
        # orbgpu_proj.h
        L.orbgpu_is_in_frustum_device.argtypes = [vp, i, vp, vp, vp, vp, f, vp, vp, vp, vp]
        L.orbgpu_search_by_projection_batch_device.argtypes = [i, vp, i, vp, vp, vp]
        L.orbgpu_search_by_projection.argtypes = [vp, vp, vp]
        L.orbgpu_search_by_sim3.argtypes = [vp, vp, vp]
        _LIB = L
    return _LIB


def last_error() -> str:
    return lib().orbgpu_last_error().decode(errors="replace")


def _check(rc: int, what: str) -> None:
    if rc != OK:
        raise OrbGpuError(rc, what)


def device_arch() -> str:
    buf = ctypes.create_string_buffer(64)
    _check(lib().orbgpu_device_arch(buf, 64), "orbgpu_device_arch")
    return buf.value.decode()


def device_count() -> int:
    """visible HIP devices (0 without any)"""
    n = ctypes.c_int()
    _check(lib().orbgpu_device_count(ctypes.byref(n)), "orbgpu_device_count")
    return n.value


def set_thread_device(device: int) -> None:
    """the calling thread's device for the host-form calls (orbgpu_set_thread_device)"""
    _check(lib().orbgpu_set_thread_device(int(device)), "orbgpu_set_thread_device")


def get_thread_device() -> int:
    d = ctypes.c_int()
    _check(lib().orbgpu_get_thread_device(ctypes.byref(d)), "orbgpu_get_thread_device")
    return d.value


def pyramid_plan_emulate(img: np.ndarray, nfeatures=1000, scale_factor=1.2, nlevels=8):
    """Levels 1..nlevels-1 of `img` computed on the CPU by the fused pyramid
    kernel's own plan (orbgpu_debug_pyramid_emulate: same LDS ring slots, row
    records and per-lane columns, with slot-ownership checks), and the plan's
    figures.  Needs no GPU."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    # level sizes as ORBextractor computes them (cvRound of float products)
    sizes, s = [], np.float32(1.0)
    for l in range(1, nlevels):
        s = np.float32(s * np.float32(scale_factor))
        inv = np.float32(np.float32(1.0) / s)
        sizes.append((int(np.rint(np.float32(h) * inv)), int(np.rint(np.float32(w) * inv))))
    out = np.zeros(sum(a * b for a, b in sizes) + 64, np.uint8)
    info = np.zeros(8, np.int32)
    _check(lib().orbgpu_debug_pyramid_emulate(nfeatures, scale_factor, nlevels, w, h, img.ctypes.data, img.strides[0],
                                              out.ctypes.data, out.size, info.ctypes.data),
           "orbgpu_debug_pyramid_emulate")
    levels, o = [], 0
    for lh, lw in sizes:
        levels.append(out[o:o + lw * lh].reshape(lh, lw).copy())
        o += lw * lh
    keys = ("ticks", "rows_per_chunk", "compute_waves", "producer_waves", "loads_per_lane", "entries_per_lane",
            "lds_bytes", "ring0_rows")
    return levels, dict(zip(keys, (int(v) for v in info)))


def _ptr(a) -> int:
    """data pointer of a numpy array or a torch tensor"""
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    return a.ctypes.data


def _stream_ptr(stream) -> int | None:
    if stream is None:
        return None
    return getattr(stream, "cuda_stream", stream)


class DeviceEvent:
    """A device-scope hipEvent_t (orbgpu_device_event_create: no timing, no
    system-scope fence when recorded) for ordering streams of one GPU.  It has
    torch.cuda.Event's record / wait / cuda_event, so torch streams take it
    (Stream.wait_event calls event.wait(stream)) and the extractor's stage
    hook can record it.  Not for a host that synchronises on it to read host
    memory: use a default event there."""

    def __init__(self):
        h = ctypes.c_void_p()
        _check(lib().orbgpu_device_event_create(ctypes.byref(h)), "device_event_create")
        self.cuda_event = h.value
        self._lib = lib()

    @staticmethod
    def _stream(stream):
        if stream is None:
            import torch
            stream = torch.cuda.current_stream()
        return stream.cuda_stream

    def record(self, stream=None):
        _check(lib().orbgpu_device_event_record(self.cuda_event, self._stream(stream)), "device_event_record")

    def wait(self, stream=None):
        _check(lib().orbgpu_stream_wait_device_event(self._stream(stream), self.cuda_event), "stream_wait_device_event")

    def __del__(self):
        try:
            if self.cuda_event:
                self._lib.orbgpu_device_event_destroy(self.cuda_event)
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass


class Extractor:
    """ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST) for
    frames of a fixed width x height, batched up to ``max_batch`` frames."""

    def __init__(self, nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7,
                 width=640, height=480, max_batch=1, device=None):
        """device: a HIP ordinal to place the extractor on (orbgpu_extractor_create_on_device);
        None: the calling thread's current device"""
        h = ctypes.c_void_p()
        if device is None:
            _check(lib().orbgpu_extractor_create(nfeatures, scale_factor, nlevels, ini_th, min_th,
                                                 width, height, max_batch, ctypes.byref(h)),
                   "orbgpu_extractor_create")
        else:
            _check(lib().orbgpu_extractor_create_on_device(int(device), nfeatures, scale_factor, nlevels, ini_th,
                                                           min_th, width, height, max_batch, ctypes.byref(h)),
                   "orbgpu_extractor_create_on_device")
        self.h = h
        info = _Info()
        _check(lib().orbgpu_extractor_get_info(self.h, ctypes.byref(info)), "get_info")
        self.nlevels = info.nlevels
        self.width, self.height = info.width, info.height
        self.max_batch = info.max_batch
        self.max_keypoints = info.max_keypoints
        self.level_sizes = [(info.level_width[l], info.level_height[l]) for l in range(self.nlevels)]
        self.features_per_level = [info.features_per_level[l] for l in range(self.nlevels)]
        self.level_capacity = [info.level_capacity[l] for l in range(self.nlevels)]
        self.device = info.device

    def close(self):
        if getattr(self, "h", None):
            lib().orbgpu_extractor_destroy(self.h)
            self.h = None

    __del__ = close

    def scale_factors(self):
        arrs = [np.zeros(self.nlevels, np.float32) for _ in range(4)]
        _check(lib().orbgpu_extractor_get_scales(self.h, *[a.ctypes.data for a in arrs]), "get_scales")
        return arrs

    def extract(self, img: np.ndarray):
        """operator()(image) for one host image -> (keypoints, descriptors)."""
        img = np.ascontiguousarray(img, np.uint8)
        cap = self.max_keypoints
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = ctypes.c_int()
        _check(lib().orbgpu_extract(self.h, img.ctypes.data, img.shape[1], img.shape[0], img.strides[0],
                                    kps.ctypes.data, desc.ctypes.data, cap, ctypes.byref(n)), "orbgpu_extract")
        if n.value < 0:
            return None
        return kps[:n.value].copy(), desc[:n.value].copy()

    def extract_batch(self, images, kps, desc, counts, stream=None, row_step=None, frame_step=None):
        """Device path.  images: uint8 (B, H, pitch) tensor on the GPU;
        kps: (B, cap, 7) float32/int32 view of orbgpu_keypoint (28 B each);
        desc: (B, cap, 32) uint8; counts: (B,) int32.  Asynchronous."""
        B = images.shape[0]
        rs = row_step if row_step is not None else images.stride(1) * images.element_size()
        fs = frame_step if frame_step is not None else images.stride(0) * images.element_size()
        cap = desc.shape[1]
        _check(lib().orbgpu_extract_batch_device(self.h, _ptr(images), B, rs, fs, _ptr(kps), _ptr(desc),
                                                 _ptr(counts), cap, _stream_ptr(stream)),
               "orbgpu_extract_batch_device")

    def sync(self, stream=None):
        _check(lib().orbgpu_extractor_sync(self.h, _stream_ptr(stream)), "orbgpu_extractor_sync")

    STAGES = ("pyramid", "fast_cells", "octree", "describe")

    def profile(self, enable: bool = True):
        _check(lib().orbgpu_extractor_profile(self.h, int(enable)), "profile")

    def set_stage_event(self, stage: str, event=None):
        """record `event` (a torch.cuda.Event, or None to clear) on the extraction
        stream right after `stage` (one of STAGES) of every later batch"""
        ptr = None
        if event is not None:
            event.record()  # torch creates the HIP event lazily; make sure it exists
            ptr = event.cuda_event
        _check(lib().orbgpu_extractor_set_stage_event(self.h, self.STAGES.index(stage), ptr), "set_stage_event")
        # the library keeps the raw hipEvent_t: hold the owner so it outlives the registration
        if not hasattr(self, "_stage_events"):
            self._stage_events = {}
        self._stage_events[stage] = event

    def stage_times(self, reset: bool = True):
        """(dict stage -> summed ms, number of extractions) since last reset."""
        ms = np.zeros(4, np.float32)
        n = ctypes.c_int()
        _check(lib().orbgpu_extractor_stage_times(self.h, ms.ctypes.data, ctypes.byref(n), int(reset)),
               "stage_times")
        return dict(zip(self.STAGES, ms.tolist())), n.value

    def _debug_xys(self, fn, level: int, frame: int) -> np.ndarray:
        n = fn(self.h, frame, level, None, 0)
        if n < 0:
            raise OrbGpuError(n, fn.__name__)
        out = np.zeros((max(n, 1), 3), np.int32)
        fn(self.h, frame, level, out.ctypes.data, n)
        return out[:n]

    def candidates(self, level: int, frame: int = 0) -> np.ndarray:
        """FAST candidates (x, y, score) of the last extraction, oracle order."""
        return self._debug_xys(lib().orbgpu_debug_level_candidates, level, frame)

    def octree(self, level: int, frame: int = 0) -> np.ndarray:
        """DistributeOctTree output (x, y, score) in list order."""
        return self._debug_xys(lib().orbgpu_debug_level_octree, level, frame)

    def enable_octree_trace(self):
        _check(lib().orbgpu_debug_octree_trace(self.h, 1, None, 0), "octree_trace")

    def octree_trace(self):
        out = np.zeros(16 * 512, np.int32)
        _check(lib().orbgpu_debug_octree_trace(self.h, 0, out.ctypes.data, out.size), "octree_trace")
        res = []
        for l in range(self.nlevels):
            t = out[l * 512:(l + 1) * 512]
            res.append(t[2:2 + 8 * t[0]].reshape(-1, 8))
        return res

    def blurred(self, level: int, frame: int = 0) -> np.ndarray:
        """The blurred level (GaussianBlur 7x7) of `frame` of the last extraction."""
        w, h = self.level_sizes[level]
        out = np.zeros((h, w), np.uint8)
        _check(lib().orbgpu_debug_level_blur(self.h, frame, level, out.ctypes.data, w), "debug_level_blur")
        return out

    def level(self, level: int, frame: int = 0) -> np.ndarray:
        """mvImagePyramid[level] of `frame` of the last extraction."""
        w, h = self.level_sizes[level]
        out = np.zeros((h, w), np.uint8)
        _check(lib().orbgpu_extractor_copy_level(self.h, frame, level, out.ctypes.data, w), "copy_level")
        return out


def keypoints_from_raw(raw: np.ndarray) -> np.ndarray:
    """View a (N, 28) uint8 / (N, 7) 4-byte array as KP_DTYPE records."""
    return np.ascontiguousarray(raw).view(np.uint8).reshape(-1, 28).view(KP_DTYPE).reshape(-1)


def search_for_initialization(kps1, desc1, kps2, desc2, img_w, img_h, prev_xy=None, window=100,
                              nnratio=0.9, check_ori=True, annotated_histo=False, bounds=None):
    """Host form: returns (nmatches, matches12, prev_xy_updated).  bounds
    defaults to the undistorted frame [0, img_w] x [0, img_h]."""
    kps1 = np.ascontiguousarray(kps1, KP_DTYPE)
    kps2 = np.ascontiguousarray(kps2, KP_DTYPE)
    desc1 = np.ascontiguousarray(desc1, np.uint8)
    desc2 = np.ascontiguousarray(desc2, np.uint8)
    if prev_xy is None:
        prev_xy = np.stack([kps1["x"], kps1["y"]], axis=1)
    prev = np.ascontiguousarray(prev_xy, np.float32).copy()
    m12 = np.full(max(len(kps1), 1), -1, np.int32)
    n = ctypes.c_int()
    flags = (MATCH_CHECK_ORI if check_ori else 0) | (MATCH_ANNOTATED_HISTO if annotated_histo else 0)
    bd = bounds if bounds is not None else bounds_for(img_w, img_h)
    _check(lib().orbgpu_search_for_initialization(bd, kps1.ctypes.data, desc1.ctypes.data, len(kps1),
                                                  kps2.ctypes.data, desc2.ctypes.data, len(kps2),
                                                  prev.ctypes.data, window, nnratio, flags,
                                                  m12.ctypes.data, ctypes.byref(n)),
           "orbgpu_search_for_initialization")
    return n.value, m12[:len(kps1)], prev


def search_for_initialization_batch(img_w, img_h, kps1, desc1, n1, kps2, desc2, n2, matches12, nmatches,
                                    prev_xy=None, window=100, nnratio=0.9, flags=MATCH_CHECK_ORI, stream=None,
                                    bounds=None, max_level0=0):
    """Device form over B pairs (tensors on the GPU, see include/orbgpu.h).
    max_level0 > 0: a known bound on every frame's level-0 keypoints (an
    Extractor's level_capacity[0]); pairs above it report nmatches -1."""
    B = n2.shape[0]
    bd = bounds if bounds is not None else bounds_for(img_w, img_h)
    _check(lib().orbgpu_search_for_initialization_batch_device_bounded(
        B, bd, _ptr(kps1), _ptr(desc1), _ptr(n1), desc1.shape[1], _ptr(kps2), _ptr(desc2), _ptr(n2),
        desc2.shape[1], _ptr(prev_xy) if prev_xy is not None else None, window, nnratio, flags, max_level0,
        _ptr(matches12), _ptr(nmatches), _stream_ptr(stream)), "orbgpu_search_for_initialization_batch_device_bounded")


def search_for_initialization_stream(img_w, img_h, kps, desc, n, prev_kps, prev_desc, prev_n, matches12, nmatches,
                                     prev_xy=None, window=100, nnratio=0.9, flags=MATCH_CHECK_ORI, stream=None,
                                     bounds=None, max_level0=0):
    """Stream form over the B frames of one extraction (Tracking's (F_{t-1},
    F_t), Tracking.cpp:768-769): pair b matches frame b-1 against frame b, pair
    0 the frame (prev_kps (cap, 7), prev_desc (cap, 32), prev_n (1,)) before
    the batch, read in place.  matches12 (B, cap): row b has F1's keypoints."""
    B, cap = n.shape[0], desc.shape[1]
    assert kps.shape[0] >= B and desc.shape[0] >= B and prev_desc.shape[0] <= cap
    assert matches12.shape[0] >= B and matches12.shape[1] == cap and nmatches.shape[0] >= B
    bd = bounds if bounds is not None else bounds_for(img_w, img_h)
    _check(lib().orbgpu_search_for_initialization_stream_device(
        B, bd, _ptr(kps), _ptr(desc), _ptr(n), cap, _ptr(prev_kps), _ptr(prev_desc), _ptr(prev_n),
        _ptr(prev_xy) if prev_xy is not None else None, window, nnratio, flags, max_level0,
        _ptr(matches12), _ptr(nmatches), _stream_ptr(stream)), "orbgpu_search_for_initialization_stream_device")


def hamming_pairs(a, b, out, stream=None):
    """DescriptorDistance over n pairs of device descriptors (n, 32) uint8."""
    _check(lib().orbgpu_hamming_pairs_device(_ptr(a), _ptr(b), a.shape[0], _ptr(out), _stream_ptr(stream)),
           "orbgpu_hamming_pairs_device")


def pack_rows(batch: int, cap: int, items, stream=None) -> None:
    """orbgpu_pack_rows_device: items = [(rows (batch, cap, ...) tensor,
    packed tensor with >= batch * cap rows, counts int32 (batch,) tensor)];
    frame b's first counts[b] rows land at sum_{b' < b} counts[b'] of
    packed (asynchronous on `stream`)."""
    import torch
    descs = (PackDesc * len(items))()
    for d, (rows, packed, counts) in zip(descs, items):
        assert rows.is_contiguous() and packed.is_contiguous() and counts.is_contiguous()
        assert counts.dtype == torch.int32 and counts.numel() >= batch and rows.shape[1] == cap
        rb = rows[0, 0].numel() * rows.element_size()
        assert packed[0].numel() * packed.element_size() == rb and packed.shape[0] >= batch * cap
        d.rows, d.packed, d.counts, d.row_bytes = rows.data_ptr(), packed.data_ptr(), counts.data_ptr(), rb
    _check(lib().orbgpu_pack_rows_device(batch, cap, len(items), descs, _stream_ptr(stream)),
           "orbgpu_pack_rows_device")


def stereo_matches_batch(ex: "Extractor", images, npairs, kps, desc, counts, bf, min_z, uright, depth,
                         stream=None, row_step=None, frame_step=None):
    """Frame::ComputeStereoMatches (Frame.cpp:540-748) for pairs (2p, 2p+1) of
    the last ex.extract_batch() call (same images / kps / desc / counts
    tensors).  uright, depth: float32 (npairs, cap) device tensors.  min_z is
    Frame::mb at call time (0 in the reference: infinite max disparity)."""
    rs = row_step if row_step is not None else images.stride(1) * images.element_size()
    fs = frame_step if frame_step is not None else images.stride(0) * images.element_size()
    cap = desc.shape[1]
    _check(lib().orbgpu_stereo_matches_batch_device(ex.h, _ptr(images), rs, fs, npairs, _ptr(kps), _ptr(desc),
                                                    _ptr(counts), cap, float(bf), float(min_z), _ptr(uright),
                                                    _ptr(depth), _stream_ptr(stream)),
           "orbgpu_stereo_matches_batch_device")


def compute_image_bounds(cam: Camera, cols: int, rows: int) -> GridBounds:
    """Frame::ComputeImageBounds (Frame.cpp:498-530)."""
    b = GridBounds()
    _check(lib().orbgpu_compute_image_bounds(ctypes.byref(cam), cols, rows, ctypes.byref(b)), "compute_image_bounds")
    return b


def undistort_keypoints_batch(cam: Camera, kps, counts, kps_un, stream=None):
    """Frame::UndistortKeyPoints for (B, cap, 7) keypoint tensors."""
    _check(lib().orbgpu_undistort_keypoints_batch_device(ctypes.byref(cam), kps.shape[0], _ptr(kps), _ptr(counts),
                                                         kps.shape[1], _ptr(kps_un), _stream_ptr(stream)),
           "undistort_keypoints_batch_device")


def assign_features_to_grid_batch(bounds: GridBounds, kps_un, counts, cell_start, cell_items, stream=None):
    """Frame::AssignFeaturesToGrid -> CSR (cell_start (B, 64*48+1), cell_items (B, cap)) int32 tensors."""
    _check(lib().orbgpu_assign_features_to_grid_batch_device(kps_un.shape[0], bounds, _ptr(kps_un), _ptr(counts),
                                                             kps_un.shape[1], _ptr(cell_start), _ptr(cell_items),
                                                             _stream_ptr(stream)),
           "assign_features_to_grid_batch_device")
