"""Host-side mirror of LoopClosing::ComputeSim3's hot loop over the C ABI in
include/orbgpu_loop.h (csrc/loop.hip) and include/orbgpu_bow.h.

* ``Keyframes`` -- the keyframe data the loop closer reads (descriptors,
  angles, octaves, MapPoint flags and world positions, pose, K), resident in
  HBM, plus their DBoW2 FeatureVectors (KeyFrame::ComputeBoW).
* ``LoopBurst`` -- a batch of ComputeSim3 calls (src/LoopClosing.cpp:273-420):
  per query, SearchByBoW(mpCurrentKF, pKF) with ORBmatcher(0.75, true) for
  every candidate (:311), the Sim3Solver constructors of the candidates with
  >= 20 matches (:314-324), then the round-robin iterate(5) RANSAC until the
  first candidate returns a Sim3 (:339-356; the SearchBySim3/OptimizeSim3
  verification that follows is outside the hot path and taken to pass).

Everything runs on the GPU in four launches per step (SearchByBoW batch,
Sim3Solver set-up, ComputeSim3); there is no host fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np

import bow
import orbgpu
import ransac

_BOUND = False


class LoopKeyframe(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("pad", ctypes.c_int), ("Rcw", ctypes.c_float * 9), ("tcw", ctypes.c_float * 3),
                ("K", ctypes.c_float * 4), ("mp_world", ctypes.c_void_p), ("mp_valid", ctypes.c_void_p),
                ("octave", ctypes.c_void_p), ("sigma2", ctypes.c_void_p)]


class Sim3Candidate(ctypes.Structure):
    _fields_ = [("kf1", ctypes.c_int), ("kf2", ctypes.c_int)]


class ComputeSim3Query(ctypes.Structure):
    _fields_ = [("first_cand", ctypes.c_int), ("n_cand", ctypes.c_int), ("rng", ransac.RandState)]


class Sim3RansacParams(ctypes.Structure):
    _fields_ = [("probability", ctypes.c_double), ("min_inliers", ctypes.c_int), ("max_iterations", ctypes.c_int),
                ("iterations_per_call", ctypes.c_int), ("fix_scale", ctypes.c_int)]


class ComputeSim3Result(ctypes.Structure):
    _fields_ = [("matched", ctypes.c_int), ("round", ctypes.c_int), ("n_inliers", ctypes.c_int),
                ("hypotheses", ctypes.c_int), ("draws", ctypes.c_int), ("pad", ctypes.c_int),
                ("T12", ctypes.c_float * 16), ("R12", ctypes.c_float * 9), ("t12", ctypes.c_float * 3),
                ("s12", ctypes.c_float), ("rng_after", ransac.RandState)]


class Sim3CandidateState(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("max_iterations", ctypes.c_int), ("iterations", ctypes.c_int),
                ("best_inliers", ctypes.c_int), ("discarded", ctypes.c_int), ("pad", ctypes.c_int)]


MAX_CANDIDATES = 64


def _lib():
    global _BOUND
    L = orbgpu.lib()
    if not _BOUND:
        vp, i = ctypes.c_void_p, ctypes.c_int
        L.orbgpu_sim3_setup_workspace_bytes.argtypes = [i, i]
        L.orbgpu_sim3_setup_workspace_bytes.restype = ctypes.c_size_t
        L.orbgpu_sim3_setup_batch_device.argtypes = [i, vp, vp, vp, i, vp, i, vp, vp, vp]
        L.orbgpu_compute_sim3_batch_device.argtypes = [i, vp, i, vp, vp, i, vp, vp, Sim3RansacParams, vp, vp, vp, vp]
        L.orbgpu_sim3_corr_kf1_slots.argtypes = [vp, i, i, i]
        L.orbgpu_sim3_corr_kf1_slots.restype = ctypes.c_void_p
        _BOUND = True
    return L


def _struct_rows(tensor_u8, ctype, n):
    raw = tensor_u8.cpu().numpy().tobytes()
    return (ctype * n).from_buffer_copy(raw[:ctypes.sizeof(ctype) * n])


class Keyframes:
    """n_kf keyframes of up to `stride` keypoints in HBM.  Host inputs (numpy):
    desc (n_kf, stride, 32) u8, angle (n_kf, stride) f32, octave (n_kf, stride)
    i32, valid (n_kf, stride) u8 (MapPoint present and good), mp_world (n_kf,
    stride, 3) f32, Tcw (n_kf, 12) f32 (Rcw row-major, tcw), K (4,) f32,
    sigma2 (nlevels,) f32, counts (n_kf,) (default all stride)."""

    def __init__(self, desc, angle, octave, valid, mp_world, Tcw, K, sigma2, counts=None, device="cuda"):
        import torch
        n_kf, S = desc.shape[:2]
        self.n_kf, self.stride, self.device = n_kf, S, torch.device(device)
        self.counts_host = np.full(n_kf, S, np.int32) if counts is None else np.asarray(counts, np.int32)
        up = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dt)).to(self.device)  # noqa: E731
        self.desc = up(desc, np.uint8)
        self.angle = up(angle, np.float32)
        self.octave = up(octave, np.int32)
        self.valid = up(valid, np.uint8)
        self.mp_world = up(mp_world, np.float32)
        self.sigma2 = up(sigma2, np.float32)
        self.counts = up(self.counts_host, np.int32)
        tab = (LoopKeyframe * n_kf)()
        for k in range(n_kf):
            r = tab[k]
            r.n = int(self.counts_host[k])
            r.Rcw[:] = [float(v) for v in Tcw[k, :9]]
            r.tcw[:] = [float(v) for v in Tcw[k, 9:12]]
            r.K[:] = [float(v) for v in K]
            r.mp_world = self.mp_world.data_ptr() + 12 * S * k
            r.mp_valid = self.valid.data_ptr() + S * k
            r.octave = self.octave.data_ptr() + 4 * S * k
            r.sigma2 = self.sigma2.data_ptr()
        self.d_table = bow.to_device_table(tab, self.device)
        self.tf = None

    def compute_bow(self, voc: bow.Vocabulary, levelsup=4, stream=None):
        """KeyFrame::ComputeBoW for every keyframe (mFeatVec, levelsup 4)."""
        self.tf = bow.BatchTransform(self.n_kf, self.stride, self.device)
        bow.transform_batch(voc, self.desc, self.counts, self.tf, levelsup, stream)
        self.frames = bow.frame_table(self.tf, self.desc, self.angle, self.valid, self.counts_host)
        return self.tf


class LoopBurst:
    """ComputeSim3 for `queries` = list of (current_kf, [candidate kfs], rng
    state or seed): all SearchByBoW pairs in one batch, then the Sim3Solver
    set-up and the round-robin RANSAC of every query on the GPU."""

    def __init__(self, kfs: Keyframes, queries, nnratio=0.75, check_ori=True, min_matches=20, probability=0.99,
                 min_inliers=20, max_iterations=300, iterations_per_call=5, fix_scale=False):
        import torch
        if kfs.tf is None:
            raise ValueError("Keyframes.compute_bow() first")
        self.kfs = kfs
        dev = kfs.device
        self.nnratio, self.check_ori, self.min_matches = nnratio, check_ori, min_matches
        self.params = Sim3RansacParams(probability, min_inliers, max_iterations, iterations_per_call, int(fix_scale))
        pairs, qtab = [], (ComputeSim3Query * max(len(queries), 1))()
        for qi, (cur, cands, rng) in enumerate(queries):
            if len(cands) > MAX_CANDIDATES:
                raise ValueError(f"at most {MAX_CANDIDATES} candidates per query")
            qtab[qi].first_cand = len(pairs)
            qtab[qi].n_cand = len(cands)
            if isinstance(rng, ransac.RandState):
                qtab[qi].rng = rng
            else:
                orbgpu.lib().orbgpu_srand_r(ctypes.byref(qtab[qi].rng), int(rng) & 0xFFFFFFFF)
            pairs.extend((cur, c) for c in cands)
        self.n_queries, self.n_pairs = len(queries), len(pairs)
        self.pairs = np.array(pairs, np.int32).reshape(-1, 2)
        fa = (bow.BowFrame * max(self.n_pairs, 1))()
        fb = (bow.BowFrame * max(self.n_pairs, 1))()
        ctab = (Sim3Candidate * max(self.n_pairs, 1))()
        for p, (a, b) in enumerate(pairs):
            fa[p], fb[p] = kfs.frames[a], kfs.frames[b]
            ctab[p].kf1, ctab[p].kf2 = a, b
        self.d_fa, self.d_fb = bow.to_device_table(fa, dev), bow.to_device_table(fb, dev)
        self.d_cands = bow.to_device_table(ctab, dev)
        self.d_queries = bow.to_device_table(qtab, dev)
        S = kfs.stride
        P = max(self.n_pairs, 1)
        self.match = torch.zeros((P, S), dtype=torch.int32, device=dev)
        self.nmatches = torch.zeros(P, dtype=torch.int32, device=dev)
        self.n_corr = torch.zeros(P, dtype=torch.int32, device=dev)
        wbytes = _lib().orbgpu_sim3_setup_workspace_bytes(P, S)
        self.workspace = torch.zeros(wbytes, dtype=torch.uint8, device=dev)
        self.results = torch.zeros(max(self.n_queries, 1) * ctypes.sizeof(ComputeSim3Result), dtype=torch.uint8,
                                   device=dev)
        self.states = torch.zeros(P * ctypes.sizeof(Sim3CandidateState), dtype=torch.uint8, device=dev)
        self.inliers = torch.zeros((P, S), dtype=torch.uint8, device=dev)

    def search_by_bow(self, stream=None):
        """SearchByBoW(mpCurrentKF, pKF, vpMatches12) for every pair."""
        bow.search_by_bow_batch(bow.KF_KF, self.d_fa, self.d_fb, self.n_pairs, self.nnratio, self.check_ori,
                                self.kfs.stride, self.match, self.nmatches, stream)

    def setup(self, stream=None):
        """Sim3Solver(pKF1, pKF2, vpMatched12, bFixScale) per candidate."""
        orbgpu._check(_lib().orbgpu_sim3_setup_batch_device(
            self.n_pairs, self.d_cands.data_ptr(), self.kfs.d_table.data_ptr(), self.match.data_ptr(),
            self.kfs.stride, self.nmatches.data_ptr(), self.min_matches, self.workspace.data_ptr(),
            self.n_corr.data_ptr(), orbgpu._stream_ptr(stream)), "orbgpu_sim3_setup_batch_device")

    def compute_sim3(self, stream=None):
        """The round-robin RANSAC of every query."""
        orbgpu._check(_lib().orbgpu_compute_sim3_batch_device(
            self.n_queries, self.d_queries.data_ptr(), self.n_pairs, self.d_cands.data_ptr(),
            self.kfs.d_table.data_ptr(), self.kfs.stride, self.workspace.data_ptr(), self.n_corr.data_ptr(),
            self.params, self.results.data_ptr(), self.states.data_ptr(), self.inliers.data_ptr(),
            orbgpu._stream_ptr(stream)), "orbgpu_compute_sim3_batch_device")

    def step(self, stream=None):
        self.search_by_bow(stream)
        self.setup(stream)
        self.compute_sim3(stream)

    # ---- results (host) ---------------------------------------------------
    def query_results(self):
        return _struct_rows(self.results, ComputeSim3Result, self.n_queries)

    def candidate_states(self):
        return _struct_rows(self.states, Sim3CandidateState, self.n_pairs)

    def corr_kf1_slots(self, c: int) -> np.ndarray:
        """mvnIndices1 of candidate c (KF1 slot of each correspondence)."""
        n = int(self.n_corr[c].item())
        if n <= 0:
            return np.zeros(0, np.int32)
        S = self.kfs.stride
        ws = _lib().orbgpu_sim3_corr_kf1_slots(self.workspace.data_ptr(), self.n_pairs, S, c)
        off = (ws - self.workspace.data_ptr()) // 4
        import torch
        flat = self.workspace.view(torch.int32)
        return flat[off:off + n].cpu().numpy()

    def vb_inliers(self, q: int, res=None) -> np.ndarray:
        """vbInliers (size KF1.N) of query q's returned Sim3, or all False."""
        res = res if res is not None else self.query_results()
        r = res[q]
        cur = int(self.pairs[0, 0]) if self.n_pairs else 0
        out = np.zeros(self.kfs.stride, bool)
        if r.matched < 0:
            return out
        c = self.d_first(q) + r.matched
        cur = int(self.pairs[c, 0])
        slots = self.corr_kf1_slots(c)
        mask = self.inliers[c, :len(slots)].cpu().numpy().astype(bool)
        out[slots[mask]] = True
        return out[:int(self.kfs.counts_host[cur])]

    def d_first(self, q: int) -> int:
        tab = _struct_rows(self.d_queries, ComputeSim3Query, self.n_queries)
        return tab[q].first_cand
