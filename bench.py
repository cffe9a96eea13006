#!/usr/bin/env python3
"""bench.py -- ORB-SLAM2 front-end hot path on MI355X: frames/sec of ORB
extract + match (BASELINE.json metric).

A step = one pass of the hot path over one batch of B synthetic frames per
GPU, inputs already resident in HBM:
  * ORBextractor::operator() on all B frames (pyramid -> FAST cells ->
    octree -> angle/blur/rBRIEF), and
  * ORBmatcher(0.9, true).SearchForInitialization(F_{t-1}, F_t, window 100)
    for the B consecutive pairs, the reference's map-free matcher
    (Tracking.cpp:768-769).
value = frames processed by all ranks / max-over-ranks wall time.
The matcher runs on a second HIP stream one step behind: step k-1's
SearchForInitialization starts when step k's FAST pass is done (never during
the pyramid pass, which fills every CU) and overlaps step k's octree /
describe (the extractor's stage-event hook, orbgpu_extractor_set_stage_event);
the last step's match is issued before the timed region closes, so all K
steps' work is inside it.

Ranks.  `python3 bench.py --gpus N` with N > 1 and no WORLD_SIZE in the
environment starts `python -m torch.distributed.run --nproc-per-node N`
on this same command line as a CHILD process (the parent never touches the
GPU) and exits with its status; under torchrun (the driver's own N > 1 form)
each rank reads RANK / LOCAL_RANK / WORLD_SIZE and checks WORLD_SIZE == N.
One process per GPU, RCCL ("nccl") process group.

The frames are ONE stream (shard.py): at step s rank r owns
global frames [(s*N + r)*B, +B) -- contiguous chunks; the chunk-boundary
frame's keypoints/descriptors go to rank r+1 (RCCL send/recv) so the (t-1, t)
pair across ranks is matched; every step's outputs are gathered to rank 0
(send/recv, overlapped with the next step).  Both are inside the timed
region.  The frames come from a pool of 4 steps per rank rendered up front
(a fresh batch every step, > the 256 MB MALL).

Stereo (--config euroc_stereo / kitti_stereo, and the `stereo_euroc_sharded`
leg of the default line at every N): the unit is the L/R pair one stereo
Frame is built from (src/Frame.cpp:84-98): each rank extracts the L and R
images of its contiguous chunk of pairs in one batch and runs
Frame::ComputeStereoMatches on them; the pair never straddles ranks, there is
no cross-pair dependency, and every step's keypoints / descriptors / uRight /
depth are gathered to rank 0.

Also reported:
  * roofline: the pyramid pass (the HBM-bound stage named by BASELINE.json),
    algorithmic bytes = sum_{l>=1} |P_{l-1}| + |P_l| per frame, divided by the
    pyramid launches' summed duration from HIP events recorded on the launch
    stream during the timed region; traffic = PMC-measured HBM bytes from
    profiles/ when a matching summary exists;
  * cpu_baseline: the oracle (a scalar C++ restatement, oracle/liborbref.so --
    NOT the reference's SIMD OpenCV code) on the host cores, rank 0 at N=1
    only, on a bounded sample;
  * single_frame / drop_in: the drop-in C++ classes timed as Tracking calls
    them (tests/cpp/adapter_main --time);
  * other_geometries: the 1241x376 / 2000-feature mono stream with its own
    pyramid roofline, and KITTI / EuRoC stereo pairs/s;
  * loop_burst: SURVEY config 5 (LoopClosing::ComputeSim3 bursts) on the
    bench mix and two harder mixes, queries round-robin over the ranks.
--config loopburst runs config 5 alone as the headline.

--cpu-dry-run ENGINE.py (tests only): the same launcher, rank logic,
sharding and gather over gloo on the CPU, with ENGINE.py providing the
orbgpu surface (tests/dryrun_orbgpu.py wraps the CPU oracle as the checker);
--dump DIR makes rank 0 write the gathered outputs of every step.
"""
from __future__ import annotations

import argparse
import contextlib
import gc
import importlib.util
import json
import math
import os
import socket
import struct
import subprocess
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path[:0] = [str(ROOT / "orb-slam2-annotation_amd"), str(ROOT / "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "frames/sec ORB extract+match (1000 feat, 640×480 mono) at 1/2/4/8 GPU; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
PYR_KERNEL = ("pyramid_tick_kernel (one frame per block; all levels advance together in ticks through LDS rings: "
              "level 0 read once, levels 1..7 written once, nothing read back)")
PYR_KERNEL_ID = "pyramid_tick_kernel"
POOL_STEPS = 4

CONFIGS = {
    # name: (width, height, nfeatures, description)
    "mono640": (640, 480, 1000, "synthetic 640x480 mono stream, 1000 feat, 8 levels x1.2, FAST 20/7 "
                                "(TUM1.yaml params), extract + SearchForInitialization(t-1,t)"),
    "kitti": (1241, 376, 2000, "synthetic 1241x376 mono stream, 2000 feat (KITTI00-02.yaml params), "
                               "extract + SearchForInitialization(t-1,t)"),
    "euroc": (752, 480, 1200, "synthetic 752x480 mono stream, 1200 feat (EuRoC.yaml params), "
                              "extract + SearchForInitialization(t-1,t)"),
    "euroc_stereo": (752, 480, 1200, "synthetic rectified 752x480 stereo stream, 1200 feat (EuRoC.yaml params), "
                                     "per pair: extract L+R + Frame::ComputeStereoMatches, pairs sharded "
                                     "per rank in contiguous chunks"),
    "kitti_stereo": (1241, 376, 2000, "synthetic rectified 1241x376 stereo stream, 2000 feat (KITTI00-02.yaml), "
                                      "per pair: extract L+R + Frame::ComputeStereoMatches, pairs sharded per "
                                      "rank in contiguous chunks"),
    "loopburst": (None, None, 1000, "LoopClosing::ComputeSim3 bursts: 100 queries x 5 candidate keyframes "
                                    "(500 KF pairs, 1000 keypoints each, 40% true correspondences under a "
                                    "known Sim3, the rest geometric outliers), SearchByBoW(KF,KF) over a "
                                    "k=10 L=6 DBoW2 vocabulary + Sim3Solver(0.99,20,300) round-robin iterate(5)"),
}
STEREO = {  # config -> (Camera.bf, synthetic baseline px)
    "kitti_stereo": (0.54 * 718.856, 30.0),           # Examples/Stereo/KITTI00-02.yaml
    "euroc_stereo": (47.90639384423901, 18.0),        # Examples/Stereo/EuRoC.yaml
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None,
                    help="frames (stereo: pairs) per GPU per step (default 512 mono640, 256 kitti, 128 stereo)")
    ap.add_argument("--config", default="mono640", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="bounded CPU-baseline budget per config")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="headline only (no extra legs)")
    ap.add_argument("--match-after", default="fast_cells", choices=["pyramid", "fast_cells", "octree"],
                    help="extraction stage of step k after which step k-1's match starts")
    ap.add_argument("--deliver", default="gpu0", choices=["host", "gpu0"],
                    help="where each step's outputs go (shard.Delivery): host = every rank copies its trimmed "
                         "outputs over its own PCIe link to pinned host memory (the Tracking thread's side); "
                         "gpu0 = counts then used rows sent to rank 0's HBM")
    ap.add_argument("--feed", default="hbm", choices=["hbm", "host"],
                    help="headline input: frames resident in HBM (default) or copied from pinned host memory "
                         "every step (the host_fed leg of the default line)")
    ap.add_argument("--parts", type=int, default=1,
                    help="headline step as this many sub-batches on their own streams, each started once the "
                         "previous one has passed --part-stage (1: one extraction of the whole batch)")
    ap.add_argument("--part-stage", default="pyramid", choices=["pyramid", "fast_cells", "octree"])
    ap.add_argument("--match-priority", type=int, default=0, choices=[0, -1],
                    help="matcher stream priority (0: default, below the extraction streams; -1: high)")
    ap.add_argument("--sustained-steps", type=int, default=None,
                    help="length of the mono line's sustained leg (default: BENCH_SUSTAINED_STEPS or 400 with the "
                         "extra legs on a GPU, none otherwise; > 0 forces it, e.g. in the CPU launcher tests)")
    ap.add_argument("--other-delivery", type=int, default=1, choices=[0, 1],
                    help="N > 1: also run the stream with the other --deliver mode (a second leg in the line)")
    ap.add_argument("--traffic-json", default=str(ROOT / "profiles" / "pmc_traffic.json"))
    ap.add_argument("--cpu-dry-run", default=None, metavar="ENGINE.py",
                    help="tests only: gloo on the CPU with ENGINE.py standing in for orbgpu")
    ap.add_argument("--dump", default=None, metavar="DIR", help="rank 0 writes every step's gathered outputs")
    return ap.parse_args(argv)


SUSTAINED_STEPS = int(os.environ.get("BENCH_SUSTAINED_STEPS", "400"))  # the sustained leg of the mono line
HEADLINE_PROFILED = 5  # a timed leg's stage and match times: HIP events on its last 5 steps
PROF_STEPS = int(os.environ.get("BENCH_PROF_STEPS", "-1"))  # diagnostics: overrides HEADLINE_PROFILED
SETTLE_STEPS = int(os.environ.get("BENCH_SETTLE_STEPS", "0"))  # diagnostics: an untimed leg before the headline
PROFILED_TAIL = 40     # a deferred leg's stage times: its last steps only (StreamBench.run)
STEP_TRACE = [os.environ.get("BENCH_STEP_TRACE") == "1"]  # diagnostics: per-step times of each timed leg
MATCH_AFTER = ["fast_cells"]  # set from --match-after
MATCH_PRIORITY = [0]  # set from --match-priority (0: default, -1: high, as the extraction streams)
DEVICE_EVENTS = os.environ.get("BENCH_DEVICE_EVENTS", "1") != "0"  # Dev.event: device-scope ordering events


# ---------------------------------------------------------------------------
# launcher: one process per GPU
# ---------------------------------------------------------------------------

def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(n: int, argv) -> int:
    """Run this command line under torchrun with n ranks as a child process
    (never exec: the parent has not touched the GPU, but a child is the
    pattern the GPU box allows everywhere) and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(Path(__file__).resolve())] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


class _NullStream:
    """CPU stand-in for a HIP stream (dry run)."""
    cuda_stream = None

    def wait_event(self, ev):
        pass


class _NullEvent:
    def record(self, stream=None):
        pass

    def elapsed_time(self, other):
        return 0.0


class Dev:
    """The rank's device: a GPU (HIP streams / events) or, for --cpu-dry-run,
    the CPU with no-op streams and events."""

    def __init__(self, device: torch.device):
        self.device = device
        self.cuda = device.type == "cuda"

    def stream(self, priority=0):
        return torch.cuda.Stream(self.device, priority=priority) if self.cuda else _NullStream()

    def current_stream(self):
        return torch.cuda.current_stream(self.device) if self.cuda else _NullStream()

    def event(self, timing=False):
        """a timing event (torch), or for stream-to-stream ordering a device-scope
        one (orbgpu.DeviceEvent: a default event's system-scope fence stalled the
        extraction stream ~7 us per record, profiles/r06_notes_ab.txt r6x;
        BENCH_DEVICE_EVENTS=0 restores torch's)"""
        if not self.cuda:
            return _NullEvent()
        if timing or not DEVICE_EVENTS:
            return torch.cuda.Event(enable_timing=timing)
        import orbgpu
        return orbgpu.DeviceEvent()

    def synchronize(self):
        if self.cuda:
            torch.cuda.synchronize(self.device)

    def use_stream(self, s):
        return torch.cuda.stream(s) if self.cuda else contextlib.nullcontext()

    def empty_cache(self):
        if self.cuda:
            torch.cuda.empty_cache()


def load_engine(path):
    """orbgpu (the HIP library; raises when liborbgpu.so or the GPU is
    missing), or the dry-run stand-in a test names."""
    if path is None:
        import orbgpu
        orbgpu.lib()
        return orbgpu
    spec = importlib.util.spec_from_file_location("orbgpu_dryrun_engine", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def pyramid_bytes_per_frame(level_sizes):
    px = [w * h for (w, h) in level_sizes]
    return sum(px[l - 1] + px[l] for l in range(1, len(px)))


def aggregate(elapsed: float, frames_local: int, device=None):
    """Whole-job numbers across ranks: max elapsed (the job ends when the
    slowest rank ends) and the sum of frames.  No-op without a process group."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return elapsed, frames_local
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    n = torch.tensor([frames_local], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(n, op=dist.ReduceOp.SUM)
    return float(t.item()), int(n.item())


def gather_delivery_stats(rep, world, device=None):
    """per-rank delivery numbers -> rank 0: the bytes every rank moved per
    step and the owner waits, max over ranks (no-op at N = 1)"""
    import torch.distributed as dist
    keys = ["bytes_per_step", "recv_bytes_per_step", "owner_wait_ms_per_step", "delivery_latency_ms", "ms_per_step"]
    if not (dist.is_available() and dist.is_initialized()) or world == 1:
        return {**rep, "per_rank": [{k: rep[k] for k in keys if k in rep}]}
    t = torch.tensor([float(rep.get(k, 0.0)) for k in keys], dtype=torch.float64, device=device)
    allt = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(allt, t)
    per = [{k: (int(v) if "bytes" in k else round(float(v), 4)) for k, v in zip(keys, x.tolist())} for x in allt]
    out = {"mode": rep["mode"], "per_rank": per}
    for k in keys:
        out[k + "_max"] = max(p[k] for p in per)
    return out


def _barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


class _Dumper:
    """rank 0: collects gathered outputs per global unit (frame or pair)."""

    def __init__(self, path, name):
        self.path, self.name, self.rows = path, name, {}

    def add(self, unit, **arrays):
        self.rows[int(unit)] = {k: np.asarray(v) for k, v in arrays.items()}

    def write(self):
        if not self.path:
            return
        Path(self.path).mkdir(parents=True, exist_ok=True)
        units = sorted(self.rows)
        keys = sorted(self.rows[units[0]]) if units else []
        out = {"units": np.array(units, np.int64)}
        for k in keys:
            out[k] = np.stack([self.rows[u][k] for u in units])
        np.savez(Path(self.path) / f"{self.name}.npz", **out)


# ---------------------------------------------------------------------------
# mono stream: extract + SearchForInitialization(t-1, t)
# ---------------------------------------------------------------------------

NSETS = 3  # output sets in rotation (StreamBench)


class OutSet:
    """One step's outputs in HBM: keypoints (B, cap, 7) f32 (orbgpu_keypoint),
    descriptors (B, cap, 32) u8, counts (B,), SearchForInitialization's m12
    (B, cap) / nmatch (B,), the F1 count of each pair (B,: the delivery trims
    m12 rows to it), and `inb`, the boundary frame received from another rank
    (kps (cap, 7), desc (cap, 32), count (1,)).  `prev` names the frame
    before the set's batch (pair 0's F1), read in place wherever it lives."""

    def __init__(self, B, cap, dev):
        z = torch.zeros
        self.kps = z((B, cap, 7), dtype=torch.float32, device=dev)
        self.desc = z((B, cap, 32), dtype=torch.uint8, device=dev)
        self.counts = z(B, dtype=torch.int32, device=dev)
        self.m12 = z((B, cap), dtype=torch.int32, device=dev)
        self.nmatch = z(B, dtype=torch.int32, device=dev)
        self.c1 = z(B, dtype=torch.int32, device=dev)
        self.inb = (z((cap, 7), dtype=torch.float32, device=dev), z((cap, 32), dtype=torch.uint8, device=dev),
                    z(1, dtype=torch.int32, device=dev))
        self.prev = None   # (kps, desc, count) of the frame before this set's batch
        self.pidx = None   # pool index of the step the set holds
        self.ev_ext = None  # end of the step's extraction (and boundary exchange)
        self.dslot = 0      # delivery ring slot of the set's last step

    def last(self):
        """the set's last frame, in place"""
        B = self.counts.shape[0]
        return self.kps[B - 1], self.desc[B - 1], self.counts[B - 1:B]


class StreamBench:
    """Extract + SearchForInitialization over one sharded frame stream.

    Output sets rotate over NSETS = 3 steps.  Step k extracts into set k % 3;
    its match (pairs (F_{t-1}, F_t) over the batch, src/Tracking.cpp:768-769)
    runs on the matcher stream one step behind, and pair 0's F1 -- the frame
    before the batch -- is read in place: at N = 1 the previous step's last
    frame in set (k-1) % 3, at N > 1 the boundary frame received straight into
    the set's `inb` buffers (rank r > 0: rank r-1's last frame of the same
    step; rank 0: rank N-1's last frame of the previous step).  So nothing is
    copied on the extraction stream.  Step k writes set k % 3, which the
    matches of steps k-3 (as F2) and k-2 (its last frame as pair 0's F1) read:
    it waits for the last match issued before it, step k-2's (matches run in
    order on one stream) -- the same distance as with two sets and the copy.
    """

    def __init__(self, og, D: Dev, W, H, NF, B, rank, world, stream, dump=None, deliver="host", feed="hbm",
                 parts=1, part_stage="pyramid", dump_tag=""):
        import shard
        import synth
        self.og, self.D = og, D
        self.deliver, self.feed = deliver, feed
        self.W, self.H, self.NF, self.B, self.rank, self.world = W, H, NF, B, rank, world
        dev = D.device
        self.dev, self.stream = dev, stream
        self.pitch = (W + 15) // 16 * 16
        # --parts P: the step's B frames as P sub-batches, each on an extractor and a stream
        # of its own; sub-batch i starts once sub-batch i-1 has passed `part_stage` (the
        # first one after the previous step's last), so stages with different limits
        # overlap (P = 1: one extraction of B frames on `stream`)
        if B % parts:
            raise SystemExit(f"--parts {parts} does not divide the batch {B}")
        self.parts, self.part_n = parts, B // parts
        self.exs = [og.Extractor(nfeatures=NF, width=W, height=H, max_batch=self.part_n) for _ in range(parts)]
        self.ex = self.exs[0]
        self.pstreams = [stream] + [D.stream(priority=-1) for _ in range(parts - 1)]
        # the step's tail (boundary exchange, the event the matcher waits for) on a stream of
        # its own when the step is split: the next step's first sub-batch then waits only for
        # the stage event, not for this step's last sub-batch to finish
        self.tstream = D.stream(priority=-1) if parts > 1 else stream
        cap = self.cap = self.ex.max_keypoints
        # pool: this rank's chunks of POOL_STEPS steps of the global stream
        self.pool_t0 = [shard.chunk_frames(s, rank, world, B)[0] for s in range(POOL_STEPS)]
        self.pool = [synth.torch_stream(B, W, H, device=dev, pitch=self.pitch, bounded=True, t0=t0)
                     for t0 in self.pool_t0]
        if feed == "host":
            # host-fed stream (TrackMonocular's images arrive from host memory,
            # mono_tum.cc:79-90): the pool lives in pinned host memory; every step's B
            # frames are copied into one of two HBM input buffers on a copy stream, the
            # next step's copy overlapping this step's extraction
            self.pool = [p.cpu().pin_memory() if D.cuda else p.cpu() for p in self.pool]
            self.inbuf = [torch.empty_like(self.pool[0], device=dev) for _ in range(2)]
            self.h2d = D.stream()
            self.ev_h2d = [D.event() for _ in range(2)]
            self.ev_in_read = [None, None]  # the extraction that last read each input buffer
            self.h2d_time = []  # (start, end) timing events per copy in the timed region
            self.h2d_issued = -1
        self.sets = [OutSet(B, cap, dev) for _ in range(NSETS)]
        z = torch.zeros
        self.empty = (z((cap, 7), dtype=torch.float32, device=dev), z((cap, 32), dtype=torch.uint8, device=dev),
                      z(1, dtype=torch.int32, device=dev))  # before the stream's first frame: no keypoints
        self.bx = shard.BoundaryExchange(rank, world)
        # every step's keypoints, descriptors (trimmed to the counts) and m12 rows (trimmed to the
        # matched-against frames' counts) plus counts / match counts go to the Tracking owner
        # (shard.Delivery: "host" over each rank's own PCIe link, or "gpu0" to rank 0's HBM)
        groups = None
        if deliver == "gpu0" and world > 1:
            import torch.distributed as dist
            groups = (dist.new_group(list(range(world))), dist.new_group(list(range(world))))
        S0 = self.sets[0]
        self.delivery = shard.Delivery(deliver, rank, world, dev,
                                       [shard.RowSpec("kps", 0), shard.RowSpec("desc", 0), shard.RowSpec("m12", 1)],
                                       B, cap, [S0.kps, S0.desc, S0.m12], 3 * B, groups=groups,
                                       packer=getattr(og, "pack_rows", None))
        self.flags = og.MATCH_CHECK_ORI
        self.step_no = 0
        # dumps (tests): host mode -- every rank its own delivered frames; gpu0 -- rank 0 all ranks'
        per_rank = deliver == "host" and world > 1
        self.dump = (_Dumper(dump, f"mono_{W}x{H}{dump_tag}" + (f"_rank{rank}" if per_rank else ""))
                     if (dump and (rank == 0 or per_rank)) else None)
        self.dump_all = bool(dump)
        # The matcher runs on its own stream, one step behind: SearchForInitialization of
        # step k-1 (a few hundred latency-bound blocks) starts once step k's FAST pass is
        # done (--match-after; never during the pyramid pass, which wants every CU).
        # run() flushes the last match inside the timed region.
        self.mstream = D.stream(priority=MATCH_PRIORITY[0])
        self.ev_pyr = D.event()
        # the previous step's match starts once the first sub-batch has passed MATCH_AFTER
        self.exs[0].set_stage_event(MATCH_AFTER[0], self.ev_pyr)
        self.ev_part = [None] * parts
        self.ev_part_done = [D.event() for _ in range(parts)]
        if parts > 1:
            for i, e in enumerate(self.exs):
                if i == 0 and part_stage == MATCH_AFTER[0]:
                    self.ev_part[i] = self.ev_pyr  # one event per (extractor, stage)
                else:
                    self.ev_part[i] = D.event()
                    e.set_stage_event(part_stage, self.ev_part[i])
        for S in self.sets:
            S.ev_ext = D.event()
        self.ev_match_last = None  # the last match issued (with its delivery packing)
        self.pending = None  # (set index, timing events) of the step whose match is not issued yet
        self.timing_h2d = False
        self._sus = None  # a deferred leg (run(defer=True)) whose stage times the next run() reads

    def _match(self, si, after, ev=None):
        S = self.sets[si]
        ms = self.mstream
        ms.wait_event(after)
        if after is not S.ev_ext:
            ms.wait_event(S.ev_ext)  # its step's tail (on its own stream when the step is split)
        pk, pd, pn = S.prev
        with self.D.use_stream(ms):  # F1 count of each pair (the delivery's m12 rows), beside the matcher
            torch.cat([pn, S.counts[:-1]], out=S.c1)
        if ev is not None:
            ev[0].record(ms)
        self.og.search_for_initialization_stream(self.W, self.H, S.kps, S.desc, S.counts, pk, pd, pn, S.m12,
                                                 S.nmatch, flags=self.flags, stream=ms,
                                                 max_level0=self.ex.level_capacity[0])
        if ev is not None:
            ev[1].record(ms)
        # delivery (packing on this stream, after the match; the copies or sends on the
        # delivery's own stream)
        S.dslot = self.delivery.start([S.kps, S.desc, S.m12], [S.counts, S.c1, S.nmatch], [S.counts, S.c1],
                                      stream=None if not self.D.cuda else ms)
        em = self.D.event()
        em.record(ms)  # the extraction two steps later (into the set this match read) waits for it
        self.ev_match_last = em

    def step(self, ev=None):
        B, st = self.B, self.stream
        k = self.step_no
        si = k % NSETS
        S = self.sets[si]
        if self.ev_match_last is not None:  # step k-2's match: it read S's last frame (k-3's read all of S)
            st.wait_event(self.ev_match_last)
        pidx = k % POOL_STEPS
        S.pidx = pidx
        frames = self.pool[pidx] if self.feed == "hbm" else self._fed(k)
        n = self.part_n
        for i, (e, ps) in enumerate(zip(self.exs, self.pstreams)):
            if i > 0 and self.ev_match_last is not None:
                ps.wait_event(self.ev_match_last)
            if self.parts > 1 and (i > 0 or k > 0):
                ps.wait_event(self.ev_part[i - 1])  # i = 0: the previous step's last sub-batch
            lo, hi = i * n, (i + 1) * n
            e.extract_batch(frames[lo:hi], S.kps[lo:hi], S.desc[lo:hi], S.counts[lo:hi],
                            stream=ps, row_step=self.pitch, frame_step=self.pitch * self.H)
        ts = self.tstream
        if self.parts > 1:  # the rest of the step (exchange, match) after every sub-batch
            for i in range(self.parts):
                self.ev_part_done[i].record(self.pstreams[i])
                ts.wait_event(self.ev_part_done[i])
        if self.feed == "host":  # the input buffer is free again after this extraction
            e_in = self.D.event()
            e_in.record(ts)
            self.ev_in_read[k % 2] = e_in
        # the frame before this batch (pair 0's F1), read in place
        if self.world == 1:
            S.prev = self.sets[(k - 1) % NSETS].last() if k > 0 else self.empty
        else:
            with self.D.use_stream(ts):
                if self.rank == 0:  # rank N-1's last frame: the one before our NEXT chunk
                    self.bx.exchange(S.last(), self.sets[(k + 1) % NSETS].inb)
                    S.prev = S.inb if k > 0 else self.empty
                else:
                    self.bx.exchange(S.last(), S.inb)
                    S.prev = S.inb
        S.ev_ext.record(ts)
        if self.pending is not None:  # step k-1's match, after step k's FAST pass
            self._match(self.pending[0], self.ev_pyr, self.pending[1])
        self.pending = (si, ev)
        if self.dump_all:  # test mode: finish the step and record what was delivered
            self.flush()
            self.delivery.finish()
            if self.dump is not None:
                self._record(si)
        self.step_no += 1

    def _issue_h2d(self, k):
        """copy step k's frames from pinned host memory into input buffer k % 2 on
        the copy stream, after the extraction that last read that buffer (step k-2)"""
        b = k % 2
        h = self.h2d
        if self.ev_in_read[b] is not None:
            h.wait_event(self.ev_in_read[b])
        timed = self.timing_h2d
        if timed:
            e0, e1 = self.D.event(True), self.D.event(True)
            e0.record(h)
        with self.D.use_stream(h):
            self.inbuf[b].copy_(self.pool[k % POOL_STEPS], non_blocking=True)
        if timed:
            e1.record(h)
            self.h2d_time.append((e0, e1))
        self.ev_h2d[b].record(h)
        self.h2d_issued = k

    def _fed(self, k):
        """input buffer of step k (its copy issued, the next step's copy issued behind it)"""
        if self.h2d_issued < k:
            self._issue_h2d(k)
        for ps in self.pstreams:
            ps.wait_event(self.ev_h2d[k % 2])
        self._issue_h2d(k + 1)  # prefetch: overlaps this step's extraction
        return self.inbuf[k % 2]

    def _record(self, si):
        import shard
        B, cap = self.B, self.cap
        S = self.sets[si]

        def unpack(rows, small):
            sm = small.cpu().numpy()
            c, cp, nm = sm[:B], sm[B:2 * B], sm[2 * B:]
            k = shard.unpack_rows(rows[0].cpu().numpy(), c, cap)
            d = shard.unpack_rows(rows[1].cpu().numpy(), c, cap)
            m = shard.unpack_rows(rows[2].cpu().numpy(), cp, cap)
            return k, d, c, m, nm

        if self.deliver == "host":
            rows, small = self.delivery.host_rows(S.dslot)
            chunks = [(self.rank, unpack([r for r, _ in rows], small))]
        else:
            own = [t.cpu().numpy() for t in (S.kps, S.desc, S.counts, S.m12, S.nmatch)]
            chunks = [(0, own)] + [(r + 1, unpack(rows, small))
                                   for r, (rows, small) in enumerate(self.delivery.received(S.dslot))]
        for r, (k, d, c, m, n) in chunks:
            for b, f in enumerate(shard.chunk_frames(S.pidx, r, self.world, self.B)):
                self.dump.add(f, count=int(c[b]), kps=k[b], desc=d[b], nmatch=int(n[b]), m12=m[b])

    def flush(self):
        """issue the match of the last extracted step"""
        if self.pending is not None:
            si, ev = self.pending
            self._match(si, self.sets[si].ev_ext, ev)
            self.pending = None

    def run(self, warmup, steps, defer=False):
        """W untimed warm-up steps, then exactly `steps` timed steps bracketed by a
        barrier + synchronisation on both sides.  defer=True (the sustained leg,
        run straight before the headline): return at once after the timed region,
        with profiling switched off, and a function that produces the leg's
        numbers later -- its stage times come from the next run()'s stage-times
        reset (profiling was off for that run's warm-up), its statistics and
        collectives run after the next leg -- so the GPU goes from this leg into
        the next one's warm-up without the host bookkeeping in between (an idle
        gap of >= 10 ms leaves the next ~60 steps ~5 % slower,
        profiles/r05_notes_ab.txt r5n)."""
        D = self.D
        # no garbage-collector pause inside a leg (collected between legs, in _finish)
        gc.disable()
        # timing events on the profiled tail only (PROFILED_TAIL / HEADLINE_PROFILED steps): every
        # timed HIP event between the step's kernels costs the stream time (r7e: events on all 20
        # headline steps 373-388k frames/s, on the last one 391.4-391.8k, one box)
        n_prof = min(steps, PROFILED_TAIL if defer else (PROF_STEPS if PROF_STEPS >= 0 else HEADLINE_PROFILED))
        evs = [(D.event(True), D.event(True)) for _ in range(n_prof)]  # created before the warm-up
        for _ in range(warmup):
            self.step()
        self.flush()
        self.delivery.finish()
        D.synchronize()
        t_idle = time.perf_counter()  # the GPU is idle from here until the timed steps start
        self.delivery.reset_stats()
        sus, self._sus = self._sus, None
        if sus is not None:
            sus["stage_ms"], sus["nb"] = {}, 0
        for e, ps in zip(self.exs, self.pstreams):
            e.sync(ps)
            e.profile(True)
            ms_i, nb_i = e.stage_times(reset=True)
            if sus is not None:  # a deferred leg's own launches (profiling was off since)
                for k, v in ms_i.items():
                    sus["stage_ms"][k] = sus["stage_ms"].get(k, 0.0) + v
                sus["nb"] = nb_i
        if self.feed == "host":
            self.timing_h2d, self.h2d_time = True, []
        # stage times over the last n_prof steps only (a deferred leg: so the next leg's
        # stage-times reset, between its warm-up and its timed steps, also reads few events)
        if n_prof < steps:
            for e in self.exs:
                e.profile(False)
        _barrier(self.world)
        D.synchronize()
        if defer and self._event_timed_ok():
            # one rank, nothing to deliver: the leg is timed by events on the streams (its
            # first step's issue on the extraction stream to its last match's end on the
            # matcher stream) and the host never waits for its end -- the next leg's
            # warm-up steps are queued behind it (r5o: no idle GPU at all between them)
            e0, e1 = D.event(True), D.event(True)
            e0.record(self.stream)
            for i in range(steps):
                if i == steps - n_prof and n_prof < steps:
                    for e in self.exs:
                        e.profile(True)
                self.step(evs[i - (steps - n_prof)] if i >= steps - n_prof else None)
            self.flush()
            e1.record(self.mstream)
            last = self.sets[(self.step_no - 1) % NSETS]
            raw = {"elapsed": None, "span": (e0, e1), "steps": steps, "evs": evs,
                   "delivery": self.delivery.report(steps), "h2d": None,
                   "kp": last.counts.float().mean(), "nm": last.nmatch.float().mean()}
            for e in self.exs:
                e.profile(False)
            self._sus = raw
            return lambda: self._finish(raw)
        marks = [D.event(True) for _ in range(steps + 1)] if STEP_TRACE[0] else None
        host_t = []
        t0 = time.perf_counter()
        self.host_gap_ms = round((t0 - t_idle) * 1e3, 3)
        for i in range(steps):
            if i == steps - n_prof and n_prof < steps:
                for e in self.exs:
                    e.profile(True)
            if marks:
                marks[i].record(self.stream)
                host_t.append(time.perf_counter())
            self.step(evs[i - (steps - n_prof)] if i >= steps - n_prof else None)
        self.flush()
        if marks:
            marks[steps].record(self.mstream)
        self.delivery.finish()
        D.synchronize()
        elapsed = time.perf_counter() - t0
        self.step_ms = [round(marks[i].elapsed_time(marks[i + 1]), 4) for i in range(steps)] if marks else None
        if marks:  # the host's issue interval of each step (a cold host CPU can starve the GPU)
            host_t.append(time.perf_counter())
            self.step_ms = {"gpu": self.step_ms,
                            "host_issue": [round((host_t[i + 1] - host_t[i]) * 1e3, 4) for i in range(steps)]}
        raw_step_ms = self.step_ms
        self.timing_h2d = False
        delivery = self.delivery.report(steps)
        delivery["ms_per_step"] = round(elapsed / steps * 1e3, 4)  # this rank's own step time
        last = self.sets[(self.step_no - 1) % NSETS]
        raw = {"elapsed": elapsed, "steps": steps, "evs": evs, "delivery": delivery, "step_ms": raw_step_ms,
               "h2d": list(self.h2d_time) if self.feed == "host" else None,
               "kp": last.counts.float().mean(), "nm": last.nmatch.float().mean()}
        if defer:
            for e in self.exs:
                e.profile(False)
            self._sus = raw
            return lambda: self._finish(raw)
        raw["stage_ms"], raw["nb"] = {}, 0
        for e, ps in zip(self.exs, self.pstreams):
            e.sync(ps)
            ms_i, nb_i = e.stage_times(reset=True)
            e.profile(False)
            for k, v in ms_i.items():
                raw["stage_ms"][k] = raw["stage_ms"].get(k, 0.0) + v
            raw["nb"] = nb_i
        return self._finish(raw)

    def _event_timed_ok(self):
        """a leg may end without a host wait (run(defer=True)): one rank, nothing to
        deliver (gpu0 at N = 1 moves nothing), frames already in HBM"""
        return self.D.cuda and self.world == 1 and self.deliver == "gpu0" and self.feed == "hbm"

    def _finish(self, raw):
        """a timed leg's numbers: max elapsed / summed frames over ranks, the
        delivery numbers gathered to rank 0, stage and match times, the pyramid's
        achieved bandwidth"""
        steps, elapsed = raw["steps"], raw["elapsed"]
        if self._sus is None:  # no leg handed over to a next one: collect now, outside any timed region
            gc.enable()
            gc.collect()
        if elapsed is None:  # an event-timed leg
            self.D.synchronize()
            elapsed = raw["span"][0].elapsed_time(raw["span"][1]) / 1e3
            raw["delivery"]["ms_per_step"] = round(elapsed / steps * 1e3, 4)
        elapsed, frames_total = aggregate(elapsed, self.B * steps, device=self.dev)
        delivery = gather_delivery_stats(raw["delivery"], self.world, self.dev)
        _barrier(self.world)
        if self.dump is not None:
            self.dump.write()
        # stage times summed over the sub-batches (per launch: a stage's duration on its
        # stream; with P > 1 sub-batches overlap, so the sum exceeds the step)
        per_step = {k: v / max(raw.get("nb", 0), 1) for k, v in raw.get("stage_ms", {}).items()}
        # the matcher's time beside the extraction: the leg's last match (flushed after the
        # last extraction) runs alone, so it counts only when it is the one timed
        mev = raw["evs"][:-1] if len(raw["evs"]) > 1 else raw["evs"]
        per_step["match"] = sum(a.elapsed_time(b) for a, b in mev) / max(len(mev), 1)
        pyr_bytes = pyramid_bytes_per_frame(self.ex.level_sizes) * self.B
        pyr_s = per_step.get("pyramid", 0.0) / 1e3
        achieved = pyr_bytes / pyr_s / 1e9 if pyr_s > 0 else None
        h2d = None
        if raw["h2d"]:
            ms = [a.elapsed_time(b) for a, b in raw["h2d"]]  # the copies issued inside the timed region
            nbytes = self.inbuf[0].numel()
            h2d = {"bytes_per_step": int(nbytes), "ms_per_copy_mean": round(float(np.mean(ms)), 4),
                   "gb_per_s": round(nbytes / (float(np.mean(ms)) / 1e3) / 1e9, 2), "copies": len(ms)}
        return {"fps": frames_total / elapsed, "elapsed": elapsed, "per_step": per_step, "pyr_bytes": pyr_bytes,
                "achieved": achieved, "keypoints": float(raw["kp"].item()), "matches": float(raw["nm"].item()),
                "frames_total": frames_total, "delivery": delivery, "h2d": h2d, "step_ms": raw.get("step_ms")}

    def close(self):
        self.delivery.close()


    def parity_timed(self):
        """The timed path's own outputs against the oracle (untimed, after run()):
        in the last step's output set -- written by the very extractor, batch size and
        kernel configuration that was timed -- frames 0, 1, B-2 and B-1 (keypoints as
        bits, all 7 fields, and descriptors) and the matches of pairs (0, 1) and
        (B-2, B-1); at N = 1 also pair 0, whose F1 is the previous step's last frame
        read in place from the previous output set (src/Tracking.cpp:768-769)."""
        import orbgpu
        import orbref
        try:
            self.D.synchronize()
            B, W = self.B, self.W
            S = self.sets[(self.step_no - 1) % NSETS]
            ex = orbref.Extractor(nfeatures=self.NF)

            def ref(pidx, b):
                return ex.extract(np.ascontiguousarray(self.pool[pidx][b, :, :W].cpu().numpy()))

            def same(kd, k, d):
                return len(kd[0]) == len(k) and kd[0].tobytes() == k.tobytes() and np.array_equal(kd[1], d)

            idx = sorted({0, 1, B - 2, B - 1} & set(range(B)))
            R = {b: ref(S.pidx, b) for b in idx}
            kps, desc, cnt = S.kps.cpu().numpy(), S.desc.cpu().numpy(), S.counts.cpu().numpy()
            m12, nm = S.m12.cpu().numpy(), S.nmatch.cpu().numpy()
            got = {b: (orbgpu.keypoints_from_raw(kps[b, :cnt[b]]), desc[b, :cnt[b]]) for b in idx}
            ok_frames = {b: bool(same(got[b], *R[b])) for b in idx}

            def pair_ok(b, f1):
                n_r, m_r, _ = orbref.search_for_initialization(f1[0], f1[1], R[b][0], R[b][1], W, self.H)
                return bool(int(nm[b]) == n_r and np.array_equal(m12[b, :len(f1[0])], m_r))

            ok_pairs = {f"({b - 1},{b})": pair_ok(b, R[b - 1]) for b in idx if b - 1 in R}
            if self.world == 1 and self.step_no >= 2 and 0 in R:
                P = self.sets[(self.step_no - 2) % NSETS]
                ok_pairs["(prev step's B-1, 0)"] = pair_ok(0, ref(P.pidx, B - 1))
            ok = all(ok_frames.values()) and all(ok_pairs.values())
            return {"ok": ok, "frames": ok_frames, "pairs": ok_pairs,
                    "from": f"output set of the last timed step (batch {B}, the timed extractor and matcher)"}
        except Exception as e:  # report, never hide
            return {"ok": False, "error": str(e)}


# ---------------------------------------------------------------------------
# stereo stream: per pair extract L+R + ComputeStereoMatches, sharded by pair
# ---------------------------------------------------------------------------

class StereoBench:
    """Stereo Frames (src/Frame.cpp:66-127) over one sharded pair stream: at
    step s rank r owns pairs [(s*N + r)*P, +P); the L and R images of its
    pairs are extracted in one batch (frames 2p, 2p+1) and
    Frame::ComputeStereoMatches runs on them; outputs go to rank 0."""

    def __init__(self, og, D: Dev, config, P, rank, world, stream, dump=None):
        import shard
        import synth
        W, H, NF, _ = CONFIGS[config]
        self.bf, base_px = STEREO[config]
        self.og, self.D, self.config = og, D, config
        self.W, self.H, self.NF, self.P, self.rank, self.world = W, H, NF, P, rank, world
        dev = D.device
        self.dev, self.stream = dev, stream
        self.pitch = (W + 15) // 16 * 16
        self.ex = og.Extractor(nfeatures=NF, width=W, height=H, max_batch=2 * P)
        cap = self.cap = self.ex.max_keypoints
        self.pool = [synth.torch_stereo_stream(P, W, H, base_px, device=dev, pitch=self.pitch,
                                               t0=shard.chunk_frames(s, rank, world, P)[0])
                     for s in range(POOL_STEPS)]
        self.sets = []
        for _ in range(2):
            self.sets.append((torch.zeros((2 * P, cap, 7), dtype=torch.float32, device=dev),
                              torch.zeros((2 * P, cap, 32), dtype=torch.uint8, device=dev),
                              torch.zeros(2 * P, dtype=torch.int32, device=dev),
                              torch.zeros((P, cap), dtype=torch.float32, device=dev),
                              torch.zeros((P, cap), dtype=torch.float32, device=dev)))
        self.gather = shard.OwnerGather(rank, world, list(self.sets[0]))
        self.ev_done = [None, None]
        self.step_no = 0
        self.dump = _Dumper(dump, f"stereo_{W}x{H}") if (dump and rank == 0) else None
        self.dump_all = bool(dump)

    def step(self):
        st = self.stream
        si = self.step_no % 2
        kps, desc, counts, ur, dp = self.sets[si]
        self.gather.finish(si)
        pidx = self.step_no % POOL_STEPS
        imgs = self.pool[pidx]
        self.ex.extract_batch(imgs, kps, desc, counts, stream=st, row_step=self.pitch, frame_step=self.pitch * self.H)
        self.og.stereo_matches_batch(self.ex, imgs, self.P, kps, desc, counts, self.bf, 0.0, ur, dp, stream=st,
                                     row_step=self.pitch, frame_step=self.pitch * self.H)
        with self.D.use_stream(st):
            self.gather.start(si, [kps, desc, counts, ur, dp])
        if self.dump_all:
            self.gather.finish()
            if self.dump is not None:
                self._record(si, pidx)
        self.step_no += 1

    def _record(self, si, pidx):
        import shard
        own = [t.cpu() for t in self.sets[si]]
        chunks = [(0, own)] + [(r + 1, [t.cpu() for t in ts]) for r, ts in enumerate(self.gather.received(si))]
        for r, (k, d, c, u, z) in chunks:
            for p, pair in enumerate(shard.chunk_frames(pidx, r, self.world, self.P)):
                self.dump.add(pair, count=c[2 * p:2 * p + 2].numpy(), kps=k[2 * p:2 * p + 2].numpy(),
                              desc=d[2 * p:2 * p + 2].numpy(), uright=u[p].numpy(), depth=z[p].numpy())

    def run(self, warmup, steps):
        D = self.D
        for _ in range(warmup):
            self.step()
        self.gather.finish()
        D.synchronize()
        _barrier(self.world)
        D.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            self.step()
        self.gather.finish()
        D.synchronize()
        elapsed = time.perf_counter() - t0
        elapsed, pairs_total = aggregate(elapsed, self.P * steps, device=self.dev)
        _barrier(self.world)
        if self.dump is not None:
            self.dump.write()
        kps, desc, counts, ur, dp = self.sets[(self.step_no - 1) % 2]
        n = counts.cpu().numpy()
        urh = ur.cpu().numpy()
        with_depth = float(np.mean([(urh[p, :n[2 * p]] >= 0).mean() if n[2 * p] else 0.0 for p in range(self.P)]))
        return {"pairs_per_s": pairs_total / elapsed, "elapsed": elapsed, "pairs_total": pairs_total,
                "keypoints_per_frame": float(n.mean()), "left_keypoints_with_depth": with_depth}

    def parity_timed(self):
        """The timed path's own outputs against the oracle (untimed, after run()):
        in the last step's output set -- written by the timed extractor (batch
        2P) and the timed ComputeStereoMatches launch (P pairs, so the kernel's
        S-blocks-per-pair split of csrc/stereo.hip is the timed one) -- pairs 0,
        1, P-2 and P-1: both frames' keypoints (all 7 fields as bits) and
        descriptors, and uRight / depth as bits against the C++ oracle's stereo
        Frame (oracle/stereo_ref.cpp, src/Frame.cpp:540-748).  Rank 0's own
        pairs."""
        import orbgpu
        import orbref
        try:
            self.D.synchronize()
            P, W = self.P, self.W
            si = (self.step_no - 1) % 2
            pidx = (self.step_no - 1) % POOL_STEPS
            kps, desc, counts, ur, dp = [t.cpu().numpy() for t in self.sets[si]]
            exL, exR = orbref.Extractor(nfeatures=self.NF), orbref.Extractor(nfeatures=self.NF)
            imgs = self.pool[pidx]
            out = {}
            for p in sorted({0, 1, P - 2, P - 1} & set(range(P))):
                left = np.ascontiguousarray(imgs[2 * p, :, :W].cpu().numpy())
                right = np.ascontiguousarray(imgs[2 * p + 1, :, :W].cpu().numpy())
                kl, dl, kr, dr, ur_r, dp_r = orbref.stereo_frame(exL, exR, left, right, self.bf)
                nl, nr = int(counts[2 * p]), int(counts[2 * p + 1])
                gl = orbgpu.keypoints_from_raw(kps[2 * p, :nl])
                gr = orbgpu.keypoints_from_raw(kps[2 * p + 1, :nr])
                frames_ok = (nl == len(kl) and nr == len(kr) and gl.tobytes() == kl.tobytes() and
                             gr.tobytes() == kr.tobytes() and np.array_equal(desc[2 * p, :nl], dl) and
                             np.array_equal(desc[2 * p + 1, :nr], dr))
                n = min(nl, len(ur_r))
                stereo_ok = (n == len(ur_r) and ur[p, :n].view(np.uint32).tobytes() == ur_r.view(np.uint32).tobytes()
                             and dp[p, :n].view(np.uint32).tobytes() == dp_r.view(np.uint32).tobytes())
                out[f"pair {p}"] = {"frames": bool(frames_ok), "uright_depth": bool(stereo_ok),
                                    "with_depth": int((ur_r >= 0).sum())}
            ok = all(v["frames"] and v["uright_depth"] for v in out.values())
            return {"ok": ok, "pairs": out,
                    "from": f"output set of the last timed step ({P} pairs, the timed extractor and stereo launch)"}
        except Exception as e:  # report, never hide
            return {"ok": False, "error": str(e)}

    def summary(self, r, steps):
        return {"pairs_per_s": round(r["pairs_per_s"], 1), "ms_per_step": round(r["elapsed"] / steps * 1e3, 3),
                "pairs_per_gpu_per_step": self.P, "n_gpus": self.world, "width": self.W, "height": self.H,
                "nfeatures": self.NF, "keypoints_per_frame": round(r["keypoints_per_frame"], 1),
                "left_keypoints_with_depth": round(r["left_keypoints_with_depth"], 3),
                "workload": CONFIGS[self.config][3] + f" (bf {self.bf:.3f})",
                "parallelism": f"contiguous pair chunks x{self.world}, L/R of a pair on one rank, "
                               f"per-step gather to rank 0"}


# ---------------------------------------------------------------------------
# CPU baselines (oracle on the host cores; rank 0 at N=1 only)
# ---------------------------------------------------------------------------

def _cgroup_cpu_quota():
    """CPUs granted by the cgroup CPU controller (cpu.max of cgroup v2, or
    cpu.cfs_quota_us / cpu.cfs_period_us of v1) on this process's cgroup
    path, or None when no quota is set or readable."""
    paths = []
    try:
        for line in open("/proc/self/cgroup"):
            parts = line.strip().split(":", 2)
            if len(parts) == 3 and (parts[1] == "" or "cpu" in parts[1].split(",")):
                paths.append((parts[1] == "", parts[2]))
    except OSError:
        pass
    for v2, rel in paths + [(True, "/"), (False, "/")]:
        root = "/sys/fs/cgroup" if v2 else "/sys/fs/cgroup/cpu"
        rel = rel.lstrip("/")
        # walk up from the process's own cgroup: a limit set on an ancestor applies
        while True:
            d = os.path.join(root, rel)
            try:
                if v2:
                    q, per = open(os.path.join(d, "cpu.max")).read().split()[:2]
                    if q != "max":
                        return float(q) / float(per), os.path.join(d, "cpu.max")
                else:
                    q = int(open(os.path.join(d, "cpu.cfs_quota_us")).read())
                    per = int(open(os.path.join(d, "cpu.cfs_period_us")).read())
                    if q > 0:
                        return q / per, os.path.join(d, "cpu.cfs_quota_us")
            except (OSError, ValueError):
                pass
            if not rel:
                break
            rel = os.path.dirname(rel)
    return None


def cpu_info():
    """The CPU share the all-core baseline runs on: the cgroup CPU quota when
    one is set (rounded down, at least 1), else the affinity mask; both are
    reported, with OMP_NUM_THREADS (the box's documented share) beside them."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    quota = _cgroup_cpu_quota()
    if quota is not None:
        threads, source = max(1, min(avail, int(quota[0]))), f"cgroup CPU quota ({quota[1]})"
    elif omp > 0:
        threads, source = min(avail, omp), "OMP_NUM_THREADS (no cgroup CPU quota readable)"
    else:
        threads, source = avail, "affinity mask (no cgroup CPU quota, no OMP_NUM_THREADS)"
    return {"cpu_model": model, "host_cpus": os.cpu_count(), "cpus_available_to_process": avail,
            "cgroup_cpu_quota": None if quota is None else round(quota[0], 2), "omp_num_threads": omp or None,
            "threads_used": max(1, threads), "threads_source": source}


def _timed_threads(fn, threads, seconds):
    """fn(j, stop_at, out) per thread; returns (units, elapsed)."""
    res = []
    t0 = time.perf_counter()
    stop = t0 + seconds
    ths = [threading.Thread(target=fn, args=(j, stop, res)) for j in range(threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return sum(res), time.perf_counter() - t0


def cpu_baseline_mono(frames_np, W, H, nf, seconds, info):
    """Oracle extract + match (t-1, t) on host cores: one extractor per thread."""
    import orbref

    def run(j, stop_at, out, step=1):
        ex = orbref.Extractor(nfeatures=nf)
        prev = None
        n = 0
        i = j
        while time.perf_counter() < stop_at:
            k, d = ex.extract(frames_np[i % len(frames_np)])
            if prev is not None:
                orbref.search_for_initialization(prev[0], prev[1], k, d, W, H)
            prev = (k, d)
            n += 1
            i += step
        out.append(n)

    n1, e1 = _timed_threads(run, 1, seconds / 3)
    T = info["threads_used"]
    nN, eN = _timed_threads(lambda j, s, o: run(j, s, o, T), T, 2 * seconds / 3)
    return {"value": round(nN / eN, 2), "unit": "frames/s", "cores": T, "kind": "port",
            "single_thread_value": round(n1 / e1, 2), "single_thread_ms_per_frame": round(1e3 * e1 / max(n1, 1), 2),
            "cpu_model": info["cpu_model"], "host_cpus": info["host_cpus"],
            "cpus_available_to_process": info["cpus_available_to_process"],
            "cgroup_cpu_quota": info["cgroup_cpu_quota"], "omp_num_threads": info["omp_num_threads"],
            "threads_used": T, "threads_source": info["threads_source"],
            "note": "scalar C++ restatement of the reference's arithmetic (oracle/orbref.cpp: full corner score on "
                    "every pixel, no SIMD); the reference itself uses OpenCV 2.4's SSE FAST/resize/blur and would "
                    "be faster per core. cores = threads_used: the cgroup CPU quota when one is set, else "
                    "OMP_NUM_THREADS, else the affinity mask (threads_source says which); the reference's own "
                    "timing mode is single_thread_value (mono_tum.cc:79-120, one thread per sequence)",
            "sample": f"oracle extract+match on {len(frames_np)} distinct synthetic {W}x{H} frames, "
                      f"~{seconds:.0f}s bounded ({n1} frames on 1 thread, {nN} on {T})"}


def cpu_baseline_stereo(config, seconds, info):
    """Oracle stereo Frame (extract L, R + ComputeStereoMatches, C++) on host cores."""
    import orbref
    import synth
    W, H, NF, _ = CONFIGS[config]
    bf, base_px = STEREO[config]
    pairs = synth.stereo_stream(4, W, H, 0x5E7, base_px)

    def run(j, stop_at, out, step=1):
        ex = [orbref.Extractor(nfeatures=NF), orbref.Extractor(nfeatures=NF)]
        n, i = 0, j
        while time.perf_counter() < stop_at:
            lr = pairs[i % len(pairs)]
            orbref.stereo_frame(ex[0], ex[1], lr[0], lr[1], bf)
            n += 1
            i += step
        out.append(n)

    n1, e1 = _timed_threads(run, 1, seconds / 3)
    T = info["threads_used"]
    nN, eN = _timed_threads(lambda j, s, o: run(j, s, o, T), T, 2 * seconds / 3)
    return {"value": round(nN / eN, 2), "unit": "pairs/s", "cores": T, "kind": "port",
            "single_thread_value": round(n1 / e1, 2), "single_thread_ms_per_pair": round(1e3 * e1 / max(n1, 1), 2),
            "sample": f"oracle stereo Frame (extract L + R, ComputeStereoMatches; oracle/orbref.cpp) on 4 synthetic "
                      f"{W}x{H} pairs, ~{seconds:.0f}s bounded ({n1} pairs on 1 thread, {nN} on {T})"}


def cpu_baseline_mono_geometry(config, seconds, info):
    W, H, NF, _ = CONFIGS[config]
    import synth
    frames = synth.mono_stream(6, W, H)
    r = cpu_baseline_mono(frames, W, H, NF, seconds, info)
    return {k: r[k] for k in ("value", "unit", "cores", "kind", "single_thread_value", "single_thread_ms_per_frame",
                              "sample")}


# ---------------------------------------------------------------------------
# drop-in latency (the C++ classes, as Tracking calls them)
# ---------------------------------------------------------------------------

class DropIn:
    """The drop-in C++ classes timed as the reference's threads call them:
    tests/cpp/adapter_main (the include/orbslam2_amd/ headers over
    liborbgpu.so) with ADAPTER_REPS / ADAPTER_TIME_LOG, at per-frame sizes:
      * ORBextractor::operator() on a 640x480 frame (Frame::ExtractORB), with
        and without the mvImagePyramid host copy;
      * ORBmatcher::SearchForInitialization (Tracking.cpp:769);
      * the stereo Frame (two extractors on two threads + ComputeStereoMatches
        on their HBM pyramids) at 752x480 / 1200 features;
      * ORBmatcher::SearchByProjection(F, localMPs, th) (Tracking.cpp:1560,
        ~2000 local MapPoints) and (F, LastFrame) (:1152);
      * ORBmatcher::SearchByBoW(KF, F) (:990) and (KF1, KF2) (LoopClosing:311);
      * PnPsolver::iterate(5) of a fresh solver (Relocalization, :1822);
      * Initializer::Initialize (MonocularInitialization, :790).
    The scenarios come from synth.py (FeatureVectors and isInFrustum flags
    from the GPU library itself)."""

    def __init__(self, workdir: Path, reps: int = 100):
        self.dir, self.reps = workdir, reps
        self.scen = {}

    def _run(self, *args, timeout=300):
        exe = ROOT / "tests" / "cpp" / "adapter_main"
        env = dict(os.environ, ADAPTER_REPS=str(self.reps), ADAPTER_TIME_LOG=str(self.dir / "times.jsonl"))
        r = subprocess.run([str(exe), *map(str, args)], capture_output=True, text=True, timeout=timeout, env=env)
        if r.returncode != 0:
            raise RuntimeError(f"adapter_main {args[0]}: rc {r.returncode}: {r.stderr[-400:]}")

    def run(self):
        sys.path.insert(0, str(ROOT))
        import bow
        import proj
        import synth
        from tools import adapter_io as aio
        d = self.dir
        d.mkdir(parents=True, exist_ok=True)
        (d / "times.jsonl").unlink(missing_ok=True)
        # extraction + SearchForInitialization (640x480, 1000 features)
        fr = synth.mono_stream(2, 640, 480)
        self.scen["mono"] = fr
        for k in range(2):
            (d / f"f{k}.raw").write_bytes(fr[k].tobytes())
        self._run("extract", 640, 480, 1000, d / "f0.raw", d / "f1.raw", d / "extract.out")
        # stereo Frame (EuRoC geometry)
        bf = float(np.float32(STEREO["euroc_stereo"][0]))
        st = synth.stereo_stream(1, 752, 480, 0x5E7, STEREO["euroc_stereo"][1])[0]
        self.scen["stereo"] = (st, bf)
        (d / "l.raw").write_bytes(st[0].tobytes())
        (d / "r.raw").write_bytes(st[1].tobytes())
        self._run("stereo", 752, 480, 1200, repr(bf), d / "l.raw", d / "r.raw", d / "stereo.out")
        # SearchByProjection: local map (LOCAL, th 1 as Tracking with a recent relocalisation off)
        tgt, pts = synth.projection_scenario(2000, 600, 91)
        fl, tr, lv = proj.is_in_frustum(tgt, pts, 0.5)
        pts_l = dict(pts, flags=fl, track=tr, track_level=lv)
        self.scen["proj_local"] = (tgt, pts_l)
        (d / "proj0.in").write_bytes(aio.proj_blob(1.0, dict(nnratio=0.8), tgt, pts_l, tgt["Tcw"]))
        self._run("proj", 0, d / "proj0.in", d / "proj0.out")
        tgt2, pts2 = synth.projection_scenario(1000, 400, 92)
        last = np.asarray(tgt2["Tcw"], np.float32).copy()
        last[:3, 3] += np.float32(0.05)
        self.scen["proj_last"] = (tgt2, pts2, last)
        (d / "proj2.in").write_bytes(aio.proj_blob(15.0, dict(check_ori=True, mono=True), tgt2, pts2, last))
        self._run("proj", 2, d / "proj2.in", d / "proj2.out")
        # SearchByBoW: 1000-feature frames over a k=10, L=6 vocabulary (ORBvoc.txt's shape; GPU
        # transform, levelsup 4: the FeatureVector nodes are the 100 level-2 nodes)
        par, leaf, vdesc, w = synth.synthetic_vocabulary_fast(10, 6, 7)
        voc = bow.Vocabulary.from_arrays(10, 6, 0, 0, par, leaf, vdesc, w)
        d1, a1, d2, a2 = synth.bow_frame_pair(vdesc[leaf == 1], 1000, 0.6, seed=41)
        fv1, fv2 = voc.transform(d1, 4)[3], voc.transform(d2, 4)[3]
        rng = np.random.default_rng(23)
        s1 = rng.choice([0, 1, 1, 1, 1, 1, 1, 2], 1000).astype(np.uint8)
        s2 = rng.choice([0, 1, 1, 1, 1, 1, 1, 2], 1000).astype(np.uint8)
        self.scen["bow"] = (par, leaf, vdesc, w, d1, a1, s1, d2, a2, s2)
        (d / "bow.in").write_bytes(aio.bow_blob(0.7, True, (d1, a1, s1, fv1), (d2, a2, s2, fv2)))
        self._run("bow", d / "bow.in", d / "bow.out")
        # PnPsolver: 300 correspondences, half inliers (Relocalization's SearchByBoW output size)
        P = synth.pnp_problem(300, 0.5, seed=80)
        self.scen["pnp"] = P
        blob, _, _ = aio.pnp_frame(P, seed=1)
        (d / "pnp.in").write_bytes(struct.pack("<I", 0) + blob)
        self._run("pnp", d / "pnp.in", d / "pnp.out")
        # Initializer: 1000 matches
        kp1, kp2, m12 = aio.init_scene(1000, 3)
        self.scen["init"] = (kp1, kp2, m12)
        (d / "init.in").write_bytes(aio.init_blob(aio.K_TUM, kp1, kp2, m12))
        self._run("init", d / "init.in", d / "init.out")
        out = {}
        for line in (d / "times.jsonl").read_text().splitlines():
            r = json.loads(line)
            out[r.pop("op")] = {k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}
        return out

    def cpu_oracle(self, ops):
        """Single-thread time of the oracle doing the same call on the same
        scenario (C++ oracle where it exists, else the numpy/Python one)."""
        import orbref
        res = {}

        def t(fn, n=3):
            ts = []
            for _ in range(n):
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            return round(1e6 * float(np.median(ts)), 1)

        fr = self.scen["mono"]
        ex = orbref.Extractor(1000)
        k0, d0 = ex.extract(fr[0])
        k1, d1 = ex.extract(fr[1])
        res["ORBextractor::operator()"] = (t(lambda: ex.extract(fr[1])), "C++ oracle (scalar)")
        res["ORBmatcher::SearchForInitialization"] = (
            t(lambda: orbref.search_for_initialization(k0, d0, k1, d1, 640, 480)), "C++ oracle")
        st, bf = self.scen["stereo"]
        eL, eR = orbref.Extractor(1200), orbref.Extractor(1200)
        kl, dl, kr, dr, _, _ = orbref.stereo_frame(eL, eR, st[0], st[1], bf)
        res["stereo Frame: ORBextractor L || R + ComputeStereoMatches"] = (
            t(lambda: orbref.stereo_frame(eL, eR, st[0], st[1], bf)), "C++ oracle, L and R sequential")
        res["stereo Frame: ORBextractor::ExtractPair (both frames from one thread) + ComputeStereoMatches"] = \
            res["stereo Frame: ORBextractor L || R + ComputeStereoMatches"]
        res["ComputeStereoMatches"] = (t(lambda: orbref.stereo_matches(eL, eR, kl, dl, kr, dr, bf)), "C++ oracle")
        tgt, pts = self.scen["proj_local"]
        res["ORBmatcher::SearchByProjection(F, vpLocalMapPoints, th)"] = (
            t(lambda: orbref.search_by_projection(0, tgt, pts, 1.0, nnratio=0.8), 5),
            "C++ oracle (oracle/proj_ref.cpp, equal to proj_ref.py)")
        tgt2, pts2, last = self.scen["proj_last"]
        res["ORBmatcher::SearchByProjection(F, LastFrame, th, bMono)"] = (
            t(lambda: orbref.search_by_projection(2, tgt2, pts2, 15.0, check_ori=True, mono=True, last_Tcw=last),
              5), "C++ oracle (oracle/proj_ref.cpp, equal to proj_ref.py)")
        par, leaf, vdesc, w, d1_, a1, s1, d2_, a2, s2 = self.scen["bow"]
        cv = orbref.Vocabulary(10, 6, par, leaf, vdesc, w)
        res["ORBmatcher::SearchByBoW(KF1, KF2)"] = (
            t(lambda: orbref.search_by_bow_kf_kf(cv, d1_, a1, s1 == 1, d2_, a2, s2 == 1, 0.7)),
            "C++ oracle (includes the two BoW transforms)")
        import loop_ref
        av = loop_ref.ArrayVocabulary(10, 6, 0, 0, par, leaf, vdesc, w)
        f1, f2 = av.transform(d1_, 4)[3], av.transform(d2_, 4)[3]
        res["ORBmatcher::SearchByBoW(KF, F)"] = (
            t(lambda: orbref.search_by_bow_kf_f(f1, d1_, a1, s1 == 1, f2, d2_, a2, 0.7, True), 5),
            "C++ oracle (oracle/loop_ref.cpp, FeatureVectors given as in TrackReferenceKeyFrame)")
        P = self.scen["pnp"]
        maxerr = (P["sigma2"] * np.float32(5.991)).astype(np.float32)
        rng = np.random.default_rng(0)
        # a fresh solver's iterate(5) runs hypotheses until the first Refine
        # that passes (the || loop condition, up to mRansacMaxIts = 300)
        smp = np.array([rng.choice(len(P["P2"]), 4, replace=False) for _ in range(300)], np.int32)
        o = orbref.pnp_ransac_call(P["P3w"], P["P2"], maxerr, P["cam"], 150, 0, smp)
        res["PnPsolver::iterate(5)"] = (
            t(lambda: orbref.pnp_ransac_call(P["P3w"], P["P2"], maxerr, P["cam"], 150, 0, smp), 5),
            f"C++ oracle (oracle/pnp_ref.cpp, equal to pnp_ref.py): {o['consumed']} hypotheses + Refine until "
            f"the first pass, found={o['found']}")
        return {op: {"cpu_oracle_single_thread_us": v[0], "cpu_oracle_kind": v[1]} for op, v in res.items()
                if op in ops}


def drop_in_latency(with_cpu=True):
    import tempfile
    with tempfile.TemporaryDirectory(prefix="orbgpu_dropin_") as td:
        di = DropIn(Path(td))
        try:
            ops = di.run()
        except Exception as e:  # report, never hide
            return {"error": str(e)}
        if with_cpu:
            try:
                for op, v in di.cpu_oracle(ops).items():
                    ops[op].update(v)
            except Exception as e:
                ops["cpu_oracle_error"] = str(e)
    return {"unit": "us per call (wall, steady_clock around the class member call, median of repetitions)",
            "path": "tests/cpp/adapter_main: include/orbslam2_amd/*.h over liborbgpu.so, host inputs and outputs, "
                    "per-thread stream / arena / pinned staging (no hipMalloc, hipFree or device-wide sync per call)",
            "ops": ops}


# ---------------------------------------------------------------------------
# loop burst (SURVEY config 5)
# ---------------------------------------------------------------------------

LOOP_MIXES = {
    # name: (inlier fractions per candidate slot, outlier fractions, fixed scale, description)
    "bench": (0.4, 0.6, False, "40% true correspondences, the rest geometric outliers"),
    "several_rounds": ([0.0, 0.0, 0.03, 0.4, 0.4], [0.0, 0.08, 0.05, 0.5, 0.5], False,
                       "unrelated / false loop / weak / two true loops with 50% outliers"),
    "false_loops": (0.0, [0.0, 0.06, 0.08, 0.1, 0.05], False,
                    "false loops only: every solver runs to its maximum iterations, no Sim3 returned"),
}


class LoopLeg:
    """ComputeSim3 bursts (src/LoopClosing.cpp:273-356): 100 queries x 5
    candidates per mix, queries round-robin over the ranks."""

    def __init__(self, rank, world, dev, nq_total=100, nc=5):
        import bow
        import synth
        self.rank, self.world, self.dev, self.nq, self.nc = rank, world, dev, nq_total, nc
        t_set = time.perf_counter()
        self.voc_arrays = synth.synthetic_vocabulary_fast(10, 6, 0x70C)
        p, l, d, w = self.voc_arrays
        vpath = Path(os.environ.get("TMPDIR", "/tmp")) / f"orbgpu_voc_k10_L6_{os.getpid()}.txt"
        synth.write_vocabulary_text_fast(vpath, 10, 6, 0, 0, p, l, d, w)
        t_load = time.perf_counter()
        self.voc = bow.Vocabulary.load_text(str(vpath))
        self.t_load = time.perf_counter() - t_load
        vpath.unlink()
        self.t_voc = time.perf_counter() - t_set
        self.scenes = {}

    def scene(self, mix):
        import synth
        if mix not in self.scenes:
            fr, ofr, fix, _ = LOOP_MIXES[mix]
            p, l, d, w = self.voc_arrays
            seed = {"bench": 55, "several_rounds": 56, "false_loops": 57}[mix]
            self.scenes[mix] = synth.loop_burst_scene(self.nq, self.nc, d[l == 1], n_kp=1000, inlier_frac=fr,
                                                      outlier_frac=ofr, seed=seed, fix_scale=fix)
        return self.scenes[mix]

    def run(self, mix, steps, warmup):
        import loop
        nq, nc, dev = self.nq, self.nc, self.dev
        scene = self.scene(mix)
        fix = LOOP_MIXES[mix][2]
        my_q = list(range(self.rank, nq, self.world))
        kf_ids = []
        for q in my_q:
            kf_ids += [q] + [nq + q * nc + c for c in range(nc)]
        sel = np.array(kf_ids)
        kfs = loop.Keyframes(scene["desc"][sel], scene["angle"][sel], scene["octave"][sel], scene["valid"][sel],
                             scene["mp_world"][sel], scene["Tcw"][sel], scene["K"], scene["sigma2"], device=dev)
        st = torch.cuda.current_stream(dev)
        kfs.compute_bow(self.voc, stream=st)
        queries = [(j * (1 + nc), [j * (1 + nc) + 1 + c for c in range(nc)], 1000 + q) for j, q in enumerate(my_q)]
        lb = loop.LoopBurst(kfs, queries, fix_scale=fix)
        for _ in range(warmup):
            lb.step(st)
        torch.cuda.synchronize(dev)
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(steps)]
        _barrier(self.world)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(steps):
            ev[i][0].record(st)
            lb.search_by_bow(st)
            ev[i][1].record(st)
            lb.setup(st)
            ev[i][2].record(st)
            lb.compute_sim3(st)
            ev[i][3].record(st)
        torch.cuda.synchronize(dev)
        elapsed = time.perf_counter() - t0
        elapsed, pairs_total = aggregate(elapsed, len(my_q) * nc * steps, device=dev)
        stage = {k: sum(e[j].elapsed_time(e[j + 1]) for e in ev) / steps
                 for j, k in enumerate(["search_by_bow", "sim3_setup", "compute_sim3"])}
        res = lb.query_results()
        states = lb.candidate_states()
        # the timed burst's own outputs against the oracle (untimed): rank 0's first and last query
        self.last_parity = self.parity_timed(lb, mix, my_q, res, states) if self.rank == 0 else None
        n_kp = 1000
        npairs = len(my_q) * nc
        sbb_bytes = 2 * n_kp * (32 + 4 + 1 + 4 + 4) + n_kp * 4
        kern_bytes = {"search_by_bow": sbb_bytes * npairs,
                      "sim3_setup": npairs * n_kp * (4 + 2 * (12 + 1 + 4)) + npairs * 300 * 36,
                      "compute_sim3": sum(max(s.n, 0) for s in states) * 36}
        dominant = max(stage, key=stage.get)
        achieved = kern_bytes[dominant] / (stage[dominant] / 1e3) / 1e9
        return {"kf_pairs_per_s": round(pairs_total / elapsed, 1), "ms_per_step": round(elapsed / steps * 1e3, 4),
                "kf_pairs_per_step": pairs_total // steps, "mix": LOOP_MIXES[mix][3],
                "stages_ms_per_step_rank0": {k: round(v, 4) for k, v in stage.items()},
                "dominant_kernel": dominant,
                "dominant_hbm_frac": round(achieved / HBM_PEAK_GBS, 5),
                "queries_matched_rank0": int(sum(r.matched >= 0 for r in res)),
                "mean_round_of_match_rank0": round(float(np.mean([r.round for r in res if r.matched >= 0] or [0])), 2),
                "ransac_iterations_per_step_rank0": int(sum(r.hypotheses for r in res)),
                "mean_searchbybow_matches": round(float(lb.nmatches.float().mean().item()), 1),
                "parity_vs_oracle": self.last_parity}

    def oracle_vocabulary(self):
        import orbref
        if getattr(self, "_ovoc", None) is None:
            p, l, d, w = self.voc_arrays
            self._ovoc = orbref.Vocabulary(10, 6, p, l, d, w)
        return self._ovoc

    def parity_timed(self, lb, mix, my_q, res, states):
        """The timed burst's outputs (the last timed step's LoopBurst: the batch
        size, kernels and launch configuration that were timed) against the C++
        oracle (oracle/loop_ref.cpp, random_r stream per query) for this rank's
        first and last query (queries 0 and 99 at N = 1): every candidate's
        SearchByBoW(KF, KF) match count and vpMatches12, the solvers' (N, max
        iterations, iterations, best inliers), the matched candidate, round,
        inlier count, hypotheses and draws, the stream after the draws, and the
        returned Sim3 within tests/test_ransac.py's tolerance
        (src/LoopClosing.cpp:273-356)."""
        import ctypes
        import orbgpu
        import orbref
        import ransac
        try:
            scene = self.scene(mix)
            fix = LOOP_MIXES[mix][2]
            nq, nc = self.nq, self.nc
            voc = self.oracle_vocabulary()
            match, nm = lb.match.cpu().numpy(), lb.nmatches.cpu().numpy()
            out = {}
            for j in sorted({0, len(my_q) - 1}):
                q = my_q[j]
                r = orbref.compute_sim3_query_ex(voc, scene, q, [nq + q * nc + c for c in range(nc)], 1000 + q, fix)
                g = res[j]
                chk = {}
                chk["searchbybow"] = bool(all(int(nm[j * nc + c]) == int(r["nmatches"][c]) and
                                              np.array_equal(match[j * nc + c, :1000], r["m12"][c])
                                              for c in range(nc)))
                chk["solvers"] = bool(all((states[j * nc + c].n, states[j * nc + c].max_iterations,
                                           states[j * nc + c].iterations, states[j * nc + c].best_inliers) ==
                                          tuple(int(v) for v in r["cand_state"][c][:4])
                                          for c in range(nc) if r["nmatches"][c] >= 20))
                chk["outcome"] = bool((g.matched, g.round, g.n_inliers, g.hypotheses) ==
                                      (r["matched"], r["round"], r["n_inliers"], r["hypotheses"])
                                      and g.draws == 3 * r["hypotheses"])
                after = ransac.RandState.from_buffer_copy(bytes(g.rng_after))
                chk["stream_after"] = bool(orbgpu.lib().orbgpu_rand_r(ctypes.byref(after)) == r["rand_after"])
                if r["matched"] >= 0:
                    tol = 2e-4 * (1 + float(np.abs(r["t12"]).max()))
                    chk["pose"] = bool(np.abs(np.array(g.R12) - r["R12"].reshape(9)).max() <= 2e-4 and
                                       abs(g.s12 - r["s12"]) <= 2e-4 and
                                       np.abs(np.array(g.t12) - r["t12"]).max() <= tol)
                out[f"query {q}"] = {"ok": all(chk.values()), **chk, "matched": r["matched"]}
            return {"ok": all(v["ok"] for v in out.values()), "queries": out,
                    "from": f"the last timed step's LoopBurst ({len(my_q)} queries x {nc} candidates on this rank)",
                    "tolerance": "integers and matches exact; R12, s12 to 2e-4, t12 to 2e-4*(1+|t|)"}
        except Exception as e:  # report, never hide
            return {"ok": False, "error": str(e)}

    def cpu_baseline(self, mix, seconds, info):
        """The oracle pipeline in C++ (oracle/liborbref.so: DBoW2 transform,
        SearchByBoW(KF,KF), Sim3Solver set-up and the round-robin iterate(5)
        with host glibc rand()) over whole queries, 1 thread and all threads."""
        import orbref
        scene = self.scene(mix)
        voc = self.oracle_vocabulary()
        nq, nc = self.nq, self.nc
        fix = LOOP_MIXES[mix][2]

        def run(j, stop_at, out, step=1):
            n, q = 0, j
            while time.perf_counter() < stop_at:
                qq = q % nq
                orbref.compute_sim3_query(voc, scene, qq, [nq + qq * nc + c for c in range(nc)], 1000 + qq, fix)
                n += nc
                q += step
            out.append(n)

        n1, e1 = _timed_threads(run, 1, seconds / 3)
        T = info["threads_used"]
        nN, eN = _timed_threads(lambda j, s, o: run(j, s, o, T), T, 2 * seconds / 3)
        return {"value": round(nN / eN, 2), "unit": "KF pairs/s", "cores": T, "kind": "port",
                "single_thread_value": round(n1 / e1, 2),
                "sample": f"C++ oracle ComputeSim3 queries (BoW transform of the query and its {nc} candidates, "
                          f"SearchByBoW(KF,KF), Sim3Solver set-up, round-robin iterate(5)), ~{seconds:.0f}s bounded "
                          f"({n1} KF pairs on 1 thread, {nN} on {T}); rand() is process-global in glibc, so the "
                          f"threads' draws interleave (timing only)"}


def run_loop_leg(args, rank, world, dev, mixes, info=None):
    leg = LoopLeg(rank, world, dev)
    out = {"vocabulary": "k=10 L=6 (1,111,111 nodes), DBoW2 text format, loaded by orbgpu_vocabulary_load_text",
           "setup_s": round(leg.t_voc, 2), "vocabulary_text_load_s": round(leg.t_load, 2)}
    steps, warm = max(5, min(args.steps, 20)), 2
    for mix in mixes:
        out[mix] = leg.run(mix, steps, warm)
    if info is not None:
        for mix in mixes:
            out[mix]["cpu_baseline"] = leg.cpu_baseline(mix, args.cpu_seconds / 2, info)
    return out, leg


def traffic_for(path, config, batch):
    p = Path(path)
    if not p.exists():
        return None
    try:
        tj = json.loads(p.read_text())
        if tj.get("config") == config and tj.get("batch") == batch and \
                str(tj.get("kernel_name", "")).startswith(PYR_KERNEL_ID):
            return tj.get("pyramid_hbm_bytes_per_step")
    except Exception:
        return None
    return None


def common_line(args, world):
    return {"n_gpus": world, "steps": args.steps, "warmup": args.warmup, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "data": "synthetic"}


def main_loopburst(args, rank, world, dev):
    info = cpu_info() if (world == 1 and not args.no_cpu_baseline and rank == 0) else None
    legs, _ = run_loop_leg(args, rank, world, dev, ["bench", "several_rounds", "false_loops"], info)
    if rank != 0:
        return None
    b = legs["bench"]
    line = {"metric": "KF pairs/s LoopClosing::ComputeSim3 burst (SearchByBoW(KF,KF) + Sim3Solver RANSAC)",
            "value": b["kf_pairs_per_s"], "unit": "KF pairs/s", **common_line(args, world),
            "ms_per_step": b["ms_per_step"], "dtype": "u8/f32/f64",
            "config": {"workload": CONFIGS["loopburst"][3], "config": "loopburst", "queries": 100,
                       "candidates_per_query": 5, "kf_pairs_per_step": b["kf_pairs_per_step"],
                       "parallelism": f"queries round-robin x{world}"},
            "roofline": {"bound": "hbm", "kernel": b["dominant_kernel"], "frac": b["dominant_hbm_frac"],
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "traffic": None,
                         "note": "latency-bound (sequential per-node merge walks / per-query RANSAC chain)"},
            "mixes": legs,
            "parity_vs_oracle": {m: legs[m].get("parity_vs_oracle") for m in legs if isinstance(legs[m], dict)
                                 and "parity_vs_oracle" in legs[m]}}
    if "cpu_baseline" in b:
        line["cpu_baseline"] = b["cpu_baseline"]
    return line


def main_stereo(args, og, D, rank, world, stream):
    P = args.batch or 128
    sb = StereoBench(og, D, args.config, P, rank, world, stream, dump=args.dump)
    r = sb.run(args.warmup, args.steps)
    if rank != 0:
        return None
    parity = sb.parity_timed()
    W, H, NF, desc = CONFIGS[args.config]
    line = {"metric": f"pairs/sec stereo Frame (extract L+R + ComputeStereoMatches, {W}x{H}, {NF} feat)",
            "value": round(r["pairs_per_s"], 1), "unit": "pairs/s", **common_line(args, world),
            "ms_per_step": round(r["elapsed"] / args.steps * 1e3, 3), "dtype": "u8",
            "config": {"workload": desc, "config": args.config, "pairs_per_gpu_per_step": P, "width": W, "height": H,
                       "nfeatures": NF, "parallelism": sb.summary(r, args.steps)["parallelism"]},
            "keypoints_per_frame": round(r["keypoints_per_frame"], 1),
            "left_keypoints_with_depth": round(r["left_keypoints_with_depth"], 3),
            "parity_vs_oracle": parity}
    if D.cuda and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline_stereo(args.config, args.cpu_seconds, cpu_info())
    return line


def main_mono(args, og, D, rank, world, stream):
    W, H, NF, desc_cfg = CONFIGS[args.config]
    B = args.batch or (512 if args.config == "mono640" else 256)
    MATCH_AFTER[0] = args.match_after
    MATCH_PRIORITY[0] = args.match_priority
    sb = StreamBench(og, D, W, H, NF, B, rank, world, stream, dump=args.dump, deliver=args.deliver, feed=args.feed,
                     parts=args.parts, part_stage=args.part_stage)
    extras = {}
    n_sus = args.sustained_steps if args.sustained_steps is not None else (
        max(args.steps, SUSTAINED_STEPS) if not args.no_extras and D.cuda else 0)
    if n_sus > 0:
        # sustained leg, before the headline: the same stream for SUSTAINED_STEPS steps
        # (~0.55 s at 640x480; the headline's timed region is steps x ms_per_step, ~30 ms at
        # the driver's 20).  Run first, it also brings the GPU to the clock it holds under
        # this load (5 warm-up steps after an idle GPU leave the 20 timed steps
        # ~4 % slower than the same steps after 60)
        # straight into the headline's warm-up steps: the leg's bookkeeping after the headline
        sustained_done = sb.run(args.warmup, n_sus, defer=True)
        settle = sb.run(args.warmup, SETTLE_STEPS) if SETTLE_STEPS > 0 else None
        r = sb.run(args.warmup, args.steps)
        rs = sustained_done()
        extras["sustained"] = {"steps": n_sus, "warmup": args.warmup, "seconds": round(rs["elapsed"], 3),
                               "frames_per_s": round(rs["fps"], 1),
                               "ms_per_step": round(rs["elapsed"] / n_sus * 1e3, 3),
                               "stages_ms_per_step": {k: round(v, 4) for k, v in rs["per_step"].items()},
                               "stages_over_last_steps": min(n_sus, PROFILED_TAIL),
                               "headline_host_gap_ms": sb.host_gap_ms,
                               "settle_leg": None if settle is None else {
                                   "steps": SETTLE_STEPS, "frames_per_s": round(settle["fps"], 1),
                                   "step_ms": settle.get("step_ms")},
                               "order": "run before the headline's warm-up and timed steps, its bookkeeping "
                                        "after them (no host work between its last step and their first)"}
    else:
        r = sb.run(args.warmup, args.steps)
    # the timed configuration's own outputs against the oracle (rank 0, untimed)
    parity = sb.parity_timed() if rank == 0 else None
    sb.close()
    del sb
    D.empty_cache()
    if world > 1 and args.other_delivery:
        # the other delivery mode on the same stream (N > 1): per rank ms_per_step and the
        # owner's waits for both modes in one line
        other = "host" if args.deliver == "gpu0" else "gpu0"
        ob = StreamBench(og, D, W, H, NF, B, rank, world, stream, dump=args.dump, deliver=other, feed=args.feed,
                         dump_tag="_other")
        orr = ob.run(args.warmup, args.steps)
        ob.close()
        del ob
        D.empty_cache()
        extras["delivery_other_mode"] = {
            "mode": other, "frames_per_s": round(orr["fps"], 1),
            "ms_per_step": round(orr["elapsed"] / args.steps * 1e3, 3), "delivery": orr["delivery"],
            "stages_ms_per_step_rank0": {k: round(v, 4) for k, v in orr["per_step"].items()},
            "note": "the same stream and steps with the other delivery mode, run after the headline"}
    if not args.no_extras and D.cuda and args.feed == "hbm":
        # host-fed leg: the same stream with every step's frames copied from pinned host
        # memory (double-buffered H2D on a copy stream, overlapped with extraction) and the
        # outputs delivered to host memory, as TrackMonocular consumes them
        hb = StreamBench(og, D, W, H, NF, B, rank, world, stream, deliver="host", feed="host")
        hr = hb.run(2, max(10, args.steps))
        hb.close()
        del hb
        D.empty_cache()
        h2d_ms = hr["h2d"]["ms_per_copy_mean"] if hr["h2d"] else None
        compute_ms = r["elapsed"] / args.steps * 1e3
        extras["host_fed"] = {
            "frames_per_s": round(hr["fps"], 1), "ms_per_step": round(hr["elapsed"] / max(10, args.steps) * 1e3, 3),
            "frames_per_gpu_per_step": B, "h2d": hr["h2d"], "delivery": hr["delivery"],
            "hbm_resident_ms_per_step": round(compute_ms, 3),
            "bound": ("pcie_h2d" if h2d_ms and h2d_ms > compute_ms else "kernels"),
            "workload": desc_cfg + "; frames copied from pinned host memory every step (H2D on a copy stream, "
                                   "double-buffered), outputs delivered to pinned host memory"}
    if not args.no_extras and D.cuda:
        # config 4: EuRoC stereo sharded over all ranks (every N)
        esb = StereoBench(og, D, "euroc_stereo", 128, rank, world, stream)
        er = esb.run(2, 10)
        extras["stereo_euroc_sharded"] = esb.summary(er, 10)
        if rank == 0:
            extras["stereo_euroc_sharded"]["parity_vs_oracle"] = esb.parity_timed()
        del esb
        D.empty_cache()
        # config 5: loop-closure bursts, queries round-robin over all ranks
        info = cpu_info() if (world == 1 and not args.no_cpu_baseline and rank == 0) else None
        loop_legs, _ = run_loop_leg(args, rank, world, D.device, ["bench", "several_rounds", "false_loops"], info)
        extras["loop_burst"] = loop_legs
        D.empty_cache()
    if rank != 0:
        return None
    achieved = r["achieved"]
    line = {
        "metric": METRIC,
        "value": round(r["fps"], 1),
        "unit": "frames/s",
        **common_line(args, world),
        "ms_per_step": round(r["elapsed"] / args.steps * 1e3, 3),
        "dtype": "u8",
        "config": {"workload": desc_cfg, "config": args.config, "frames_per_gpu_per_step": B,
                   "width": W, "height": H, "nfeatures": NF,
                   "sub_batches": {"parts": args.parts, "frames_each": B // args.parts,
                                   "next_starts_after": args.part_stage if args.parts > 1 else None},
                   "parallelism": f"one stream in contiguous per-rank chunks x{world}, boundary frame send/recv, "
                                  + ("per-rank delivery of trimmed outputs to pinned host memory"
                                     if args.deliver == "host" else "per-step counts-first gather to rank 0")},
        "roofline": {"bound": "hbm", "kernel": PYR_KERNEL,
                     "achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                     "traffic": traffic_for(args.traffic_json, args.config, B),
                     "algorithmic_bytes_per_step": r["pyr_bytes"]},
        "stages_ms_per_step": {k: round(v, 4) for k, v in r["per_step"].items()},
        "stages_over_last_steps": min(args.steps, PROF_STEPS if PROF_STEPS >= 0 else HEADLINE_PROFILED),
        **({"step_ms": r["step_ms"]} if r.get("step_ms") else {}),
        "keypoints_per_frame": round(r["keypoints"], 1),
        "matches_per_pair": round(r["matches"], 1),
        "parity_vs_oracle": parity,
        "parity_frame0_vs_oracle": None if parity is None else bool(parity.get("ok")),
        "world_size_checked": world,
        "input": "frames resident in HBM" if args.feed == "hbm" else
                 "frames copied from pinned host memory every step (double-buffered H2D)",
        "delivery": r["delivery"],
    }
    if r.get("h2d"):
        line["h2d"] = r["h2d"]
    tr = line["roofline"]["traffic"]
    if tr and r["per_step"].get("pyramid"):
        line["roofline"]["traffic_frac"] = round(tr / (r["per_step"]["pyramid"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
    line.update(extras)
    if world == 1 and not args.no_extras and D.cuda:
        line["drop_in"] = drop_in_latency(with_cpu=not args.no_cpu_baseline)
        ex_op = line["drop_in"].get("ops", {}).get("ORBextractor::operator()")
        if ex_op:
            line["single_frame"] = {"median_ms": round(ex_op["median_us"] / 1e3, 4),
                                    "path": "ORB_SLAM2::ORBextractor::operator() (C++ drop-in class, 640x480, host "
                                            "image in, keypoints + descriptors out, no host pyramid copy)"}
        other = {}
        kb = StreamBench(og, D, *CONFIGS["kitti"][:3], 256, 0, 1, stream, deliver=args.deliver)
        kr = kb.run(2, 10)
        k_par = kb.parity_timed()
        kb.close()
        other["mono1241x376"] = {
            "frames_per_s": round(kr["fps"], 1), "ms_per_step": round(kr["elapsed"] / 10 * 1e3, 3),
            "frames_per_step": 256, "nfeatures": CONFIGS["kitti"][2],
            "pyramid_roofline": {"achieved": round(kr["achieved"], 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": round(kr["achieved"] / HBM_PEAK_GBS, 4),
                                 "algorithmic_bytes_per_step": kr["pyr_bytes"]},
            "stages_ms_per_step": {k: round(v, 4) for k, v in kr["per_step"].items()},
            "keypoints_per_frame": round(kr["keypoints"], 1), "matches_per_pair": round(kr["matches"], 1),
            "parity_vs_oracle": k_par, "workload": CONFIGS["kitti"][3]}
        del kb
        D.empty_cache()
        ksb = StereoBench(og, D, "kitti_stereo", 128, 0, 1, stream)
        other["stereo_kitti"] = ksb.summary(ksb.run(2, 10), 10)
        other["stereo_kitti"]["parity_vs_oracle"] = ksb.parity_timed()
        del ksb
        D.empty_cache()
        line["other_geometries"] = other
    if world == 1 and not args.no_cpu_baseline and D.cuda:
        import synth
        info = cpu_info()
        frames_np = np.stack([synth.torch_stream(1, W, H, device=D.device, t0=t, bounded=True)[0].cpu().numpy()
                              for t in range(24)])
        line["cpu_baseline"] = cpu_baseline_mono(frames_np, W, H, NF, args.cpu_seconds, info)
        if "other_geometries" in line:
            og_ = line["other_geometries"]
            og_["mono1241x376"]["cpu_baseline"] = cpu_baseline_mono_geometry("kitti", args.cpu_seconds / 2, info)
            og_["stereo_kitti"]["cpu_baseline"] = cpu_baseline_stereo("kitti_stereo", args.cpu_seconds / 2, info)
        if "stereo_euroc_sharded" in line:
            line["stereo_euroc_sharded"]["cpu_baseline"] = cpu_baseline_stereo("euroc_stereo", args.cpu_seconds / 2,
                                                                               info)
    return line


def main():
    argv = sys.argv[1:]
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args.gpus, argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    dry = args.cpu_dry_run is not None
    og = load_engine(args.cpu_dry_run)
    if dry:
        device = torch.device("cpu")
    else:
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    D = Dev(device)
    if world > 1:
        import torch.distributed as dist
        if dry:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
    if args.config == "loopburst":
        if dry:
            raise SystemExit("--cpu-dry-run covers the frame and pair streams, not loopburst")
        line = main_loopburst(args, rank, world, device)
    else:
        # extraction on a high-priority stream (the matcher's stream has the default, lower
        # priority): when both have work ready, the extraction's workgroups dispatch first
        stream = D.stream(priority=-1)
        if D.cuda:
            torch.cuda.set_stream(stream)
        if args.config in STEREO:
            line = main_stereo(args, og, D, rank, world, stream)
        else:
            line = main_mono(args, og, D, rank, world, stream)
    if line is not None:
        line["world_size_checked"] = world
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
