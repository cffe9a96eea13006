"""Frame sharding across the GPUs of one node.

One frame stream is split into contiguous chunks: at step s, rank r owns
global frames [(s*N + r)*B, (s*N + r + 1)*B).  Extraction is independent per
frame; the only cross-rank dependency of the path is the (t-1, t) pair that
SearchForInitialization matches (src/Tracking.cpp:768-769), so each rank sends
the last frame of its chunk -- keypoints, descriptors, count, ~60 KB -- to
rank r+1 over the process group (RCCL send/recv on GPUs, gloo on the CPU).
Rank r > 0 pairs its first frame with rank r-1's last frame of the same
step; rank 0 with rank N-1's last frame of the previous step.  A stereo
pair (L, R) is one unit of a chunk, so it never straddles two ranks
(src/Frame.cpp:84-87).

Every step's outputs (keypoints, descriptors, counts, matches) go to their
consumer, the Tracking thread (src/Tracking.cpp:280-317), in one of two ways
(``Delivery``):

* ``host`` -- each rank packs the rows its frames actually hold (trimmed to
  the keypoint counts) and copies them over its OWN PCIe link into pinned
  host memory: nothing funnels through one GPU, so the per-rank cost does
  not grow with N;
* ``gpu0`` -- the rows go to rank 0's HBM with point-to-point sends (a
  gather emulated with send/recv: only rank 0 needs them, so an all-gather
  would move N times the bytes), the counts first so only used rows travel.

There is no all-reduce on the data path.  Both modes record the bytes each
rank moves per step and how long the owner thread waited for a delivery.

The classes take torch tensors on whatever device the process group uses,
so the same code runs over RCCL in bench.py and over gloo in
tests/test_distributed.py.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def chunk_frames(step: int, rank: int, world: int, per_rank: int) -> range:
    """Global frame indices rank `rank` processes at `step`."""
    first = (step * world + rank) * per_rank
    return range(first, first + per_rank)


def _pg_active(world: int) -> bool:
    return world > 1 and dist.is_available() and dist.is_initialized()


class BoundaryExchange:
    """The chunk-boundary frame between ranks, with no copies.
    ``exchange(last, into)`` sends this rank's last frame (`last`: its
    keypoints, descriptors and count, read in place from the output set) to
    rank+1 and receives rank-1's last frame of the same step straight into
    `into`, the buffers the matcher then reads as the frame before this
    rank's first frame.  For rank 0 that frame is rank N-1's last frame of
    the step, i.e. the one before rank 0's NEXT chunk: the caller passes the
    next step's buffers as `into`.  At N = 1 there is nothing to exchange
    (the previous step's last frame is read in place from its output set)
    and ``exchange`` returns False."""

    def __init__(self, rank: int, world: int):
        self.rank, self.world = rank, world

    def exchange(self, last, into) -> bool:
        if not _pg_active(self.world):
            return False
        nxt, prv = (self.rank + 1) % self.world, (self.rank - 1) % self.world
        ops = [dist.P2POp(dist.isend, t, nxt) for t in last]
        ops += [dist.P2POp(dist.irecv, t, prv) for t in into]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        return True


class OwnerGather:
    """Gather of every rank's step outputs to rank 0 (send/recv).  Two
    buffer sets alternate so the transfer of step k overlaps the compute of
    step k+1; ``start`` returns immediately, ``finish`` (called before a
    buffer set is reused, or at the end) completes it.  On rank 0
    ``received(k)`` is the list over ranks of the tensors of step k's set."""

    def __init__(self, rank: int, world: int, templates, sets: int = 2):
        self.rank, self.world, self.sets = rank, world, sets
        self.pending = [[] for _ in range(sets)]
        self.recv = None
        if rank == 0 and world > 1:
            self.recv = [[[torch.zeros_like(t) for t in templates] for _ in range(world - 1)] for _ in range(sets)]

    def start(self, set_idx: int, tensors):
        self.finish(set_idx)
        if not _pg_active(self.world):
            return
        if self.rank == 0:
            ops = [dist.P2POp(dist.irecv, buf, src + 1)
                   for src, bufs in enumerate(self.recv[set_idx]) for buf in bufs]
        else:
            ops = [dist.P2POp(dist.isend, t.contiguous(), 0) for t in tensors]
        self.pending[set_idx] = dist.batch_isend_irecv(ops)

    def finish(self, set_idx: int | None = None):
        idx = range(self.sets) if set_idx is None else [set_idx]
        for i in idx:
            for w in self.pending[i]:
                w.wait()
            self.pending[i] = []

    def received(self, set_idx: int):
        """rank 0: [tensors of rank 1, ..., rank N-1] of that buffer set."""
        return self.recv[set_idx] if self.recv is not None else []


# ---------------------------------------------------------------------------
# Delivery of each step's outputs to the Tracking owner
# ---------------------------------------------------------------------------

class RowSpec:
    """One output of a step: `rows` is (B, cap, *row_shape); the B frames'
    rows are trimmed to counts[which] (0: the frames' own counts, 1: the
    counts of the frames they were matched against -- SearchForInitialization's
    m12 has a row per keypoint of F1)."""

    def __init__(self, name, which=0):
        self.name, self.which = name, which


def clamped_counts(counts, cap):
    """per-frame row counts as the pack kernel uses them: clamped to [0, cap]
    (csrc/pack.hip), so an out-of-range count cannot shift other frames' rows"""
    return counts.to(torch.int64).clamp(0, cap)


def pack_offsets(counts, cap):
    """exclusive prefix sums of the clamped per-frame counts (device, int64)"""
    c = clamped_counts(counts, cap)
    return torch.cumsum(c, 0) - c


def pack_rows(rows, counts, out):
    """out[offsets[b] + j] = rows[b, j] for j < counts[b] (device-side, static
    shapes, no host sync); out has B * cap + 1 rows, the last one a dump slot
    for the rows past each frame's count.  Returns nothing: the number of
    used rows is sum(counts), which the caller learns from the counts copy."""
    B, cap = rows.shape[0], rows.shape[1]
    off = pack_offsets(counts, cap)
    j = torch.arange(cap, device=rows.device, dtype=torch.int64)
    idx = torch.where(j[None, :] < clamped_counts(counts, cap)[:, None], off[:, None] + j[None, :],
                      torch.full((), B * cap, device=rows.device, dtype=torch.int64))
    out.index_copy_(0, idx.reshape(-1), rows.reshape(B * cap, *rows.shape[2:]))


class Delivery:
    """Per-rank delivery of a step's outputs (``mode`` "host" or "gpu0") to
    the Tracking owner, driven from the owner thread with no helper thread
    (no lock or interpreter contention with the thread issuing the kernels).

    ``start(rows, small_parts, counts, stream)`` is called right after the
    step's producers are issued on `stream`: on `stream` the rows are packed
    (trimmed to the counts; the HIP pack kernel on a GPU) and the per-frame
    scalars (counts, match counts) gathered into one small int tensor, whose
    copy to pinned host memory (host) or send to rank 0 (gpu0) is queued on a
    copy stream.  Every later ``start`` / ``poll`` advances the queued slots
    without blocking: once a slot's small tensor has landed the owner knows
    how many rows are used and queues exactly those --
      host: copies into pinned host memory, over this rank's own PCIe link;
      gpu0: rank r > 0 sends them to rank 0, which receives each rank's
            rows after its counts.  Point-to-point operations between a pair
            of ranks are matched in the order they are posted, and the two
            sides post them at different times (rank r posts step k's rows as
            soon as its own counts are out, rank 0 only after step k's counts
            have arrived, possibly after posting step k+1's counts receive), so
            the counts and the rows travel on TWO process groups: on each, both
            sides post one kind of operation in step order.
    Slots form a ring of `sets` (the producer's device buffers are free
    again once the packing on `stream` is done); a slot is waited for only
    when it is reused or at ``finish()``: that wait is the owner's wait.
    """

    def __init__(self, mode, rank, world, device, specs, B, cap, row_templates, small_len, sets=4, groups=None,
                 packer=None, on_delivered=None):
        import collections
        import time
        assert mode in ("host", "gpu0"), mode
        self.mode, self.rank, self.world, self.device = mode, rank, world, device
        # packer(B, cap, [(rows, packed, counts)], stream): the HIP pack kernel on a GPU
        # (orbgpu.pack_rows); pack_rows (torch ops) where the engine has none (CPU dry run)
        self.packer = packer
        self.specs, self.B, self.cap, self.sets = specs, B, cap, sets
        self.cuda = device.type == "cuda"
        self._time = time.perf_counter
        # gpu0 with N > 1: (counts group, rows group) -- see the class comment
        self.remote = mode == "gpu0" and _pg_active(world)
        if self.remote:
            assert groups is not None and len(groups) == 2 and groups[0] is not groups[1], \
                "gpu0 delivery needs two process groups (counts, rows)"
        self.g_small, self.g_rows = groups if groups is not None else (None, None)
        # on_delivered(slot, seq): called when the seq-th start()'s rows are delivered, before
        # the slot can be reused (tests read rank 0's received rows there)
        self.on_delivered = on_delivered
        self.owner_local = mode == "gpu0" and rank == 0  # the owner's own rows stay where they are
        pin = self.cuda
        self.packed = [[torch.zeros((B * cap + 1, *t.shape[2:]), dtype=t.dtype, device=device) for t in row_templates]
                       for _ in range(sets)]
        self.small = [torch.zeros(small_len, dtype=torch.int32, device=device) for _ in range(sets)]
        self.small_host = [torch.zeros(small_len, dtype=torch.int32, pin_memory=pin) for _ in range(sets)]
        if mode == "host":
            self.host = [[torch.zeros((B * cap, *t.shape[2:]), dtype=t.dtype, pin_memory=pin) for t in row_templates]
                         for _ in range(sets)]
        if self.remote and rank == 0:
            self.recv_rows = [[[torch.zeros((B * cap, *t.shape[2:]), dtype=t.dtype, device=device)
                                for t in row_templates] for _ in range(world - 1)] for _ in range(sets)]
            self.recv_small = [[torch.zeros(small_len, dtype=torch.int32, device=device) for _ in range(world - 1)]
                               for _ in range(sets)]
            self.recv_small_host = [[torch.zeros(small_len, dtype=torch.int32, pin_memory=pin)
                                     for _ in range(world - 1)] for _ in range(sets)]
        self.counts_which = [spec.which for spec in specs]
        self.used = [[0] * len(row_templates) for _ in range(sets)]
        self.copy_stream = torch.cuda.Stream(device) if self.cuda else None
        self.queue = collections.deque()  # slots in flight, oldest first: [slot, stage, works, t0, ev...]
        self.state = [None] * sets
        self.next = 0
        self.stats = self._zero()

    @staticmethod
    def _zero():
        return {"bytes": 0, "steps": 0, "wait_s": 0.0, "recv_bytes": 0, "copy_ms": 0.0, "latency_s": 0.0}

    # ---- helpers -----------------------------------------------------------
    def _ctx(self):
        return torch.cuda.stream(self.copy_stream) if self.cuda else _null()

    def _event(self, timing=False):
        if not self.cuda:
            return None
        e = torch.cuda.Event(enable_timing=timing)
        e.record(self.copy_stream)
        return e

    @staticmethod
    def _ready(ev, works=()):
        return (ev is None or ev.query()) and all(w.is_completed() for w in works)

    def _used_rows(self, small_host):
        B = self.B
        c = clamped_counts(small_host[:2 * B], self.cap)
        tot = [int(c[:B].sum()), int(c[B:2 * B].sum())]
        return [tot[w] for w in self.counts_which]

    # ---- owner thread ------------------------------------------------------
    def start(self, rows, small_parts, counts, stream=None):
        """rows: one (B, cap, ...) tensor per spec; small_parts: per-frame int
        tensors concatenated into the small tensor (counts first); counts:
        [own counts (B,), matched-against counts (B,)].  Returns the slot."""
        import torch.distributed as dist
        self.poll()
        si = self.next % self.sets
        self.next += 1
        self.finish(si)
        ctx = torch.cuda.stream(stream) if (self.cuda and stream is not None) else _null()
        with ctx:
            if self.owner_local:
                pass
            elif self.packer is not None:
                self.packer(self.B, self.cap, [(t, out, counts[spec.which])
                                               for spec, t, out in zip(self.specs, rows, self.packed[si])], stream)
            else:
                for spec, t, out in zip(self.specs, rows, self.packed[si]):
                    pack_rows(t, counts[spec.which], out)
            torch.cat([p.to(torch.int32).reshape(-1) for p in small_parts], out=self.small[si])
            ready = None
            if self.cuda:
                ready = torch.cuda.Event()
                ready.record(stream if stream is not None else torch.cuda.current_stream(self.device))
        st = {"slot": si, "seq": self.next - 1, "t0": self._time(), "works": [], "ev": None, "bytes": 0}
        with self._ctx():
            if self.cuda:
                self.copy_stream.wait_event(ready)
            if self.remote and self.rank > 0:
                st["works"] = [dist.isend(self.small[si], 0, group=self.g_small)]
                self.small_host[si].copy_(self.small[si], non_blocking=self.cuda)
                st["stage"] = "sent_small"
            elif self.remote:  # rank 0: every other rank's small tensor for this step
                st["works"] = [dist.irecv(self.recv_small[si][r - 1], r, group=self.g_small)
                               for r in range(1, self.world)]
                st["stage"] = "recv_small"
            else:
                self.small_host[si].copy_(self.small[si], non_blocking=self.cuda)
                st["stage"] = "small"
            st["ev"] = self._event()
        self.state[si] = st
        self.queue.append(st)
        self.poll()
        return si

    def poll(self, block=False):
        """advance the slots in flight, oldest first, without blocking unless
        `block` (then until the oldest slot is delivered)"""
        import torch.distributed as dist
        while self.queue:
            st = self.queue[0]
            si = st["slot"]
            if not block and not self._ready(st["ev"], st["works"]):
                return
            if block:
                for w in st["works"]:
                    w.wait()
                if st["ev"] is not None:
                    st["ev"].synchronize()
            stage = st["stage"]
            with self._ctx():
                if stage == "small":  # host / local: counts known -> the used rows
                    used = self._used_rows(self.small_host[si])
                    self.used[si] = used
                    nbytes = self.small[si].numel() * 4
                    if self.mode == "host":
                        e0 = self._event(True)
                        for out, dev, n in zip(self.host[si], self.packed[si], used):
                            if n:
                                out[:n].copy_(dev[:n], non_blocking=self.cuda)
                            nbytes += n * dev[0].numel() * dev.element_size()
                        st["copy"] = (e0, self._event(True))
                    else:
                        nbytes = 0  # gpu0 at N = 1: the owner's own HBM, nothing moves
                    st["bytes"], st["stage"], st["works"], st["ev"] = nbytes, "rows", [], self._event()
                elif stage == "sent_small":  # rank r > 0: the counts of our own rows
                    used = self._used_rows(self.small_host[si])
                    works = []
                    nbytes = self.small[si].numel() * 4
                    for dev, n in zip(self.packed[si], used):
                        if n:
                            works.append(dist.isend(dev[:n], 0, group=self.g_rows))
                        nbytes += n * dev[0].numel() * dev.element_size()
                    st["bytes"], st["stage"], st["works"], st["ev"] = nbytes, "rows", works, None
                elif stage == "recv_small":  # rank 0: the counts received -> to the host
                    for r in range(1, self.world):
                        self.recv_small_host[si][r - 1].copy_(self.recv_small[si][r - 1], non_blocking=self.cuda)
                    st["stage"], st["works"], st["ev"] = "recv_small_host", [], self._event()
                elif stage == "recv_small_host":  # rank 0: each rank's used rows after its counts
                    works, rb = [], 0
                    for r in range(1, self.world):
                        smh = self.recv_small_host[si][r - 1]
                        for buf, n in zip(self.recv_rows[si][r - 1], self._used_rows(smh)):
                            if n:
                                works.append(dist.irecv(buf[:n], r, group=self.g_rows))
                            rb += n * buf[0].numel() * buf.element_size()
                    st["recv_bytes"] = rb
                    st["stage"], st["works"], st["ev"] = "rows", works, None
                else:  # rows delivered
                    self.queue.popleft()
                    self.stats["bytes"] += st["bytes"]
                    self.stats["recv_bytes"] += st.get("recv_bytes", 0)
                    self.stats["steps"] += 1
                    self.stats["latency_s"] += self._time() - st["t0"]
                    if "copy" in st and self.cuda:
                        self.stats["copy_ms"] += st["copy"][0].elapsed_time(st["copy"][1])
                    self.state[si] = None
                    if self.on_delivered is not None:
                        self.on_delivered(si, st["seq"])
                    if block:
                        return

    def finish(self, si=None):
        """wait until slot si (None: every slot) is delivered"""
        t0 = self._time()
        while self.queue and (si is None or self.state[si] is not None):
            self.poll(block=True)
        self.stats["wait_s"] += self._time() - t0

    def close(self):
        self.finish()

    def host_rows(self, si):
        """host mode: this rank's delivered rows of slot si, one (rows, used)
        pair per spec, and the small per-frame tensor."""
        return list(zip(self.host[si], self.used[si])), self.small_host[si]

    def received(self, si):
        """gpu0, rank 0: per source rank r > 0, (rows per spec, small host
        tensor); each spec's used rows are the first sum(counts) rows."""
        if not hasattr(self, "recv_rows"):  # N = 1, or not rank 0: nothing received
            return []
        return list(zip(self.recv_rows[si], self.recv_small_host[si]))

    def report(self, steps):
        s = self.stats
        n = max(steps, 1)
        out = {"mode": self.mode, "bytes_per_step": int(s["bytes"] / max(s["steps"], 1)),
               "recv_bytes_per_step": int(s["recv_bytes"] / max(s["steps"], 1)),
               "owner_wait_ms_per_step": round(1e3 * s["wait_s"] / n, 4),
               "delivery_latency_ms": round(1e3 * s["latency_s"] / max(s["steps"], 1), 4),
               "ring_slots": self.sets}
        if self.mode == "host" and s["copy_ms"] > 0:  # the D2H copies alone (events on the copy stream)
            out["copy_ms_per_step"] = round(s["copy_ms"] / max(s["steps"], 1), 4)
            out["copy_gb_per_s"] = round(s["bytes"] / (s["copy_ms"] / 1e3) / 1e9, 2)
        return out

    def reset_stats(self):
        self.finish()
        self.stats = self._zero()


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def unpack_rows(packed, counts, cap):
    """inverse of pack_rows on the host (tests and dumps): (B, cap, ...) with
    zero rows past each count"""
    import numpy as np
    packed = np.asarray(packed)
    counts = np.clip(np.asarray(counts, np.int64), 0, cap)
    out = np.zeros((len(counts), cap, *packed.shape[1:]), packed.dtype)
    off = 0
    for b, c in enumerate(counts):
        out[b, :c] = packed[off:off + c]
        off += c
    return out
