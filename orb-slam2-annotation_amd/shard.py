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

Every step's outputs (keypoints, descriptors, counts, matches) are gathered
to rank 0, the Tracking owner, with point-to-point sends (a gather emulated
with send/recv: only rank 0 needs them, so an all-gather would move N times
the bytes).  There is no all-reduce on the data path.

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
    """The chunk-boundary frame: ``exchange(last)`` sends this rank's last
    frame to rank+1 and returns the frame that precedes this rank's first
    frame (for rank 0: the one received at the previous step; an empty
    frame -- count 0 -- before the first step)."""

    def __init__(self, rank: int, world: int, templates):
        """templates: tensors shaped like one frame's outputs (e.g. kps
        (cap, 7) f32, desc (cap, 32) u8, count (1,) i32)."""
        self.rank, self.world = rank, world
        self.incoming = [torch.zeros_like(t) for t in templates]
        self.stored = [torch.zeros_like(t) for t in templates]  # rank 0: previous step's boundary

    def exchange(self, last):
        if not _pg_active(self.world):
            prev = [s.clone() for s in self.stored]
            for s, t in zip(self.stored, last):
                s.copy_(t)
            return prev
        nxt, prv = (self.rank + 1) % self.world, (self.rank - 1) % self.world
        ops = [dist.P2POp(dist.isend, t.contiguous(), nxt) for t in last]
        ops += [dist.P2POp(dist.irecv, t, prv) for t in self.incoming]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        if self.rank > 0:
            return self.incoming
        prev = [s.clone() for s in self.stored]
        for s, t in zip(self.stored, self.incoming):
            s.copy_(t)
        return prev


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
