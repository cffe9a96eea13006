"""Multi-process (world_size 2, gloo on CPU) coverage of bench.py's N>1 path:
independent per-rank streams, max-over-ranks elapsed time and the whole-job
frame count.  The data path has no collective (frame-sharded, weak scaling)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    elapsed, frames = bench.aggregate(1.0 + rank, 100 * (rank + 1))
    dist.barrier()
    q.put((rank, elapsed, frames, bench.rank_seed(rank)))
    dist.destroy_process_group()


def test_aggregate_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [2.0, 2.0]        # max over ranks
    assert [r[2] for r in res] == [300, 300]        # whole-job frames
    assert res[0][3] != res[1][3]                   # independent streams


def test_aggregate_single_process_is_identity():
    import bench
    assert bench.aggregate(3.5, 42) == (3.5, 42)
