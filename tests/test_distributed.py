"""Multi-process (world_size 2, gloo on CPU) coverage of the N>1 path
(orb-slam2-annotation_amd/shard.py):

* one frame stream in contiguous per-rank chunks; the chunk-boundary frame's
  keypoints/descriptors go to the next rank (send/recv) so the (t-1, t) pair
  across ranks is matched; every step's outputs are gathered to rank 0;
* the gathered keypoints, descriptors and SearchForInitialization matches
  equal a single-process run over the same frames (computed with the CPU
  oracle: the sharding logic is device independent);
* bench.aggregate: max-over-ranks elapsed time and the whole-job frame count.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

CAP = 1100


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _worker(rank, world, port, q):
    _init(rank, world, port)
    import bench
    elapsed, frames = bench.aggregate(1.0 + rank, 100 * (rank + 1))
    dist.barrier()
    q.put((rank, elapsed, frames))
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


def test_aggregate_single_process_is_identity():
    import bench
    assert bench.aggregate(3.5, 42) == (3.5, 42)


def _extract(ex, img):
    k, d = ex.extract(img)
    kp = torch.zeros((CAP, 7), dtype=torch.float32)
    de = torch.zeros((CAP, 32), dtype=torch.uint8)
    n = len(k)
    kp[:n] = torch.from_numpy(k.view(np.float32).reshape(n, 7).copy())
    de[:n] = torch.from_numpy(d.copy())
    return kp, de, n


def _match(kp1, de1, n1, kp2, de2, n2):
    import orbgpu
    import orbref
    m = torch.full((CAP,), -1, dtype=torch.int32)
    if n1 == 0 or n2 == 0:
        return m, 0
    k1 = kp1[:n1].numpy().copy().view(orbgpu.KP_DTYPE).reshape(n1)
    k2 = kp2[:n2].numpy().copy().view(orbgpu.KP_DTYPE).reshape(n2)
    nm, m12, _ = orbref.search_for_initialization(k1, de1[:n1].numpy(), k2, de2[:n2].numpy(), 640, 480)
    m[:n1] = torch.from_numpy(m12)
    return m, nm


def _shard_worker(rank, world, port, steps, B, q):
    _init(rank, world, port)
    import orbref
    import shard
    import synth
    frames = synth.mono_stream(steps * world * B)
    ex = orbref.Extractor()
    bx = shard.BoundaryExchange(rank, world)

    def frame_bufs():
        return (torch.zeros((CAP, 7)), torch.zeros((CAP, 32), dtype=torch.uint8), torch.zeros(1, dtype=torch.int32))

    inb = [frame_bufs() for _ in range(3)]  # per step (mod 3), as bench.py's output sets
    empty = frame_bufs()
    tmpl = [torch.zeros((B, CAP, 7)), torch.zeros((B, CAP, 32), dtype=torch.uint8), torch.zeros(B, dtype=torch.int32),
            torch.zeros((B, CAP), dtype=torch.int32), torch.zeros(B, dtype=torch.int32)]
    gather = shard.OwnerGather(rank, world, tmpl)
    out = {}
    for s in range(steps):
        ids = list(shard.chunk_frames(s, rank, world, B))
        kps, desc, cnt = (torch.zeros_like(t) for t in tmpl[:3])
        for b, f in enumerate(ids):
            kps[b], desc[b], n = _extract(ex, frames[f])
            cnt[b] = n
        last = (kps[B - 1], desc[B - 1], cnt[B - 1:B])
        if rank == 0:  # rank N-1's last frame precedes our next chunk
            assert bx.exchange(last, inb[(s + 1) % 3])
            prev = inb[s % 3] if s > 0 else empty
        else:
            assert bx.exchange(last, inb[s % 3])
            prev = inb[s % 3]
        m12, nm = torch.full((B, CAP), -1, dtype=torch.int32), torch.zeros(B, dtype=torch.int32)
        for b in range(B):
            p = (prev[0], prev[1], int(prev[2][0])) if b == 0 else (kps[b - 1], desc[b - 1], int(cnt[b - 1]))
            m12[b], nm[b] = _match(*p, kps[b], desc[b], int(cnt[b]))
        sidx = s % 2
        gather.start(sidx, [kps, desc, cnt, m12, nm])
        gather.finish(sidx)
        if rank == 0:
            chunks = [(0, [kps, desc, cnt, m12, nm])] + [(r + 1, t) for r, t in enumerate(gather.received(sidx))]
            for r, (k, d, c, m, n) in chunks:
                for b, f in enumerate(shard.chunk_frames(s, r, world, B)):
                    cc = int(c[b])
                    out[f] = (cc, k[b, :cc].numpy().tobytes(), d[b, :cc].numpy().tobytes(), int(n[b]),
                              m[b, :cc].numpy().tobytes())
    gather.finish()
    dist.barrier()
    if rank == 0:
        q.put(out)
    dist.destroy_process_group()


def test_sharded_stream_equals_single_process():
    import orbref
    import synth
    world, steps, B = 2, 2, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, steps, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    # single process, frames in stream order, (t-1, t) pairs
    frames = synth.mono_stream(steps * world * B)
    ex = orbref.Extractor()
    prev = (torch.zeros((CAP, 7)), torch.zeros((CAP, 32), dtype=torch.uint8), 0)
    assert sorted(got) == list(range(len(frames)))
    cross = 0
    for f in range(len(frames)):
        k, d, n = _extract(ex, frames[f])
        m, nm = _match(*prev, k, d, n)
        g = got[f]
        assert g[0] == n and g[1] == k[:n].numpy().tobytes() and g[2] == d[:n].numpy().tobytes(), f
        assert g[3] == nm and g[4] == m[:n].numpy().tobytes(), f
        cross += f > 0 and f % B == 0 and nm > 0  # pairs that straddle two chunks
        prev = (k, d, n)
    assert cross >= 2


def test_pack_rows_torch_path_matches_unpack():
    """shard.pack_rows (the torch packing used where the engine has no HIP
    packer: the CPU dry run) puts frame b's first counts[b] rows at the
    exclusive prefix sum of the counts; shard.unpack_rows inverts it.  Ragged
    counts, empty and full frames, rows of keypoint (7 f32), descriptor
    (32 u8) and match (i32) shape."""
    import shard
    rng = np.random.default_rng(11)
    B, cap = 9, 17
    counts = rng.integers(0, cap + 1, B).astype(np.int32)
    counts[[1, 4]] = 0
    counts[7] = cap
    for shape, dt in (((7,), torch.float32), ((32,), torch.uint8), ((), torch.int32)):
        rows = torch.from_numpy(rng.integers(0, 200, (B, cap, *shape)).astype(np.float32)).to(dt)
        out = torch.zeros((B * cap + 1, *shape), dtype=dt)
        shard.pack_rows(rows, torch.from_numpy(counts), out)
        n = int(counts.sum())
        back = shard.unpack_rows(out[:n].numpy(), counts, cap)
        ref = rows.numpy().copy()
        for b in range(B):
            ref[b, counts[b]:] = 0
        assert np.array_equal(back, ref)
        assert np.array_equal(shard.pack_offsets(torch.from_numpy(counts), cap).numpy(),
                              np.concatenate([[0], np.cumsum(counts)[:-1]]))


def test_pack_rows_clamps_out_of_range_counts():
    """A count below 0 or above cap (an error sentinel, or counts from a
    foreign producer) is clamped to [0, cap] for the frame's own rows AND for
    every later frame's offset (csrc/pack.hip does the same), so the other
    frames' rows neither overlap nor leave gaps."""
    import shard
    B, cap = 5, 6
    counts = np.array([3, -1, cap + 4, 2, 0], np.int32)
    rows = torch.arange(B * cap, dtype=torch.int32).reshape(B, cap)
    out = torch.full((B * cap + 1,), -7, dtype=torch.int32)
    shard.pack_rows(rows, torch.from_numpy(counts), out)
    cl = np.clip(counts, 0, cap)
    n = int(cl.sum())
    assert np.array_equal(shard.pack_offsets(torch.from_numpy(counts), cap).numpy(),
                          np.concatenate([[0], np.cumsum(cl)[:-1]]))
    exp = np.concatenate([rows[b, :cl[b]].numpy() for b in range(B)])
    assert np.array_equal(out[:n].numpy(), exp)
    back = shard.unpack_rows(out[:n].numpy(), counts, cap)
    for b in range(B):
        assert np.array_equal(back[b, :cl[b]], rows[b, :cl[b]].numpy())


def test_delivery_host_mode_single_process_round_trip():
    """shard.Delivery in host mode on the CPU (world 1): the ring of slots,
    back-pressure and the delivered rows / counts of every step."""
    import shard
    rng = np.random.default_rng(12)
    B, cap, steps = 4, 10, 7
    tmpl = [torch.zeros((B, cap, 7)), torch.zeros((B, cap, 32), dtype=torch.uint8),
            torch.zeros((B, cap), dtype=torch.int32)]
    d = shard.Delivery("host", 0, 1, torch.device("cpu"),
                       [shard.RowSpec("kps", 0), shard.RowSpec("desc", 0), shard.RowSpec("m12", 1)],
                       B, cap, tmpl, 3 * B, sets=3)
    for s in range(steps):
        c = torch.from_numpy(rng.integers(0, cap + 1, B).astype(np.int32))
        cp = torch.from_numpy(rng.integers(0, cap + 1, B).astype(np.int32))
        nm = torch.from_numpy(rng.integers(0, 5, B).astype(np.int32))
        k = torch.randn(B, cap, 7)
        de = torch.from_numpy(rng.integers(0, 255, (B, cap, 32)).astype(np.uint8))
        m = torch.from_numpy(rng.integers(-1, 50, (B, cap)).astype(np.int32))
        si = d.start([k, de, m], [c, cp, nm], [c, cp])
        d.finish(si)
        rows, small = d.host_rows(si)
        assert np.array_equal(small.numpy(), np.concatenate([c.numpy(), cp.numpy(), nm.numpy()]))
        for (h, n), t, cnt in zip(rows, (k, de, m), (c, c, cp)):
            assert n == int(cnt.sum())
            back = shard.unpack_rows(h[:n].numpy(), cnt.numpy(), cap)
            ref = t.numpy().copy()
            for b in range(B):
                ref[b, int(cnt[b]):] = 0
            assert np.array_equal(back, ref)
    rep = d.report(steps)
    assert rep["mode"] == "host" and rep["bytes_per_step"] > 0
    d.close()


def _gpu0_pipeline_worker(rank, world, port, steps, sets, adversarial, q):
    """shard.Delivery("gpu0") driven like bench.py's headline: start() every
    step with no finish() in between, ranks staggered by different delays, so
    rank r > 0 posts step k's rows while rank 0 may already have posted the
    counts receive of step k+1.  `adversarial` forces that order: rank 0 posts
    every step's counts receive first (a ring as long as the run), while the
    other ranks start late and push each step's rows out before the next
    step's counts."""
    import time
    _init(rank, world, port)
    import shard
    B, cap = 3, 8
    groups = (dist.new_group(list(range(world))), dist.new_group(list(range(world))))
    tmpl = [torch.zeros((B, cap, 7)), torch.zeros((B, cap, 32), dtype=torch.uint8),
            torch.zeros((B, cap), dtype=torch.int32)]
    got = {}

    def on_delivered(si, seq):  # rank 0: what arrived for step `seq`, before the slot is reused
        if rank == 0:
            got[seq] = [(smh.numpy().copy(), [r.numpy().copy() for r in rows])
                        for rows, smh in d.received(si)]

    d = shard.Delivery("gpu0", rank, world, torch.device("cpu"),
                       [shard.RowSpec("kps", 0), shard.RowSpec("desc", 0), shard.RowSpec("m12", 1)],
                       B, cap, tmpl, 3 * B, sets=sets, groups=groups, on_delivered=on_delivered)
    rng = np.random.default_rng(100 + rank)
    delays = [0.002, 0.013, 0.005][rank % 3]
    if adversarial and rank > 0:
        time.sleep(0.3)
    for s in range(steps):
        g = np.random.default_rng(1000 * s + rank)  # the data rank r sends at step s (rank 0 can rebuild it)
        c = torch.from_numpy(g.integers(0, cap + 1, B).astype(np.int32))
        cp = torch.from_numpy(g.integers(0, cap + 1, B).astype(np.int32))
        nm = torch.from_numpy(g.integers(0, 5, B).astype(np.int32))
        k = torch.from_numpy(g.standard_normal((B, cap, 7)).astype(np.float32))
        de = torch.from_numpy(g.integers(0, 255, (B, cap, 32)).astype(np.uint8))
        m = torch.from_numpy(g.integers(-1, 50, (B, cap)).astype(np.int32))
        d.start([k, de, m], [c, cp, nm], [c, cp])
        if adversarial:
            if rank > 0:
                d.poll(block=True)  # this step's rows are posted before the next step's counts
            continue
        time.sleep(delays * (1 + rng.random()))
        d.poll()
    d.finish()
    dist.barrier()
    if rank == 0:
        q.put(got)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,sets,adversarial", [(2, 2, False), (3, 3, False), (2, 9, True), (3, 9, True)])
def test_delivery_gpu0_pipelined_ranks(world, sets, adversarial):
    """with the counts and the rows of gpu0 delivery on one group,
    the two sides could post their point-to-point operations in different
    orders; on two groups every step's rows reach rank 0 intact while the
    ring is kept full (no finish() per step) and the ranks run at different
    speeds."""
    import shard
    steps, B, cap = 9, 3, 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu0_pipeline_worker, args=(r, world, port, steps, sets, adversarial, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert sorted(got) == list(range(steps))
    for s in range(steps):
        assert len(got[s]) == world - 1
        for r in range(1, world):
            g = np.random.default_rng(1000 * s + r)
            c = g.integers(0, cap + 1, B).astype(np.int32)
            cp = g.integers(0, cap + 1, B).astype(np.int32)
            nm = g.integers(0, 5, B).astype(np.int32)
            k = g.standard_normal((B, cap, 7)).astype(np.float32)
            de = g.integers(0, 255, (B, cap, 32)).astype(np.uint8)
            m = g.integers(-1, 50, (B, cap)).astype(np.int32)
            small, rows = got[s][r - 1]
            assert np.array_equal(small, np.concatenate([c, cp, nm])), (s, r)
            for t, ref, cnt in zip(rows, (k, de, m), (c, c, cp)):
                n = int(cnt.sum())
                back = shard.unpack_rows(t[:n], cnt, cap)
                exp = ref.copy()
                for b in range(B):
                    exp[b, cnt[b]:] = 0
                assert np.array_equal(back, exp), (s, r)
