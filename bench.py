#!/usr/bin/env python3
"""bench.py -- ORB-SLAM2 front-end hot path on MI355X: frames/sec of ORB
extract + match (BASELINE.json metric).

A step = one pass of the hot path over one batch of B synthetic frames per
GPU, inputs already resident in HBM:
  * ORBextractor::operator() on all B frames (pyramid -> FAST cells ->
    octree -> angle/blur/rBRIEF), and
  * ORBmatcher(0.9, true).SearchForInitialization(F_{t-1}, F_t, window 100)
    for the B consecutive pairs (the first pair uses the previous step's
    last frame), the reference's map-free matcher (Tracking.cpp:768-769).
value = frames processed by all ranks / max-over-ranks wall time.

Multi-GPU (launched by torch.distributed.run): every rank owns an independent
frame stream (weak scaling, no collective on the data path); one barrier
before/after the timed region and an all-reduce(MAX) of the elapsed time.

Also reported (Measurement):
  * roofline: the pyramid pass (the HBM-bound stage named by BASELINE.json),
    algorithmic bytes = sum_{l>=1} |P_{l-1}| + |P_l| per frame, divided by the
    pyramid launches' summed duration from HIP events recorded on the launch
    stream during the timed region; traffic = PMC-measured HBM bytes from
    profiles/ when a matching summary exists;
  * cpu_baseline: the oracle (CPU restatement, oracle/liborbref.so) on the
    host cores, rank 0 at N=1 only, on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path[:0] = [str(ROOT / "orb-slam2-annotation_amd"), str(ROOT / "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

PYR_KERNEL_LABEL = {
    "stream": "pyramid_stream_kernel (one frame per block; source rows staged through LDS per 4-row step)",
    "frame": "pyramid_frame_kernel (one frame per block; per-lane buffer-load windows)",
    "band": "pyramid_kernel (frame bands, all levels in LDS)",
}
METRIC = "frames/sec ORB extract+match (1000 feat, 640×480 mono) at 1/2/4/8 GPU; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

CONFIGS = {
    # name: (width, height, nfeatures, description)
    "mono640": (640, 480, 1000, "synthetic 640x480 mono stream, 1000 feat, 8 levels x1.2, FAST 20/7 "
                                "(TUM1.yaml params), extract + SearchForInitialization(t-1,t)"),
    "kitti": (1241, 376, 2000, "synthetic 1241x376 stream, 2000 feat (KITTI00-02.yaml params), "
                               "extract + SearchForInitialization(t-1,t)"),
    "euroc": (752, 480, 1200, "synthetic 752x480 stream, 1200 feat (EuRoC.yaml params), "
                              "extract + SearchForInitialization(t-1,t)"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=512, help="frames per GPU per step")
    ap.add_argument("--config", default="mono640", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=str(ROOT / "profiles" / "pmc_traffic.json"))
    return ap.parse_args()


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


def rank_seed(rank: int) -> int:
    """Each rank renders its own independent synthetic stream (weak scaling)."""
    return 0x0B5E + 1009 * rank


def cpu_baseline(frames_np, W, H, nf, seconds):
    """Oracle extract + match on host cores: one extractor per thread."""
    import orbref

    def run(idx_iter, stop_at, out):
        ex = orbref.Extractor(nfeatures=nf)
        prev = None
        n = 0
        for i in idx_iter:
            if time.perf_counter() > stop_at:
                break
            k, d = ex.extract(frames_np[i % len(frames_np)])
            if prev is not None:
                orbref.search_for_initialization(prev[0], prev[1], k, d, W, H)
            prev = (k, d)
            n += 1
        out.append(n)

    # single thread (the reference's own per-frame mode)
    t0 = time.perf_counter()
    res1 = []
    run(iter(range(10 ** 9)), t0 + seconds / 3, res1)
    fps1 = res1[0] / (time.perf_counter() - t0)
    # all host cores granted to this process (16 on a one-GPU box)
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16") or 16), os.cpu_count() or 1, 16))
    res = []
    t0 = time.perf_counter()
    stop = t0 + 2 * seconds / 3
    ths = [threading.Thread(target=run, args=(iter(range(j, 10 ** 9, threads)), stop, res)) for j in range(threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    fpsN = sum(res) / (time.perf_counter() - t0)
    return {"value": round(fpsN, 2), "unit": "frames/s", "cores": threads, "kind": "port",
            "single_thread_value": round(fps1, 2),
            "sample": f"oracle extract+match on {len(frames_np)} distinct synthetic {W}x{H} frames, "
                      f"~{seconds:.0f}s bounded ({res1[0]} frames on 1 thread, {sum(res)} on {threads})"}


def main():
    args = parse()
    W, H, NF, desc_cfg = CONFIGS[args.config]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    import orbgpu
    import synth

    B = args.batch
    pitch = (W + 15) // 16 * 16
    ex = orbgpu.Extractor(nfeatures=NF, width=W, height=H, max_batch=B)
    cap = ex.max_keypoints
    frames = synth.torch_stream(B, W, H, seed=rank_seed(rank), device=dev, pitch=pitch)
    # frame slots 0..B: slot 0 holds the previous step's last frame, slots
    # 1..B this step's frames, so all B (t-1, t) pairs are one matcher launch
    kps_all = torch.zeros((B + 1, cap, 7), dtype=torch.float32, device=dev)
    desc_all = torch.zeros((B + 1, cap, 32), dtype=torch.uint8, device=dev)
    counts_all = torch.zeros(B + 1, dtype=torch.int32, device=dev)
    kps, desc, counts = kps_all[1:], desc_all[1:], counts_all[1:]
    m12 = torch.zeros((B, cap), dtype=torch.int32, device=dev)
    nmatch = torch.zeros(B, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    flags = orbgpu.MATCH_CHECK_ORI

    def step(ev=None):
        ex.extract_batch(frames, kps, desc, counts, stream=stream, row_step=pitch, frame_step=pitch * H)
        if ev is not None:
            ev[0].record(stream)
        orbgpu.search_for_initialization_batch(W, H, kps_all[:-1], desc_all[:-1], counts_all[:-1], kps_all[1:],
                                               desc_all[1:], counts_all[1:], m12, nmatch, flags=flags, stream=stream)
        if ev is not None:
            ev[1].record(stream)
        kps_all[0].copy_(kps_all[B])
        desc_all[0].copy_(desc_all[B])
        counts_all[0].copy_(counts_all[B])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ex.sync(stream)

    # parity spot check of this rank's frame 0 against the oracle (untimed)
    parity = None
    if rank == 0:
        try:
            import orbref
            ref = orbref.Extractor(nfeatures=NF)
            f0 = frames[0, :, :W].cpu().numpy()
            kr, dr = ref.extract(f0)
            n0 = int(counts[0].item())
            kg = orbgpu.keypoints_from_raw(kps[0, :n0].cpu().numpy())
            parity = bool(n0 == len(kr) and kg.tobytes() == kr.tobytes() and
                          np.array_equal(desc[0, :n0].cpu().numpy(), dr))
        except Exception as e:  # report, never hide
            parity = f"error: {e}"

    ex.profile(True)
    ex.stage_times(reset=True)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(evs[i])
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    elapsed, frames_total = aggregate(elapsed, B * args.steps, device=dev)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    ex.sync(stream)
    stage_ms, nb = ex.stage_times(reset=True)
    ex.profile(False)
    match_ms = sum(a.elapsed_time(b) for a, b in evs)

    if rank != 0:
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return

    fps = frames_total / elapsed
    per_step = {k: v / max(nb, 1) for k, v in stage_ms.items()}
    per_step["match"] = match_ms / args.steps
    pyr_bytes = pyramid_bytes_per_frame(ex.level_sizes) * B
    pyr_s = per_step["pyramid"] / 1e3
    achieved = pyr_bytes / pyr_s / 1e9 if pyr_s > 0 else None
    traffic = None
    tpath = Path(args.traffic_json)
    if tpath.exists():
        try:
            tj = json.loads(tpath.read_text())
            if tj.get("config") == args.config and tj.get("batch") == B:
                traffic = tj.get("pyramid_hbm_bytes_per_step")
        except Exception:
            traffic = None
    line = {
        "metric": METRIC,
        "value": round(fps, 1),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": desc_cfg, "config": args.config, "frames_per_gpu_per_step": B,
                   "width": W, "height": H, "nfeatures": NF, "parallelism": f"frame-sharded x{world}"},
        "roofline": {"bound": "hbm", "kernel": PYR_KERNEL_LABEL.get(os.environ.get("ORBGPU_PYR_MODE", "stream"),
                                                               PYR_KERNEL_LABEL["stream"]),
                     "achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                     "traffic": traffic, "algorithmic_bytes_per_step": pyr_bytes},
        "stages_ms_per_step": {k: round(v, 4) for k, v in per_step.items()},
        "keypoints_per_frame": round(float(counts.float().mean().item()), 1),
        "matches_per_pair": round(float(nmatch.float().mean().item()), 1),
        "parity_frame0_vs_oracle": parity,
    }
    if world == 1 and not args.no_cpu_baseline:
        frames_np = frames[: min(B, 24), :, :W].cpu().numpy()
        line["cpu_baseline"] = cpu_baseline(frames_np, W, H, NF, args.cpu_seconds)
    print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
