"""bench.py's multi-rank path end to end on the CPU:

`python bench.py --gpus 2 --cpu-dry-run tests/dryrun_orbgpu.py ...` goes
through the same launcher a driver's `bench.py --gpus N` uses (no
WORLD_SIZE -> a torchrun child with N ranks, gloo here instead of RCCL), the
same per-rank chunking, boundary exchange and gather to rank 0 as the GPU
run, with the CPU oracle standing in for the kernels.  Rank 0 dumps what it
gathered; the test recomputes the whole stream in one process and requires
equality:

* mono: every frame's keypoints / descriptors and SearchForInitialization
  (t-1, t) matches, including the pairs that straddle two ranks' chunks and
  two steps;
* stereo (EuRoC geometry): every pair's L/R keypoints, descriptors and the
  ComputeStereoMatches uRight / depth, pairs on both sides of a chunk
  boundary;
* the JSON line reports n_gpus == world_size_checked == 2.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
ENGINE = ROOT / "tests" / "dryrun_orbgpu.py"


def _run_bench(tmp_path, *args, timeout=420, world=2):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    env["OMP_NUM_THREADS"] = "2"
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", str(world), "--cpu-dry-run", str(ENGINE), "--dump",
           str(tmp_path), "--no-cpu-baseline", "--no-extras", *args]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=str(ROOT))
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-3000:]
    return json.loads(lines[0])


def test_gpus_flag_rejects_mismatched_world_size():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--cpu-dry-run", str(ENGINE)],
                         capture_output=True, text=True, timeout=120, env=env, cwd=str(ROOT))
    assert out.returncode != 0 and "WORLD_SIZE=1" in out.stderr


def _merge_rank_dumps(tmp_path, name, world):
    parts = [np.load(tmp_path / f"{name}_rank{r}.npz") for r in range(world)]
    units = np.concatenate([p["units"] for p in parts])
    order = np.argsort(units)
    return {k: np.concatenate([p[k] for p in parts])[order] for k in parts[0].files}


def _oracle_stream(world, B, steps):
    """the whole stream in one process: per global frame (keypoints,
    descriptors, nmatches, m12 over the previous frame's keypoints)"""
    import orbref
    import shard
    import synth
    frames = {}
    for s in range(steps):
        for r in range(world):
            ids = shard.chunk_frames(s, r, world, B)
            imgs = synth.torch_stream(B, 640, 480, device="cpu", pitch=640, bounded=True, t0=ids[0])
            for b, f in enumerate(ids):
                frames[f] = imgs[b].numpy()
    ex = orbref.Extractor(1000)
    out, prev = [], None
    for f in range(world * B * steps):
        k, d = ex.extract(frames[f])
        if prev is None:
            nm, m12 = 0, np.full(0, -1, np.int32)
        else:
            nm, m12, _ = orbref.search_for_initialization(prev[0], prev[1], k, d, 640, 480)
        out.append((k, d, nm, m12))
        prev = (k, d)
    return out


def _check_stream(got, ref, B):
    assert list(got["units"]) == list(range(len(ref)))
    cross = 0
    for f, (k, d, nm, m12) in enumerate(ref):
        n = len(k)
        assert got["count"][f] == n, f
        assert got["kps"][f][:n].tobytes() == k.tobytes(), f
        assert np.array_equal(got["desc"][f][:n], d), f
        assert got["nmatch"][f] == nm, f
        assert np.array_equal(got["m12"][f][:len(m12)], m12), f
        cross += f % B == 0 and f > 0 and nm > 0
    assert cross == len(ref) // B - 1  # every chunk's first frame matched against another rank's / step's last


def _load_dump(tmp_path, deliver, world, tag=""):
    if deliver == "host":  # every rank's own delivered frames
        return _merge_rank_dumps(tmp_path, f"mono_640x480{tag}", world)
    return np.load(tmp_path / f"mono_640x480{tag}.npz")  # what rank 0 received


@pytest.mark.parametrize("deliver,parts", [("host", 1), ("gpu0", 1), ("gpu0", 2)])
def test_mono_stream_two_ranks_equals_single_process(tmp_path, deliver, parts):
    """both delivery modes (shard.Delivery): host -- each rank's trimmed
    outputs in its own host memory (merged here from the per-rank dumps);
    gpu0 -- counts first, then the used rows, received by rank 0; and the
    step as two sub-batches (--parts 2: each on its own extractor and stream).
    At N > 1 the line also runs the OTHER delivery mode over the same stream
    (`delivery_other_mode`, per-rank ms_per_step and owner waits); its
    delivered frames are checked the same way.  Pair 0 of every chunk reads
    the frame before it in place (the previous step's set at N = 1, the
    boundary frame received straight into the set at N > 1)."""
    world, B, steps = 2, 2 * parts, 2
    line = _run_bench(tmp_path, "--config", "mono640", "--batch", str(B), "--steps", str(steps), "--warmup", "0",
                      "--deliver", deliver, "--parts", str(parts))
    assert line["n_gpus"] == 2 and line["world_size_checked"] == 2
    assert line["config"]["frames_per_gpu_per_step"] == B
    assert line["config"]["sub_batches"]["parts"] == parts
    assert line["parity_vs_oracle"]["ok"] is True and line["parity_frame0_vs_oracle"] is True
    other = "gpu0" if deliver == "host" else "host"
    ol = line["delivery_other_mode"]
    assert ol["mode"] == other and ol["frames_per_s"] > 0
    for dl, mode in ((line["delivery"], deliver), (ol["delivery"], other)):
        assert dl["mode"] == mode and len(dl["per_rank"]) == 2
        assert all(p["ms_per_step"] > 0 for p in dl["per_rank"])
        if mode == "host":  # every rank moves its own outputs
            assert all(p["bytes_per_step"] > 0 for p in dl["per_rank"])
        else:  # rank 1 sends, rank 0 receives exactly that
            assert dl["per_rank"][1]["bytes_per_step"] > 0 and dl["per_rank"][0]["bytes_per_step"] == 0
            assert dl["per_rank"][0]["recv_bytes_per_step"] + 4 * 3 * B == dl["per_rank"][1]["bytes_per_step"]
    ref = _oracle_stream(world, B, steps)
    _check_stream(_load_dump(tmp_path, deliver, world), ref, B)
    _check_stream(_load_dump(tmp_path, other, world, "_other"), ref, B)


def test_sustained_leg_deferred_two_ranks(tmp_path):
    """The sustained leg handed over to the headline without host bookkeeping in
    between (StreamBench.run(defer=True); at N > 1 its collectives and
    statistics run after the headline, in the same order on every rank): with
    two gloo ranks the run completes (no collective mismatched between the
    ranks), the line carries both legs, and the headline's output set equals
    the oracle."""
    world, B, steps = 2, 2, 2
    line = _run_bench(tmp_path, "--config", "mono640", "--batch", str(B), "--steps", str(steps), "--warmup", "1",
                      "--deliver", "gpu0", "--sustained-steps", "3", "--other-delivery", "0")
    sus = line["sustained"]
    assert sus["steps"] == 3 and sus["frames_per_s"] > 0 and sus["ms_per_step"] > 0
    assert sus["headline_host_gap_ms"] >= 0 and line["value"] > 0
    # the headline's own output set (the last step) against the oracle, pairs across the
    # chunk boundary included (bench.py parity_timed)
    assert line["parity_vs_oracle"]["ok"] is True and line["n_gpus"] == world


def test_mono_stream_four_ranks_equals_single_process(tmp_path):
    """Four ranks (the driver's N = 4 launch, gloo here): the boundary frame
    passes along a ring of three chunk boundaries per step plus the step
    boundary, and in gpu0 mode rank 0 takes counts and rows from three senders
    at once (two process groups, each one op type in step order).  Both
    delivery legs equal the single-process oracle stream frame by frame, and
    rank 0's received bytes equal the three senders' rows."""
    world, B, steps = 4, 2, 2
    line = _run_bench(tmp_path, "--config", "mono640", "--batch", str(B), "--steps", str(steps), "--warmup", "0",
                      "--deliver", "gpu0", world=world, timeout=600)
    assert line["n_gpus"] == world and line["world_size_checked"] == world
    dl, ol = line["delivery"], line["delivery_other_mode"]
    assert dl["mode"] == "gpu0" and ol["mode"] == "host" and len(dl["per_rank"]) == world
    sent = [p["bytes_per_step"] for p in dl["per_rank"]]
    assert sent[0] == 0 and all(b > 0 for b in sent[1:])
    assert dl["per_rank"][0]["recv_bytes_per_step"] + 4 * 3 * B * (world - 1) == sum(sent[1:])
    assert all(p["bytes_per_step"] > 0 for p in ol["delivery"]["per_rank"])
    ref = _oracle_stream(world, B, steps)
    _check_stream(_load_dump(tmp_path, "gpu0", world), ref, B)
    _check_stream(_load_dump(tmp_path, "host", world, "_other"), ref, B)


def test_stereo_pairs_two_ranks_equal_single_process(tmp_path):
    import orbref
    import shard
    import synth
    world, P = 2, 2
    line = _run_bench(tmp_path, "--config", "euroc_stereo", "--batch", str(P), "--steps", "1", "--warmup", "0")
    assert line["n_gpus"] == 2 and line["world_size_checked"] == 2 and line["unit"] == "pairs/s"
    got = np.load(tmp_path / "stereo_752x480.npz")
    assert list(got["units"]) == list(range(world * P))
    exL, exR = orbref.Extractor(1200), orbref.Extractor(1200)
    for r in range(world):
        ids = shard.chunk_frames(0, r, world, P)
        imgs = synth.torch_stereo_stream(P, 752, 480, 18.0, device="cpu", t0=ids[0], pitch=752)
        for p, pair in enumerate(ids):
            kl, dl, kr, dr, ur, dp = orbref.stereo_frame(exL, exR, imgs[2 * p].numpy(), imgs[2 * p + 1].numpy(),
                                                         47.90639384423901)
            c = got["count"][pair]
            assert (c[0], c[1]) == (len(kl), len(kr)), pair
            assert got["kps"][pair][0][:len(kl)].tobytes() == kl.tobytes()
            assert got["kps"][pair][1][:len(kr)].tobytes() == kr.tobytes()
            assert np.array_equal(got["desc"][pair][0][:len(kl)], dl)
            assert np.array_equal(got["desc"][pair][1][:len(kr)], dr)
            assert got["uright"][pair][:len(kl)].tobytes() == ur.tobytes()
            assert got["depth"][pair][:len(kl)].tobytes() == dp.tobytes()
            assert (ur >= 0).sum() > 0.3 * len(kl)  # a real stereo scene


@pytest.mark.gpu
@pytest.mark.parametrize("deliver", ["host", "gpu0"])
def test_gpu_host_fed_stream_frames_equal_oracle(tmp_path, deliver):
    """The host-fed path on the GPU (bench.py --feed host: frames copied from
    pinned host memory through the double-buffered H2D stream) with each
    delivery mode: every delivered frame's keypoints, descriptors and matches
    equal the CPU oracle on the same frames."""
    import orbref
    import synth
    import torch
    B, steps = 3, 2
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, str(ROOT / "bench.py"), "--feed", "host", "--deliver", deliver, "--batch", str(B),
           "--steps", str(steps), "--warmup", "0", "--dump", str(tmp_path), "--no-cpu-baseline", "--no-extras"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=str(ROOT))
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    line = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert line["h2d"]["bytes_per_step"] == B * 480 * 640 and line["delivery"]["mode"] == deliver
    got = np.load(tmp_path / "mono_640x480.npz")
    assert list(got["units"]) == list(range(B * steps))
    ex = orbref.Extractor(1000)
    prev = None
    for s in range(steps):
        imgs = synth.torch_stream(B, 640, 480, device="cuda", pitch=640, bounded=True, t0=s * B).cpu()
        for b in range(B):
            f = s * B + b
            k, d = ex.extract(imgs[b].numpy())
            n = len(k)
            assert got["count"][f] == n and got["kps"][f][:n].tobytes() == k.tobytes(), f
            assert np.array_equal(got["desc"][f][:n], d), f
            if prev is not None:
                nm, m12, _ = orbref.search_for_initialization(prev[0], prev[1], k, d, 640, 480)
                assert got["nmatch"][f] == nm and np.array_equal(got["m12"][f][:len(prev[0])], m12), f
            prev = (k, d)
