#!/usr/bin/env python3
"""Per-step times (events on the extraction stream, BENCH_STEP_TRACE) of the
mono640 stream: a 400-step leg, then 5 warm-up + 20 timed steps, repeated, to
see where inside the 20 steps the driver-shaped leg loses time against the
long one.  usage (GPU box): BENCH_STEP_TRACE=1 python3 tools/warm_probe2.py"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import torch  # noqa: E402


def main():
    og = bench.load_engine(None)
    torch.cuda.set_device(0)
    D = bench.Dev(torch.device("cuda", 0))
    stream = D.stream(priority=-1)
    torch.cuda.set_stream(stream)
    W, H, NF, _ = bench.CONFIGS["mono640"]
    sb = bench.StreamBench(og, D, W, H, NF, 512, 0, 1, stream, deliver="gpu0")
    for rep in range(2):
        for name, w, k in (("long", 5, 1000), ("short", 5, 20), ("short", 5, 20)):
            r = sb.run(w, k)
            st = sb.step_ms["gpu"]
            print(json.dumps({"rep": rep, "leg": name, "fps": round(r["fps"], 1),
                              "stages": {a: round(b, 4) for a, b in r["per_step"].items()},
                              "first10": st[:10], "last10": st[-10:],
                              "mean_mid": round(sum(st[5:-5]) / max(len(st) - 10, 1), 4),
                              "means_per_50": [round(sum(st[i:i + 50]) / len(st[i:i + 50]), 4)
                                               for i in range(0, len(st), 50)]}), flush=True)
    sb.close()


if __name__ == "__main__":
    main()
