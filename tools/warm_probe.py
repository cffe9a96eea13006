#!/usr/bin/env python3
"""Why the driver's headline (20 timed steps after 5 warm-up steps) runs ~6 %
below the sustained rate: the mono640 stream of bench.py run back to back
with different warm-up lengths and idle gaps, per-step wall times from events
on the extraction stream, and the per-stage times of each run.

usage (GPU box): python3 tools/warm_probe.py > gpurun_out/x.json"""
import json
import sys
import time
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
    out = []

    def leg(name, warmup, steps, idle_before=0.0):
        if idle_before:
            time.sleep(idle_before)
        r = sb.run(warmup, steps)
        out.append({"leg": name, "warmup": warmup, "steps": steps, "idle_before_s": idle_before,
                    "fps": round(r["fps"], 1), "ms_per_step": round(r["elapsed"] / steps * 1e3, 4),
                    "stages": {k: round(v, 4) for k, v in r["per_step"].items()}})
        print(json.dumps(out[-1]), flush=True)

    leg("cold W5 K20", 5, 20)
    leg("again W5 K20", 5, 20)
    leg("W60 K20", 60, 20)
    leg("W5 K20 after 10 ms idle", 5, 20, 0.01)
    leg("W5 K20 after 100 ms idle", 5, 20, 0.1)
    leg("W5 K20 after 1 s idle", 5, 20, 1.0)
    leg("W5 K400", 5, 400)
    leg("W5 K20 right after", 5, 20)
    leg("W0 K20 right after", 0, 20)
    leg("W5 K100", 5, 100)
    sb.close()


if __name__ == "__main__":
    main()
