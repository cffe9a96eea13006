"""Time the batched Initializer scorer (csrc/init.hip): one FindHomography +
one FindFundamental worth of hypotheses (mMaxIterations = 200) over n
matches, per monocular initialisation attempt.  Prints one JSON line."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "orb-slam2-annotation_amd")]

import torch  # noqa: E402

import initializer  # noqa: E402


def main(n=1000, nhyp=200, iters=200):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    pts = (torch.rand((n, 4), generator=g) * 600).to(dev)
    H21 = (torch.eye(3) + 1e-3 * torch.randn((nhyp, 3, 3), generator=g)).to(dev).contiguous()
    H12 = torch.linalg.inv(H21).contiguous()
    F21 = (1e-3 * torch.randn((nhyp, 3, 3), generator=g)).to(dev).contiguous()
    sh = torch.empty(nhyp, device=dev)
    sf = torch.empty(nhyp, device=dev)
    ih = torch.empty((nhyp, n), dtype=torch.uint8, device=dev)
    i_f = torch.empty((nhyp, n), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()

    def step():
        initializer.check_both_batch(pts, H21, H12, F21, 1.0, sh, ih, sf, i_f, stream=s)

    for _ in range(10):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        step()
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / iters
    print(json.dumps({"what": "CheckHomography+CheckFundamental x nhyp", "n": n, "nhyp": nhyp,
                      "us_per_attempt": round(us, 2), "attempts_per_s": round(1e6 / us, 1)}))


if __name__ == "__main__":
    main()
