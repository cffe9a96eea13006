"""D2H path probe: a 33 MB device -> pinned host copy on a side stream, alone
and beside a compute-bound kernel stream, timed with events.  Run under
`rocprofv3 --kernel-trace --memory-copy-trace` to see whether HIP moves it with
an SDMA engine or a blit kernel (a __amd_rocclr_copyBuffer dispatch on CUs)."""
import json
import sys
import time

import torch

n = 33 << 20
dev = torch.device("cuda", 0)
src = torch.randint(0, 255, (n,), dtype=torch.uint8, device=dev)
dst = torch.empty(n, dtype=torch.uint8, pin_memory=True)
cs = torch.cuda.Stream(dev)
out = {}
for it in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(cs):
        e0.record(cs)
        dst.copy_(src, non_blocking=True)
        e1.record(cs)
    cs.synchronize()
    out[f"alone_ms_{it}"] = round(e0.elapsed_time(e1), 4)
a = torch.randn(4096, 4096, device=dev)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    a = torch.tanh(a @ a * 1e-3)
torch.cuda.synchronize()
out["compute_alone_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
t0 = time.perf_counter()
for _ in range(20):
    a = torch.tanh(a @ a * 1e-3)
    with torch.cuda.stream(cs):
        dst.copy_(src, non_blocking=True)
torch.cuda.synchronize()
out["compute_with_copies_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
out["gb_per_s_alone"] = round(n / (min(out[f"alone_ms_{i}"] for i in range(3)) / 1e3) / 1e9, 2)
print(json.dumps(out))
