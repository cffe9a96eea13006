"""The drop-in C++ classes' latency (bench.py's drop_in leg without the CPU
column): one JSON line of per-op median / p90 / p99 microseconds."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402

r = bench.drop_in_latency(with_cpu=False)
ops = r.get("ops", r)
print(json.dumps({k: ({kk: v[kk] for kk in ("median_us", "p90_us", "p99_us") if kk in v} if isinstance(v, dict) else v)
                  for k, v in ops.items()}), flush=True)
