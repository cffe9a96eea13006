"""Drop-in class latencies alone (bench.py's DropIn, no CPU oracle): for
rocprofv3 kernel traces of the per-call paths.  usage: python tools/dropin_profile.py [reps]"""
import json
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
with tempfile.TemporaryDirectory(prefix="orbgpu_dropin_") as td:
    ops = bench.DropIn(Path(td), reps=reps).run()
print(json.dumps({k: ({f: v.get(f) for f in ("median_us", "p90_us", "p99_us", "max_us")} if isinstance(v, dict) else v)
                  for k, v in ops.items()}, indent=1))
