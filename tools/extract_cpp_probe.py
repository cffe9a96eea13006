"""ORB_SLAM2::ORBextractor::operator() (the C++ drop-in class over
liborbgpu.so, tests/cpp/adapter_main) latency: ADAPTER_REPS calls (default
1000) per run, runs interleaved over the environment variants given as
label=ENV=V[,ENV=V] (label alone: the environment as is), ROUNDS rounds.
Prints one line per run: label, median / p90 / p99 us."""
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "orb-slam2-annotation_amd"))
import synth  # noqa: E402

variants = []
for a in sys.argv[1:]:
    label, _, envs = a.partition("=")
    env = dict(kv.split("=", 1) for kv in envs.split(",") if kv) if envs else {}
    variants.append((label, env))
with tempfile.TemporaryDirectory(prefix="orbgpu_xp_") as td:
    d = Path(td)
    fr = synth.mono_stream(2, 640, 480)
    for k in range(2):
        (d / f"f{k}.raw").write_bytes(fr[k].tobytes())
    for r in range(int(os.environ.get("ROUNDS", "3"))):
        for label, extra in variants:
            log = d / f"t_{label}_{r}.jsonl"
            env = dict(os.environ, ADAPTER_REPS=os.environ.get("REPS", "1000"), ADAPTER_TIME_LOG=str(log), **extra)
            subprocess.run([str(ROOT / "tests" / "cpp" / "adapter_main"), "extract", "640", "480", "1000",
                            str(d / "f0.raw"), str(d / "f1.raw"), str(d / "x.out")], check=True, env=env,
                           capture_output=True, timeout=300)
            for line in log.read_text().splitlines():
                j = json.loads(line)
                if j.get("op") == "ORBextractor::operator()":
                    print(f"{label:12s} round {r}: median {j['median_us']:7.1f}  p90 {j['p90_us']:7.1f}  "
                          f"p99 {j['p99_us']:7.1f} us", flush=True)
