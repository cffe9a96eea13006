#!/usr/bin/env python3
"""Table of bench lines from gpurun_out/<tag>_<lib>_<round>.log files:
frames/s and stage ms per library, each round."""
import glob
import json
import re
import sys

tag = sys.argv[1]
rows = {}
for f in sorted(glob.glob(f"gpurun_out/{tag}_*.log")):
    m = re.match(rf"gpurun_out/{re.escape(tag)}_(.+)_(\d+)\.log$", f)
    if not m:
        continue
    for line in open(f):
        if line.startswith("{"):
            j = json.loads(line)
            st = j["stages_ms_per_step"]
            rows.setdefault(m.group(1), []).append((int(m.group(2)), j["value"], st))
for lib, rs in rows.items():
    for r, v, st in sorted(rs):
        print(f"{lib:16s} r{r} {v:10.1f}  " + "  ".join(f"{k} {x:.4f}" for k, x in st.items()))
