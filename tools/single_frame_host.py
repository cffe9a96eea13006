#!/usr/bin/env python3
"""Host-side breakdown of the single-frame drop-in call from a rocprofv3
--kernel-trace --hip-runtime-trace run of tools/single_frame_probe.py: per
call (cut at each hipStreamSynchronize), the medians of
  pre      previous sync's end -> this call's first kernel launch API start
           (host work before the GPU sees the frame: result copies of the
           previous call, Python, the image memcpy into pinned staging)
  launch   first launch API start -> first kernel start
  kernels  first kernel start -> last kernel end
  wake     last kernel end -> hipStreamSynchronize end
  apis     summed duration of the launch API calls of the call
usage: single_frame_host.py <rocprofv3 output dir> [--skip N]
"""
import csv
import glob
import os
import statistics
import sys


def _rows(d, pat):
    out = []
    for p in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def main():
    d = sys.argv[1]
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 20
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in _rows(d, "*kernel_trace.csv"))
    api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Function", r.get("Operation", "")))
                 for r in _rows(d, "*hip_api_trace.csv"))
    syncs = [a for a in api if a[2] in ("hipStreamSynchronize", "hipEventSynchronize", "hipDeviceSynchronize")]
    launches = [a for a in api if "Launch" in a[2]]
    rows = []
    prev_end = None
    for s in syncs:
        if prev_end is None:
            prev_end = s[1]
            continue
        kk = [k for k in ks if prev_end <= k[0] <= s[1]]
        ll = [a for a in launches if prev_end <= a[0] <= s[0]]
        if kk and ll:
            rows.append({"pre": ll[0][0] - prev_end, "launch": kk[0][0] - ll[0][0],
                         "kernels": max(k[1] for k in kk) - kk[0][0], "wake": s[1] - max(k[1] for k in kk),
                         "apis": sum(a[1] - a[0] for a in ll), "nlaunch": len(ll), "total": s[1] - ll[0][0]})
        prev_end = s[1]
    rows = rows[skip:]
    print(f"{len(rows)} calls (after skipping {skip})")
    for key in ("pre", "launch", "kernels", "wake", "apis", "total"):
        v = [r[key] / 1e3 for r in rows]
        if v:
            print(f"  {key:8s} median {statistics.median(v):8.2f} us")
    if rows:
        print(f"  launches per call: {statistics.median([r['nlaunch'] for r in rows])}")
    names = {}
    for a in api:
        names.setdefault(a[2], []).append((a[1] - a[0]) / 1e3)
    for n, v in sorted(names.items(), key=lambda kv: -sum(kv[1]))[:12]:
        print(f"  api {n:36s} n {len(v):6d}  median {statistics.median(v):7.2f} us")


if __name__ == "__main__":
    main()
