#!/usr/bin/env python3
"""Per-call timeline of a traced drop-in run (tools/gpu_r4_dropin.sh): the
kernel and memory-copy records merged by start time, cut into calls at each
host-to-device copy that follows a device-to-host one, then for every
position in a call the median duration and the median gap since the
previous event ended.

usage: dropin_timeline.py <rocprofv3 output dir> [--skip N]
       [--anchor NAME --before B --after A]   (calls found around a kernel)
"""
import csv
import glob
import os
import statistics
import sys


def _rows(pattern):
    out = []
    for p in glob.glob(pattern, recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def main():
    d = sys.argv[1]
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 20
    ev = []
    for r in _rows(os.path.join(d, "**", "*kernel_trace.csv")):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-48:]))
    for r in _rows(os.path.join(d, "**", "*memory_copy_trace.csv")):
        name = r.get("Direction", "copy")
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    ev.sort()
    if "--anchor" in sys.argv:
        # calls without copy-engine transfers: the events from `before` events ahead
        # of each event whose name contains ANCHOR to `after` events behind it
        anchor = sys.argv[sys.argv.index("--anchor") + 1]
        before = int(sys.argv[sys.argv.index("--before") + 1]) if "--before" in sys.argv else 1
        after = int(sys.argv[sys.argv.index("--after") + 1]) if "--after" in sys.argv else 3
        idx = [i for i, e in enumerate(ev) if anchor in e[2] and i >= before and i + after < len(ev)]
        group = [ev[i - before:i + after + 1] for i in idx]
        group = group[skip:] if len(group) > 2 * skip else group
        key = tuple(x[2] for x in group[0])
        group = [c for c in group if tuple(x[2] for x in c) == key]
        _report(key, group, len(idx))
        return
    calls, cur, last_d2h = [], [], False
    for e in ev:
        h2d = "HOST_TO_DEVICE" in e[2].upper()
        if h2d and last_d2h and cur:
            calls.append(cur)
            cur = []
        cur.append(e)
        last_d2h = "DEVICE_TO_HOST" in e[2].upper()
    if cur:
        calls.append(cur)
    shape = {}
    for c in calls:
        shape.setdefault(tuple(x[2] for x in c), []).append(c)
    key, group = max(shape.items(), key=lambda kv: len(kv[1]))
    group = group[skip:] if len(group) > 2 * skip else group
    _report(key, group, len(calls))


def _report(key, group, ncalls):
    print(f"{ncalls} calls, {len(group)} of the most common shape ({len(key)} events)")
    spans = [c[-1][1] - c[0][0] for c in group]
    print(f"call span (first event start -> last event end): median {statistics.median(spans) / 1e3:.1f} us, "
          f"p90 {sorted(spans)[int(0.9 * len(spans))] / 1e3:.1f} us")
    for i, name in enumerate(key):
        dur = statistics.median(c[i][1] - c[i][0] for c in group) / 1e3
        gap = statistics.median(c[i][0] - c[i - 1][1] for c in group) / 1e3 if i else 0.0
        print(f"  {i:2d} {name:50s} dur {dur:7.1f} us   gap before {gap:6.1f} us")
    if len(group) > 1:
        between = statistics.median(group[j + 1][0][0] - group[j][-1][1] for j in range(len(group) - 1)) / 1e3
        print(f"between calls (last event end -> next call's first start): median {between:.1f} us")


if __name__ == "__main__":
    main()
