#!/usr/bin/env python3
"""Per-launch durations of selected kernels from a rocprofv3 kernel trace
(ks_kernel_trace.csv): for each kernel whose name contains one of the given
substrings (and, optionally, a given number of workgroups), the launch count and the
median / min / max / mean duration in microseconds; plus, with --between,
the kernels launched on the extraction's stream between consecutive launches
of a marker kernel (e.g. copies between 512-frame pyramid launches).

usage: kernel_launches.py TRACE.csv [--kernel SUBSTR[:GRID_X]]... [--between SUBSTR:GRID_X] [--json OUT]
"""
import csv
import json
import statistics
import sys


def main():
    args = sys.argv[1:]
    path = args[0]
    kernels, between, out = [], None, None
    i = 1
    while i < len(args):
        if args[i] == "--kernel":
            kernels.append(args[i + 1])
            i += 2
        elif args[i] == "--between":
            between = args[i + 1]
            i += 2
        elif args[i] == "--json":
            out = args[i + 1]
            i += 2
        else:
            sys.exit(f"unknown argument {args[i]}")
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))

    def match(r, spec):
        name, _, grid = spec.partition(":")
        blocks = int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1)  # GRID = workgroups
        return name in r["Kernel_Name"] and (not grid or blocks == int(grid))

    res = {"trace": path, "kernels": {}}
    for spec in kernels:
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if match(r, spec)]
        if not d:
            res["kernels"][spec] = {"launches": 0}
            continue
        res["kernels"][spec] = {"launches": len(d), "median_us": round(statistics.median(d), 2),
                                "min_us": round(min(d), 2), "max_us": round(max(d), 2),
                                "mean_us": round(statistics.mean(d), 2)}
    if between:
        marks = [r for r in rows if match(r, between)]
        if marks:
            q = marks[0]["Queue_Id"]
            gaps = []
            for a, b in zip(marks, marks[1:]):
                t0, t1 = int(a["Start_Timestamp"]), int(b["Start_Timestamp"])
                mid = [r["Kernel_Name"][:60] for r in rows if r["Queue_Id"] == q and t0 < int(r["Start_Timestamp"]) < t1]
                gaps.append(mid)
            names = {}
            for g in gaps:
                for n in g:
                    names[n] = names.get(n, 0) + 1
            res["between"] = {"marker": between, "queue": q, "intervals": len(gaps),
                              "kernels_per_interval": {n: round(c / max(len(gaps), 1), 2) for n, c in names.items()}}
    s = json.dumps(res, indent=1)
    if out:
        open(out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
