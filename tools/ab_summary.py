"""Summaries of a tools/gpu_r4_ab.sh run: bench stage times per variant and
the per-launch PMC counters of the extraction kernels.
usage: python tools/ab_summary.py <tag> <variant>..."""
import csv
import glob
import json
import sys
from collections import defaultdict

tag, variants = sys.argv[1], ["base"] + sys.argv[2:]
for v in variants:
    for f in sorted(glob.glob(f"gpurun_out/{tag}_{v}_*.log")):
        try:
            d = json.loads([l for l in open(f) if l.startswith("{")][-1])
            print(f"{f:40s} {d['value']:10.1f} {d['stages_ms_per_step']}")
        except Exception as e:
            print(f, "no line", e)
    par = glob.glob(f"gpurun_out/{tag}_par_{v}.log")
    if par:
        print("  parity:", open(par[0]).read().strip().splitlines()[-1])
for v in variants:
    p = glob.glob(f"gpurun_out/{tag}_pmc_{v}/q_counter_collection.csv") + \
        glob.glob(f"gpurun_out/{tag}_pmc_{v}/*/q_counter_collection.csv")
    if not p:
        continue
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(p[0])):
        k = r["Kernel_Name"]
        for key in ("pyramid_tick", "fast_cells", "describe_kernel", "octree_kernel<256>", "match_init_kernel<512>"):
            if key in k:
                acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[key].add(r["Dispatch_Id"])
    print(f"PMC {v} (per launch):")
    for key, c in acc.items():
        n = max(len(disp[key]), 1)
        print("  ", key, {kk: round(vv / n / 1e6, 3) for kk, vv in sorted(c.items())}, "(M)")
