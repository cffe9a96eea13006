"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel (largest
grid only, i.e. the full-batch launches), mean of each counter per dispatch."""
import csv
import sys
from collections import defaultdict


def load(path):
    rows = list(csv.DictReader(open(path)))
    per = defaultdict(lambda: defaultdict(list))
    grid = {}
    for r in rows:
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1]
        g = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
        key = (k, g)
        per[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        grid[k] = max(grid.get(k, 0), g)
    out = {}
    for (k, g), cs in per.items():
        if g != grid[k]:
            continue
        # counter rows are per dispatch (already summed over XCDs/SEs by rocprofv3)
        out[k] = {c: sum(v) / max(1, len(v)) for c, v in cs.items()}
        out[k]["_grid"] = g
    return out


if __name__ == "__main__":
    merged = defaultdict(dict)
    for p in sys.argv[1:]:
        for k, d in load(p).items():
            merged[k].update(d)
    for k, d in sorted(merged.items()):
        print(k)
        for c, v in sorted(d.items()):
            print(f"   {c:28s} {v:16.0f}")
        if "SQ_WAVE_CYCLES" in d:
            wc = d["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if c in d:
                    print(f"   {c:28s} {100 * d[c] / wc:6.1f} % of wave cycles")
