"""Per-basic-block instruction counts of one kernel in a .s file
(usage: asm_blocks.py file.s kernel_substring)."""
import sys

lines = open(sys.argv[1]).read().splitlines()
key = sys.argv[2]
start = next(i for i, l in enumerate(lines) if key in l and l.endswith(":") or (key in l and ": ;" in l))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
blocks = [{"name": "entry", "v": 0, "s": 0, "ds": 0, "vm": 0, "line": start + 1, "loop": ""}]
for i in range(start + 1, end):
    l = lines[i]
    t = l.strip()
    if l.startswith(".LBB") or t.startswith("; %bb."):
        blocks.append({"name": l.split()[0] if l.startswith(".LBB") else t.split()[1], "v": 0, "s": 0, "ds": 0,
                       "vm": 0, "line": i + 1, "loop": "LOOP" if "Loop" in l else ""})
        continue
    b = blocks[-1]
    if t.startswith("v_"):
        b["v"] += 1
    elif t.startswith("s_"):
        b["s"] += 1
    elif t.startswith("ds_"):
        b["ds"] += 1
    elif t.startswith(("global_", "buffer_", "flat_")):
        b["vm"] += 1
tot = {"v": 0, "s": 0, "ds": 0}
for b in blocks:
    for k in tot:
        tot[k] += b[k]
    if b["v"] + b["ds"] + b["vm"] >= int(sys.argv[3] if len(sys.argv) > 3 else 6):
        print(f'{b["name"]:12s} line {b["line"]:5d} valu {b["v"]:4d} salu {b["s"]:3d} ds {b["ds"]:3d} vmem {b["vm"]:3d} {b["loop"]}')
print("total", tot)
