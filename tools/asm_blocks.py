#!/usr/bin/env python3
"""Per-basic-block instruction counts of one kernel in a device .s file
(hipcc -S --cuda-device-only): VALU / SALU / LDS / VMEM / SMEM per block and
the block's most frequent VALU opcodes -- to attribute a kernel's
SQ_INSTS_VALU per launch to its phases.

usage: asm_blocks.py FILE.s KERNEL_SUBSTRING [--top N]
"""
import collections
import re
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 6
    s = open(path).read()
    m = re.search(r"^(\S*%s\S*):" % re.escape(name), s, re.M)
    if not m:
        sys.exit("kernel not found")
    end = s.index(".Lfunc_end", m.end())
    blocks, cur = [], ["entry", []]
    for raw in s[m.end():end].splitlines():
        l = raw.split(";")[0].strip()
        if not l or l.startswith("."):
            if re.match(r"^\.LBB\S*:", raw.strip()):
                blocks.append(cur)
                cur = [raw.strip().rstrip(":"), []]
            continue
        cur[1].append(l)
        if l.startswith(("s_cbranch", "s_branch")):  # fall-through: a block of its own
            blocks.append(cur)
            cur = [cur[0].split("+")[0] + "+", []]
    blocks.append(cur)
    tot = collections.Counter()
    for lab, ins in blocks:
        c = collections.Counter()
        ops = collections.Counter()
        for l in ins:
            op = l.split()[0]
            if op.startswith("v_"):
                c["valu"] += 1
                ops[op] += 1
            elif op.startswith("s_"):
                k = "smem" if op.startswith(("s_load", "s_buffer_load")) else "salu"
                c[k] += 1
            elif op.startswith("ds_"):
                c["lds"] += 1
            elif op.startswith(("global_", "buffer_", "flat_")):
                c["vmem"] += 1
        tot.update(c)
        tail = ins[-1].split()[0] if ins else ""
        print("%-14s valu %4d salu %4d lds %3d vmem %3d smem %3d  end %-22s %s" % (
            lab, c["valu"], c["salu"], c["lds"], c["vmem"], c["smem"], tail,
            " ".join("%s:%d" % kv for kv in ops.most_common(top))))
    print("total", dict(tot))


if __name__ == "__main__":
    main()
