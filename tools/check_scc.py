"""Guard against a ROCm 7.2 (LLVM 22) gfx950 miscompile found in this repo.

Pattern: a value loaded from LDS at a wave-uniform address is compared with
a VALU `v_cmp_* vcc, ...`, and the select that consumes the comparison is
emitted as a scalar `s_cselect_*`, which reads SCC -- a flag the v_cmp never
wrote -- so the select takes a stale SCC from an earlier scalar op
(reproducer: tools/scc_repro.hip).  This script scans device assembly
(`hipcc -S --cuda-device-only`) and reports every s_cselect / s_cbranch_scc*
whose nearest preceding definition of SCC-or-VCC in the same basic block is
a VALU compare into VCC, unless the compare's VCC is read by an instruction before the consumer or
by the consumer itself (vcc / vcc_lo / vcc_hi as a source operand),
or after it before VCC is redefined in the same block (then the compare has its own user and the
consumer's SCC comes from an earlier scalar op), or the SCC the consumer actually reads was set
in that block by `s_and_b64 s, vcc, exec` -- the compiler's uniform lowering
of an earlier compare (a later v_cmp into VCC for another purpose may sit
in between).  build() runs it over every kernel and fails the build on a
hit.
"""
from __future__ import annotations

import re
import sys

SCC_WRITERS = re.compile(
    r"^\s*s_(cmp|cmpk|and|or|xor|andn2|orn2|nand|nor|xnor|add|addc|sub|subb|min|max|lshl|lshr|ashr|bfe|"
    r"not|abs|bitcmp|absdiff|lshl\d_add|mul_hi|cselect_b|movk)_?")
VCC_CMP = re.compile(r"^\s*v_cmp\w*_e32\s+vcc")
UNIFORM_AND = re.compile(r"^\s*s_and_b64\s+s\[\d+:\d+\],\s*(vcc,\s*exec|exec,\s*vcc)\s*$")
CONSUMER = re.compile(r"^\s*(s_cselect_b(32|64)|s_cbranch_scc[01])\b")
LABEL = re.compile(r"^\S+:")


def vcc_read(lines, lo, hi):
    """True when an instruction in lines[lo:hi] reads VCC (v_cndmask, s_and, ...): the compare
    then feeds that reader, and the SCC consumer's flag comes from an earlier scalar op."""
    for k in range(lo, hi):
        ins = lines[k].strip()
        if ins.startswith(";") or VCC_CMP.match(ins):
            continue
        ops = ins.split(None, 1)
        if len(ops) == 2 and re.search(r"\bvcc(_lo|_hi)?\b", ops[1].split(",", 1)[1] if "," in ops[1] else ""):
            return True
    return False


def vcc_read_after(lines, i):
    """True when VCC (as left by the compare) is read after the consumer at line i, before it is
    redefined or the basic block ends."""
    for k in range(i + 1, min(len(lines), i + 60)):
        ins = lines[k].strip()
        if LABEL.match(ins) or ins.startswith("s_cbranch") or ins.startswith("s_branch"):
            return False
        if ins.startswith(";") or not ins:
            continue
        if VCC_CMP.match(ins):
            return False
        ops = ins.split(None, 1)
        if len(ops) < 2:
            continue
        args = [a.strip() for a in ops[1].split(",")]
        if "vcc" in args[1:]:
            return True
        if args[0] == "vcc":
            return False
    return False


def scan(lines):
    hits = []
    for i, line in enumerate(lines):
        if not CONSUMER.match(line):
            continue
        cmp_at = None  # nearest v_cmp into VCC above the consumer, if it comes before any SCC writer
        for j in range(i - 1, max(-1, i - 60), -1):
            prev = lines[j]
            if LABEL.match(prev):
                break
            if prev.lstrip().startswith(";"):
                continue
            if SCC_WRITERS.match(prev) and not prev.lstrip().startswith("s_cselect"):
                if cmp_at is not None and not UNIFORM_AND.match(prev):
                    hits.append((i + 1, line.strip(), cmp_at + 1, lines[cmp_at].strip()))
                cmp_at = None
                break
            # (the consumer itself reading VCC as a source, e.g. s_cselect_b32 s, vcc_hi, 0
            # after s_cmp: the compare's mask is its data, its SCC the earlier scalar compare)
            if VCC_CMP.match(prev) and cmp_at is None and not vcc_read(lines, j + 1, i + 1) and \
                    not vcc_read_after(lines, i):
                cmp_at = j
        if cmp_at is not None:  # reached the block start: SCC comes from another block
            hits.append((i + 1, line.strip(), cmp_at + 1, lines[cmp_at].strip()))
    return hits


def main(paths) -> int:
    bad = 0
    for p in paths:
        with open(p) as fh:
            lines = fh.read().splitlines()
        for ln, ins, pln, pins in scan(lines):
            print(f"{p}:{ln}: '{ins}' consumes SCC but the flag was last computed by VALU '{pins}' (line {pln})")
            bad += 1
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
