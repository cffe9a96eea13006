"""VGPR / SGPR / scratch / LDS per kernel from the device assembly the build
emits (build/*.s, amdhsa metadata).  usage: python tools/kernel_resources.py [build_dir] [pattern]"""
import re
import sys
from pathlib import Path

d = Path(sys.argv[1] if len(sys.argv) > 1 else "orb-slam2-annotation_amd/build")
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for s in sorted(d.glob("*.s")):
    txt = s.read_text(errors="ignore")
    for m in re.finditer(r"\.name:\s+(\S+)\n(.*?)(?=\n  - |\n\.end_amdgpu_metadata)", txt, re.S):
        name, body = m.group(1), m.group(2)
        if pat not in name:
            continue
        get = lambda k: (re.search(rf"\.{k}:\s+(\d+)", body) or [None, "?"])[1]  # noqa: E731
        # static LDS lives in the kernel descriptor (.amdhsa_group_segment_fixed_size)
        km = re.search(r"\.amdhsa_kernel " + re.escape(name) + r"\n(.*?)\.end_amdhsa_kernel", txt, re.S)
        lds = (re.search(r"\.amdhsa_group_segment_fixed_size (\d+)", km.group(1)) if km else None)
        lds = lds.group(1) if lds else "?"
        print(f"{s.stem:18s} {name[:70]:70s} vgpr={get('vgpr_count'):>4} agpr={get('agpr_count'):>3} "
              f"sgpr={get('sgpr_count'):>3} scratch={get('private_segment_fixed_size'):>5} "
              f"lds={lds:>6} (static; dynamic LDS is set at launch)")
