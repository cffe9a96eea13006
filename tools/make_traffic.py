"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs,
they do not fit one pass on gfx950) into profiles/pmc_traffic.json, which
bench.py reports as roofline.traffic.

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE counts
half the bytes of a wide coalesced streaming read, so read bytes =
2 x FETCH_SIZE; WRITE_SIZE is exact for 16-B-per-lane stores.  Both are in
KiB per dispatch.

usage: make_traffic.py FETCH.csv WRITE.csv --config mono640 --batch 512 [--out F]
"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_summary import load  # noqa: E402

KERNEL = "pyramid_tick"  # matched as a prefix (pyramid_tick_kernel<E, NP>)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--config", default="mono640")
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--algorithmic", type=int, default=None, help="algorithmic bytes per launch")
    ap.add_argument("--out", default=str(Path(__file__).resolve().parents[1] / "profiles" / "pmc_traffic.json"))
    a = ap.parse_args()
    f = load(a.fetch_csv)
    w = load(a.write_csv)
    kf = next(k for k in f if k.startswith(KERNEL))
    kw = next(k for k in w if k.startswith(KERNEL))
    fetch_kib = f[kf]["FETCH_SIZE"]
    write_kib = w[kw]["WRITE_SIZE"]
    read_b = 2.0 * fetch_kib * 1024.0
    write_b = write_kib * 1024.0
    out = {
        "kernel": KERNEL,
        "kernel_name": kf,
        "config": a.config,
        "batch": a.batch,
        "fetch_size_kib_raw": fetch_kib,
        "write_size_kib_raw": write_kib,
        "read_bytes_corrected": read_b,
        "write_bytes": write_b,
        "pyramid_hbm_bytes_per_step": int(read_b + write_b),
        "correction": "read = 2 x FETCH_SIZE (gfx950 half-count on wide streaming reads); write = WRITE_SIZE",
        "sources": [a.fetch_csv, a.write_csv],
    }
    if a.algorithmic:
        out["algorithmic_bytes_per_step"] = a.algorithmic
        out["traffic_over_algorithmic"] = (read_b + write_b) / a.algorithmic
    Path(a.out).write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
