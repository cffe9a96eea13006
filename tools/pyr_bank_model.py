#!/usr/bin/env python3
"""Analytic LDS bank-conflict model of the tick pyramid's horizontal pass
(VERDICT r4 #7): lane c of a 32-lane half takes the 8-pixel output column c,
i.e. quads 2c and 2c+1, and reads each quad's 12-byte source window as three
dwords.  A quad q of a 1.2x downscale starts at source pixel
floor(4.8 q + 0.1), so its window's first dword is d(q) = floor(that / 4) and
consecutive lanes' windows sit 2.4 dwords apart: 32 lanes span ~77 dwords,
more than the 32 banks of ds_read_b32 ((a/4) mod 32, MI355X_MICROARCH.md
§LDS), so every window read is 2-way conflicted whatever the row's LDS base
or pitch (the row base only rotates the banks).  Padding ring rows per level
cannot remove it; only a lane order that keeps each half within 32 dwords of
one row (about 13 columns) or interleaves rows whose bases are ~13 dwords
apart could, and round 4 measured that mixing row groups in a wave costs more
(tick imbalance) than the conflicts (hidden behind VALU issue).

usage: pyr_bank_model.py [W H]   (default 640 480)"""
import collections
import math
import sys


def d(q):
    return math.floor(math.floor(4.8 * q + 0.1) / 4)


def main():
    W, H = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (640, 480)
    tot = n = 0
    worst = collections.Counter()
    for c0 in range(0, 200, 7):
        for base in range(0, 32, 5):
            for which in (0, 1):
                for j in range(3):
                    banks = collections.Counter((base + d(2 * (c0 + c) + which) + j) % 32 for c in range(32))
                    m = max(banks.values())
                    worst[m] += 1
                    tot += m - 1
                    n += 1
    print(f"max bank multiplicity per 32-lane half: {dict(sorted(worst.items()))}")
    print(f"mean extra LDS cycles per half per window dword read: {tot / n:.2f}")
    sizes = [(W, H)]
    s = 1.0
    for _ in range(7):
        s *= 1.2
        sizes.append((round(W / s), round(H / s)))
    lane_reads = sum(h * math.ceil(w / 4) * 1.2 * 3 for w, h in sizes[1:])
    wi = lane_reads / 64 * 512
    print(f"window dword reads per 512 frames: {wi / 1e6:.2f} M wave-instructions")
    print(f"modelled conflict cycles per launch: {wi * 2 * tot / n / 1e6:.1f} M "
          f"(measured SQ_LDS_BANK_CONFLICT, round 4: 16.5 M incl. the vertical pass and table reads)")


if __name__ == "__main__":
    main()
