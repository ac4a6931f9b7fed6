"""Idle gaps of the GPU timeline in a rocprofv3 kernel trace: for the last
`--steps` training steps (split at the AdamW kernels), the time between one
kernel's end and the next kernel's start, summed and listed by the kernel
pair around the largest gaps.

    python scripts/trace_gaps.py <rocprofv3 output dir> [--top 25]
"""
import argparse
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    p = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))
    if not p:
        sys.exit(f"no kernel_trace.csv under {d}")
    rows = []
    with open(p[-1]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = load(a.dir)
    # step boundaries: the last kernel of each step is the final AdamW launch
    # before the next step's first forward kernel (embedding gather)
    starts = [i for i, r in enumerate(rows) if "gather" in r[2] or "embed_fwd" in r[2]]
    if len(starts) < 2:
        starts = [0]
    lo = starts[-2] if len(starts) >= 2 else 0
    seg = rows[lo:starts[-1]] if len(starts) >= 2 else rows
    busy = sum(e - s for s, e, _ in seg)
    wall = seg[-1][1] - seg[0][0]
    gaps = defaultdict(lambda: [0, 0])
    big = []
    end = seg[0][1]
    for (s, e, n), (_, _, prev) in zip(seg[1:], seg[:-1]):
        g = s - end
        if g > 0:
            key = (prev[:60], n[:60])
            gaps[key][0] += g
            gaps[key][1] += 1
            big.append((g, prev[:60], n[:60]))
        end = max(end, e)
    idle = sum(v[0] for v in gaps.values())
    print(f"step window: {len(seg)} kernels, wall {wall / 1e6:.2f} ms, kernel busy {busy / 1e6:.2f} ms, "
          f"idle gaps {idle / 1e6:.2f} ms")
    print("largest gaps (us): prev -> next")
    for g, p, n in sorted(big, reverse=True)[:a.top]:
        print(f"  {g / 1e3:9.1f}  {p} -> {n}")
    print("gap totals by kernel pair (us, count):")
    for k, (t, c) in sorted(gaps.items(), key=lambda kv: -kv[1][0])[:a.top]:
        print(f"  {t / 1e3:9.1f} {c:5d}  {k[0]} -> {k[1]}")


if __name__ == "__main__":
    main()
