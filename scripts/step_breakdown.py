"""Per-step kernel table from a rocprofv3 --kernel-trace CSV: the kernels
between the last two launches whose name contains MARKER (one per step).

    python scripts/step_breakdown.py <rocprof out dir> <marker>
"""
import collections
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
marker = sys.argv[2]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
if len(idx) < 2:
    raise SystemExit(f"fewer than two '{marker}' kernels in the trace")
# one step = from the kernel after the second-to-last marker to the last marker
s, e = idx[-2] + 1, idx[-1] + 1
d = collections.defaultdict(lambda: [0, 0.0])
for r in rows[s:e]:
    k = r["Kernel_Name"][:110]
    d[k][0] += 1
    d[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
tot = sum(v[1] for v in d.values())
span = (int(rows[e - 1]["End_Timestamp"]) - int(rows[s]["Start_Timestamp"])) / 1e6
print(f"one step: kernel time {tot:.2f} ms, span {span:.2f} ms")
for k, (c, t) in sorted(d.items(), key=lambda kv: -kv[1][1])[:40]:
    print(f"{t:8.3f} ms  {100 * t / tot:5.1f}%  n={c:4d}  {k}")
