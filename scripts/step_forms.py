"""Per-step kernel table keyed by (kernel, grid size) from a rocprofv3
--kernel-trace CSV: the GEMM forms of the Llama step share a kernel name and
differ by grid, so this separates e.g. qkv.fwd from o.fwd in-model.

    python scripts/step_forms.py <rocprof out dir> <marker> [--top 40]
"""
import argparse
import collections
import csv
import glob

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("marker")
ap.add_argument("--top", type=int, default=40)
a = ap.parse_args()
f = glob.glob(f"{a.dir}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
if len(idx) < 2:
    raise SystemExit(f"fewer than two '{a.marker}' kernels in the trace")
s, e = idx[-2] + 1, idx[-1] + 1
gkey = next(k for k in ("Grid_Size", "Grid_Size_X", "grid_size") if k in rows[0])
d = collections.defaultdict(lambda: [0, 0.0])
for r in rows[s:e]:
    name = r["Kernel_Name"].split("(")[0][:70]
    k = f"{name} grid={r[gkey]}"
    d[k][0] += 1
    d[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
tot = sum(v[1] for v in d.values())
print(f"one step: kernel time {tot:.2f} ms")
for k, (c, t) in sorted(d.items(), key=lambda kv: -kv[1][1])[:a.top]:
    print(f"{t:8.3f} ms  {100 * t / tot:5.1f}%  n={c:4d}  {t / c:7.3f} ms/call  {k}")
