"""Per-kernel-name summary of a rocprofv3 --kernel-trace CSV: dispatches,
grid (workgroups), LDS bytes, mean / min duration in us.

    python scripts/probes/trace_summary.py <dir with *_kernel_trace.csv> [name-substring ...]
"""
import collections
import csv
import glob
import sys


def main():
    root, keys = sys.argv[1], sys.argv[2:]
    per = collections.defaultdict(list)
    for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if keys and not any(k in n for k in keys):
                continue
            wg = int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1)
            per[(n[:72], wg, r["LDS_Block_Size"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for (n, wg, lds), d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"{len(d):5d} wg={wg:6d} lds={lds:>6s} mean={sum(d) / len(d) / 1e3:9.1f}us min={min(d) / 1e3:9.1f}us  {n}")


if __name__ == "__main__":
    main()
