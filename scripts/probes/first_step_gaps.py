"""Host-side stalls of the first training steps from a rocprofv3 kernel
trace: every gap of more than --min-ms between consecutive kernels, with the
kernels on either side, and the span / busy time of each step window.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- \
        python3 bench.py --direct --steps 1 --warmup 1
    python scripts/probes/first_step_gaps.py OUT/run_kernel_trace.csv
"""
import csv
import sys


def main():
    path = sys.argv[1]
    min_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    t0 = ks[0][0]
    print(f"{len(ks)} kernels, span {(ks[-1][1] - t0) / 1e6:.1f} ms, busy {sum(e - s for s, e, _ in ks) / 1e6:.1f} ms")
    end = ks[0][1]
    total_gap = 0.0
    for i in range(1, len(ks)):
        s, e, n = ks[i]
        gap = (s - end) / 1e6
        if gap > min_ms:
            total_gap += gap
            print(f"  t={(end - t0) / 1e6:9.1f} ms  gap {gap:8.2f} ms  before {n[:70]}  (after {ks[i - 1][2][:50]})")
        end = max(end, e)
    print(f"gaps > {min_ms} ms: {total_gap:.1f} ms")


if __name__ == "__main__":
    main()
