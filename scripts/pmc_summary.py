"""Mean-per-dispatch counter table from a rocprofv3 --pmc run, for kernels
whose name contains any of the given substrings; adds the MFMA-pipe busy
fraction SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs over GRBM_GUI_ACTIVE / 8 XCDs
(the same formula as profiles/r1_attn_pmc/summary.md).

    python scripts/pmc_summary.py <rocprof out dir> attn_fwd attn_bwd_dq attn_bwd_dkdv
"""
import collections
import csv
import glob
import sqlite3
import sys


def _rows(root):
    """(kernel, dispatch, counter, value, duration_ns) from CSV or rocpd
    SQLite (rocprofv3's default output format) results."""
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            dur = float(r["End_Timestamp"]) - float(r["Start_Timestamp"]) if "End_Timestamp" in r else 0.0
            yield r["Kernel_Name"], f + r["Dispatch_Id"], r["Counter_Name"], float(r["Counter_Value"]), dur
    for f in glob.glob(f"{root}/**/*results.db", recursive=True):
        c = sqlite3.connect(f)
        try:
            q = c.execute("select kernel_name, dispatch_id, counter_name, value, duration from counters_collection")
        except sqlite3.OperationalError:
            continue
        for k, d, n, v, dur in q:
            yield k, f + str(d), n, float(v), float(dur or 0)


def main():
    root, keys = sys.argv[1], sys.argv[2:]
    per = collections.defaultdict(lambda: collections.defaultdict(dict))  # kernel -> dispatch -> counter
    for name, disp, ctr, val, dur in _rows(root):
        k = next((k for k in keys if k in name), None)
        if k is None:
            continue
        per[k][disp][ctr] = val
        if dur:
            per[k][disp]["duration_us"] = dur / 1e3
    if not per:
        raise SystemExit(f"no counter rows for {keys} under {root}")
    cols = sorted({c for d in per.values() for v in d.values() for c in v})
    print("| kernel | dispatches | " + " | ".join(cols) + " | MFMA busy | clock GHz |")
    print("|---" * (len(cols) + 4) + "|")
    for k in keys:
        ds = per.get(k)
        if not ds:
            continue
        mean = {}
        for c in cols:  # over the dispatches (of the pass) that collected c
            vals = [v[c] for v in ds.values() if c in v]
            mean[c] = sum(vals) / len(vals) if vals else 0.0
        busy = ""
        if mean.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
            busy = f"{100 * (mean['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024) / (mean['GRBM_GUI_ACTIVE'] / 8):.0f}%"
        clk = ""
        if mean.get("GRBM_GUI_ACTIVE") and mean.get("duration_us"):
            clk = f"{mean['GRBM_GUI_ACTIVE'] / 8 / (mean['duration_us'] * 1e3):.2f}"
        print(f"| {k} | {len(ds)} | " + " | ".join(f"{mean[c]:.3g}" for c in cols) + f" | {busy} | {clk} |")


if __name__ == "__main__":
    main()
