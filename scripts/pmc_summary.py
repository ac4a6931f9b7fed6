"""Mean-per-dispatch counter table from a rocprofv3 --pmc run, for kernels
whose name contains any of the given substrings; adds the MFMA-pipe busy
fraction SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs over GRBM_GUI_ACTIVE / 8 XCDs
(the same formula as profiles/r1_attn_pmc/summary.md).

    python scripts/pmc_summary.py <rocprof out dir> attn_fwd attn_bwd_dq attn_bwd_dkdv
"""
import collections
import csv
import glob
import sys


def main():
    root, keys = sys.argv[1], sys.argv[2:]
    files = glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {root}")
    per = collections.defaultdict(lambda: collections.defaultdict(dict))  # kernel -> dispatch -> counter
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            k = next((k for k in keys if k in name), None)
            if k is None:
                continue
            per[k][r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    cols = sorted({c for d in per.values() for v in d.values() for c in v})
    print("| kernel | dispatches | " + " | ".join(cols) + " | MFMA busy |")
    print("|---" * (len(cols) + 3) + "|")
    for k in keys:
        ds = per.get(k)
        if not ds:
            continue
        mean = {c: sum(v.get(c, 0.0) for v in ds.values()) / len(ds) for c in cols}
        busy = ""
        if mean.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
            busy = f"{100 * (mean['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024) / (mean['GRBM_GUI_ACTIVE'] / 8):.0f}%"
        print(f"| {k} | {len(ds)} | " + " | ".join(f"{mean[c]:.3g}" for c in cols) + f" | {busy} |")


if __name__ == "__main__":
    main()
