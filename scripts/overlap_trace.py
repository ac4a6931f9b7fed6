"""How the emulated collectives (emu_xfer_kernel, parallel/emulate.py) and
the GEMMs share the GPU, from a rocprofv3 --kernel-trace CSV.

    python scripts/overlap_trace.py <dir with *_kernel_trace.csv> [--out summary.json]

Reports, over the traced steps:
* the emulated collectives: count, mean / max duration, and the fraction of
  their lifetime spent beside a GEMM (interleaved) rather than between GEMMs;
* every GEMM family (hipBLASLt Cijk, the framework's wgrad_nt): mean
  duration with and without an emulated collective running beside it;
* the span of the trace and the time the last collective ends after the
  last GEMM ("collective tail").
"""
import argparse
import csv
import glob
import json
import statistics


def load(root):
    rows = []
    for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort(key=lambda x: x[1])
    return rows


def family(name):
    if "emu_xfer_kernel" in name:
        return "collective"
    if "Cijk" in name:
        return "hipblaslt"
    if "wgrad_nt" in name:
        return "wgrad_nt"
    return None


def overlap(a0, a1, ivs):
    t = 0
    for b0, b1 in ivs:
        if b1 <= a0 or b0 >= a1:
            continue
        t += min(a1, b1) - max(a0, b0)
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = load(a.root)
    if not rows:
        raise SystemExit(f"no kernel trace under {a.root}")
    coll = [(s, e) for n, s, e in rows if family(n) == "collective"]
    gemm = {f: [(s, e) for n, s, e in rows if family(n) == f] for f in ("hipblaslt", "wgrad_nt")}
    all_gemm = sorted(gemm["hipblaslt"] + gemm["wgrad_nt"])
    out = {"span_ms": round((rows[-1][2] - rows[0][1]) / 1e6, 2), "kernels": len(rows)}
    if coll:
        d = [e - s for s, e in coll]
        beside = sum(overlap(s, e, all_gemm) for s, e in coll)
        out["collective"] = {"count": len(coll), "mean_us": round(statistics.mean(d) / 1e3, 1),
                             "max_us": round(max(d) / 1e3, 1), "total_ms": round(sum(d) / 1e6, 2),
                             "beside_gemm_fraction": round(beside / max(sum(d), 1), 3)}
        if all_gemm:
            out["collective_tail_after_last_gemm_us"] = round((max(e for _, e in coll) - max(e for _, e in all_gemm))
                                                              / 1e3, 1)
    for f, ivs in gemm.items():
        if not ivs:
            continue
        w = [e - s for s, e in ivs if overlap(s, e, coll) > 0]
        wo = [e - s for s, e in ivs if overlap(s, e, coll) == 0]
        out[f] = {"count": len(ivs), "total_ms": round(sum(e - s for s, e in ivs) / 1e6, 2),
                  "with_collective": len(w), "mean_us_with": round(statistics.mean(w) / 1e3, 1) if w else None,
                  "mean_us_without": round(statistics.mean(wo) / 1e3, 1) if wo else None}
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
