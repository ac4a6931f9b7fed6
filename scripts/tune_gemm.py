"""Measure the fastest hipBLASLt solution for every GEMM form of the
Llama-3-8B training step (T = micro-batch x seq tokens) and write the table
that tf_operator_amd.ops.gemm installs at start-up.

    python scripts/tune_gemm.py [--tokens 24576] [--out path] [--exclude-streamk]

--exclude-streamk keeps only non-stream-K solutions and writes the ``nosk``
table (ops/gemm.py TABLE_NOSK) by default.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tf_operator_amd.ops import gemm  # noqa: E402

LLAMA3_8B = {"qkv": (4096, 6144), "o": (4096, 4096), "gate_up": (4096, 28672), "down": (14336, 4096),
             "lm_head": (4096, 128256)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, nargs="+", default=[24576])
    ap.add_argument("--out", default=None)
    ap.add_argument("--exclude-streamk", action="store_true")
    ap.add_argument("--forms", default="fwd,dgrad_wt", help="comma list of fwd,dgrad,dgrad_wt,wgrad")
    ap.add_argument("--merge", action="store_true", help="keep existing entries of other forms")
    a = ap.parse_args()
    if a.out is None:
        a.out = gemm.TABLE_NOSK if a.exclude_streamk else gemm.TABLE
    forms = set(a.forms.split(","))
    entries = {}
    if a.merge and os.path.exists(a.out):
        for e in json.load(open(a.out)).get("entries", []):
            entries[tuple(e[k] for k in ("ta", "tb", "m", "n", "k", "lda", "ldb", "ldc", "beta_nz"))] = e
    for T in a.tokens:
        for name, form, key in gemm.form_keys(T, LLAMA3_8B):
            if form not in forms:
                continue
            t0 = time.time()
            idx, best, dflt, n = gemm.tune_form(key, exclude_streamk=a.exclude_streamk)
            ta, tb, m, n_, k, lda, ldb, ldc, beta_nz = key
            fl = 2.0 * m * n_ * k
            e = {"name": f"{name}.{form}", "tokens": T, "ta": ta, "tb": tb, "m": m, "n": n_, "k": k, "lda": lda,
                 "ldb": ldb, "ldc": ldc, "beta_nz": beta_nz, "out_f32": 0, "index": idx, "ms": round(best, 4),
                 "default_ms": round(dflt, 4), "tflops": round(fl / best / 1e9, 1),
                 "default_tflops": round(fl / dflt / 1e9, 1), "candidates": n,
                 "kernel": gemm.kernel_name(key)}
            entries[key] = e
            print(json.dumps(e), f"({time.time() - t0:.1f}s)", flush=True)
    gemm.save_table(list(entries.values()), a.out)
    print("wrote", a.out)


if __name__ == "__main__":
    main()
