"""One line per form from an asm_gemm_bench.py log: TF/s of every arm."""
import json
import sys

for line in open(sys.argv[1]):
    if not line.startswith("{") or '"tokens"' in line or '"check"' in line:
        continue
    d = json.loads(line)
    for form, rec in d.items():
        if form == "mlp_ms":
            print(form, rec)
            continue
        arms = {k: v["TFps"] for k, v in rec.items() if isinstance(v, dict) and "TFps" in v}
        diff = [k for k, v in rec.get("variants_bit_identical", {}).items() if not v]
        print(f"{form:16s}", " ".join(f"{k}={v:.0f}" for k, v in arms.items()), ("differs: " + ",".join(diff)) if diff else "")
