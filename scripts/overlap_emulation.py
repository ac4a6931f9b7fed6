"""World-8 ZeRO-1 step on ONE GPU with emulated collective traffic, under
several GEMM policies (verdict r2, "Next round" item 1).

Each variant is one ``bench.py --direct --zero 1`` process with
``TOA_EMULATE_WORLD=8`` (parallel/emulate.py): rank 0's world-8 step -- 1/8
of AdamW, a reduce-scatter per gradient bucket during backward and an
all-gather per bucket before the next forward -- with every collective
replaced by paced traffic on a high-priority side stream.  Variants:

    <policy>.traffic   the collectives move (N-1)/N of each bucket at --gbps
    <policy>.quiet     same step, collectives moving nothing (TOA_EMULATE_BYTES=0)

for each entry of --policies: a GEMM policy (asm = the assembly kernel, the
default; torch = hipBLASLt heuristic, i.e. its stream-K kernels; nosk = the
non-stream-K table, ops/gemm.py), optionally followed by "+VAR=VALUE" extra
environment, e.g. ``asm+TOA_ZERO_PIPE=0`` for the unpipelined ZeRO-1 tail.  The overlap cost of a
policy is traffic - quiet; policies are compared on traffic.

    python scripts/overlap_emulation.py --out gpurun_out/r3_overlap [--steps 4] [--gbps 350]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(name, env_extra, args, out_dir):
    env = dict(os.environ, TOA_EMULATE_WORLD=str(args.world), TOA_EMULATE_GBPS=str(args.gbps),
               TOA_EMULATE_CHANNELS=str(args.channels), **env_extra)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--direct", "--zero", "1", "--steps", str(args.steps),
           "--warmup", str(args.warmup), "--latency-probes", "0"]
    t0 = time.time()
    log = os.path.join(out_dir, f"{name}.log")
    with open(log, "w") as f:
        p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=f, timeout=args.timeout, text=True)
    line = next((ln for ln in p.stdout.splitlines() if ln.startswith("{")), None)
    res = json.loads(line) if line else {"error": f"rc={p.returncode}", "stdout": p.stdout[-2000:]}
    res["_variant"], res["_wall_s"] = name, round(time.time() - t0, 1)
    print(f"[overlap] {name}: {res.get('ms_per_step')} ms/step ({res['_wall_s']} s)", flush=True)
    if p.returncode != 0:
        raise SystemExit(f"{name} failed rc={p.returncode}; see {log}")
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--gbps", type=float, default=350.0)
    ap.add_argument("--channels", type=int, default=32)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--policies", default="asm,asm+TOA_ZERO_PIPE=0")
    ap.add_argument("--timeout", type=float, default=240)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    rows = []
    for pol in a.policies.split(","):
        gemm, *assigns = pol.split("+")
        env = {"TOA_GEMM": gemm, **dict(x.split("=", 1) for x in assigns)}
        for kind, extra in (("traffic", {}), ("quiet", {"TOA_EMULATE_BYTES": "0"})):
            rows.append(run(f"{pol}.{kind}", {**env, **extra}, a, a.out))
    by = {r["_variant"]: r for r in rows}
    summary = {"world": a.world, "gbps": a.gbps, "channels": a.channels, "steps": a.steps, "variants": {}}
    for pol in a.policies.split(","):
        t, q = by[f"{pol}.traffic"]["ms_per_step"], by[f"{pol}.quiet"]["ms_per_step"]
        summary["variants"][pol] = {"traffic_ms": t, "quiet_ms": q, "overlap_cost_ms": round(t - q, 2),
                                    "overlap_cost_pct": round(100 * (t - q) / q, 2)}
    with open(os.path.join(a.out, "summary.json"), "w") as f:
        json.dump({"summary": summary, "runs": rows}, f, indent=1)
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
