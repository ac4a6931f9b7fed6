"""Trainer profiling on MI355X (SURVEY section 5 "Tracing / profiling").

The reference has only the payloads' TF FULL_TRACE run metadata every 100th
step and TensorBoard summaries (mnist_with_summaries.py:162-171,
multi_worker_strategy-with-keras.py:107).  Here:

* :func:`rocprof_argv` / ``python -m tf_operator_amd.utils.profiling`` -- a
  launcher that runs a trainer under ``rocprofv3`` (kernel trace + per-kernel
  stats, or one PMC counter pass) as a CHILD process -- never by exec: the
  profiler's preloaded library initialises the GPU, so the program goes
  straight after ``--`` -- and then writes ``summary.md`` (top kernels by
  time, with calls and average duration).  The operator wraps a replica's
  command with it when the job carries the annotation
  ``amd.com/rocprof: kernel-trace | stats | pmc:COUNTER,...`` (C++ core,
  ``reconcile.cc``), writing under ``amd.com/rocprof-dir``/<pod>.
* :class:`StepTimer` -- per-step wall time from HIP events without a host
  sync per step (the first-step timestamp is the latency metric);
* :func:`trace_step` -- the FULL_TRACE analog: one step under
  ``torch.profiler`` (roctracer) exported as a Chrome trace.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

MODES = ("kernel-trace", "stats", "pmc")
LAUNCHERS = ("env", "bash", "sh", "dash", "zsh", "taskset", "numactl", "nohup", "exec", "time")


def is_launcher(argv0: str) -> bool:
    """True for a shell or launcher (by basename: /usr/bin/env too) -- a hop
    that would re-exec under the profiler's preloaded library."""
    return os.path.basename(argv0) in LAUNCHERS


def rocprof_argv(program: list, out_dir: str, mode: str = "stats", counters=None, name: str = "run") -> list:
    """rocprofv3 command line for `program` (argv list).  `mode`:
    kernel-trace (trace only), stats (trace + per-kernel stats), pmc (one
    counter pass with `counters`; counters need a run of their own, without
    runtime / memory-copy tracing)."""
    if mode not in MODES:
        raise ValueError(f"mode {mode!r} not in {MODES}")
    exe = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    argv = [exe, "--kernel-trace", "--output-format", "csv", "-d", out_dir, "-o", name]
    if mode == "stats":
        argv.insert(2, "--stats")
    if mode == "pmc":
        if not counters:
            raise ValueError("pmc mode needs counters")
        argv[1:1] = ["--pmc", *counters]
    if not program or is_launcher(program[0]):
        raise ValueError("put the program itself after `--` (no launcher hops under the profiler)")
    return argv + ["--"] + list(program)


def summarize(out_dir: str, top: int = 25) -> str:
    """Markdown table of the heaviest kernels from rocprofv3's
    *_kernel_stats.csv (or aggregated from *_kernel_trace.csv)."""
    stats = glob.glob(os.path.join(out_dir, "**", "*kernel_stats.csv"), recursive=True)
    rows = []
    if stats:
        with open(stats[0]) as f:
            for r in csv.DictReader(f):
                rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"])))
    else:
        agg = {}
        for tr in glob.glob(os.path.join(out_dir, "**", "*kernel_trace.csv"), recursive=True):
            with open(tr) as f:
                for r in csv.DictReader(f):
                    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                    c, t = agg.get(r["Kernel_Name"], (0, 0.0))
                    agg[r["Kernel_Name"]] = (c + 1, t + d)
        rows = [(k, c, t) for k, (c, t) in agg.items()]
    rows.sort(key=lambda x: -x[2])
    total = sum(r[2] for r in rows) or 1.0
    lines = [f"# Kernel time summary ({out_dir})", "", f"Total kernel time: {total / 1e6:.2f} ms", "",
             "| % | total ms | calls | avg us | kernel |", "|---|---|---|---|---|"]
    for name, calls, t in rows[:top]:
        short = name.split("(")[0][:100].replace("|", "/")
        lines.append(f"| {100 * t / total:.1f} | {t / 1e6:.2f} | {calls} | {t / max(calls, 1) / 1e3:.1f} | `{short}` |")
    return "\n".join(lines) + "\n"


class StepTimer:
    """HIP-event step timer: record() after each step costs no host sync;
    summary() synchronises once and returns per-step milliseconds."""

    def __init__(self):
        import torch

        self.torch = torch
        self.events = []

    def record(self):
        torch = self.torch
        if torch.cuda.is_available():
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.events.append(e)

    def summary(self) -> dict:
        if len(self.events) < 2:
            return {}
        self.events[-1].synchronize()
        ms = [a.elapsed_time(b) for a, b in zip(self.events, self.events[1:])]
        ms_sorted = sorted(ms)
        return {"steps": len(ms), "mean_ms": sum(ms) / len(ms), "p50_ms": ms_sorted[len(ms) // 2],
                "max_ms": ms_sorted[-1]}


def trace_step(fn, path: str):
    """Run fn() once under torch.profiler (CPU + GPU activities) and export a
    Chrome trace to `path`.  Returns fn's result; if the profiler is not
    usable on this build the step still runs and no trace is written."""
    import torch

    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    try:
        with torch.profiler.profile(activities=acts, record_shapes=False) as prof:
            out = fn()
            if torch.cuda.is_available():
                torch.cuda.synchronize()
    except RuntimeError:
        return fn()
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    prof.export_chrome_trace(path)
    return out


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if "--" not in argv:
        raise SystemExit("usage: python -m tf_operator_amd.utils.profiling [--mode M] [--out DIR] -- program args...")
    cut = argv.index("--")
    p = argparse.ArgumentParser()
    p.add_argument("--mode", default="stats", help="kernel-trace | stats | pmc:COUNTER,COUNTER")
    p.add_argument("--out", default=os.environ.get("TOA_ROCPROF_DIR", "rocprof_out"))
    a = p.parse_args(argv[:cut])
    program = argv[cut + 1:]
    mode, counters = a.mode, None
    if mode.startswith("pmc:"):
        mode, counters = "pmc", [c for c in a.mode[4:].split(",") if c]
    os.makedirs(a.out, exist_ok=True)
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    if shutil.which("rocprofv3") is None and not os.path.exists("/opt/rocm/bin/rocprofv3"):
        print("[profiling] rocprofv3 not found: running unprofiled", file=sys.stderr)
        return subprocess.call(program, env=env)
    if not program or is_launcher(program[0]):
        # the operator core already skips such commands; a hand-written pod
        # spec still gets its job run, just unprofiled, instead of exit 1
        print(f"[profiling] {program[:1]} is a launcher hop: running unprofiled", file=sys.stderr)
        return subprocess.call(program, env=env) if program else 2
    rc = subprocess.call(rocprof_argv(program, a.out, mode, counters), env=env)
    try:
        with open(os.path.join(a.out, "summary.md"), "w") as f:
            f.write(summarize(a.out))
        with open(os.path.join(a.out, "launcher.json"), "w") as f:
            json.dump({"mode": a.mode, "program": program, "rc": rc}, f)
    except OSError as e:  # pragma: no cover - best effort
        print(f"[profiling] summary failed: {e}", file=sys.stderr)
    return rc


if __name__ == "__main__":
    sys.exit(main())
