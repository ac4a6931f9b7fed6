"""Back-to-back Llama-3-8B probe TFJobs through the local operator stack,
cold or warm-started (kubelet fork server), with the driver's VRAM counter
sampled every 50 ms: shows when a finished job's HBM is released and scrubbed
relative to the kubelet's exit report and to the next job's start-up phases.

    python scripts/probes/warm_vram.py [--warm 1] [--jobs 3]
"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from tf_operator_amd.bench import flagship  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--warm", default="1")
    ap.add_argument("--jobs", type=int, default=3)
    ap.add_argument("--micro-batch", type=int, default=6)
    ap.add_argument("--gap", type=float, default=0.0, help="idle seconds between jobs (after the drain wait)")
    a = ap.parse_args()
    args = flagship.parser().parse_args(["--micro-batch", str(a.micro_batch)])
    t0 = time.time()
    samples, stop = [], threading.Event()

    def sampler():
        while not stop.is_set():
            samples.append((round(time.time() - t0, 3), round((flagship.vram_used_bytes() or 0) / 2**30, 1)))
            time.sleep(0.05)

    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    c = flagship._cluster(1, a.warm == "1")
    events = [("cluster_ready", round(time.time() - t0, 3))]
    base = flagship.vram_used_bytes()
    try:
        for i in range(a.jobs):
            events.append((f"submit_{i}", round(time.time() - t0, 3)))
            r = flagship._run_job(c, f"probe-{i}", 1, flagship._payload(args), 180, vram_baseline=base)
            events.append((f"cleaned_{i}", round(time.time() - t0, 3)))
            r.pop("_logs", None)
            print(json.dumps({"job": i, **r}), flush=True)
            time.sleep(a.gap)
    finally:
        c.stop()
        stop.set()
        th.join()
    print(json.dumps({"events": events}))
    last = None
    for t, v in samples:  # only changes
        if v != last:
            print(f"t={t:8.3f}s vram={v:7.1f} GiB")
            last = v


if __name__ == "__main__":
    main()
