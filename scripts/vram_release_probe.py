"""Where does a back-to-back job's extra start-up time go?  Runs the 8B
payload (one step) twice in a row as child processes while sampling the
driver's VRAM usage (sysfs mem_info_vram_used) every 100 ms, so the log
shows whether the second job waits for the first job's memory to be
released/cleared by the driver.

    python scripts/vram_release_probe.py [--gap 0] [--runs 3]
"""
import argparse
import glob
import json
import os
import subprocess
import sys
import threading
import time


def vram_used():
    out = {}
    for p in sorted(glob.glob("/sys/class/drm/card*/device/mem_info_vram_used")):
        try:
            out[p.split("/")[4]] = int(open(p).read()) / 2**30
        except OSError:
            pass
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gap", type=float, default=0.0)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--model", default="llama3-8b")
    a = ap.parse_args()
    t0 = time.time()
    samples = []
    stop = threading.Event()

    def sampler():
        while not stop.is_set():
            samples.append((round(time.time() - t0, 2), vram_used()))
            time.sleep(0.1)

    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    runs = []
    for i in range(a.runs):
        s = time.time()
        p = subprocess.run([sys.executable, "-m", "tf_operator_amd.examples.llama_train", "--model", a.model,
                            "--steps", "1", "--seq-len", "4096", "--micro-batch", "6"],
                           capture_output=True, text=True, env=dict(os.environ, TOA_LOG_PHASES="1"))
        e = time.time()
        phases = [ln for ln in p.stdout.splitlines() if "start-up phases" in ln]
        runs.append({"run": i, "start": round(s - t0, 2), "end": round(e - t0, 2), "rc": p.returncode,
                     "phases": phases[-1] if phases else p.stdout[-500:] + p.stderr[-1500:]})
        print(json.dumps(runs[-1]), flush=True)
        if a.gap:
            time.sleep(a.gap)
    time.sleep(3)
    stop.set()
    th.join()
    # condensed VRAM trace: only samples where the total changed by > 1 GiB
    last = None
    for t, v in samples:
        tot = round(sum(v.values()), 1)
        if last is None or abs(tot - last) > 1.0:
            print(f"t={t:7.2f}s vram_used_total={tot} GiB", flush=True)
            last = tot


if __name__ == "__main__":
    main()
