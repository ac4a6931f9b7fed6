"""Box-speed evidence for the benchmark record (verdict r4 item 4).

MI355X boxes differ by up to a few percent on identical code: the chip holds
a lower clock under a dense MFMA load on some devices than on others
(MI355X_MICROARCH.md, DVFS give-back item 5), so a step time alone cannot say
whether a change of code or a change of box moved it.  Two measurements go
into ``bench.py``'s JSON line next to the step time:

* a fixed-shape bf16 GEMM (8192^3) on hipBLASLt (``torch.matmul``) and on the
  hand-written assembly kernel (``toa_gemm_asm``), just before and just after
  the timed region (outside it): PF/s of each;
* the GPU's graphics clock, power and busy percentage sampled from the
  amdgpu sysfs counters every 50 ms on a helper thread during the timed
  region (no HIP call, so nothing is added to the GPU's queue): mean / min /
  max.  sysfs reports the DPM level the firmware selected; the in-kernel
  clock under a dense MFMA loop can read up to ~10 % lower, so the GEMM
  rates are the primary normaliser and the clock the explanation.

A step time divided by the ratio of two boxes' calibration GEMM rates gives
the calibration-normalised comparison ``BASELINE.md`` reports.
"""
from __future__ import annotations

import glob
import os
import re
import statistics
import threading
import time

SHAPE = (8192, 8192, 8192)
SYSFS_DRM = "/sys/class/drm"


def _read(path: str):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def sysfs_device_dir(dev) -> str | None:
    """The amdgpu sysfs device directory of torch device `dev` (matched by
    PCI domain / bus / device)."""
    import torch

    p = torch.cuda.get_device_properties(dev)
    want = (int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id))
    for card in glob.glob(os.path.join(SYSFS_DRM, "card*")):
        if not re.fullmatch(r"card\d+", os.path.basename(card)):
            continue
        bdf = os.path.basename(os.path.realpath(os.path.join(card, "device")))
        m = re.fullmatch(r"([0-9a-f]+):([0-9a-f]+):([0-9a-f]+)\.([0-9a-f])", bdf)
        if m and (int(m.group(1), 16), int(m.group(2), 16), int(m.group(3), 16)) == want:
            return os.path.join(card, "device")
    return None


def read_sclk_mhz(devdir: str) -> tuple[float | None, str]:
    """Current graphics clock: hwmon freq1_input (Hz), else the active
    pp_dpm_sclk level (the line marked '*')."""
    for hw in sorted(glob.glob(os.path.join(devdir, "hwmon", "hwmon*"))):
        lab = _read(os.path.join(hw, "freq1_label"))
        v = _read(os.path.join(hw, "freq1_input"))
        if v is not None and (lab is None or lab.lower() == "sclk"):
            try:
                return float(v) / 1e6, "hwmon freq1_input"
            except ValueError:
                pass
    s = _read(os.path.join(devdir, "pp_dpm_sclk"))
    if s:
        for line in s.splitlines():
            if line.rstrip().endswith("*"):
                m = re.search(r"(\d+)\s*Mhz", line, re.I)
                if m:
                    return float(m.group(1)), "pp_dpm_sclk"
    return None, "unavailable"


def read_power_w(devdir: str) -> float | None:
    for hw in sorted(glob.glob(os.path.join(devdir, "hwmon", "hwmon*"))):
        for name in ("power1_average", "power1_input"):
            v = _read(os.path.join(hw, name))
            if v is not None:
                try:
                    return float(v) / 1e6
                except ValueError:
                    pass
    return None


class ClockSampler:
    """Samples clock / power / busy of one GPU on a thread between start()
    and stop(); stop() returns the summary dict (empty without sysfs)."""

    def __init__(self, devdir: str | None, period_s: float = 0.05):
        self.devdir, self.period = devdir, period_s
        self.clk, self.pw, self.busy = [], [], []
        self.source = "unavailable"
        self._stop = threading.Event()
        self._t = None

    def _run(self):
        while not self._stop.is_set():
            c, self.source = read_sclk_mhz(self.devdir)
            if c is not None:
                self.clk.append(c)
            p = read_power_w(self.devdir)
            if p is not None:
                self.pw.append(p)
            b = _read(os.path.join(self.devdir, "gpu_busy_percent"))
            if b is not None:
                try:
                    self.busy.append(float(b))
                except ValueError:
                    pass
            self._stop.wait(self.period)

    def start(self):
        if self.devdir:
            self._t = threading.Thread(target=self._run, name="toa-clock-sampler", daemon=True)
            self._t.start()
        return self

    def stop(self) -> dict:
        if self._t is None:
            return {}
        self._stop.set()
        self._t.join(timeout=2.0)
        out = {"source": self.source, "samples": len(self.clk)}
        if self.clk:
            out.update(gfxclk_mhz_mean=round(statistics.fmean(self.clk), 1), gfxclk_mhz_min=round(min(self.clk), 1),
                       gfxclk_mhz_max=round(max(self.clk), 1))
        if self.pw:
            out["power_w_mean"] = round(statistics.fmean(self.pw), 1)
        if self.busy:
            out["busy_pct_mean"] = round(statistics.fmean(self.busy), 1)
        return out


def gemm_rates(dev, reps: int = 10, rounds: int = 2) -> dict:
    """PF/s of the fixed-shape GEMM on hipBLASLt and on the assembly kernel,
    alternating arms, median over rounds.  Missing arms are left out."""
    import torch

    from ..ops import _lib

    M, N, K = SHAPE
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16, generator=g)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    arms = {"hipblaslt": lambda: torch.matmul(x, w.t(), out=y)}
    if _lib.available() and _lib.has("toa_gemm_asm"):
        def asm():
            _lib.call("toa_gemm_asm", _lib.ptr(x), K, _lib.ptr(w), K, _lib.ptr(y), N, M, N, K, _lib.stream(x))
        arms["asm"] = asm
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    times = {k: [] for k in arms}
    for _ in range(rounds):
        for k, fn in arms.items():
            fn()
            fn()
            ev[0].record()
            for _ in range(reps):
                fn()
            ev[1].record()
            torch.cuda.synchronize(dev)
            times[k].append(ev[0].elapsed_time(ev[1]) / reps)
    del x, w, y
    fl = 2.0 * M * N * K
    return {f"{k}_pfs": round(fl / statistics.median(v) / 1e12, 4) for k, v in times.items()}


class Calibration:
    """before() / sampling around the timed region / after() -> record()."""

    def __init__(self, dev, enabled: bool = True):
        self.dev, self.on = dev, enabled and getattr(dev, "type", "") == "cuda"
        self.rec: dict = {}
        self.sampler = None
        if self.on:
            try:
                self.devdir = sysfs_device_dir(dev)
            except (RuntimeError, AttributeError):
                self.devdir = None

    def before(self):
        if self.on:
            t = time.perf_counter()
            self.rec["before"] = gemm_rates(self.dev)
            self.rec["calibration_s"] = round(time.perf_counter() - t, 3)

    def start(self):
        if self.on:
            self.sampler = ClockSampler(self.devdir).start()

    def stop(self):
        if self.sampler is not None:
            self.rec["timed_region_clock"] = self.sampler.stop()
            self.sampler = None

    def after(self):
        if self.on:
            self.rec["after"] = gemm_rates(self.dev)

    def record(self) -> dict | None:
        if not self.on:
            return None
        out = {"gemm_shape_mnk": list(SHAPE), **self.rec}
        b, a = self.rec.get("before", {}), self.rec.get("after", {})
        for k in set(b) & set(a):
            out[f"{k[:-4]}_pfs_mean"] = round((b[k] + a[k]) / 2, 4)
        return out
