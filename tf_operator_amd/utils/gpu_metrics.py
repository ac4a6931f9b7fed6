"""Per-pod GPU device metrics for MI355X nodes (SURVEY 5 "metrics /
logging"; the reference documents the cAdvisor accelerator series for
NVIDIA GPUs: ``container_accelerator_memory_used_bytes`` per pod,
docs/monitoring/README.md:26-29).

The same series, for AMD Instinct GPUs, straight from the amdgpu driver's
sysfs counters -- no HIP context, no SMI daemon, cheap enough to scrape
every few seconds on a node that is training:

    container_accelerator_memory_used_bytes{make="amd",model=...,acc_id=...,namespace,pod,container}
    container_accelerator_memory_total_bytes{...}
    container_accelerator_duty_cycle{...}              (percent busy, gpu_busy_percent)
    toa_gpu_power_watts{acc_id}                        (hwmon power1_average / power1_input)
    toa_gpu_temperature_celsius{acc_id,sensor}         (hwmon temp*_input)
    toa_gpu_info{acc_id,bdf,model}                     (1)

Pod attribution: the node agent that hands out ``amd.com/gpu`` device
indices (the local kubelet here, the device plugin + kubelet pod-resources
API in a cluster) passes ``owners`` = {device index: (namespace, pod,
container)}; unassigned devices carry empty pod labels, like cAdvisor's
node-level series.

    python -m tf_operator_amd.utils.gpu_metrics --port 9400 [--owners owners.json]

serves ``/metrics`` (an amd-smi-free exporter for nodes without the AMD
device-metrics exporter).  ``amd-smi metric --json`` output can be parsed
with :func:`from_amd_smi` for the fields sysfs lacks (UMC activity, ECC).
"""
from __future__ import annotations

import argparse
import glob
import http.server
import json
import os
import re

SYSFS_DRM = "/sys/class/drm"


def _read(path: str):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _num(s):
    try:
        return float(s)
    except (TypeError, ValueError):
        return None


def accessible_devices(root: str = SYSFS_DRM, dev_dri: str = "/dev/dri") -> set[str]:
    """PCI devices (sysfs realpaths) of the render nodes this process can
    open.  sysfs lists every GPU of the host; a container or a shared box
    exposes only its own render nodes under /dev/dri."""
    out = set()
    for node in glob.glob(os.path.join(dev_dri, "renderD*")):
        if os.access(node, os.R_OK | os.W_OK):
            out.add(os.path.realpath(os.path.join(root, os.path.basename(node), "device")))
    return out


def read_devices(root: str = SYSFS_DRM, accessible_only: bool = False, dev_dri: str = "/dev/dri") -> list[dict]:
    """One record per amdgpu device with VRAM (compute GPUs), ordered by
    card number = the HIP device order on a node with only these GPUs.
    ``accessible_only``: only the GPUs whose render node this process can
    open (:func:`accessible_devices`)."""
    out = []
    own = accessible_devices(root, dev_dri) if accessible_only else None
    cards = [p for p in glob.glob(os.path.join(root, "card*")) if re.fullmatch(r"card\d+", os.path.basename(p))]
    for card in sorted(cards, key=lambda p: int(os.path.basename(p)[4:])):
        dev = os.path.join(card, "device")
        if own is not None and os.path.realpath(dev) not in own:
            continue
        total = _num(_read(os.path.join(dev, "mem_info_vram_total")))
        if not total:
            continue
        rec = {"acc_id": os.path.basename(card), "index": len(out),
               "memory_total_bytes": total,
               "memory_used_bytes": _num(_read(os.path.join(dev, "mem_info_vram_used"))) or 0.0,
               "duty_cycle": _num(_read(os.path.join(dev, "gpu_busy_percent"))),
               "bdf": os.path.basename(os.path.realpath(dev)), "power_watts": None, "temperature_celsius": {}}
        for hw in sorted(glob.glob(os.path.join(dev, "hwmon", "hwmon*"))):
            for name in ("power1_average", "power1_input"):
                v = _num(_read(os.path.join(hw, name)))
                if v is not None and rec["power_watts"] is None:
                    rec["power_watts"] = v / 1e6  # microwatts
            for t in sorted(glob.glob(os.path.join(hw, "temp*_input"))):
                v = _num(_read(t))
                if v is None:
                    continue
                label = _read(t.replace("_input", "_label")) or os.path.basename(t)[:-6]
                rec["temperature_celsius"][label] = v / 1000.0  # millidegrees
        out.append(rec)
    return out


def from_amd_smi(doc) -> list[dict]:
    """Records from ``amd-smi metric --json`` (list or {"gpu_data": [...]})."""
    rows = doc.get("gpu_data", []) if isinstance(doc, dict) else doc
    out = []

    def val(d, *path):
        for k in path:
            if not isinstance(d, dict):
                return None
            d = d.get(k)
        if isinstance(d, dict):
            d = d.get("value")
        return _num(d)

    for g in rows:
        mb = 1 << 20
        used, total = val(g, "mem_usage", "used_vram"), val(g, "mem_usage", "total_vram")
        temps = {k: v for k in ("edge", "hotspot", "mem") if (v := val(g, "temperature", k)) is not None}
        out.append({"acc_id": f"card{g.get('gpu', len(out))}", "index": int(g.get("gpu", len(out))),
                    "memory_used_bytes": used * mb if used is not None else 0.0,
                    "memory_total_bytes": total * mb if total is not None else 0.0,
                    "duty_cycle": val(g, "usage", "gfx_activity"),
                    "umc_activity": val(g, "usage", "umc_activity"),
                    "power_watts": val(g, "power", "socket_power"), "temperature_celsius": temps,
                    "ecc_uncorrectable": val(g, "ecc", "total_uncorrectable_count"), "bdf": ""})
    return out


def _esc(v) -> str:
    return str(v).replace("\\", "\\\\").replace('"', '\\"').replace("\n", "\\n")


def _labels(d: dict) -> str:
    return "{" + ",".join(f'{k}="{_esc(v)}"' for k, v in d.items()) + "}"


def exposition(devices: list[dict], owners: dict | None = None, model: str = "MI355X") -> str:
    """Prometheus text format.  `owners`: device index -> (namespace, pod, container)."""
    owners = owners or {}
    fams = {
        "container_accelerator_memory_used_bytes": ("gauge", "GPU HBM in use (bytes)"),
        "container_accelerator_memory_total_bytes": ("gauge", "GPU HBM capacity (bytes)"),
        "container_accelerator_duty_cycle": ("gauge", "Percent of time the GPU was busy"),
        "toa_gpu_power_watts": ("gauge", "GPU socket power (W)"),
        "toa_gpu_temperature_celsius": ("gauge", "GPU temperature sensors (C)"),
        "toa_gpu_info": ("gauge", "GPU identity"),
    }
    lines = {k: [] for k in fams}
    for d in devices:
        ns, pod, ctr = owners.get(d["index"], owners.get(str(d["index"]), ("", "", "")))
        base = {"make": "amd", "model": model, "acc_id": d["acc_id"], "namespace": ns, "pod": pod, "container": ctr}
        lines["container_accelerator_memory_used_bytes"].append((base, d["memory_used_bytes"]))
        lines["container_accelerator_memory_total_bytes"].append((base, d["memory_total_bytes"]))
        if d.get("duty_cycle") is not None:
            lines["container_accelerator_duty_cycle"].append((base, d["duty_cycle"]))
        if d.get("power_watts") is not None:
            lines["toa_gpu_power_watts"].append(({"acc_id": d["acc_id"]}, d["power_watts"]))
        for sensor, v in (d.get("temperature_celsius") or {}).items():
            lines["toa_gpu_temperature_celsius"].append(({"acc_id": d["acc_id"], "sensor": sensor}, v))
        lines["toa_gpu_info"].append(({"acc_id": d["acc_id"], "bdf": d.get("bdf", ""), "model": model}, 1))
    out = []
    for name, (typ, help_) in fams.items():
        if not lines[name]:
            continue
        out.append(f"# HELP {name} {help_}")
        out.append(f"# TYPE {name} {typ}")
        out += [f"{name}{_labels(lab)} {float(v):g}" for lab, v in lines[name]]
    return "\n".join(out) + "\n"


def serve(port: int, owners_path: str | None = None, root: str = SYSFS_DRM, accessible_only: bool = False):
    class H(http.server.BaseHTTPRequestHandler):
        def do_GET(self):
            if self.path.split("?")[0] != "/metrics":
                self.send_response(404)
                self.end_headers()
                return
            owners = {}
            if owners_path and os.path.exists(owners_path):
                with open(owners_path) as f:
                    owners = {int(k): tuple(v) for k, v in json.load(f).items()}
            body = exposition(read_devices(root, accessible_only), owners).encode()
            self.send_response(200)
            self.send_header("Content-Type", "text/plain; version=0.0.4")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass

    http.server.ThreadingHTTPServer(("", port), H).serve_forever()


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--port", type=int, default=9400)
    ap.add_argument("--owners", default=None, help="JSON {device index: [namespace, pod, container]}")
    ap.add_argument("--once", action="store_true", help="print one scrape and exit")
    ap.add_argument("--accessible-only", action="store_true",
                    help="only the GPUs whose /dev/dri render node this process can open (shared hosts)")
    a = ap.parse_args(argv)
    if a.once:
        print(exposition(read_devices(accessible_only=a.accessible_only)), end="")
        return 0
    serve(a.port, a.owners, accessible_only=a.accessible_only)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
