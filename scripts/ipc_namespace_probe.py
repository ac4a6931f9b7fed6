"""Does a HIP IPC memory handle open across Linux namespaces?  (Decides the
node-local layout's IPC mode: csrc/core/nodelocal.cc.)

Each node-local rank is its own pod, so on a real cluster two ranks differ in
their PID, network, mount and UTS namespaces.  With HSA_ENABLE_IPC_MODE_LEGACY=0
(DMA-BUF IPC, the only mode the MI355X hosts of this pool support) the
exporter's dmabuf fd has to reach the importer: this probe finds out which of
those namespaces that transfer crosses.

    python scripts/ipc_namespace_probe.py [--modes same,userns,pidns,netns,ipcns]

ROCm 7.2's runtime imports a DMA-BUF handle by opening /proc/<exporter
pid>/fd/<fd>, so the PID namespace is the one expected to matter.  Creating
the namespaces needs unprivileged user namespaces; where the host forbids
them (`unshare: ... No space left on device`, max_user_namespaces = 0) only
the `same` arm runs.

The driver (this process) never touches the GPU.  It starts the exporter as a
child, then one importer per mode, each under `unshare` (the exec happens
before the importer's first HIP call), and prints one JSON line per mode:
{"mode", "ok", "detail"}.  `userns` is the control for the others (each
needs a user namespace to be created without root).
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import tempfile
import time

N = 1 << 20
PATTERN = 0x5A


class IpcHandle(ctypes.Structure):
    """hipIpcMemHandle_t: 64 bytes, passed BY VALUE to hipIpcOpenMemHandle."""
    _fields_ = [("reserved", ctypes.c_char * 64)]


def _hip():
    for name in ("libamdhip64.so", "libamdhip64.so.7", "/opt/rocm/lib/libamdhip64.so"):
        try:
            return ctypes.CDLL(name)
        except OSError:
            continue
    raise OSError("libamdhip64 not found")


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed: hipError {rc}")


def exporter(handle_path: str, done_path: str, timeout: float):
    hip = _hip()
    _check(hip.hipSetDevice(0), "hipSetDevice")
    ptr = ctypes.c_void_p()
    _check(hip.hipMalloc(ctypes.byref(ptr), ctypes.c_size_t(N)), "hipMalloc")
    _check(hip.hipMemset(ptr, PATTERN, ctypes.c_size_t(N)), "hipMemset")
    _check(hip.hipDeviceSynchronize(), "hipDeviceSynchronize")
    handle = IpcHandle()
    _check(hip.hipIpcGetMemHandle(ctypes.byref(handle), ptr), "hipIpcGetMemHandle")
    tmp = handle_path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(bytes(handle))
    os.replace(tmp, handle_path)
    t0 = time.time()
    while not os.path.exists(done_path) and time.time() - t0 < timeout:
        time.sleep(0.05)
    hip.hipFree(ptr)


def importer(handle_path: str):
    hip = _hip()
    _check(hip.hipSetDevice(0), "hipSetDevice")
    raw = open(handle_path, "rb").read()
    handle = IpcHandle.from_buffer_copy(raw)
    dptr = ctypes.c_void_p()
    hip.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), IpcHandle, ctypes.c_uint]
    _check(hip.hipIpcOpenMemHandle(ctypes.byref(dptr), handle, ctypes.c_uint(1)), "hipIpcOpenMemHandle")
    host = (ctypes.c_ubyte * N)()
    _check(hip.hipMemcpy(host, dptr, ctypes.c_size_t(N), ctypes.c_int(2)), "hipMemcpy D2H")
    bad = sum(1 for i in range(0, N, 4093) if host[i] != PATTERN)
    hip.hipIpcCloseMemHandle(dptr)
    print(json.dumps({"pid": os.getpid(), "bad_samples": bad}), flush=True)
    sys.exit(0 if bad == 0 else 3)


UNSHARE = {
    "same": [],
    "userns": ["unshare", "--user", "--map-root-user"],
    "pidns": ["unshare", "--user", "--map-root-user", "--pid", "--fork"],
    "netns": ["unshare", "--user", "--map-root-user", "--net"],
    "ipcns": ["unshare", "--user", "--map-root-user", "--ipc"],
    "mntns": ["unshare", "--user", "--map-root-user", "--mount"],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--role", default="driver", choices=("driver", "exporter", "importer"))
    ap.add_argument("--handle", default="")
    ap.add_argument("--done", default="")
    ap.add_argument("--modes", default="same,userns,pidns,netns,ipcns,mntns")
    ap.add_argument("--timeout", type=float, default=60.0)
    a = ap.parse_args()
    if a.role == "exporter":
        return exporter(a.handle, a.done, a.timeout)
    if a.role == "importer":
        return importer(a.handle)
    d = tempfile.mkdtemp(prefix="toa_ipcns_")
    hp, dp = os.path.join(d, "handle"), os.path.join(d, "done")
    me = os.path.abspath(__file__)
    exp = subprocess.Popen([sys.executable, me, "--role", "exporter", "--handle", hp, "--done", dp,
                            "--timeout", str(a.timeout * 4)])
    t0 = time.time()
    while not os.path.exists(hp):
        if exp.poll() is not None or time.time() - t0 > a.timeout:
            print(json.dumps({"mode": "exporter", "ok": False, "detail": f"no handle (rc={exp.poll()})"}))
            exp.kill()
            return 1
        time.sleep(0.05)
    results = {}
    for mode in a.modes.split(","):
        cmd = UNSHARE[mode] + [sys.executable, me, "--role", "importer", "--handle", hp]
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=a.timeout)
            ok = r.returncode == 0
            detail = (r.stdout.strip().splitlines() or [""])[-1] if ok else (r.stderr.strip()[-300:] or f"rc={r.returncode}")
            if not ok and mode != "same" and "unshare" in detail:
                detail = "namespace unavailable: " + detail
        except subprocess.TimeoutExpired:
            ok, detail = False, "timeout"
        results[mode] = ok
        print(json.dumps({"mode": mode, "ok": ok, "detail": detail}), flush=True)
    open(dp, "w").close()
    exp.wait(timeout=a.timeout)
    print(json.dumps({"summary": results}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main() or 0)
