"""Node agent: pull the GPU code objects a trainer's first step needs into
the page cache, WITHOUT touching the GPU.

A replica's first step loads code objects lazily: hipBLASLt / Tensile
solution libraries for gfx950 (~0.5 GB under /opt/rocm/lib/hipblaslt),
the HIP / HSA / RCCL runtimes, torch's ROCm libraries and this framework's
libtoa_hip.so.  On a freshly booted node those come off disk during the
first job's first step (the round-2 driver saw one 8.2 s probe on a fresh
box against 1.5 s after it).  A real node pre-pulls the trainer image; the
local kubelet runs this module once at node start, in the background, as
its analogue: ``posix_fadvise(WILLNEED)`` on each file (the kernel reads
ahead asynchronously; nothing is mapped, imported or executed, so no HIP
runtime is initialised here).

    python -m tf_operator_amd.localkubelet.pagecache [--dry-run]
"""
from __future__ import annotations

import glob
import json
import os
import sys
import time

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def candidate_files(rocm: str | None = None, arch: str = "gfx950") -> list[str]:
    rocm = rocm or os.environ.get("ROCM_PATH", "/opt/rocm")
    pats = [os.path.join(rocm, "lib", "hipblaslt", "library", f"*{arch}*"),
            os.path.join(rocm, "lib", "rocblas", "library", f"*{arch}*"),
            os.path.join(rocm, "lib", "libamdhip64.so*"), os.path.join(rocm, "lib", "libhsa-runtime64.so*"),
            os.path.join(rocm, "lib", "libhipblaslt.so*"), os.path.join(rocm, "lib", "librccl.so*"),
            os.path.join(REPO_ROOT, "tf_operator_amd", "lib", "*.so")]
    try:
        import importlib.util

        spec = importlib.util.find_spec("torch")  # locates the package; does not import it
        if spec and spec.submodule_search_locations:
            tdir = list(spec.submodule_search_locations)[0]
            pats += [os.path.join(tdir, "lib", n) for n in ("libtorch_hip.so", "libc10_hip.so", "libtorch_cpu.so")]
    except Exception:  # noqa: BLE001
        pass
    out, seen = [], set()
    for p in pats:
        for f in sorted(glob.glob(p)):
            r = os.path.realpath(f)
            if os.path.isfile(r) and r not in seen:
                seen.add(r)
                out.append(r)
    return out


def warm(files: list[str]) -> dict:
    t0, n, nbytes = time.time(), 0, 0
    for f in files:
        try:
            fd = os.open(f, os.O_RDONLY)
        except OSError:
            continue
        try:
            size = os.fstat(fd).st_size
            os.posix_fadvise(fd, 0, size, os.POSIX_FADV_WILLNEED)
            n, nbytes = n + 1, nbytes + size
        except OSError:
            pass
        finally:
            os.close(fd)
    return {"files": n, "bytes": nbytes, "advise_s": round(time.time() - t0, 3)}


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    files = candidate_files()
    if "--dry-run" in argv:
        print(json.dumps({"files": len(files), "bytes": sum(os.path.getsize(f) for f in files)}))
        return 0
    print(json.dumps(warm(files)), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
