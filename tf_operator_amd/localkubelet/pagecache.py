"""Node agent: pull the GPU code objects a trainer's first step needs into
the page cache, WITHOUT touching the GPU.

A replica's first step loads code objects lazily: hipBLASLt / Tensile
solution libraries for gfx950 (~0.5 GB under /opt/rocm/lib/hipblaslt),
the HIP / HSA / RCCL runtimes, torch's ROCm libraries and this framework's
libtoa_hip.so.  On a freshly booted node those come off disk during the
first job's first step (the round-2 driver saw one 8.2 s probe on a fresh
box against 1.5 s after it).  A real node pre-pulls the trainer image; the
local kubelet runs this module once at node start, in the background, as
its analogue: it reads each file through once (nothing is mapped, imported
or executed, so no HIP runtime is initialised here) and exits; the kubelet
reports when it is done (``LocalKubelet.node_warm``), which is when a real
node would have finished pulling the image.

    python -m tf_operator_amd.localkubelet.pagecache [--dry-run]
"""
from __future__ import annotations

import glob
import json
import os
import sys
import time

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _torch_lib_dir() -> str | None:
    try:
        import importlib.util

        spec = importlib.util.find_spec("torch")  # locates the package; does not import it
        if spec and spec.submodule_search_locations:
            return os.path.join(list(spec.submodule_search_locations)[0], "lib")
    except Exception:  # noqa: BLE001
        pass
    return None


# the ROCm runtime a trainer maps at its first GPU call and first kernel: the
# HIP / HSA runtimes, the code-object manager HIP parses every module with
# (160 MB), the GEMM libraries and RCCL.  torch bundles its own copies (same
# SONAMEs, so a process that imports torch first uses those for this
# framework's libraries too); both trees are listed
RUNTIME_LIBS = ("libamdhip64.so*", "libhsa-runtime64.so*", "libamd_comgr.so*", "libhipblaslt.so*",
                "librocroller.so*", "librccl.so*", "librocblas.so*", "librocprofiler-register.so*",
                "libroctx64.so*")
TORCH_LIBS = ("libtorch_hip.so", "libc10_hip.so")


def candidate_files(rocm: str | None = None, arch: str = "gfx950") -> list[str]:
    rocm = rocm or os.environ.get("ROCM_PATH", "/opt/rocm")
    pats = [os.path.join(REPO_ROOT, "tf_operator_amd", "lib", "*.so"),
            os.path.join(REPO_ROOT, "tf_operator_amd", "core", "*.so")]
    tdir = _torch_lib_dir()
    # the trainer imports torch first, so torch's copies are the ones it maps;
    # the system tree only without a torch that bundles ROCm
    bundled = bool(tdir) and bool(glob.glob(os.path.join(tdir, "libamdhip64.so*")))
    for lib in [tdir] if bundled else [os.path.join(rocm, "lib")]:
        pats += [os.path.join(lib, n) for n in RUNTIME_LIBS]
        pats += [os.path.join(lib, "hipblaslt", "library", f"*{arch}*"),
                 os.path.join(lib, "rocblas", "library", f"*{arch}*")]
    if tdir:
        pats += [os.path.join(tdir, n) for n in TORCH_LIBS]
    out, seen = [], set()
    for p in pats:
        for f in sorted(glob.glob(p)):
            r = os.path.realpath(f)
            if os.path.isfile(r) and r not in seen:
                seen.add(r)
                out.append(r)
    return out


def warm(files: list[str], chunk: int = 8 << 20) -> dict:
    """Read every file through once (the page cache keeps it; nothing is
    mapped or executed).  A POSIX_FADV_WILLNEED hint alone returned before
    the pages were in, and the first job on a fresh node still read them from
    disk (profiles/r4_fresh2: the first probe's first forward 1.68 s against
    0.12 s after it)."""
    t0, n, nbytes = time.time(), 0, 0
    for f in files:
        try:
            fd = os.open(f, os.O_RDONLY)
        except OSError:
            continue
        try:
            size = os.fstat(fd).st_size
            os.posix_fadvise(fd, 0, size, os.POSIX_FADV_SEQUENTIAL)
            while os.read(fd, chunk):
                pass
            n, nbytes = n + 1, nbytes + size
        except OSError:
            pass
        finally:
            os.close(fd)
    return {"files": n, "bytes": nbytes, "read_s": round(time.time() - t0, 3)}


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
