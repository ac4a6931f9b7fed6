"""In-tree native build for tf_operator_amd.

Two native artefacts, both built IN the source tree so they travel with the
repo snapshot to the GPU box:

* ``tf_operator_amd/lib/libtoa_hip.so`` -- every ``csrc/hip/*.hip`` kernel,
  compiled by ``hipcc --offload-arch=gfx950`` (no torch headers; bound with
  ctypes by :mod:`tf_operator_amd.ops._lib`).
* ``tf_operator_amd/core/_toa_core<EXT_SUFFIX>`` -- the C++17 operator core
  (``csrc/core/*.cc``: API types, defaulting, validation, reconcile engine,
  status engines, cluster-spec / RCCL env generation) exposed via pybind11.

Usage: ``python -m tf_operator_amd._build [--force] [--only hip|core]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "tf_operator_amd")
HIP_SRC = os.path.join(ROOT, "csrc", "hip")
CORE_SRC = os.path.join(ROOT, "csrc", "core")
BUILD = os.path.join(ROOT, "build")
HIP_LIB = os.path.join(PKG, "lib", "libtoa_hip.so")
ARCH = os.environ.get("TOA_OFFLOAD_ARCH", "gfx950")


# extra hipcc flags per source file (none at present; an A/B of attention.hip
# with -fno-honor-nans -mno-amdgpu-ieee measured 9 % slower forward and a
# spilling dK/dV kernel, profiles/r2_attention/ab_valu.log)
PER_FILE_FLAGS: dict[str, list[str]] = {}


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    return "hipcc"


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def _jobs():
    try:
        return max(1, min(16, int(os.environ.get("MAX_JOBS", "0")) or (os.cpu_count() or 4)))
    except ValueError:
        return 4


def build_hip(force=False, verbose=False):
    srcs = sorted(glob.glob(os.path.join(HIP_SRC, "*.hip")))
    hdrs = glob.glob(os.path.join(HIP_SRC, "*.h"))
    os.makedirs(os.path.join(BUILD, "hip"), exist_ok=True)
    os.makedirs(os.path.dirname(HIP_LIB), exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=fast", "-Wno-unused-result",
             "-munsafe-fp-atomics"]
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(BUILD, "hip", os.path.basename(s) + ".o")
        objs.append(o)
        if force or _stale(o, [s] + hdrs + [os.path.abspath(__file__)]):
            todo.append([_hipcc()] + flags + PER_FILE_FLAGS.get(os.path.basename(s), []) + ["-c", s, "-o", o])
    with cf.ThreadPoolExecutor(_jobs()) as ex:
        for out in ex.map(_run, todo):
            if verbose and out.strip():
                print(out)
    if force or todo or _stale(HIP_LIB, objs):
        _run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", HIP_LIB] + objs +
             ["-L/opt/rocm/lib", "-lhipblaslt", "-Wl,-rpath,/opt/rocm/lib"])
    return HIP_LIB


def core_target():
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG, "core", "_toa_core" + suffix)


def build_core(force=False, verbose=False, sanitize=None):
    import pybind11

    srcs = sorted(glob.glob(os.path.join(CORE_SRC, "*.cc")))
    hdrs = glob.glob(os.path.join(CORE_SRC, "*.h"))
    if not srcs:
        return None
    target = core_target()
    os.makedirs(os.path.join(BUILD, "core"), exist_ok=True)
    inc = [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}", f"-I{CORE_SRC}"]
    flags = ["-O2", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-fvisibility=hidden"]
    if sanitize:
        flags += [f"-fsanitize={sanitize}", "-fno-omit-frame-pointer", "-g"]
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(BUILD, "core", os.path.basename(s) + (f".{sanitize}" if sanitize else "") + ".o")
        objs.append(o)
        if force or _stale(o, [s] + hdrs):
            todo.append([os.environ.get("CXX", "g++")] + flags + inc + ["-c", s, "-o", o])
    with cf.ThreadPoolExecutor(_jobs()) as ex:
        for out in ex.map(_run, todo):
            if verbose and out.strip():
                print(out)
    if sanitize:
        return objs
    if force or todo or _stale(target, objs):
        _run([os.environ.get("CXX", "g++"), "-shared", "-fPIC", "-o", target] + objs)
    return target


def build_all(force=False, verbose=False):
    return {"core": build_core(force, verbose), "hip": build_hip(force, verbose)}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["hip", "core"])
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    if a.only in (None, "core"):
        print("core:", build_core(a.force, a.verbose))
    if a.only in (None, "hip"):
        print("hip:", build_hip(a.force, a.verbose))


if __name__ == "__main__":
    sys.exit(main())
