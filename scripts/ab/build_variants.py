"""Build variants of one HIP source into separate .so files for in-process
A/B timing (guide §5.4 rule 24: compare arms in one process, interleaved).

    python scripts/ab/build_variants.py csrc/hip/attention.hip base: noslp:-fno-slp-vectorize
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(ROOT, "build", "variants")


def build(src, name, flags):
    os.makedirs(OUT, exist_ok=True)
    so = os.path.join(OUT, f"{os.path.splitext(os.path.basename(src))[0]}_{name}.so")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-ffp-contract=fast", "-munsafe-fp-atomics", f"-I{os.path.join(ROOT, 'csrc', 'hip')}"] + flags + [src, "-o", so]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(f"{name}: {r.stderr[-3000:]}")
    return so


if __name__ == "__main__":
    src = os.path.join(ROOT, sys.argv[1])
    specs = [a.split(":", 1) for a in sys.argv[2:]]
    with ThreadPoolExecutor(8) as ex:
        for so in ex.map(lambda s: build(src, s[0], [f for f in s[1].split(",") if f]), specs):
            print(so)
