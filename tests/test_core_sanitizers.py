"""Build the native core self-test under ASan+UBSan and TSan and run it
(race detection / sanitizers for the C++ core)."""
import glob
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CORE = os.path.join(ROOT, "csrc", "core")


def _build_and_run(tmp_path, flags, iters):
    srcs = [os.path.join(CORE, "tests", "core_selftest.cc")] + sorted(
        s for s in glob.glob(os.path.join(CORE, "*.cc")) if not s.endswith("bindings.cc"))
    exe = str(tmp_path / "selftest")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer"] + flags + srcs + ["-o", exe, "-lpthread"]
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    env = dict(os.environ, TOA_SELFTEST_ITERS=str(iters), TSAN_OPTIONS="halt_on_error=1",
               ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "core selftest OK" in r.stdout


def test_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"], 300)


def test_tsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=thread"], 20)
