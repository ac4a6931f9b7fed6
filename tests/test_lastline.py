"""The pre-rendered last line (csrc/hip/lastline.hip, utils/lastline.py):
a fatal signal during bench.py's optional collectives A/B still writes the
headline JSON line, with the signal's number in it, and leaves with the
armed status; disarmed, the previous disposition is back.  Host code only:
runs without a GPU, each case in its own interpreter."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_PRE = """
import os, signal, sys, json
from tf_operator_amd.ops import _lib
if not _lib.has("toa_lastline_arm"):
    print("NOLIB"); sys.exit(0)
from tf_operator_amd.utils import lastline
"""


def _run(body: str):
    p = subprocess.run([sys.executable, "-c", _PRE + body], cwd=ROOT, capture_output=True, text=True, timeout=120)
    if p.stdout.strip() == "NOLIB":
        pytest.skip("libtoa_hip.so has no toa_lastline_arm (library not built)")
    return p


@pytest.mark.parametrize("sig,code", [("SIGSEGV", 0), ("SIGTERM", 3), ("SIGABRT", 0)])
def test_signal_writes_the_armed_line(sig, code):
    p = _run(f"""
line = json.dumps({{"metric": "m", "value": 1.5, "collectives_ab": {{"error": "signal " + lastline.SIGNO}}}})
assert lastline.arm(line + "\\n", {code})
print("before", flush=True)
os.kill(os.getpid(), signal.{sig})
print("not reached", flush=True)
""")
    import signal
    assert p.returncode == code, (p.returncode, p.stderr[-2000:])
    out = p.stdout.splitlines()
    assert out[0] == "before" and "not reached" not in p.stdout
    rec = json.loads(out[1])
    assert rec["collectives_ab"]["error"] == f"signal {int(getattr(signal, sig)):02d}"
    assert "fatal signal" in p.stderr


def test_rearm_empty_and_disarm():
    # re-armed with no text: leaves silently with the status
    p = _run("""
lastline.arm("first\\n", 0)
lastline.arm("", 5)
os.kill(os.getpid(), signal.SIGTERM)
""")
    assert p.returncode == 5 and "first" not in p.stdout
    # disarmed: SIGTERM has its default effect again
    p = _run("""
lastline.arm("armed\\n", 0)
lastline.disarm()
os.kill(os.getpid(), signal.SIGTERM)
""")
    assert p.returncode == -15 and "armed" not in p.stdout
