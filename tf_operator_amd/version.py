"""Version info (reference: pkg/version/version.go:21-43)."""
import os
import subprocess

__version__ = "0.1.0"


def _git_sha():
    try:
        here = os.path.dirname(os.path.abspath(__file__))
        return subprocess.run(["git", "-C", here, "rev-parse", "--short", "HEAD"], capture_output=True, text=True,
                              timeout=5).stdout.strip() or "unknown"
    except Exception:
        return "unknown"


GIT_SHA = os.environ.get("TOA_GIT_SHA") or "unknown"


def info():
    sha = GIT_SHA if GIT_SHA != "unknown" else _git_sha()
    return f"tf_operator_amd version: {__version__}, git SHA: {sha}"
