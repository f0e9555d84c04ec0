"""Version metadata (reference: ``version/version.go:3-6``, injected by
``-ldflags -X`` in ``Makefile:22-26``).  Here ``GIT_SHA`` is resolved from the
repository at runtime when not baked in by the build."""
import os
import platform
import subprocess
import sys

__version__ = "0.1.0"
VERSION = __version__
GIT_SHA = os.environ.get("KFA_GIT_SHA", "")


def git_sha() -> str:
    if GIT_SHA:
        return GIT_SHA
    try:
        here = os.path.dirname(os.path.abspath(__file__))
        return subprocess.run(["git", "-C", here, "rev-parse", "--short", "HEAD"], capture_output=True,
                              text=True, timeout=5).stdout.strip() or "unknown"
    except Exception:
        return "unknown"


def version_info() -> dict:
    return {"version": VERSION, "gitSHA": git_sha(), "python": sys.version.split()[0],
            "platform": f"{platform.system().lower()}/{platform.machine()}"}
