"""Test configuration: register the `gpu` marker and make the package / oracle importable.

For the multi-process GPU tests (test_gpu_multiproc.py) the rank processes are started by
tests/rank_launcher.py, which this file starts when the session begins — before any test
initialises the GPU, because a process that has initialised the GPU must not fork + exec
another program.  The launcher is not started when GPU tests are deselected (-m "not gpu").
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gpu-randomized-block-lanczos_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

_LAUNCHER = None


def pytest_configure(config):
    global _LAUNCHER
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librbl_hip.so)")
    markexpr = getattr(config.option, "markexpr", "") or ""
    if "not gpu" in markexpr or _LAUNCHER is not None:
        return
    _LAUNCHER = subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "rank_launcher.py")],
                                 stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)


def pytest_unconfigure(config):
    global _LAUNCHER
    if _LAUNCHER is not None:
        try:
            _LAUNCHER.stdin.close()
            _LAUNCHER.wait(timeout=30)
        except Exception:  # noqa: BLE001
            _LAUNCHER.kill()
        _LAUNCHER = None


class RankLauncher:
    """Runs one command per rank through the pre-started launcher; returns (rcs, outputs)."""

    def __init__(self, proc):
        self.proc = proc

    def run(self, cmds, timeout=240, env=None):
        self.proc.stdin.write(json.dumps({"cmds": cmds, "timeout": timeout, "env": env or {}}) + "\n")
        self.proc.stdin.flush()
        reply = json.loads(self.proc.stdout.readline())
        return reply["rc"], reply["out"]


@pytest.fixture(scope="session")
def rank_launcher():
    if _LAUNCHER is None or _LAUNCHER.poll() is not None:
        pytest.skip("rank launcher not running (GPU tests deselected)")
    return RankLauncher(_LAUNCHER)
