"""bench.py's output contract on the CPU (no GPU needed): the N > 1 watchdog
prints the partial line and exits non-zero when a phase stalls, and the
argument defaults the driver relies on."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STALL = r"""
import sys, time
sys.path.insert(0, {root!r})
import bench
res = {{"metric": bench.METRIC, "value": 12.5, "n_gpus": 2}}
state, emit = bench.start_watchdog(res, 0, 0.5)
state["phase"] = "config4"
time.sleep(30)          # a stalled phase
print("not reached")
"""

DONE = r"""
import sys
sys.path.insert(0, {root!r})
import bench
res = {{"metric": bench.METRIC, "value": 12.5, "n_gpus": 2}}
state, emit = bench.start_watchdog(res, 0, 30.0)
emit()
emit()                  # printed once
"""


def _run(code):
    return subprocess.run([sys.executable, "-c", code.format(root=ROOT)], capture_output=True,
                          text=True, timeout=60)


def test_watchdog_stall_exits_nonzero_with_partial_line():
    r = _run(STALL)
    assert r.returncode == 3, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1 and "not reached" not in r.stdout
    d = json.loads(lines[0])
    assert d["value"] == 12.5 and "config4" in d["incomplete"]


def test_completed_line_printed_once():
    r = _run(DONE)
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1 and "incomplete" not in json.loads(lines[0])


def test_defaults_single_gpu_within_minutes():
    sys.path.insert(0, ROOT)
    import bench
    old = sys.argv
    try:
        sys.argv = ["bench.py"]
        a = bench.parse()
    finally:
        sys.argv = old
    assert a.gpus == 1 and a.nreduce == 64 << 20 and 0 < a.steps <= 100 and 0 <= a.warmup
