"""The three ways PE threads that share one GPU split a team call
(shmem_reduce.cpp run_team, OSGPU_TEAM_LOCAL): `merge` (the default: the
run's first member launches one grid for all of it) runs through every other
GPU test; `shards` (contiguous shards), `tiles` (member k of m folds tiles
k, k + m, ... of the union of their shards) and `merge` with the blocking
completion wait (OSGPU_SYNC=block instead of the default word) are replayed
here over every
golden case of tests/golden/reduce_cases.json, bit-exact against the
reference's digests, each mode in its own process (the mode is read once
per process)."""
import json
import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import json, os, sys
root = sys.argv[1]
sys.path[:0] = [os.path.join(root, "tests"), os.path.join(root, "oracle"),
                os.path.join(root, "test-resilient-osss-ucx_amd")]
import torch
assert torch.cuda.is_available()
import test_gpu_parity as G
if os.environ.get("TEST_MAX_LAUNCH_THREADS"):  # the multi-launch path (a test hook)
    import ctypes
    import osgpu
    L = osgpu.load()
    L.osgpu_test_max_launch_threads.argtypes = [ctypes.c_longlong]
    assert L.osgpu_test_max_launch_threads(int(os.environ["TEST_MAX_LAUNCH_THREADS"])) == 0
tm = G.team()
bad, paths, n = [], {}, 0
for c in G.CASES:
    out = G.run_case(tm, c)
    try:
        G.check(c, out)
    except AssertionError as e:
        bad.append(str(e))
    for p in tm.last_paths.values():
        paths[p] = paths.get(p, 0) + 1
    n += 1
print(json.dumps({"cases": n, "nbad": len(bad), "bad": bad[:5], "paths": paths}))
"""


@pytest.mark.parametrize("mode", ["shards", "tiles", "merge+block", "tiles+small"])
def test_team_local_modes_match_golden(mode):
    # +block: OSGPU_SYNC=block (hipStreamSynchronize) instead of the default
    # completion word (runtime.cpp stream_wait); +small: at most 2048 threads
    # per launch (test hook), so the tiles of every member k of m run over
    # several launches (team.hip team_launch_p: runs of whole multiples of m)
    local, _, extra = mode.partition("+")
    env = dict(os.environ, OSGPU_TEAM_LOCAL=local)
    if extra == "block":
        env["OSGPU_SYNC"] = extra
    elif extra == "small":
        env.update(OSGPU_TEST_HOOKS="1", TEST_MAX_LAUNCH_THREADS="2048")
    r = subprocess.run([sys.executable, "-c", SCRIPT, ROOT], env=env, capture_output=True,
                       text=True, timeout=280)
    assert r.returncode == 0, (r.stdout + r.stderr)[-2000:]
    res = json.loads([line for line in r.stdout.splitlines() if line.startswith("{")][-1])
    assert res["nbad"] == 0, res["bad"]
    assert res["cases"] > 100
    assert res["paths"].get("team", 0) > 100, res["paths"]


SWITCH = r"""
import ctypes, json, os, queue, sys, threading
root = sys.argv[1]
sys.path[:0] = [os.path.join(root, "tests"), os.path.join(root, "oracle"),
                os.path.join(root, "test-resilient-osss-ucx_amd")]
import numpy as np
import torch
assert torch.cuda.is_available()
import oracle as O
from support import team as T
P, n = 3, 40_003
tm = T.Team(P, 2 * n * 8 + 8192, device=True)
toff = (n * 8 + 4095) // 4096 * 4096
fn = tm.osgpu.to_all("double", "sum")
pwrk = (ctypes.c_byte * 4096)()
def call(pe):
    tm.pet.pet_set_me(pe)
    fn(tm.ptr(pe, toff), tm.ptr(pe, 0), n, 0, 0, P, ctypes.addressof(pwrk), tm.psync_ptr(pe))
# PE 0 keeps one thread for every call; PEs 1 and 2 get a fresh thread per
# call (a thread pool handing a PE's calls to different threads)
jobs, done = queue.Queue(), queue.Queue()
def pe0_loop():
    while jobs.get():
        call(0)
        done.put(1)
t0 = threading.Thread(target=pe0_loop)
t0.start()
bad = 0
for r in range(4):
    src = O.team_inputs("double", P, n, 0x7100 + r, "wide")
    for pe in range(P):
        tm.write(pe, 0, src[pe])
    want = O.to_all("double", "sum", src)
    jobs.put(1)
    ths = [threading.Thread(target=call, args=(pe,)) for pe in (1, 2)]
    for th in ths: th.start()
    for th in ths: th.join()
    done.get()
    for pe in range(P):
        got = tm.read(pe, toff, n * 8).view(np.uint64)
        bad += int(np.sum(got != want[pe].view(np.uint64)))
jobs.put(0)
t0.join()
print(json.dumps({"bad": bad}))
"""


def test_merge_matches_calls_when_threads_switch():
    """OSGPU_TEAM_LOCAL=merge matches a call across a process's members by a
    sequence number kept per PE, not per OS thread: PE 0 calls
    from one thread, PEs 1 and 2 from a new thread every call.  Every call
    is bit-exact against the oracle, and every call after the first still
    forms ONE merged run of all 3 members (the debug log's "tiles k of 3";
    a per-thread count would have split calls 2-4 into runs of 1 and 2)."""
    env = dict(os.environ, OSGPU_TEAM_LOCAL="merge", OSGPU_DEBUG="1")
    r = subprocess.run([sys.executable, "-c", SWITCH, ROOT], env=env, capture_output=True,
                       text=True, timeout=200)
    assert r.returncode == 0, (r.stdout + r.stderr)[-2000:]
    res = json.loads([line for line in r.stdout.splitlines() if line.startswith("{")][-1])
    assert res["bad"] == 0, res
    # (the PE threads' debug lines may interleave: match the messages, not lines)
    runs = re.findall(r"team path, \[\d+, \d+\) of \d+, tiles (\d+) of (\d+), P=3", r.stderr)
    assert len(runs) == 4 * 3, runs
    assert all(m == "3" for _, m in runs), runs
