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


@pytest.mark.parametrize("mode", ["shards", "tiles", "merge+block"])
def test_team_local_modes_match_golden(mode):
    # +block: OSGPU_SYNC=block (hipStreamSynchronize) instead of the default
    # completion word (runtime.cpp stream_wait)
    local, _, sync = mode.partition("+")
    env = dict(os.environ, OSGPU_TEAM_LOCAL=local)
    if sync:
        env["OSGPU_SYNC"] = sync
    r = subprocess.run([sys.executable, "-c", SCRIPT, ROOT], env=env, capture_output=True,
                       text=True, timeout=280)
    assert r.returncode == 0, (r.stdout + r.stderr)[-2000:]
    res = json.loads([line for line in r.stdout.splitlines() if line.startswith("{")][-1])
    assert res["nbad"] == 0, res["bad"]
    assert res["cases"] > 100
    assert res["paths"].get("team", 0) > 100, res["paths"]
