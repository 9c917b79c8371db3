#!/usr/bin/env python3
"""heap_leak_run.py -- run the `heapleak` worker mode (tests/support/
mp_worker.py) in 2 processes: create / destroy MP_LEAK_GIB GiB heaps
MP_LEAK_CYCLES times and report how many cycles succeeded.  Not a test."""
import json
import os
import pathlib
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "test-resilient-osss-ucx_amd")]
from test_multiproc import launch  # noqa: E402

res = launch("heapleak", 2, pathlib.Path(tempfile.mkdtemp()), timeout=500)
print(json.dumps(res))
