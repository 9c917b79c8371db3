"""The PE-thread runtime's barrier (tests/support/pe_threads.c, the stand-in
for shmem_barrier, src/barrier.c:21-27): polling by default, as the
reference's (src/shmemc/barrier.c:32,47), sleeping under PET_SLEEP_BARRIER=1.
No thread may leave round r before every thread has entered it, with more
PE threads than cores and with active sets that skip PEs.  CPU only."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

SCRIPT = r"""
import ctypes, sys, threading
sys.path.insert(0, sys.argv[1])
from support import team as T
P = T.pet()
npes, rounds, stride_log = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
assert P.pet_init(64) == 0
members = list(range(0, npes << stride_log, 1 << stride_log))
count = [0] * len(members)
errs = []
def body(i, pe):
    P.pet_set_me(pe)
    for r in range(rounds):
        count[i] = r + 1
        P.pet_barrier(0, stride_log, len(members), None)
        if min(count) < r + 1:
            errs.append((pe, r, list(count)))
        P.pet_barrier(0, stride_log, len(members), None)
ths = [threading.Thread(target=body, args=(i, pe)) for i, pe in enumerate(members)]
[t.start() for t in ths]
[t.join() for t in ths]
assert not errs, errs[:3]
print("ok", P.pet_barrier_calls(members[-1]))
"""


@pytest.mark.parametrize("sleep", ["0", "1"])
@pytest.mark.parametrize("npes,stride_log", [(2, 0), (16, 0), (5, 1)])
def test_barrier_holds_every_round(sleep, npes, stride_log):
    from support import team as T
    T.build_pet()
    env = dict(os.environ, PET_SLEEP_BARRIER=sleep)
    rounds = 200
    r = subprocess.run([sys.executable, "-c", SCRIPT, HERE, str(npes), str(rounds),
                        str(stride_log)], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-1500:]
    assert r.stdout.split() == ["ok", str(2 * rounds)]
