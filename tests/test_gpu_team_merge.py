"""The merged team launch of co-resident PE threads (csrc/shmem_reduce.cpp
run_team): PE threads of one process on one GPU launch the team kernel
ONCE per run of consecutive active-set members, by the run's lowest index,
instead of once per member.  Each mode runs in its own process (the switch
OSGPU_TEAM_LOCAL_MERGE is read once): 8 PE threads, the whole set and a
strided subset (PE_start 1, stride 2, 3 members), double sum / float prod /
int xor / complexd prod, ragged sizes -- both modes bit-exact against the
oracle's per-PE fold (src/reductions.c:79-111), and the OSGPU_DEBUG lines
show who launched: merged, member 0 covers every shard and the others none.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import sys, numpy as np
sys.path[:0] = [%r, %r, %r]
import torch
import oracle as O
from support import team as T
tm = T.Team(8, 17 << 20, device=True)
ok = True
for t, op, n, (ps, ls, sz) in (("double", "sum", 1000003, (0, 0, 8)),
                                ("float", "prod", 77777, (1, 1, 3)),
                                ("int", "xor", 4097, (0, 0, 8)),
                                ("complexd", "prod", 65541, (0, 0, 5))):
    srcs = [O.gen_input(t, n, O.pe_seed(0x3E, pe), "wide") for pe in range(8)]
    want = O.to_all(t, op, srcs, ps, ls, sz)
    nb = srcs[0].nbytes
    toff = (nb + 4095) // 4096 * 4096
    assert toff + nb <= tm.psync_off, "source and target must fit in every PE's heap slice"
    for pe in range(8):
        tm.write(pe, 0, srcs[pe])
        tm.fill(pe, toff, nb, 0)
    torch.cuda.synchronize()
    tm.run(t, op, toff, 0, n, ps, ls, sz)
    for pe in O.active_set(ps, ls, sz):
        got = tm.read(pe, toff, nb)
        good = np.array_equal(got, np.ascontiguousarray(want[pe]).view(np.uint8).reshape(-1))
        ok = ok and good
        print("CASE", t, op, n, ps, ls, sz, pe, tm.last_paths[pe], good, flush=True)
print("ALLOK" if ok else "MISMATCH", flush=True)
"""


def _run(merge):
    code = SCRIPT % (os.path.join(ROOT, "tests"), os.path.join(ROOT, "test-resilient-osss-ucx_amd"),
                     os.path.join(ROOT, "oracle"))
    env = dict(os.environ, OSGPU_TEAM_LOCAL_MERGE=merge, OSGPU_DEBUG="1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    return r.stdout, r.stderr


@pytest.mark.parametrize("merge", ["1", "0"])
def test_merged_team_launch_bit_exact(merge):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out, err = _run(merge)
    assert "ALLOK" in out, out[-3000:]
    cases = [l.split() for l in out.splitlines() if l.startswith("CASE")]
    assert len(cases) == 8 + 3 + 8 + 5
    assert all(c[8] == "team" for c in cases), out
    runs = [l for l in err.splitlines() if "team path, members" in l]
    assert runs, err[-2000:]
    if merge == "1":
        # every call: one leader (index 0) over the whole set, the rest none
        assert all(("members 0.." in l) or ("members -1..-1" in l) for l in runs), runs[:20]
        leads = [l for l in runs if "members 0.." in l]
        assert len(leads) == 4, leads
        assert any("members 0..7" in l for l in leads) and any("members 0..2" in l for l in leads)
    else:
        # one launch per member: every member's own shard
        assert not any("members -1..-1" in l for l in runs), runs[:20]
