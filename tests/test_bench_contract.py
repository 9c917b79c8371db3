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


def _spawn(*extra, ndev="0", world=3, hwq=None):
    env = dict(os.environ, BENCH_NDEV=ndev, BENCH_RANK_GRACE_S="5")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
              "GPU_MAX_HW_QUEUES"):
        env.pop(k, None)
    if hwq is not None:
        env["GPU_MAX_HW_QUEUES"] = hwq
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world),
                           "--dry-ranks", "--deadline", "60", *extra],
                          capture_output=True, text=True, timeout=240, env=env)


def test_spawn_without_torchrun_plumbs_every_rank():
    """`python bench.py --gpus N` with no RANK: the parent starts N ranks
    itself (no torchrun), each with the torch.distributed.run environment;
    they meet over gloo at MASTER_ADDR:MASTER_PORT and rank 0's line is
    relayed once.  3 ranks on 1 GPU: each gets the 16-queue share."""
    r = _spawn(ndev="1")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["dry"] and d["n_gpus"] == 3
    ranks = d["ranks"]
    assert [x["RANK"] for x in ranks] == ["0", "1", "2"]
    assert [x["LOCAL_RANK"] for x in ranks] == ["0", "1", "2"]
    assert {x["WORLD_SIZE"] for x in ranks} == {"3"}
    assert {x["MASTER_ADDR"] for x in ranks} == {"127.0.0.1"}
    assert {x["GPU_MAX_HW_QUEUES"] for x in ranks} == {"5"}      # 16 // 3
    assert len({x["pid"] for x in ranks}) == 3


def test_spawn_lowers_an_exported_queue_count():
    """The GPU box exports HIP's default GPU_MAX_HW_QUEUES=4: 6 ranks sharing
    one GPU must still get 16 // 6 = 2 each (else 24 queues time-slice)."""
    r = _spawn(ndev="1", world=6, hwq="4")
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert {x["GPU_MAX_HW_QUEUES"] for x in d["ranks"]} == {"2"}


def test_spawn_no_queue_cap_with_a_gpu_per_rank():
    r = _spawn(ndev="8")
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert {x["GPU_MAX_HW_QUEUES"] for x in d["ranks"]} == {None}


def test_spawn_fails_loudly_when_a_rank_fails():
    r = _spawn("--dry-fail-rank", "2")
    assert r.returncode == 7, (r.returncode, r.stderr[-2000:])
    assert "rank exit codes" in r.stderr


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


def test_bench_names_the_shipped_lds_tile():
    """bench.py looks the LDS team kernel up by its rocprof name, whose last
    template argument is team.hip's OSGPU_TEAM_LDS_U: the two must agree."""
    import re
    sys.path.insert(0, ROOT)
    import bench
    src = open(os.path.join(ROOT, "test-resilient-osss-ucx_amd", "csrc", "team.hip")).read()
    m = re.search(r"#ifndef OSGPU_TEAM_LDS_U\s*\n#define OSGPU_TEAM_LDS_U (\d+)", src)
    assert m and int(m.group(1)) == bench.TEAM_LDS_U
    lo = re.search(r"#define OSGPU_TEAM_LDS_MIN_P (\d+)", src)
    hi = re.search(r"#define OSGPU_TEAM_LDS_MAX_P (\d+)", src)
    assert (int(lo.group(1)), int(hi.group(1))) == bench.TEAM_LDS_P
    comb = open(os.path.join(ROOT, "test-resilient-osss-ucx_amd", "csrc", "combine.hip")).read()
    on = re.search(r"#define OSGPU_COMBINE_LDS (\d+)", comb)
    u2 = re.search(r"#define OSGPU_COMBINE_LDS_U2 (\d+)", comb)
    assert on and int(on.group(1)) == 1
    assert u2 and bench.COMBINE_KERNEL == f"combine_lds_kernel<double, 0, 2, {u2.group(1)}>"
