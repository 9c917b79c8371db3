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
    # the 8-member LDS rule for real types (TeamShape kLds) and bench's mirror
    assert ("((P == 5 || P == 6 || P == 8) && !kComplex && !kFpMinMax)" in src
            and bench.TEAM_LDS_EXTRA_P == (5, 6, 8))
    assert bench.team_lds(8) and not bench.team_lds(8, remote=True) and not bench.team_lds(7)
    comb = open(os.path.join(ROOT, "test-resilient-osss-ucx_amd", "csrc", "combine.hip")).read()
    kmax = re.search(r"constexpr int kCombineLdsMaxK = (\d+);", comb)
    u2 = re.search(r"#define OSGPU_COMBINE_LDS_U2 (\d+)", comb)
    assert kmax and int(kmax.group(1)) >= 2      # K = 2 takes the LDS-staged form
    assert u2 and bench.COMBINE_KERNEL == f"combine_lds_kernel<double, 0, 2, {u2.group(1)}>"


# ---------------------------------------------------------------- line cap
# The driver parses ONE JSON line of bounded size: round 5's 21.7 KB line
# went unparsed (missing 1).  bench.fit_line() keeps it at most
# bench.LINE_CAP bytes and writes the full result to the detail file.

CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
            "roofline", "cpu_baseline")


def _bulky(seed, width=120):
    """A side measurement that survives _shrink at full size: many numeric
    fields, nested, no detail-only keys."""
    return {f"field_{seed}_{i}": {"ms_per_call": 1.234567 * i, "GBs": 4567.891 * i,
                                  "frac": 0.7654321, "correct": True}
            for i in range(width)}


def _maximal(n_gpus):
    import bench
    res = {"metric": bench.METRIC, "value": 6543.21, "unit": "GiB/s", "n_gpus": n_gpus,
           "steps": 20, "warmup": 5, "ms_per_step": 0.2359, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f64",
           "data": "synthetic: uniform [1,2) doubles resident in HBM",
           "config": {"workload": "x" * 2000, "nreduce": 64 << 20, "K": 2},
           "roofline": {"bound": "hbm", "achieved": 6850.0, "peak": 8000.0, "unit": "GB/s",
                        "frac": 0.856, "traffic": 1610641408, "kernel": "k" * 300,
                        "addresses": ["0x7f0000000000"] * 64},
           "cpu_baseline": {"value": 23.6, "unit": "GiB/s", "cores": 2, "kind": "reference",
                            "sample": "s" * 3000},
           "heap_preflight": {str(r): {"status": "ok", "remote_write": "ok"} for r in range(8)},
           "launch": {"ranks": [{"pci_bus_id": "0000:%02x:00.0" % r, "uuid": "u" * 40}
                                for r in range(8)]}}
    for i, k in enumerate(bench.DROP_ORDER + ("extra_a", "extra_b")):
        res[k] = _bulky(i)
    res["team_by_members"] = {str(P): {"frac": 0.8, "trials": [
        {"frac": 0.8, "copy_frac": 0.82, "of_copy": 0.97, "canary": [0.79, 0.8], "label": "ok",
         "src": ["0x7f0000000000"] * 8}] * 3, "placements": [_bulky(P)]} for P in (2, 4, 8)}
    return res


def test_line_cap_on_maximal_results(tmp_path):
    import bench
    for n in (1, 2, 8):
        res = _maximal(n)
        det = tmp_path / f"detail_{n}.json"
        text = bench.fit_line(res, str(det))
        assert len(text.encode()) <= bench.LINE_CAP, (n, len(text))
        assert "\n" not in text
        d = json.loads(text)
        for k in CONTRACT:
            assert k in d, (n, k)
        assert d["roofline"]["frac"] == 0.856 and d["cpu_baseline"]["kind"] == "reference"
        assert "dropped_to_fit" in d
        # the detail file holds everything, the line names it
        full = json.loads(det.read_text())
        assert set(full) >= set(res) and d["detail"].endswith(det.name)


def test_line_cap_on_round5_line():
    """The round-5 N=1 line that the driver could not parse (21.7 KB) fits
    without dropping any contract field."""
    import bench
    p = os.path.join(ROOT, "profiles", "r05_bench_run8.log")
    if not os.path.exists(p):
        import pytest
        pytest.skip("round-5 log absent")
    res = json.loads([l for l in open(p) if l.startswith("{")][-1])
    assert len(json.dumps(res)) > 20000
    text = bench.fit_line(res)
    assert len(text.encode()) <= bench.LINE_CAP
    d = json.loads(text)
    for k in CONTRACT:
        assert k in d


def test_watchdog_line_is_capped(tmp_path):
    code = r"""
import sys
sys.path.insert(0, {root!r})
import bench
sys.path.insert(0, {tests!r})
from test_bench_contract import _maximal
res = _maximal(8)
state, emit = bench.start_watchdog(res, 0, 30.0, {det!r})
emit()
""".format(root=ROOT, tests=os.path.join(ROOT, "tests"), det=str(tmp_path / "d.json"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    import bench
    assert len(lines) == 1 and len(lines[0].encode()) <= bench.LINE_CAP


def test_trial_labels():
    """A slow trial is a box transient when the canary around it was slow,
    a placement when the canary was normal."""
    import bench
    tr = [{"frac": 0.78, "copy_frac": 0.80, "canary": [0.80, 0.80], "spread": [1.0, 1.0]},
          {"frac": 0.30, "copy_frac": 0.80, "canary": [0.31, 0.79], "spread": [1.0, 1.0]},
          {"frac": 0.79, "copy_frac": 0.25, "canary": [0.80, 0.81], "spread": [1.0, 1.02]},
          {"frac": 0.80, "copy_frac": 0.81, "canary": [0.80, 0.79], "spread": [1.0, 1.0]},
          {"frac": 0.79, "copy_frac": 0.20, "canary": [0.80, 0.79], "spread": [1.0, 4.1]}]
    by = {"4": {"trials": tr}, "canary": {"median": 0.8}}
    counts = bench.label_trials(by, 0.8)
    assert [t["label"] for t in tr] == ["ok", "transient", "placement", "ok", "transient"]
    assert counts == {"ok": 2, "transient": 2, "placement": 1}


def test_compile_time_knobs_bounded():
    """at most 10 `#ifndef OSGPU_*` knobs in the product
    sources, none of them a rejected experiment, and no environment variable
    read per call (every getenv of a knob sits in a function-local static
    initialiser or a read-once helper)."""
    import glob
    import re
    csrc = os.path.join(ROOT, "test-resilient-osss-ucx_amd", "csrc")
    knobs = []
    for f in glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.hpp")) + \
            glob.glob(os.path.join(csrc, "*.cpp")):
        knobs += re.findall(r"#ifndef (OSGPU_\w+)", open(f).read())
    assert len(knobs) <= 10, knobs
    for gone in ("OSGPU_TEAM_PIPE_FP", "OSGPU_TEAM_PIPE_FENCE", "OSGPU_TEAM_OCC_LDS",
                 "OSGPU_TEAM_LDS_ROT", "OSGPU_COMBINE_G8", "OSGPU_TEAM_XCD", "OSGPU_TEAM_GLDS"):
        assert gone not in knobs
    hdr = open(os.path.join(ROOT, "include", "osgpu_reduce.h")).read()
    for k in knobs:
        if k not in ("OSGPU_BUILD_ID", "OSGPU_HD"):
            assert k in hdr, f"{k} missing from the header's knob table"
