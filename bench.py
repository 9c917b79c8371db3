#!/usr/bin/env python3
"""bench.py -- device-resident shmem_double_sum_to_all combine on MI355X.

Metric (BASELINE.json): GiB/s of the device-resident shmem_double_sum_to_all
combine + fraction of the HBM roofline, at 1/2/4/8 GPUs.

N = 1 (default) -- BASELINE config 2: nreduce = 64 Mi doubles, 1 MI355X,
  "device-resident combine kernel only".  One step = one launch of the
  combine kernel that shmem_double_sum_to_all runs on the P2P path for a
  2-PE active set (K = 2 inputs: the PE's own source and its peer's, both in
  HBM) through the C ABI (osgpu_combine).  Algorithmic bytes per step
  B = (K + 1) * nreduce * 8 (2 reads + 1 write), value = steps * B / t.
  Extra fields: roofline (HIP events on the launch stream + PMC traffic from
  profiles/), the full C-API call (2 PEs, timed in C), the host-staged
  (PCIe-inclusive) rate, the data-movement collectives (copy kernel roofline,
  fcollect64 through the C ABI), BASELINE config 1's small call (1 Ki ints,
  2 PE processes: fused one-launch path vs host barriers vs the reference's
  loop on 2 cores), the reference's CPU loop shape on this host.

N > 1 (torchrun, one process per GPU) -- one PE per GPU, every PE calls
  shmem_double_sum_to_all(nreduce = 64 Mi per PE) over all N PEs (weak
  scaling: per-GPU data fixed).  Primary path: the exact owner-computes team
  kernel over the members' device heaps (osgpu_heap_create: one contiguous
  virtual range per PE, mapped into every member; xGMI); PE services from an
  intra-node shared-memory runtime (tests/support/pe_shm.c); a sampled
  bit-exact parity check against the oracle is reported.  value = steps *
  (N + 1) * nreduce * 8 / t (SURVEY.md 8d aggregate: sum over GPUs of the
  shard-fold bytes), t = the max over ranks.  Then, in the same run: RCCL
  allreduce on the same buffers (forced: FP sum within tolerance), BASELINE
  config 4 (nreduce = 1 Gi: the exact team kernel over the heaps, and RCCL
  beside it) and config 5 (float min/max/prod,
  128 Mi per PE, host-resident, H2D/D2H included), fcollect64 over the
  device heaps (xGMI), RCCL and host staging, and config 1's small call
  (1 Ki ints) with host barriers vs the fused one-launch path.  A watchdog prints the line
  with what has been measured if the run exceeds --deadline seconds.
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
# team.hip OSGPU_TEAM_LDS_U: vectors per lane per tile of the LDS-staged team
# kernel (its template argument, the rocprof name's last field), and the
# member counts that kernel serves (OSGPU_TEAM_LDS_MIN_P, OSGPU_TEAM_LDS_MAX_P)
TEAM_LDS_U = 1
TEAM_LDS_P = (2, 4)
# ... and the LDS form also at 5, 6 and 8 members for real types other than
# FP max/min (double sum among them), when no member is remote (TeamShape kLds)
TEAM_LDS_EXTRA_P = (5, 6, 8)


def team_lds(P, remote=False):
    """True where team.hip launches the LDS-staged kernel for double sum."""
    if remote:
        return 3 <= P <= 4
    return TEAM_LDS_P[0] <= P <= TEAM_LDS_P[1] or P in TEAM_LDS_EXTRA_P

# the headline kernel: combine.hip's LDS-staged form at K = 2 inputs
# (OSGPU_COMBINE_LDS_U2 = 2 vectors per lane), its rocprof / PMC key and label
COMBINE_KERNEL = "combine_lds_kernel<double, 0, 2, 2>"
COMBINE_LABEL = "osgpu::combine_lds_kernel<double, SUM, 2, 2>"
for sub in ("test-resilient-osss-ucx_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, sub))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec, MI355X_MICROARCH.md
XGMI_LINK_GBS = 76.8           # MI355X xGMI: 153.6 GB/s bidirectional per peer link
GIB = float(1 << 30)
HOST_FOLD_MAX_BYTES = 256 << 10  # runtime.cpp host_fold_max_bytes(): (P-1)*nreduce*size
METRIC = "GiB/s device-resident shmem_double_sum_to_all combine + %HBM peak, 1/2/4/8 GPU"


# --------------------------------------------------------------------------
# the printed line: at most LINE_CAP bytes (the driver reads one JSON line of
# bounded size; round 5's 21.7 KB line went unparsed).  The full result --
# placements with addresses, sweeps, per-rank reports, notes -- goes to the
# detail file named in the line; the line keeps every contract field plus a
# summary (min / median / max, no address lists) of each side measurement.
# --------------------------------------------------------------------------

LINE_CAP = 7168  # under the driver's 8 KiB stdout tail with room to spare
# keys whose values stay in the detail file only (anywhere in the tree)
DETAIL_ONLY = frozenset((
    "addresses", "placements", "sweep", "heap_preflight", "ranks", "note", "how", "what",
    "kernel_avg_how", "placements_note", "crossover_note", "hip_runtime", "offset_in_2MiB",
    "peak_measured_how", "bytes_convention", "rule", "copy_ceiling_same_mix",
    "after_timed_region_100_launches", "copy_ceiling_same_bytes", "traffic_source",
    "dma_state", "dma_state_after", "element_ops", "path_mode", "launch_note"))
# strings that keep their full text (up to 480 characters)
LONG_OK = frozenset(("metric", "workload", "sample", "incomplete", "detail"))
# top-level keys dropped, in this order, while the line is still over the cap
DROP_ORDER = ("host_staged_in_torch_process", "cpu_baseline_configs", "traffic_live",
              "api", "collectives", "longdouble_team_8_members", "config3_long_bitwise_256MiB",
              "north_star_double_sum_128Mi", "config5_host_staged", "host_staged",
              "roofline_call", "small_call", "team_by_members", "local_fold_no_exchange",
              "team_shapes_ab", "team_push", "xgmi_probe", "small_calls", "config5",
              "rccl_integer_auto", "launch", "config4", "rccl", "hbm_aggregate")


def _shrink(x, key=None):
    """The line's form of one value: DETAIL_ONLY keys removed, floats to 5
    significant digits, long strings cut, lists of more than 16 items cut."""
    if isinstance(x, dict):
        return {k: _shrink(v, k) for k, v in x.items() if k not in DETAIL_ONLY}
    if isinstance(x, (list, tuple)):
        return [_shrink(v) for v in x[:16]]
    if isinstance(x, float):
        return float(f"{x:.5g}") if x == x and abs(x) != float("inf") else None
    if isinstance(x, str):
        lim = 480 if key in LONG_OK else 160
        return x if len(x) <= lim else x[:lim - 3] + "..."
    return x


def _sum_cpu_configs(v):
    out = {k: v[k] for k in ("kind", "cpus_allowed") if k in v}
    for name in ("config3", "config4", "config5"):
        c = v.get(name)
        if isinstance(c, dict):
            out[name] = {op: c[op]["GiBs_per_PE"] for op in c
                         if isinstance(c[op], dict) and "GiBs_per_PE" in c[op]}
            out[name]["pes"] = c.get("pes")
            if "error" in c:
                out[name]["error"] = c["error"]
    return out


def _sum_torch_staged(v):
    return {k: v[k].get("pcie_GBs_each_way") if isinstance(v.get(k), dict) else v.get(k)
            for k in ("pinned", "pageable", "error") if k in v}


def _sum_team(v):
    out = {}
    for P, rec in v.items():
        if not isinstance(rec, dict) or "trials" not in rec:
            out[P] = rec
            continue
        r = {k: rec[k] for k in ("kernel", "achieved", "frac", "kernel_avg_us", "traffic",
                                 "copy_frac", "frac_of_copy_ceiling", "frac_min", "frac_median",
                                 "frac_max", "frac_of_copy_ceiling_min",
                                 "frac_of_copy_ceiling_median", "frac_of_copy_ceiling_max",
                                 "canary_min", "canary_median", "bit_exact_sample") if k in rec}
        r["trials"] = [{"frac": t["frac"], "copy_frac": t["copy_frac"], "canary": t["canary"],
                        "label": t.get("label")} for t in rec["trials"]]
        oa = rec.get("one_allocation_heaps_layout") or {}
        r["one_allocation_heaps_of_copy"] = oa.get("frac_of_copy_ceiling")
        out[P] = r
    return out


def _sum_small(v):
    keys = ("fused_team", "team", "host_fused_staged", "host_staged", "host_fold")
    out = {k + "_us": v.get(k + "_us_timed_in_c", v.get(k + "_us")) for k in keys}
    out["timed"] = "in C between the runtime's barriers, median"
    out["all_correct"] = all(v.get(k + "_correct", False) for k in keys)
    for k in ("cpu_reference_loop_us", "default_path_us", "default_path", "crossover_elements",
              "slower_than_reference_loop", "ratio_to_reference_loop", "error"):
        if k in v:
            out[k] = v[k]
    return out


def _pick(d, keys):
    return {k: d[k] for k in keys if isinstance(d, dict) and k in d}


def _sum_ld(v):
    out = _pick(v, ("kernel", "members", "error"))
    out["bound"] = "valu"
    for k in ("random_signs", "one_sign"):
        if isinstance(v.get(k), dict):
            out[k] = _pick(v[k], ("frac", "kernel_avg_us", "member0_equals_member1"))
    return out


def _sum_c3(v):
    out = _pick(v, ("nreduce", "error"))
    for k in ("and", "or", "xor"):
        if isinstance(v.get(k), dict):
            out[k] = _pick(v[k], ("frac_of_8TBs", "kernel_us", "bit_exact"))
    return out


def _sum_c5h(v):
    out = _pick(v, ("pes", "nreduce", "error"))
    for k in ("min", "max", "prod"):
        if isinstance(v.get(k), dict):
            out[k] = _pick(v[k], ("pcie_GBs_each_way", "correct_sample"))
    return out


def _sum_coll(v):
    return {"copy_kernel_frac_of_8TBps": (v.get("copy_kernel") or {}).get("frac_of_8TBps"),
            "fcollect64_device_GBps_all_pes": (v.get("fcollect64_device") or {}).get("GBps_all_pes"),
            "fcollect64_host_staged_h2d_GBs": (v.get("fcollect64_host_staged") or {}).get("pcie_h2d_GBs"),
            **_pick(v, ("error",))}


# top-level side measurements given a purpose-made summary in the line
SUMMARIZERS = {"longdouble_team_8_members": _sum_ld, "config3_long_bitwise_256MiB": _sum_c3,
               "config5_host_staged": _sum_c5h, "collectives": _sum_coll,
               "cpu_baseline_configs": _sum_cpu_configs,
               "host_staged_in_torch_process": _sum_torch_staged,
               "team_by_members": _sum_team, "small_call": _sum_small}


def fit_line(res, detail_path=None, cap=LINE_CAP):
    """The JSON line for `res` (<= cap bytes) and, when detail_path is given,
    the full `res` written there first (named in the line as `detail`)."""
    if detail_path:
        try:
            os.makedirs(os.path.dirname(detail_path) or ".", exist_ok=True)
            with open(detail_path, "w") as f:
                json.dump(res, f, indent=1, default=str)
            res = dict(res, detail=os.path.relpath(detail_path, ROOT))
        except OSError as e:  # the line still prints
            res = dict(res, detail=f"not written: {e}"[:200])
    line = {}
    for k, v in res.items():
        if k in DETAIL_ONLY:
            continue
        try:
            line[k] = _shrink(SUMMARIZERS[k](v) if k in SUMMARIZERS and isinstance(v, dict) else v, k)
        except Exception as e:  # a summary must never cost the line
            line[k] = {"summary_error": repr(e)[:120]}
    dropped = []
    text = json.dumps(line, separators=(",", ":"))
    for k in DROP_ORDER:
        if len(text) <= cap:
            break
        if k in line:
            del line[k]
            dropped.append(k)
            line["dropped_to_fit"] = dropped
            text = json.dumps(line, separators=(",", ":"))
    if len(text) > cap:   # last resort: the contract fields alone
        keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                "roofline", "cpu_baseline", "detail", "incomplete")
        line = {k: line[k] for k in keep if k in line}
        line["dropped_to_fit"] = "all side measurements (see detail)"
        text = json.dumps(line, separators=(",", ":"))
    return text


def default_detail(n_gpus):
    return os.path.join(ROOT, "gpurun_out", f"bench_detail_n{n_gpus}.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--nreduce", type=int, default=64 << 20)
    ap.add_argument("--no-rccl", action="store_true", help="N>1: skip the RCCL runs")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the side measurements (N=1: north star / config 3 "
                         "kernel rates; N>1: config 4, config 5, collectives, probes)")
    ap.add_argument("--c4-nreduce", type=int, default=1 << 30)
    ap.add_argument("--c5-nreduce", type=int, default=128 << 20)
    ap.add_argument("--deadline", type=float, default=420.0,
                    help="N>1: print what was measured and exit after this many seconds")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-live-pmc", action="store_true",
                    help="N=1: take roofline.traffic from profiles/ instead of this run's "
                         "rocprofv3 --pmc passes")
    ap.add_argument("--no-api", action="store_true")
    ap.add_argument("--cpu-n", type=int, default=64 << 20,
                    help="nreduce of the CPU-baseline sample")
    ap.add_argument("--detail", default=None,
                    help="where the full result goes (default gpurun_out/bench_detail_n<N>.json); "
                         "the printed line is its <= 8 KiB summary")
    ap.add_argument("--dry-ranks", action="store_true",
                    help="N>1 launcher check without the GPU (tests/test_bench_contract.py)")
    ap.add_argument("--dry-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    return ap.parse_args()


# --------------------------------------------------------------------------
# N = 1
# --------------------------------------------------------------------------

LIVE_TRAFFIC = {}  # filled by live_traffic() before the line's rooflines are built


def load_traffic(kernel=COMBINE_KERNEL, n=None):
    """HBM bytes per launch of `kernel` measured with rocprofv3 PMC counters:
    this run's own passes (LIVE_TRAFFIC) when they produced the kernel, else
    the newest profiles/*traffic*.json (tools/pmc_traffic.py) covering that
    kernel at that nreduce, labelled as looked up; None if neither."""
    live = LIVE_TRAFFIC.get(kernel)
    if live is not None and (n is None or live.get("nreduce") == n):
        return live
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic*.json"))):
        try:
            with open(p) as f:
                d = json.load(f)
        except Exception:
            continue
        if d.get("kernel") == kernel and (n is None or d.get("nreduce") == n):
            best = dict(d, source="looked up: profiles/" + os.path.basename(p))
    return best


def live_traffic(n, members=(2, 4, 8), reps=5, timeout=120):
    """HBM bytes per launch measured in THIS run: two child processes,
    `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (separate passes),
    over tools/pmc_probe.py -- the combine kernel and the team kernel for
    each member count, on this line's shapes, through the C ABI.  Returns
    {kernel key: tools/pmc_traffic.traffic() dict} plus "_error" on failure;
    each pass runs in its own process group, killed at `timeout`."""
    import shutil
    import signal
    import subprocess
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import pmc_traffic
    prof = shutil.which("rocprofv3")
    if not prof:
        return {"_error": "rocprofv3 not on PATH"}
    keys = {COMBINE_KERNEL: 24}
    for P in members:
        keys[(f"team_lds_kernel<double, 0, {P}, true, {TEAM_LDS_U}" if team_lds(P)
              else f"team_vec_kernel<double, 0, {P}, true>")] = 16 * P
    tmp = tempfile.mkdtemp(prefix="osgpu_pmc_")
    dirs = {}
    t0 = time.time()
    try:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, counter)
            cmd = [prof, "--pmc", counter, "-d", d, "-o", "run", "--output-format", "csv",
                   "--", sys.executable, os.path.join(ROOT, "tools", "pmc_probe.py"),
                   str(n), str(reps)] + [str(P) for P in members]
            p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                 start_new_session=True, cwd=ROOT)
            try:
                out, _ = p.communicate(timeout=timeout)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.communicate()
                return {"_error": f"{counter} pass killed after {timeout} s"}
            if p.returncode != 0:
                tail = out.decode(errors="replace").strip().splitlines()[-3:]
                return {"_error": f"{counter} pass exit {p.returncode}: {' | '.join(tail)}"}
            dirs[counter] = d
        res = {}
        for k, per_elem in keys.items():
            r = pmc_traffic.traffic(dirs["FETCH_SIZE"], dirs["WRITE_SIZE"], n, k, per_elem)
            if r is not None:
                r["source"] = "live: this run's rocprofv3 passes over tools/pmc_probe.py"
                res[k] = r
        res["_seconds"] = time.time() - t0
        return res
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def cpu_baseline(n):
    """The reference's loop shape (oracle_reduce.c: copy, barrier, 64-element
    getmem chunks, per-element function-pointer op, barrier) with 2 pthreads
    as PEs on this host's cores; the pointer is the reference's own compiled
    shmemu_sum_double_func (src/shmemu/miscops.c, oracle/_ref) when that
    library is in the tree, else the restated op."""
    import oracle as O
    src = O.team_inputs("double", 2, n, 0x5EED, "unit12")
    ref = O.ref_elem_fn("double", "sum") is not None
    # size the repetition count for ~10 s of CPU work (bounded sample)
    probe = O.cpu_baseline("double", "sum", src, reps=1, pin=True, ref_ops=ref)
    reps = max(3, min(200, int(10.0 / max(probe, 1e-3))))
    t0 = time.time()
    sec = O.cpu_baseline("double", "sum", src, reps=reps, pin=True, ref_ops=ref)
    wall = time.time() - t0
    B = 2 * 3 * n * 8  # two PE results, each (K+1)*n*8
    ops = ("the reference's own shmemu_sum_double_func (miscops.c compiled unmodified into "
           "oracle/_ref) through a pointer as src/reductions.c:95-96" if ref
           else "the restated element op (oracle/_ref absent)")
    out = {"value": B / sec / GIB, "unit": "GiB/s", "cores": 2, "kind": "port",
           "element_ops": "reference" if ref else "restatement",
           "sample": (f"src/reductions.c:79-113 loop restated (oracle/oracle_reduce.c: copy, "
                      f"barrier, 64-element getmem chunks, barrier) calling {ops}; double sum, "
                      f"2 PEs = 2 pinned pthreads, nreduce={n}, median of {reps} after 1 warm-up "
                      f"({sec*1e3:.1f} ms/call, {wall:.1f} s); bytes = 2 x 3*n*8; host "
                      f"nproc={os.cpu_count()}, usable CPUs {len(os.sched_getaffinity(0))}")}
    # the same loop with every PE's elements split over 8 threads: 16 cores,
    # this box's CPU share (a one-PE-per-core reference uses 2 for 2 PEs)
    tpp = 8
    probe = O.cpu_baseline("double", "sum", src, reps=1, pin=True, threads_per_pe=tpp,
                           ref_ops=ref)
    reps16 = max(3, min(200, int(5.0 / max(probe, 1e-3))))
    sec16 = O.cpu_baseline("double", "sum", src, reps=reps16, pin=True, threads_per_pe=tpp,
                           ref_ops=ref)
    out["same_loop_16_cores"] = {
        "value": B / sec16 / GIB, "unit": "GiB/s", "cores": 2 * tpp, "ms_per_call": sec16 * 1e3,
        "sample": f"the same loop shape, each PE's elements split over {tpp} pinned threads "
                  f"(the first {2 * tpp} CPUs this process may use), median of {reps16} after 1 warm-up"}
    return out


def cpu_baselines_configs():
    """BASELINE.md's CPU-baseline plan beyond config 2: the reference's loop
    shape (oracle_reduce.c: copy, barrier, 64-element getmem chunks, one
    indirect call per element, barrier; src/reductions.c:79-113), one pinned
    pthread per PE, on bounded samples of
      config 3  long and/or/xor, 2 PEs, nreduce = 32 Mi (256 MiB per array):
                the full size;
      config 5  float min/max/prod, 8 PEs on 8 cores, a 32 Mi-element sample
                of the 128 Mi per PE (the loop is linear in nreduce);
      config 4  double sum, 8 PEs on 8 cores, a 64 Mi-element sample of the
                1 Gi per PE (16x smaller: at full size 128 GiB of host arrays
                and ~16x this time per call).
    Rates: per-PE algbw nreduce*s/t and the fused-convention P*(P+1)*n*s/t
    (every PE's K = P inputs + 1 output)."""
    import oracle as O
    out = {"host_nproc": os.cpu_count(), "cpus_allowed": len(os.sched_getaffinity(0)),
           "kind": "port",
           "element_ops": "reference" if O.ref_lib() is not None else "restatement",
           "note": "oracle/oracle_reduce.c reference loop shape with the reference's compiled "
                   "element functions (oracle/_ref) when present, pthreads pinned to the first P "
                   "CPUs of this process's CPU set, median after 1 warm-up"}
    plans = (("config3", "long", ("and", "or", "xor"), 2, 32 << 20, "bits", 3),
             ("config5", "float", ("min", "max", "prod"), 8, 32 << 20, "unit12", 1),
             ("config4", "double", ("sum",), 8, 64 << 20, "unit12", 1))
    for name, t, ops, P, n, dist, reps in plans:
        try:
            src = O.team_inputs(t, P, n, 0xC0 + P, dist)
            es = src[0].dtype.itemsize
            res = {"pes": P, "cores": P, "nreduce_sample": n}
            for op in ops:
                sec = O.cpu_baseline(t, op, src, reps=reps, pin=True,
                                     ref_ops=O.ref_elem_fn(t, op) is not None)
                res[op] = {"ms_per_call": sec * 1e3, "GiBs_per_PE": n * es / sec / GIB,
                           "GiBs_fused_convention": P * (P + 1) * n * es / sec / GIB}
            out[name] = res
            del src
        except Exception as e:  # report, never hide
            out[name] = {"error": repr(e)[:200]}
    out["config5"]["full_nreduce"] = 128 << 20
    out["config4"]["full_nreduce"] = 1 << 30
    return out


def _timer_sig(pet):
    pet.pet_time_to_all.restype = ctypes.c_double
    pet.pet_time_to_all.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                    ctypes.c_int]


def hip_runtime_path():
    """The libamdhip64 this process has mapped: torch's bundled copy (ROCm
    7.0 in this image) once torch is imported, /opt/rocm's (7.2) in a
    process that never imports it."""
    try:
        for line in open("/proc/self/maps"):
            if "libamdhip64" in line:
                return line.split()[-1]
    except OSError:
        pass
    return None


def dma_d2h_state(nbytes=64 << 20, reps=3):
    """The DMA engine's device-to-host rate right now (best of `reps`
    64-MiB copies into pinned memory): 56-57 GB/s when the GPU's power state
    is up, 28-30 in the low state an idle box starts in (tools/
    d2h_timeline.hip).  Through the HIP runtime already in the process
    (ctypes), so it works with or without torch."""
    hip = ctypes.CDLL("libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)
    vp = ctypes.c_void_p
    d, h = vp(), vp()
    assert hip.hipMalloc(ctypes.byref(d), ctypes.c_size_t(nbytes)) == 0
    assert hip.hipHostMalloc(ctypes.byref(h), ctypes.c_size_t(nbytes), 0) == 0
    assert hip.hipMemset(d, 1, ctypes.c_size_t(nbytes)) == 0
    assert hip.hipDeviceSynchronize() == 0
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        assert hip.hipMemcpy(h, d, ctypes.c_size_t(nbytes), 2) == 0  # D2H
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    hip.hipFree(d)
    hip.hipHostFree(h)
    return {"dma_d2h_GBs": nbytes / best / 1e9, "low_state": nbytes / best / 1e9 < 40}


def host_staged_config5(n=128 << 20, P=8, reps=3, warm_s=1.5):
    """BASELINE config 5 with its H2D/D2H copies: shmem_float_{min,max,prod}
    _to_all over 8 PEs (pthreads) on one GPU, 128 Mi floats per PE in a HOST
    symmetric heap pinned with osgpu_host_register -- the STAGED path (H2D of
    each PE's source, the team exchange on the GPU, D2H of its target).  All
    8 PEs share this GPU's PCIe link: 8 * n * 4 bytes each way per call.
    Timed in C after a warm-up; every member's target sampled against its
    own fold order (numpy, src/reductions.c:79-111)."""
    import numpy as np
    import osgpu
    from support import team as T
    L = osgpu.load()
    L.osgpu_finalize()
    nb = n * 4
    tm = T.Team(P, 2 * nb + 8192, device=False)
    toff = T._align(nb)
    rng = np.random.default_rng(5)
    out = {"pes": P, "nreduce": n, "bytes_per_pe": nb, "heap": "pinned host (osgpu_host_register)",
           "pcie_bytes_each_way_per_call": P * nb, "hip_runtime": hip_runtime_path()}
    assert L.osgpu_host_register(ctypes.c_void_p(tm.base), P * tm.H) == 0
    try:
        for op, lo, hi in (("min", -1e3, 1e3), ("max", -1e3, 1e3), ("prod", 0.9, 1.1)):
            for pe in range(P):  # a 1 Mi random block per PE, tiled
                blk = rng.uniform(lo, hi, 1 << 20).astype(np.float32)
                a = tm.hoff + pe * tm.H
                tm.hbuf[a:a + nb].view(np.float32).reshape(-1, 1 << 20)[:] = blk
            fn = ctypes.cast(getattr(L, f"shmem_float_{op}_to_all"), ctypes.c_void_p)
            tgt = (ctypes.c_void_p * P)(*[tm.ptr(pe, toff) for pe in range(P)])
            src = (ctypes.c_void_p * P)(*[tm.ptr(pe, 0) for pe in range(P)])
            ps = (ctypes.c_void_p * P)(*[tm.ptr(pe, tm.psync_off) for pe in range(P)])
            _timer_sig(tm.pet)
            t_w = time.perf_counter()
            while time.perf_counter() - t_w < warm_s:
                tm.pet.pet_time_to_all(fn, P, tgt, src, ps, n, 1)
            sec = tm.pet.pet_time_to_all(fn, P, tgt, src, ps, n, reps)
            idx = rng.integers(0, n, 1 << 16)
            xs = [tm.hbuf[tm.hoff + pe * tm.H:][:nb].view(np.float32)[idx] for pe in range(P)]
            f = {"min": lambda a, b: np.where(a < b, a, b),
                 "max": lambda a, b: np.where(a > b, a, b),
                 "prod": lambda a, b: (a * b).astype(np.float32)}[op]
            ok = True
            for q in range(P):
                acc = xs[q].copy()
                for j in range(P):
                    if j != q:
                        acc = f(acc, xs[j])
                got = tm.hbuf[tm.hoff + q * tm.H + toff:][:nb].view(np.float32)[idx]
                ok = ok and bool(np.array_equal(got.view(np.int32), acc.view(np.int32)))
            out[op] = {"ms_per_call": sec * 1e3, "pcie_GBs_each_way": P * nb / sec / 1e9,
                       "correct_sample": ok}
    finally:
        L.osgpu_host_unregister(ctypes.c_void_p(tm.base))
        L.osgpu_finalize()
        del tm
    out["dma_state_after"] = dma_d2h_state()
    return out


def host_staged_child(n, timeout=240, what="host_staged_time(%d)"):
    """host_staged_time in a child process that never imports torch, so the
    library runs on /opt/rocm's HIP runtime as in a C application.  Inside a
    torch process it runs on torch's bundled ROCm 7.0 runtime, whose D2H
    copies pick an engine mask of both SDMA engines when both are idle; the
    copy is refused and redone as a blit kernel ("HSA copy failed with code
    4097, falling to Blit copy", profiles/r05_torch_runtime_d2h.txt), which
    caps the duplex pair at 41.9 GB/s each way; the staged pipeline in the
    torch process measured 44.4 pinned / 39.6 pageable in round 5 (DESIGN
    history 15.1), beside 44.5 / 41.3 here.  The 7.2 runtime picks one
    engine per direction (48.3 each way)."""
    import subprocess
    code = ("import sys, json; sys.path.insert(0, %r); import bench; "
            "print('RESULT ' + json.dumps(bench." + what + "))") % (ROOT, n)
    env = dict(os.environ, OSGPU_NO_TORCH="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT)
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
    if not line:
        return {"error": (r.stdout + r.stderr)[-600:]}
    return json.loads(line[0][7:])


def host_staged_time(n, reps=7, pes=2, warm_s=1.5):
    """The reference's data placement: sources and targets in HOST symmetric
    heaps.  shmem_double_sum_to_all over a 2-PE set on one GPU (pthreads as
    PEs), STAGED path: H2D own source -> team exchange on the GPU -> D2H,
    pipelined in 32 MiB chunks.  Timed in C, pinned heap (osgpu_host_register)
    and pageable heap.  Both PEs share this GPU's one PCIe link, so per call
    2*n*8 bytes go H2D and 2*n*8 D2H."""
    import numpy as np
    import osgpu
    from support import team as T
    L = osgpu.load()
    L.osgpu_finalize()
    P = pes
    out = {"note": f"{P} PEs (pthreads) on one GPU, host heaps, nreduce={n} doubles per PE; "
                   f"PCIe bytes per call = {P}*{n}*8 H2D + {P}*{n}*8 D2H",
           "stage_copy": os.environ.get("OSGPU_STAGE_COPY", "dma"),
           "copy_streams": os.environ.get("OSGPU_COPY_STREAMS", "prio"),
           "dma_state": dma_d2h_state(), "hip_runtime": hip_runtime_path()}
    for pinned in (True, False):
        tm = T.Team(P, 2 * n * 8 + 8192, device=False)
        toff = (n * 8 + 4095) // 4096 * 4096
        for pe in range(P):
            lo = tm.hoff + pe * tm.H
            tm.hbuf[lo:lo + n * 8].view(np.float64)[:] = 1.5 + pe
        if pinned:
            assert L.osgpu_host_register(ctypes.c_void_p(tm.base), P * tm.H) == 0
        fn = ctypes.cast(L.shmem_double_sum_to_all, ctypes.c_void_p)
        tgt = (ctypes.c_void_p * P)(*[tm.ptr(pe, toff) for pe in range(P)])
        src = (ctypes.c_void_p * P)(*[tm.ptr(pe, 0) for pe in range(P)])
        ps = (ctypes.c_void_p * P)(*[tm.ptr(pe, tm.psync_off) for pe in range(P)])
        _timer_sig(tm.pet)
        # warm-up: staged calls for warm_s seconds before the timed ones (the
        # DMA engines' device-to-host rate follows the GPU's power state,
        # dma_d2h_state; the first calls of a process also map the staging)
        t_w = time.perf_counter()
        while time.perf_counter() - t_w < warm_s:
            tm.pet.pet_time_to_all(fn, P, tgt, src, ps, n, 1)
        sec = tm.pet.pet_time_to_all(fn, P, tgt, src, ps, n, reps)
        want = sum(1.5 + pe for pe in range(P))
        ok = bool((tm.hbuf[tm.hoff + toff: tm.hoff + toff + n * 8].view(np.float64) == want).all())
        out["pinned" if pinned else "pageable"] = {
            "ms_per_call": sec * 1e3,
            "pcie_GBs_each_way": P * n * 8 / sec / 1e9,
            "algbw_GiBs_per_PE": n * 8 / sec / GIB,
            "correct": ok}
        if pinned:
            L.osgpu_host_unregister(ctypes.c_void_p(tm.base))
        L.osgpu_finalize()
        del tm
    out["dma_state_after"] = dma_d2h_state()
    return out


def collectives_single(P=4, nb=64 << 20, reps=10):
    """SURVEY.md 8f row 4 on one GPU (tools/coll_bench.py has the full
    sweep): the copy kernel alone (P ranges of nb bytes, HIP events; traffic
    2*P*nb per launch) and shmem_fcollect64 through the C ABI by P
    threads-as-PEs on this GPU (all-PE traffic 2*P*P*nb per call)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import coll_bench as CB
    t, bw = CB.kernel_rate(P, nb, reps)
    out = {"copy_kernel": {"ranges": P, "bytes_per_range": nb, "us": t * 1e6,
                           "GBps": bw / 1e9, "frac_of_8TBps": bw / 8e12}}
    t = CB.api_time("fcollect", P, nb, reps, True)
    out["fcollect64_device"] = {"pes": P, "bytes_per_pe": nb, "ms_per_call": t * 1e3,
                                "GBps_all_pes": CB.moved("fcollect", P, nb) / t / 1e9}
    # host symmetric heaps (pageable): the STAGED path, H2D / exchange / D2H
    # one after the other per chunk (a two-slot pipeline was measured and
    # reverted: profiles/r05_coll_staged_pipeline_ab.jsonl); the P PEs share
    # this GPU's PCIe link
    nh = nb // 4
    t = CB.api_time("fcollect", P, nh, 5, False)
    out["fcollect64_host_staged"] = {
        "pes": P, "bytes_per_pe": nh, "ms_per_call": t * 1e3,
        "pcie_h2d_GBs": P * nh / t / 1e9, "pcie_d2h_GBs": P * P * nh / t / 1e9}
    return out


def api_call_time(n, reps=20):
    """Full shmem_double_sum_to_all through the C ABI, timed in C
    (tests/support/pe_threads.c:pet_time_to_all): a 2-PE active set, one
    pthread per PE, both PEs' symmetric heaps in this GPU's HBM.  Includes
    the entry device sync, the two barriers and the stream syncs.  Team path
    (owner-computes, both PEs' kernels: 2*2*n*8 HBM bytes per collective)
    and pull path (each PE folds both sources: 2*3*n*8)."""
    import torch
    import osgpu
    from support import team as T
    tm = T.Team(2, 2 * n * 8 + 8192, device=True)
    toff = (n * 8 + 4095) // 4096 * 4096
    for pe in range(2):
        tm.buf[pe * tm.H: pe * tm.H + n * 8].view(torch.float64).uniform_(1, 2)
    torch.cuda.synchronize()
    fn = ctypes.cast(tm.lib.shmem_double_sum_to_all, ctypes.c_void_p)
    tgt = (ctypes.c_void_p * 2)(tm.ptr(0, toff), tm.ptr(1, toff))
    src = (ctypes.c_void_p * 2)(tm.ptr(0, 0), tm.ptr(1, 0))
    _timer_sig(tm.pet)
    out = {"note": "2 PEs (pthreads) on one GPU; one collective call, start barrier "
                   "to PE 0's return, median of %d" % reps}
    for name, path, hbm in (("team", osgpu.PATH_AUTO, 4), ("pull", osgpu.PATH_PULL, 6)):
        tm.lib.osgpu_set_path(path)
        sec = tm.pet.pet_time_to_all(fn, 2, tgt, src, None, n, reps)
        out[name] = {"ms_per_call": sec * 1e3, "hbm_bytes_per_call": hbm * n * 8,
                     "hbm_GBs": hbm * n * 8 / sec / 1e9}
    tm.lib.osgpu_set_path(osgpu.PATH_AUTO)
    return out


def span_per_launch(torch, st, launch, reps):
    """reps launches back to back on stream st, one HIP event pair around
    them all: the average launch duration, kernel boundaries included (an
    event pair around every launch would add its own gap to each)."""
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(st)
    for _ in range(reps):
        launch()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e-3 / reps


def kernel_rate(L, torch, type_code, op_code, n, esz, dtype, fill, reps=20):
    """Average launch time of osgpu_combine(K = 2) on its own stream over n
    elements of two resident inputs (HIP event span over reps launches back
    to back / reps); (K + 1) * n * esz bytes per launch."""
    dev = torch.device("cuda:0")
    a = torch.empty(n, dtype=dtype, device=dev)
    b = torch.empty(n, dtype=dtype, device=dev)
    fill(a, 1)
    fill(b, 2)
    out = torch.empty(n, dtype=dtype, device=dev)
    st = torch.cuda.Stream(device=dev)
    srcs = (ctypes.c_void_p * 2)(a.data_ptr(), b.data_ptr())
    sp = ctypes.c_void_p(st.cuda_stream)
    torch.cuda.synchronize()

    def launch():
        assert L.osgpu_combine(type_code, op_code, out.data_ptr(), srcs, 2, n, sp) == 0
    for _ in range(3):
        launch()
    return span_per_launch(torch, st, launch, reps), a, b, out


def team_arrays(torch, n, P, layout="alloc", seed=0):
    """P sources (uniform [1,2) doubles) and P targets of n doubles for the
    team kernel.  layout "alloc": every array its own allocation; "symheap":
    P symmetric heaps carved back to back out of ONE allocation (as PE
    threads' heaps in one buffer), member p's source at offset 0 of heap p
    and its target at n*8 + 2 MiB: every array shares its low 21 address bits
    and the regular high bits of one allocation -- the worst layout the sweep
    found (tools/team_layout_sweep.py symheap, profiles/r05_team_symheap.jsonl);
    heaps from osgpu_heap_create (one allocation each) do not show it
    (profiles/r05_heap_stagger_ab.jsonl)."""
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(11 + P + 100 * seed)
    if layout == "symheap":
        heap = (2 * n * 8 + (4 << 20) + (2 << 20) - 1) // (2 << 20) * (2 << 20)
        buf = torch.empty(P * heap + (2 << 20), dtype=torch.uint8, device=dev)
        b0 = (-buf.data_ptr()) % (2 << 20)
        srcs_t = [buf[b0 + p * heap: b0 + p * heap + n * 8].view(torch.float64) for p in range(P)]
        dsts_t = [buf[b0 + p * heap + n * 8 + (2 << 20): b0 + p * heap + 2 * n * 8 + (2 << 20)]
                  .view(torch.float64) for p in range(P)]
        for x in srcs_t:
            x.uniform_(1.0, 2.0, generator=g)
    else:
        srcs_t = [torch.empty(n, dtype=torch.float64, device=dev).uniform_(1.0, 2.0, generator=g)
                  for _ in range(P)]
        dsts_t = [torch.empty(n, dtype=torch.float64, device=dev) for _ in range(P)]
    return srcs_t, dsts_t


class Canary:
    """A fixed-buffer control: the copy kernel over two arrays allocated once,
    before the first placement trial, and never freed until the end.  Timed
    right before and right after every trial: a slow trial whose canary is
    slow too was the box slowing down in time (a transient); a slow trial
    with a normal canary was its own placement."""

    def __init__(self, L, torch, nbytes=512 << 20, reps=10):
        dev = torch.device("cuda:0")
        self.torch, self.L, self.reps, self.nbytes = torch, L, reps, nbytes
        self.a = torch.empty(nbytes, dtype=torch.uint8, device=dev).fill_(3)
        self.o = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        self.st = torch.cuda.Stream(device=dev)
        self.sp = ctypes.c_void_p(self.st.cuda_stream)
        self.D = (ctypes.c_void_p * 1)(self.o.data_ptr())
        self.S = (ctypes.c_void_p * 1)(self.a.data_ptr())
        self.N = (ctypes.c_size_t * 1)(nbytes)
        self.samples = []
        self()

    def __call__(self):
        def launch():
            assert self.L.osgpu_copy(self.D, self.S, self.N, 1, self.sp) == 0
        launch()
        t = span_per_launch(self.torch, self.st, launch, self.reps)
        f = 2 * self.nbytes / t / 1e9 / HBM_PEAK_GBS
        self.samples.append(f)
        return f

    def reference(self):
        v = sorted(self.samples)
        return v[len(v) // 2]


def team_kernel_rate(L, torch, n, reps, P=2, arrays=None, layout="alloc", canary=None):
    """The kernel shmem_double_sum_to_all actually dispatches on one GPU with
    registered heaps (TEAM path, csrc/team.hip): team_vec_kernel<double,SUM,P>,
    team_lds_kernel<double,SUM,P> at 2 to 4 members (TEAM_LDS_P)
    through the C ABI (osgpu_team_combine), one launch over all n elements --
    the work the P PEs' shard launches of a P-PE call do together: reads
    every source once, writes every target (PE q: x_q + the others in
    ascending order).  Algorithmic bytes 2*P*n*8 per launch.  HIP events on
    the launch stream.  Beside it the same-mix ceiling: the copy kernel
    (csrc/copy.hip) moving P ranges of n*8 bytes in one launch, its tiles
    dealt round-robin over the ranges -- P read and P write streams at once
    over the same bytes, nothing folded.  `arrays` (team_arrays) are made
    here when not given; `canary` (Canary) is timed right before and right
    after this trial's own timings."""
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(77 + P)
    srcs_t, dsts_t = arrays if arrays is not None else team_arrays(torch, n, P, layout)
    st = torch.cuda.Stream(device=dev)
    srcs = (ctypes.c_void_p * P)(*[x.data_ptr() for x in srcs_t])
    dsts = (ctypes.c_void_p * P)(*[x.data_ptr() for x in dsts_t])
    sp = ctypes.c_void_p(st.cuda_stream)
    torch.cuda.synchronize()
    can_before = canary() if canary is not None else None

    def launch():
        if L.osgpu_team_combine(5, 0, P, dsts, srcs, n, sp) != 0:
            raise RuntimeError(L.osgpu_last_error().decode())

    for _ in range(3):
        launch()
    kavg = span_per_launch(torch, st, launch, reps)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for e0, e1 in ev:
        e0.record(st)
        launch()
        e1.record(st)
    torch.cuda.synchronize()
    ks = [e0.elapsed_time(e1) * 1e-3 for e0, e1 in ev]
    # bit-exact: member q's fold order is q first, then ascending skipping q
    exact = True
    idx = torch.randint(0, n, (1 << 16,), device=dev, generator=g)
    for q in range(P):
        acc = srcs_t[q][idx].clone()
        for j in range(P):
            if j != q:
                acc = acc + srcs_t[j][idx]
        exact = exact and bool(torch.equal(dsts_t[q][idx], acc))
    # the same-mix ceiling: copy kernel, P ranges src_p -> dst_p in one launch
    S = (ctypes.c_void_p * P)(*[x.data_ptr() for x in srcs_t])
    D = (ctypes.c_void_p * P)(*[x.data_ptr() for x in dsts_t])
    N = (ctypes.c_size_t * P)(*([n * 8] * P))

    def copy():
        assert L.osgpu_copy(D, S, N, P, sp) == 0
    for _ in range(3):
        copy()
    cavg = span_per_launch(torch, st, copy, reps)
    # the team kernel again on the same arrays after the copy, then the copy
    # again: a timing that disagrees with its repeat on the SAME pages was a
    # transient of the box, not the placement (the copy is the ceiling: its
    # faster timing is the one used)
    kavg_again = span_per_launch(torch, st, launch, reps)
    cavg_again = span_per_launch(torch, st, copy, reps)
    cavg_first = cavg
    cavg = min(cavg, cavg_again)
    can_after = canary() if canary is not None else None
    B = 2 * P * n * 8
    # the form team.hip launches for double sum (TeamShape): the LDS-staged
    # kernel (U = TEAM_LDS_U) at 2 to 6 and at 8 members, the register kernel
    # otherwise
    lds = team_lds(P)
    kern = (f"team_lds_kernel<double, 0, {P}, true, {TEAM_LDS_U}" if lds    # (PMC files' key)
            else f"team_vec_kernel<double, 0, {P}, true>")
    tr = load_traffic(kern, n)
    frac = B / kavg / 1e9 / HBM_PEAK_GBS
    cfrac = B / cavg / 1e9 / HBM_PEAK_GBS
    out = {"bound": "hbm", "achieved": B / kavg / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": frac, "traffic": tr.get("bytes_per_launch") if tr else None,
           "traffic_source": tr.get("source") if tr else None,
           "kernel": ("osgpu::" + kern.replace("<double, 0,", "<double, SUM,") +
                      (">" if lds else "")),
           "members": P, "nreduce": n, "layout": layout,
           "kernel_avg_us": kavg * 1e6,
           "kernel_avg_how": "HIP event span over the launches, back to back, / launches",
           "kernel_min_us_per_launch_events": min(ks) * 1e6,
           "kernel_avg_us_again_after_copy": kavg_again * 1e6,
           "spread": {"team": max(kavg, kavg_again) / min(kavg, kavg_again),
                      "copy": max(cavg_first, cavg_again) / min(cavg_first, cavg_again)},
           "copy_us_timings": [cavg_first * 1e6, cavg_again * 1e6],
           "algorithmic_bytes_per_launch": B, "launches": reps, "bit_exact_sample": exact,
           "copy_ceiling_same_mix": {"kernel": "copy_vec_kernel (ranges dealt round-robin)",
                                     "ranges": P, "bytes_per_range": n * 8, "us": cavg * 1e6,
                                     "frac_of_8TBs": cfrac},
           "copy_frac": cfrac,
           "frac_of_copy_ceiling": frac / cfrac,
           "canary_before": can_before, "canary_after": can_after,
           # where the arrays landed (virtual; each a separate allocation):
           # base addresses and their offsets within a 2 MiB fragment
           "addresses": {"src": [hex(x.data_ptr()) for x in srcs_t],
                         "dst": [hex(x.data_ptr()) for x in dsts_t],
                         "offset_in_2MiB": [x.data_ptr() % (2 << 20) for x in srcs_t + dsts_t]},
           "note": f"one launch over all nreduce elements = the {P} PEs' shard launches of a "
                   f"{P}-PE call; {P} reads + {P} writes of 8 B per element"}
    if arrays is None:
        del srcs_t, dsts_t
        torch.cuda.empty_cache()
    return out


def team_placements(L, torch, n, reps, P, trials=3, canary=None):
    """team_kernel_rate on `trials` placements, ALL allocated up front (no
    array is freed between trials: round 5's three collapses were all trial
    1, timed right after trial 0's arrays were freed), each trial bracketed
    by the canary.  The rate of 2P streams read and written in lockstep
    depends on where the pages land -- the same kernel and the round-robin
    copy both move 0.72-0.84 of 8 TB/s at P = 2..8 across placements
    (profiles/r03_team_layouts.jsonl) -- so the line reports every trial
    (labelled by label_trials) and the medians."""
    arrs = [team_arrays(torch, n, P, seed=t) for t in range(trials)]
    runs = [team_kernel_rate(L, torch, n, reps, P, arrays=arrs[t], canary=canary)
            for t in range(trials)]
    del arrs
    torch.cuda.empty_cache()
    med = sorted(runs, key=lambda r: r["frac_of_copy_ceiling"])[len(runs) // 2]
    # (bound "hbm", peak 8000 GB/s, 2*P*nreduce*8 algorithmic bytes: the roofline's)
    out = {k: med[k] for k in ("kernel", "achieved", "frac", "kernel_avg_us", "traffic",
                               "traffic_source", "copy_frac", "frac_of_copy_ceiling")}
    out["placements"] = runs      # full records (addresses): the detail file
    out["trials"] = [{"frac": r["frac"], "copy_frac": r["copy_frac"],
                      "canary": [r["canary_before"], r["canary_after"]],
                      "spread": [r["spread"]["team"], r["spread"]["copy"]]} for r in runs]
    for key, get in (("frac", lambda r: r["frac"]),
                     ("frac_of_copy_ceiling", lambda r: r["frac_of_copy_ceiling"])):
        v = sorted(get(r) for r in runs)
        out[key + "_min"], out[key + "_median"], out[key + "_max"] = v[0], v[len(v) // 2], v[-1]
    cs = sorted(c for r in runs for c in (r["canary_before"], r["canary_after"]) if c is not None)
    if cs:
        out["canary_min"], out["canary_median"] = cs[0], cs[len(cs) // 2]
    out["placements_note"] = (f"{trials} placements allocated up front; the fields above are "
                              f"the trial with the median frac_of_copy_ceiling, *_min / *_median / "
                              f"*_max over all; canary = the fixed-buffer copy's fraction of "
                              f"8 TB/s right before / after each trial")
    out["bit_exact_sample"] = all(r["bit_exact_sample"] for r in runs)
    # heaps carved out of one allocation (equal low address bits, regular
    # high ones): the worst layout measured, reported beside the placements
    try:
        sh = team_kernel_rate(L, torch, n, reps, P, layout="symheap", canary=canary)
        out["one_allocation_heaps_layout"] = {
            "frac": sh["frac"], "copy_frac": sh["copy_frac"],
            "frac_of_copy_ceiling": sh["frac_of_copy_ceiling"],
            "bit_exact_sample": sh["bit_exact_sample"]}
    except Exception as e:  # report, never hide
        out["one_allocation_heaps_layout"] = {"error": repr(e)[:200]}
    return out


def label_trials(by_members, canary_ref, slow=0.9, box=0.9, repeat=1.25):
    """Every placement trial labelled: "ok", or -- when its frac or its copy's
    falls below `slow` x its member count's median -- "transient" (a canary
    sample around it below `box` x the run's canary median, or the team or
    copy timing disagreeing with its own repeat on the same pages by more
    than `repeat`x: the box was slow at that time) or "placement" (canary
    normal and both timings repeat: the arrays' placement itself was slow).
    Returns the count of each label."""
    counts = {"ok": 0, "transient": 0, "placement": 0}
    for rec in by_members.values():
        tr = rec.get("trials") if isinstance(rec, dict) else None
        if not tr:
            continue
        fm = sorted(t["frac"] for t in tr)[len(tr) // 2]
        cm = sorted(t["copy_frac"] for t in tr)[len(tr) // 2]
        for t in tr:
            is_slow = t["frac"] < slow * fm or t["copy_frac"] < slow * cm
            cmin = min((c for c in t["canary"] if c is not None), default=None)
            wobbly = max(t.get("spread") or [1.0]) > repeat
            if not is_slow:
                t["label"] = "ok"
            elif wobbly or (cmin is not None and canary_ref and cmin < box * canary_ref):
                t["label"] = "transient"
            else:
                t["label"] = "placement"
            counts[t["label"]] += 1
    return counts


def stream_ceiling(L, torch, nbytes, reps=20):
    """The copy kernel (csrc/copy.hip, one read + one write stream) over
    nbytes: what a streaming kernel with writes moves on this box at this
    footprint -- the practical ceiling the combine is compared with."""
    dev = torch.device("cuda:0")
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev).fill_(1)
    o = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    st = torch.cuda.Stream(device=dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    D = (ctypes.c_void_p * 1)(o.data_ptr())
    S = (ctypes.c_void_p * 1)(a.data_ptr())
    N = (ctypes.c_size_t * 1)(nbytes)
    torch.cuda.synchronize()

    def launch():
        assert L.osgpu_copy(D, S, N, 1, sp) == 0
    for _ in range(3):
        launch()
    med = span_per_launch(torch, st, launch, reps)
    del a, o
    torch.cuda.empty_cache()
    return {"kernel": "copy_vec_kernel", "bytes_copied": nbytes, "us": med * 1e6,
            "frac_of_8TBs": 2 * nbytes / med / 8e12}


def extra_kernel_rates(L, torch):
    """The north-star statement (double sum at nreduce = 128 Mi: >= 80 % of
    HBM READ bandwidth) and BASELINE config 3 (long and/or/xor, 256 MiB per
    array = 32 Mi elements, bit-exact), on the same combine kernel."""
    out = {}
    n = 128 << 20
    t, a, b, o = kernel_rate(L, torch, 5, 0, n, 8, torch.float64,
                             lambda x, k: x.uniform_(1.0, 2.0))
    ns = {"kernel_us": t * 1e6, "read_GBs": 2 * n * 8 / t / 1e9,
          "read_frac_of_8TBs": 2 * n * 8 / t / 8e12, "frac_all_bytes": 3 * n * 8 / t / 8e12}
    del a, b, o
    torch.cuda.empty_cache()
    # the same footprint through the copy kernel (1 read + 1 write stream of
    # 1.5 GiB each = the combine's 3 GiB): the box's streaming ceiling
    ceil = stream_ceiling(L, torch, 3 * n * 8 // 2)
    ns["copy_ceiling_same_bytes"] = ceil
    ns["frac_of_copy_ceiling"] = ns["frac_all_bytes"] / ceil["frac_of_8TBs"]
    out["north_star_double_sum_128Mi"] = ns
    n = 32 << 20
    c3 = {"nreduce": n, "bytes_per_array": n * 8}
    for name, code, ref in (("and", 2, lambda x, y: x & y), ("or", 3, lambda x, y: x | y),
                            ("xor", 4, lambda x, y: x ^ y)):
        t, a, b, o = kernel_rate(L, torch, 2, code, n, 8, torch.int64,
                                 lambda x, k: x.random_(-(1 << 62), 1 << 62))
        c3[name] = {"kernel_us": t * 1e6, "GBs": 3 * n * 8 / t / 1e9,
                    "frac_of_8TBs": 3 * n * 8 / t / 8e12,
                    "bit_exact": bool(torch.equal(o, ref(a, b)))}
        del a, b, o
    torch.cuda.empty_cache()
    out["config3_long_bitwise_256MiB"] = c3
    try:
        out["longdouble_team_8_members"] = longdouble_team_rate(L, torch)
    except Exception as e:  # report, never hide; the fields above stand
        out["longdouble_team_8_members"] = {"error": repr(e)[:300]}
    return out


def longdouble_team_rate(L, torch, n=4 << 20, P=8, reps=20):
    """The kernel furthest from the HBM roofline: the x87 soft-float team
    kernel (csrc/longdouble.hip ld_team_kernel, x87.hpp) for an 8-member
    long double sum -- every member's own fold order, 49 soft adds per
    element -- over n elements of 16-B slots, 2*P*n*16 bytes per launch.
    VALU-bound, so it follows the box's clock.  Data as
    tools/ld_team_rate.py: random 64-bit significands, exponents
    2^-3..2^3, random signs (the general fast add in every round) or one
    sign (the addition-only add)."""
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(5)
    st = torch.cuda.Stream(device=dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    dsts_t = [torch.empty((n, 2), dtype=torch.int64, device=dev) for _ in range(P)]
    D = (ctypes.c_void_p * P)(*[x.data_ptr() for x in dsts_t])
    B = 2 * P * n * 16
    out = {"bound": "valu (x87 soft-float; HBM roofline below)", "peak": HBM_PEAK_GBS,
           "unit": "GB/s", "members": P, "nreduce": n, "algorithmic_bytes_per_launch": B,
           "kernel": f"osgpu::x87::ld_team_kernel<SUM, {P}>"}
    for dist in ("random_signs", "one_sign"):
        srcs_t = []
        for _ in range(P):
            v = torch.empty((n, 2), dtype=torch.int64, device=dev)
            v[:, 0] = torch.randint(-(1 << 62), 1 << 62, (n,), device=dev,
                                    generator=g) | (-(1 << 63))
            e = 0x3fff + torch.randint(-3, 4, (n,), device=dev, generator=g)
            sgn = torch.randint(0, 2, (n,), device=dev, generator=g) << 15
            v[:, 1] = e | (sgn if dist == "random_signs" else 0)
            srcs_t.append(v)
        S = (ctypes.c_void_p * P)(*[x.data_ptr() for x in srcs_t])
        torch.cuda.synchronize()

        def launch():
            if L.osgpu_team_combine(6, 0, P, D, S, n, sp) != 0:
                raise RuntimeError(L.osgpu_last_error().decode())
        # warm up by time, not by count: from an idle GPU the first launches
        # of this power-hungry kernel run while the clock ramps (1.2 ms, then
        # 0.58-0.63 ms, settling at 0.53 ms for 8 Mi elements;
        # profiles/r03_clock_probe.jsonl)
        t_warm = time.time() + 1.5
        while time.time() < t_warm:
            for _ in range(20):
                launch()
            torch.cuda.synchronize()
        t = span_per_launch(torch, st, launch, reps)
        torch.cuda.synchronize()
        # members 0 and 1 fold x0 + x1 + ... and x1 + x0 + ...: the same bits
        same01 = bool(torch.equal(dsts_t[0][:, 0], dsts_t[1][:, 0]) and
                      torch.equal(dsts_t[0][:, 1] & 0xffff, dsts_t[1][:, 1] & 0xffff))
        out[dist] = {"kernel_avg_us": t * 1e6, "achieved": B / t / 1e9,
                     "frac": B / t / 1e9 / HBM_PEAK_GBS, "member0_equals_member1": same01}
        del srcs_t
    del dsts_t
    torch.cuda.empty_cache()
    out["note"] = ("every member's fold order (src/reductions.c:79-111) in x87 80-bit arithmetic "
                   "(src/shmemu/miscops.c:30); bit-exact against the reference in "
                   "tests/test_gpu_x87.py; VALU-issue-bound at ~1360 W and ~2375 MHz in steady state; "
                   "timed after a 1.5 s warm-up, as from an idle GPU the first launches run "
                   "while the clock ramps (profiles/r03_clock_probe.jsonl)")
    return out


def small_call_latency(n=1024, reps=300, sizes=(1024, 4096, 8192, 16384, 32768, 65536)):
    """BASELINE config 1's shape (shmem_int_sum_to_all, nreduce = 1 Ki, 2 PEs)
    with one PROCESS per PE, both on this GPU (IPC device heaps, the
    shared-memory PE runtime of tests/support/pe_shm.c): median per call of
    the fused one-launch path (device-side barriers) and of the host-barrier
    path, timed barrier to barrier (tools/mp_latency.py), next to the
    reference's loop shape on 2 host cores.  The same at larger sizes gives
    the crossover: the smallest nreduce at which the drop-in beats the
    reference's loop (src/reductions.c:79-113) -- below it, it is slower."""
    import subprocess
    import oracle as O
    sizes = sorted(set(sizes) | {n})
    env = dict(os.environ, MP_WORLDS="2", MP_SIZES=",".join(map(str, sizes)),
               MP_REPS=str(reps))
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "mp_latency.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        return {"error": (r.stdout + r.stderr)[-400:]}
    lat = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])["latency"]
    out = {"note": f"shmem_int_sum_to_all nreduce={n}, 2 PEs = 2 processes sharing this GPU, "
                   f"device-resident symmetric heaps, median of {reps} calls barrier to barrier"}
    for k in ("fused_team", "team", "host_fused_staged", "host_staged", "host_fold"):
        v = lat[f"{n}/{k}"]
        out[k + "_us"] = v["us_median"]
        if "us_median_timed_in_c" in v:   # the loop in C, like the CPU baseline's
            out[k + "_us_timed_in_c"] = v["us_median_timed_in_c"]
        out[k + "_correct"] = v["correct"]
    out["note"] += ("; host_* = the same call on a pinned host symmetric heap (config 1's "
                    "own placement): fused staged (one launch) vs pipelined STAGED vs the "
                    "host fold (the library's default while (P-1)*nreduce*size <= 256 KiB)")
    cpu = {}
    for m in sizes:
        src = O.team_inputs("int", 2, m, 5, "bits")
        cpu[m] = O.cpu_baseline("int", "sum", src, reps=max(50, min(2000, int(2e7 / m))),
                                pin=True, ref_ops=O.ref_elem_fn("int", "sum") is not None) * 1e6
    out["cpu_reference_loop_us"] = cpu[n]
    sweep = [{"nreduce": m, "cpu_reference_loop_us": cpu[m],
              "fused_team_us": lat[f"{m}/fused_team"]["us_median"],
              "host_fused_staged_us": lat[f"{m}/host_fused_staged"]["us_median"],
              "host_fold_us": lat[f"{m}/host_fold"].get("us_median_timed_in_c",
                                                      lat[f"{m}/host_fold"]["us_median"]),
              "host_fold_us_python": lat[f"{m}/host_fold"]["us_median"]}
             for m in sizes]
    for rec in sweep:  # the library's default on a host heap at this size
        rec["default_us"] = (rec["host_fold_us"] if (2 - 1) * rec["nreduce"] * 4 <= HOST_FOLD_MAX_BYTES
                             else rec["host_fused_staged_us"])
    out["sweep"] = sweep

    def crossover(key):
        # smallest size from which on the GPU call is faster at every larger size
        for i, rec in enumerate(sweep):
            if all(x[key] < x["cpu_reference_loop_us"] for x in sweep[i:]):
                return rec["nreduce"]
        return None
    # config 1's placement is the host heap, whose default path at 1 Ki is
    # the host fold: timed in C between the runtime's barriers, as the
    # reference's loop is
    dflt = out.get("host_fold_us_timed_in_c", out["host_fold_us"])
    out["default_path_us"] = dflt
    out["default_path"] = lat[f"{n}/host_fold"]["path"]
    out["crossover_elements"] = {"device_heaps_fused": crossover("fused_team_us"),
                                 "pinned_host_heaps_fused": crossover("host_fused_staged_us"),
                                 "pinned_host_heaps_default": crossover("default_us")}
    out["slower_than_reference_loop"] = dflt > cpu[n]
    out["ratio_to_reference_loop"] = dflt / cpu[n]
    out["best_gpu_form_us"] = min(out["fused_team_us"], out["host_fused_staged_us"])
    out["crossover_note"] = ("config 1 (1 Ki ints on host heaps): the default path is the host "
                             "fold (one getmem per peer, direct fold); the GPU forms (kernel "
                             "launch + device barriers, >= ~11 us) win from crossover_elements "
                             "on (kind: port, memcpy getmem, no UCX)")
    return out


def bench_single(args):
    import torch
    import osgpu
    L = osgpu.load()
    n = args.nreduce
    dev = torch.device("cuda:0")
    a = torch.empty(n, dtype=torch.float64, device=dev).uniform_(1.0, 2.0)
    b = torch.empty(n, dtype=torch.float64, device=dev).uniform_(1.0, 2.0)
    out = torch.empty(n, dtype=torch.float64, device=dev)
    stream = torch.cuda.Stream(device=dev)
    srcs = (ctypes.c_void_p * 2)(a.data_ptr(), b.data_ptr())
    sp = ctypes.c_void_p(stream.cuda_stream)
    torch.cuda.synchronize()  # inputs were written on torch's default stream

    def step():
        rc = L.osgpu_combine(5, 0, out.data_ptr(), srcs, 2, n, sp)
        if rc != 0:
            raise RuntimeError(L.osgpu_last_error().decode())

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # correctness spot check of the timed kernel
    idx = torch.randint(0, n, (4096,), device=dev)
    assert torch.equal(out[idx], a[idx] + b[idx])

    # timed region: the K launches back to back, one HIP event pair on the
    # launch stream around all of them (an event pair around EVERY launch
    # adds ≈ 6-8 µs per 255 µs launch, tools/warm_probe.py `gap`), so the
    # average launch duration = event span / K, kernel boundaries included
    e_beg, e_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e_beg.record(stream)
    for _ in range(args.steps):
        step()
    e_end.record(stream)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    kavg = e_beg.elapsed_time(e_end) * 1e-3 / args.steps
    # after the timed region: the per-launch spread (an event pair per launch)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    for e0, e1 in ev:
        e0.record(stream)
        step()
        e1.record(stream)
    torch.cuda.synchronize()
    kms = sorted(s.elapsed_time(e) for s, e in ev)
    # and once the clocks have settled (launches 1-100 of a process run
    # 1-3 % slower, tools/warm_probe.py): 100 more, one event pair
    ksteady = span_per_launch(torch, stream, step, 100)
    B = 3 * n * 8
    res = {
        "metric": METRIC,
        "value": args.steps * B / t / GIB,
        "unit": "GiB/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": t / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: uniform [1,2) doubles resident in HBM",
        "config": {"workload": "BASELINE config 2: shmem_double_sum_to_all combine, "
                               "nreduce=64Mi, K=2 inputs (source + peer source), 1 MI355X, "
                               "device-resident combine kernel",
                   "nreduce": n, "K": 2, "bytes_per_step": B},
    }
    del a, b, out
    torch.cuda.empty_cache()
    # this box's streaming ceiling at the same footprint (copy kernel: 1 read
    # + 1 write stream, 3*n*8 bytes moved): box-to-box spread is the memory's
    try:
        ceil64 = stream_ceiling(L, torch, 3 * n * 8 // 2, reps=args.steps)
    except Exception as e:  # report, never hide
        ceil64 = {"error": repr(e)}
    if not args.no_extra:
        try:
            res.update(extra_kernel_rates(L, torch))
        except Exception as e:  # report, never hide
            res["extra_kernels"] = {"error": repr(e)}
    # this run's own PMC passes (child processes under rocprofv3); not when
    # this process is itself being profiled (nested profilers)
    profiled = any(k.startswith("ROCPROF") for k in os.environ) or \
        "rocprof" in os.environ.get("LD_PRELOAD", "")
    if args.no_live_pmc or profiled:
        res["traffic_live"] = {"skipped": "--no-live-pmc" if args.no_live_pmc
                               else "this process runs under rocprofv3"}
    else:
        try:
            live = live_traffic(n, (2, 4, 8) if not args.no_extra else ())
        except Exception as e:  # report, never hide
            live = {"_error": repr(e)}
        LIVE_TRAFFIC.update({k: v for k, v in live.items() if not k.startswith("_")})
        res["traffic_live"] = {
            "how": "rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE, each a child process "
                   "of this run over tools/pmc_probe.py (the same kernels and shapes through "
                   "the C ABI, 5 launches each); FETCH_SIZE x2 (gfx950), KiB -> bytes",
            "kernels": {k: v["traffic_over_algorithmic"] for k, v in LIVE_TRAFFIC.items()},
            **{k: v for k, v in live.items() if k.startswith("_")}}
    tr = load_traffic(n=n)
    res["roofline"] = {
        "bound": "hbm", "achieved": B / kavg / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": B / kavg / 1e9 / HBM_PEAK_GBS,
        "traffic": tr.get("bytes_per_launch") if tr else None,
        "traffic_source": tr.get("source") if tr else None,
        "kernel": COMBINE_LABEL,
        "kernel_avg_us": kavg * 1e6,
        "kernel_avg_how": "HIP event span over the K timed launches on the launch stream / K",
        "kernel_median_us_per_launch_events": kms[len(kms) // 2] * 1e3,
        "kernel_min_us_per_launch_events": kms[0] * 1e3,
        "algorithmic_bytes_per_launch": B,
        "after_timed_region_100_launches": {
            "kernel_avg_us": ksteady * 1e6, "frac": B / ksteady / 1e9 / HBM_PEAK_GBS,
            "note": "not the timed region: 100 more launches after it (event span / 100), "
                    "once the start-of-process ramp is over"},
        "copy_ceiling_same_bytes": ceil64,
    }
    if "frac_of_8TBs" in ceil64:
        res["roofline"]["frac_of_copy_ceiling"] = res["roofline"]["frac"] / ceil64["frac_of_8TBs"]
    # the kernel the API dispatches (TEAM path), under the same roofline, for
    # 2, 4 and 8 members (config 4's 8 PEs on one GPU run it at P = 8), each
    # beside the copy kernel moving the same P read + P write streams
    res["team_by_members"] = {}
    canary = None
    try:
        canary = Canary(L, torch)
    except Exception as e:  # report, never hide; the trials run without it
        res["team_by_members"]["canary_error"] = repr(e)[:200]
    for P in ((2, 4, 8) if not args.no_extra else (2,)):
        try:
            res["team_by_members"][str(P)] = team_placements(
                L, torch, n, min(args.steps, 20), P, canary=canary)
        except Exception as e:  # report, never hide
            res["team_by_members"][str(P)] = {"error": repr(e)}
    if canary is not None:
        ref = canary.reference()
        res["team_by_members"]["canary"] = {
            "what": "copy_vec_kernel over 2 x 512 MiB allocated once before the first trial, "
                    "fraction of 8 TB/s, timed right before and after every trial",
            "median": ref, "min": min(canary.samples), "max": max(canary.samples),
            "labels": label_trials(res["team_by_members"], ref)}
        del canary
        torch.cuda.empty_cache()
    if not args.no_api:
        try:
            res["api"] = api_call_time(n)
            tcall = res["api"]["team"]["ms_per_call"] * 1e-3
            res["roofline_call"] = {
                "bound": "hbm", "achieved": 4 * n * 8 / tcall / 1e9, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": 4 * n * 8 / tcall / 1e9 / HBM_PEAK_GBS,
                "traffic": None, "ms_per_call": tcall * 1e3,
                "team_local": os.environ.get("OSGPU_TEAM_LOCAL", "merge"),
                "sync": os.environ.get("OSGPU_SYNC", "word"),
                "what": "the whole shmem_double_sum_to_all call, 2 PEs (pthreads) on one GPU, "
                        "default (TEAM) path: entry sync, 2 barriers, both PEs' shard launches, "
                        "completion waits; 4*n*8 HBM bytes per call"}
        except Exception as e:  # report, never hide
            res["api"] = {"error": repr(e)}
        try:  # as a C application runs it: /opt/rocm's HIP runtime, no torch
            res["host_staged"] = host_staged_child(n)
        except Exception as e:
            res["host_staged"] = {"error": repr(e)}
        try:  # config 5 with its H2D/D2H copies, the same child process
            res["config5_host_staged"] = host_staged_child(128 << 20, what="host_staged_config5(%d)")
        except Exception as e:
            res["config5_host_staged"] = {"error": repr(e)}
        try:  # the same inside this (torch) process: torch's bundled runtime
            res["host_staged_in_torch_process"] = host_staged_time(n)
        except Exception as e:
            res["host_staged_in_torch_process"] = {"error": repr(e)}
        try:
            res["collectives"] = collectives_single()
        except Exception as e:
            res["collectives"] = {"error": repr(e)}
        try:
            res["small_call"] = small_call_latency()
        except Exception as e:
            res["small_call"] = {"error": repr(e)}
    if not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(args.cpu_n)
        res["cpu_baseline_configs"] = cpu_baselines_configs()
    print(fit_line(res, args.detail or default_detail(1)), flush=True)


# --------------------------------------------------------------------------
# N > 1
# --------------------------------------------------------------------------

def _log(rank, msg):
    # one write per line: ranks share the stream
    sys.stderr.write(f"[bench rank {rank}] {time.strftime('%H:%M:%S')} {msg}\n")
    sys.stderr.flush()


def _sample_parity(rank, world, src, tgt, n, fn_op, dist, nsamp=1 << 15, t="double"):
    """Bit-exact check of this PE's target on a sample of elements: every
    rank contributes its source at the sampled indices (gloo), the oracle
    folds them in this PE's order (src/reductions.c:79-111).  For float /
    double also the largest difference in ulps (same-sign results: the
    distance of the bit patterns) -- the measure of DESIGN.md 3's RCCL
    tolerance."""
    import numpy as np
    import torch
    import oracle as O
    g = torch.Generator().manual_seed(1234)
    idx = torch.randint(0, n, (nsamp,), generator=g)
    mine = src[idx.to(src.device)].cpu()
    allv = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allv, mine)
    srcs = [a.numpy() for a in allv]
    want = O.fold_with(O.op_elementwise, t, fn_op, srcs, rank, 0, 0, world)
    got = tgt[idx.to(tgt.device)].cpu().numpy()
    isz = got.dtype.itemsize
    ui = {2: np.uint16, 4: np.uint32, 8: np.uint64}[isz]
    bad = int(np.count_nonzero(got.view(ui) != want.view(ui)))
    local = {"checked": nsamp, "bit_mismatches": bad}
    if t in ("float", "double"):
        si = {4: np.int32, 8: np.int64}[isz]
        rel = float(np.max(np.abs(got - want) / np.abs(want))) if nsamp else 0.0
        same = np.signbit(got) == np.signbit(want)
        d = np.abs(got.view(si).astype(np.int64)[same] - want.view(si).astype(np.int64)[same])
        local["max_rel_err"] = rel
        local["max_ulp"] = (int(d.max()) if d.size else 0) if bool(same.all()) else None
    allp = [None] * world
    dist.all_gather_object(allp, local)
    out = {"checked_per_pe": nsamp,
           "bit_mismatches": sum(p["bit_mismatches"] for p in allp)}
    if t in ("float", "double"):
        out["max_rel_err"] = max(p["max_rel_err"] for p in allp)
        ulps = [p["max_ulp"] for p in allp]
        out["max_ulp"] = None if None in ulps else max(ulps)
    return out


def _rccl_tolerance(parity, world):
    """RCCL's FP sum of same-sign inputs is within 2(P-1) ulp
    of the reference's per-PE fold."""
    bound = 2 * (world - 1)
    mu = parity.get("max_ulp")
    return {"bound_ulp": bound, "max_ulp": mu,
            "within_tolerance": mu is not None and mu <= bound,
            "rule": "same-sign sum: |RCCL - reference order| <= 2(P-1) ulp (DESIGN.md 3)"}


def _rccl_integer_legs(L, osgpu, torch, dist, rank, world, dev, psync, nint, steps=3):
    """The AUTOMATIC path's RCCL dispatch for integer (type, op)s (no heap
    holds these arrays, so shmem_reduce.cpp sends them to ncclAllReduce):
    results must be bit-exact against the oracle's per-PE fold, wrap-around
    included -- int sum near INT_MAX, long prod of full-range odd values,
    int min and long max over the full range."""
    legs = (("int", "sum", torch.int32, lambda x, gen: x.random_(2**31 - 4096, 2**31 - 1,
                                                                 generator=gen)),
            ("long", "prod", torch.int64, lambda x, gen: x.random_(-2**62, 2**62,
                                                                   generator=gen).bitwise_or_(1)),
            ("int", "min", torch.int32, lambda x, gen: x.random_(-2**31, 2**31 - 1,
                                                                 generator=gen)),
            ("long", "max", torch.int64, lambda x, gen: x.random_(-2**63, 2**63 - 1,
                                                                  generator=gen)))
    wrk = (ctypes.c_long * 64)()
    out = {"nreduce": nint, "path_mode": "auto (arrays outside every heap)"}
    L.osgpu_set_path(osgpu.PATH_AUTO)
    gen = torch.Generator(device=dev).manual_seed(7000 + rank)
    for t, op, dt, fill in legs:
        s_ = torch.empty(nint, dtype=dt, device=dev)
        d_ = torch.empty(nint, dtype=dt, device=dev)
        fill(s_, gen)
        torch.cuda.synchronize()
        fn = getattr(L, f"shmem_{t}_{op}_to_all")

        def step():
            fn(d_.data_ptr(), s_.data_ptr(), nint, 0, 0, world, wrk, psync)

        tt = _timed(step, steps, 1, dist, torch)
        par = _sample_parity(rank, world, s_, d_, nint, op, dist, t=t)
        out[f"{t}_{op}"] = {"path": osgpu.last_path(), "ms_per_call": tt / steps * 1e3,
                            "algbw_GiBs": nint * s_.element_size() * steps / tt / GIB,
                            "parity_vs_oracle": par,
                            "bit_exact": par["bit_mismatches"] == 0}
        del s_, d_
    torch.cuda.empty_cache()
    return out


def _timed(step, steps, warmup, dist, torch):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    tt = torch.tensor([t], dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return float(tt.item())


def _agree(dist, world, ok):
    """True on every rank iff ok on every rank."""
    allok = [None] * world
    dist.all_gather_object(allok, bool(ok))
    return all(allok)


def _block_sums(t, nb, world, torch):
    """int64 wrap-around sum of each nb-byte block of a uint8 tensor."""
    return [int(t[i * nb:(i + 1) * nb].view(torch.int64).sum().item()) for i in range(world)]


def _multi_fcollect(L, osgpu, torch, dist, rank, world, dev, hsrc, htgt, heap_bytes, team_ok,
                    rccl_ok, args, PES, staging_ok=True):
    """shmem_fcollect64 with one PE per GPU.  Every PE's target gathers all
    contributions: per PE (P-1)/P of the target bytes arrive over xGMI (or
    PCIe for host memory).  Parity: every nb-byte block of every target has
    the int64 checksum of the contributing PE's source, all ranks agree."""
    fc = L.shmem_fcollect64
    ps = PES.pes_heap(rank) + (1 << 20) - 4096       # symmetric pSync
    out = {"note": "fcollect64, one PE per GPU; GBps = target bytes gathered per PE / time"}

    def check(src_t, tgt_t, nb):
        mine = int(src_t[:nb].view(torch.int64).sum().item())
        allsum = [None] * world
        dist.all_gather_object(allsum, mine)
        got = _block_sums(tgt_t, nb, world, torch)
        return _agree(dist, world, got == allsum)

    nb = (heap_bytes // world) // 256 * 256          # contribution per PE (device)
    hsrc[:nb].random_(0, 256, generator=torch.Generator(device=dev).manual_seed(500 + rank))
    torch.cuda.synchronize()

    def stepd():
        fc(htgt.data_ptr(), hsrc.data_ptr(), nb // 8, 0, 0, world, ps)

    for name, path, usable in (("device_copy_xgmi", osgpu.PATH_P2P, team_ok),
                               ("rccl_allgather", osgpu.PATH_RCCL, rccl_ok)):
        if not usable:
            continue
        L.osgpu_set_path(path)
        htgt.zero_()
        torch.cuda.synchronize()
        t = _timed(stepd, 3, 1, dist, torch)
        out[name] = {"bytes_per_pe": nb, "ms_per_call": t / 3 * 1e3,
                     "GBps_per_pe": 3 * world * nb / t / 1e9,
                     "xgmi_in_GBps_per_pe": 3 * (world - 1) * nb / t / 1e9,
                     "bit_exact_blocks": check(hsrc, htgt, nb)}
    L.osgpu_set_path(osgpu.PATH_AUTO)

    if not staging_ok:
        out["host_staged_pinned"] = {"skipped": "the staging areas failed their preflight"}
        return out
    nbh = 64 << 20                                   # host: 64 MiB per PE, pinned
    hs = torch.empty(nbh, dtype=torch.uint8).pin_memory()
    ht = torch.empty(world * nbh, dtype=torch.uint8).pin_memory()
    hs.random_(0, 256, generator=torch.Generator().manual_seed(600 + rank))

    def steph():
        fc(ht.data_ptr(), hs.data_ptr(), nbh // 8, 0, 0, world, ps)

    with osgpu.host_path("staged"):
        t = _timed(steph, 3, 1, dist, torch)
    out["host_staged_pinned"] = {"bytes_per_pe": nbh, "ms_per_call": t / 3 * 1e3,
                                 "GBps_per_pe": 3 * world * nbh / t / 1e9,
                                 "pcie_GBps_per_pe": 3 * (world + 1) * nbh / t / 1e9,
                                 "bit_exact_blocks": check(hs, ht, nbh)}
    return out


def _xgmi_probe(L, torch, dist, rank, world, bases, seg_bytes, reps=5):
    """Link characteristics for the next design step: every GPU at once
    copies one chunk per peer over xGMI with the copy kernel, either PULLING
    (peer HBM -> my HBM: remote reads) or PUSHING (my HBM -> peer HBM: remote
    writes into a region only I write).  GB/s per GPU per direction."""
    chunk = (seg_bytes // world) // 4096 * 4096
    st = torch.cuda.Stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    out = {"chunk_bytes_per_peer": chunk}
    for name in ("pull_reads", "push_writes"):
        dsts, srcs, nbs = [], [], []
        for q in range(world):
            if q == rank:
                continue
            if name == "pull_reads":   # my target block q <- peer q's source block rank
                srcs.append(bases[(q, 0)] + rank * chunk)
                dsts.append(bases[(rank, 1)] + q * chunk)
            else:                      # peer q's target block rank <- my source block q
                srcs.append(bases[(rank, 0)] + q * chunk)
                dsts.append(bases[(q, 1)] + rank * chunk)
            nbs.append(chunk)
        m = len(nbs)
        D = (ctypes.c_void_p * m)(*dsts)
        S = (ctypes.c_void_p * m)(*srcs)
        N = (ctypes.c_size_t * m)(*nbs)

        def step():
            assert L.osgpu_copy(D, S, N, m, sp) == 0
            st.synchronize()

        t = _timed(step, reps, 1, dist, torch)
        out[name + "_GBs_per_gpu"] = reps * m * chunk / t / 1e9
        out[name + "_GBs_per_link"] = reps * chunk / t / 1e9
    return out


def _team_shapes_ab(L, osgpu, torch, dist, rank, world, bases, n, tgt, reps=5):
    """The team kernel's local and remote launch shapes on the real heaps:
    rank g launches shard g of the double sum over every member's source and
    target (peer HBM over xGMI when the ranks have GPUs of their own) with
    osgpu_team_combine_shape(shape), every rank at once, timed between
    barriers; max over ranks.  The targets of the two shapes must agree bit
    for bit (a position-weighted hash of every PE's whole target)."""
    lo, hi = osgpu.shard_range(n, world, rank, 8)
    m = hi - lo
    S = (ctypes.c_void_p * world)(*[bases[(pe, 0)] + lo * 8 for pe in range(world)])
    D = (ctypes.c_void_p * world)(*[bases[(pe, 1)] + lo * 8 for pe in range(world)])
    st = torch.cuda.Stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    out = {"note": "kernel only: shard of the double sum per rank, all ranks at once",
           "members": world, "shard_elems": m}
    hashes = {}
    for name, shape in (("local_shapes", 0), ("remote_shapes", 1)):
        def step():
            if m > 0:
                assert L.osgpu_team_combine_shape(5, 0, world, D, S, m, sp, shape) == 0
            st.synchronize()

        t = _timed(step, reps, 2, dist, torch)
        dist.barrier()   # every shard of every target written
        hashes[name] = osgpu.checksum("double", osgpu.CK_HASH, tgt.data_ptr(), n)
        B = 2 * world * n * 8      # the whole team's bytes per step
        out[name] = {"ms": t / reps * 1e3, "hbm_GBs_all_gpus": reps * B / t / 1e9,
                     "xgmi_in_GBs_per_gpu": reps * 2 * (world - 1) * (n * 8 // world) / t / 1e9}
    out["remote_over_local"] = out["local_shapes"]["ms"] / out["remote_shapes"]["ms"]
    out["identical_targets_all_ranks"] = _agree(
        dist, world, hashes["local_shapes"] == hashes["remote_shapes"])
    return out


def _multi_small(L, osgpu, torch, dist, rank, world, hsrc, htgt, PES, reps=200, flags_ok=True):
    """BASELINE config 1's shape with one PE per GPU: shmem_int_sum_to_all,
    nreduce = 1 Ki, device heaps over xGMI -- host barriers vs the fused
    one-launch path (device-side barriers written across GPUs).  The device
    barrier is bounded at 2 s and reported instead of fatal here; every rank
    agrees after each call, so a failure ends the phase cleanly."""
    n = 1024
    ps = PES.pes_heap(rank) + (1 << 20) - 4096       # symmetric pSync
    PES.pes_barrier.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    src = hsrc[:n * 4].view(torch.int32)
    tgt = htgt[:n * 4].view(torch.int32)
    src.copy_(torch.arange(n, dtype=torch.int32, device=hsrc.device) + rank)
    torch.cuda.synchronize()
    want = world * torch.arange(n, dtype=torch.int32) + world * (world - 1) // 2
    wrk = (ctypes.c_int * 64)()
    out = {"note": f"shmem_int_sum_to_all nreduce={n}, one PE per GPU, device heaps; "
                   f"us = max over ranks of the median call time ({reps} calls)"}
    L.osgpu_set_path(osgpu.PATH_AUTO)
    L.osgpu_set_device_barrier(2.0, 0)
    try:
        for name, lim in (("host_barriers", 0), ("fused", -1)):
            if name == "fused" and not flags_ok:
                out[name] = {"skipped": "the flag areas failed their preflight"}
                continue
            L.osgpu_set_fused_max_bytes(lim)
            ts, paths, failed = [], set(), False
            for r in range(reps + 10):
                PES.pes_barrier(0, 0, world, None)
                t0 = time.perf_counter()
                L.shmem_int_sum_to_all(tgt.data_ptr(), src.data_ptr(), n, 0, 0, world, wrk, ps)
                t = time.perf_counter() - t0
                p = osgpu.last_path()
                paths.add(p)
                bad = torch.tensor([1 if p == "fused_failed" else 0])
                dist.all_reduce(bad)
                if int(bad.item()):
                    failed = True
                    break
                if r >= 10:
                    ts.append(t)
            mine = sorted(ts)[len(ts) // 2] * 1e6 if ts else float("nan")
            tt = torch.tensor([mine], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            ok = (not failed) and bool(torch.equal(tgt.cpu(), want))
            res = {"us": float(tt.item()), "paths": sorted(paths),
                   "correct_all_ranks": _agree(dist, world, ok)}
            if failed:
                res["error"] = L.osgpu_last_error().decode()
            out[name] = res
            if failed:
                break
    finally:
        L.osgpu_set_fused_max_bytes(-1 if flags_ok else 0)
        L.osgpu_set_device_barrier(-1, 1)
    return out


def start_watchdog(res, rank, deadline, detail=None):
    """The N > 1 line's printer and deadline: emit() prints `res` once (rank
    0); if the run is still going after `deadline` seconds, the watchdog
    marks the line incomplete (naming state["phase"]), prints it and ends
    the process with status 3 -- a stalled run is never recorded as a
    success (tests/test_bench_contract.py)."""
    printed = threading.Lock()
    state = {"printed": False, "phase": "setup"}

    def emit():
        with printed:
            if rank == 0 and not state["printed"]:
                state["printed"] = True
                print(fit_line(res, detail), flush=True)

    def watchdog():
        time.sleep(deadline)
        res["incomplete"] = f"deadline {deadline}s reached during {state['phase']}"
        emit()
        os._exit(3)   # a stalled run must not be recorded as a success

    threading.Thread(target=watchdog, daemon=True).start()
    return state, emit


def bench_multi(args):
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    # ranks sharing a GPU (a rehearsal): the hardware-queue cap must be in
    # the environment before this process's first HIP call, so the devices
    # are counted without HIP (launch_ranks passes BENCH_NDEV; under
    # torch.distributed.run a child process counts them)
    ndev = device_count_without_hip()
    cap = hw_queue_cap(world, ndev)
    if cap is not None:     # the box may export HIP's default (4): lower it, never raise it
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(int(cap), int(os.environ.get(
            "GPU_MAX_HW_QUEUES", cap))))
    import torch
    import torch.distributed as dist
    import osgpu
    from support import peshm
    dev_id = local % max(ndev, 1)
    torch.cuda.set_device(dev_id)
    dev = torch.device("cuda", dev_id)
    dist.init_process_group("gloo")
    L = osgpu.load()
    PES = peshm.init(rank, world, 1 << 20, dist, tag="b")
    assert L.osgpu_set_pe_ops(PES.pes_ops()) == 0
    n = args.nreduce
    # symmetric pSync (OpenSHMEM requires it; the staging setups of the push
    # exchange and the host paths publish through it with getmem)
    psync = ctypes.c_void_p(PES.pes_heap(rank) + (1 << 20) - 8192)
    wrk = (ctypes.c_double * 64)()
    fn = L.shmem_double_sum_to_all
    B = (world + 1) * n * 8          # sum over GPUs of shard-fold bytes

    res = {
        "metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": None,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic: uniform [1,2) doubles resident in HBM",
        "config": {"workload": f"shmem_double_sum_to_all over {world} PEs, one per MI355X, "
                               f"nreduce={n} per PE",
                   "nreduce": n, "bytes_per_step": B,
                   "bytes_convention": "(P+1)*nreduce*8 per step (SURVEY.md 8d aggregate)",
                   "parallelism": f"pe{world}"},
    }
    res["launch"] = {"launcher": "bench.py (own ranks)" if "BENCH_NDEV" in os.environ
                     else "external (torch.distributed.run)",
                     "gpus_visible": ndev, "ranks_per_gpu": -(-world // max(ndev, 1)),
                     "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES")}
    # which physical GPU every PE runs on (the reference's launcher starts one
    # PE per slot, src/shmemc/oshrun.in:4): PCI bus id and UUID per rank
    try:
        ident = dict(osgpu.device_identity(), rank=rank, local_rank=local)
    except Exception as e:  # reported, never hidden
        ident = {"rank": rank, "local_rank": local, "error": repr(e)[:200]}
    idents = [None] * world
    dist.all_gather_object(idents, ident)
    res["launch"]["ranks"] = idents
    buses = [x.get("pci_bus_id") for x in idents]
    res["launch"]["distinct_gpus"] = None not in buses and len(set(buses)) == world
    state, emit = start_watchdog(res, rank, args.deadline,
                                 args.detail or default_detail(world))

    # ---- the device symmetric heap: ONE contiguous virtual range per PE
    # (osgpu_heap_create: dmabuf chunks mapped into every member), holding
    # the source and target of the main line and config 4's 1 Gi-double
    # arrays.  If it cannot be built on some rank, the old form: two HIP IPC
    # segments per PE (< 2 GiB each), and config 4 on RCCL.
    seg_bytes = (n * 8 + (2 << 20) - 1) // (2 << 20) * (2 << 20)
    n4 = args.c4_nreduce
    c4_bytes = (n4 * 8 + (2 << 20) - 1) // (2 << 20) * (2 << 20)
    with_c4 = not args.no_extra
    heap_bytes = 2 * seg_bytes + (2 * c4_bytes if with_c4 else 0)
    state["phase"] = "heap"
    mapped = []
    bases = {}
    heap_base = None
    vmm_err = None
    try:
        heap_base = osgpu.heap_create(heap_bytes, 0, 0, world, psync.value)
    except Exception as e:  # collective: the same verdict on every rank
        vmm_err = repr(e)[:300]
    team_ok = heap_base is not None
    # ---- preflight: every cross-process mapping checked with patterns at
    # both ends of every heap chunk, staging area and flag area, host copy
    # then copy kernel, BEFORE any kernel uses them (osgpu_preflight); a bad
    # mapping becomes a named entry here instead of a GPU fault later
    state["phase"] = "preflight"
    staging_ok = flags_ok = True
    try:
        prc, prep = osgpu.preflight(heap_base, 0, 0, world, psync.value)
        allrep = [None] * world
        dist.all_gather_object(allrep, {"rc": prc, "report": prep})
        res["heap_preflight"] = {str(r): x["report"] for r, x in enumerate(allrep)}
        def failed(region):   # any rank's read or remote-write leg names the region
            return any(region in str(v.get(leg, ""))
                       for x in allrep for k, v in x["report"].items() if isinstance(v, dict)
                       for leg in ("status", "remote_write"))
        heap_bad = failed("heap")
        staging_ok = not failed("staging")
        flags_ok = not failed("flags")
        res["heap_preflight_ok"] = all(x["rc"] == 0 for x in allrep)
        res["heap_preflight_remote_write"] = (
            "ok" if all(v.get("remote_write") == "ok" for x in allrep
                        for k, v in x["report"].items() if isinstance(v, dict))
            else "failed (heap_preflight)")
        if heap_bad and team_ok:
            # do not run kernels through a mapping that failed its probe
            res["heap_error"] = "preflight: some heap chunk mapping failed (heap_preflight)"
            team_ok = False
    except Exception as e:  # report, never hide
        res["heap_preflight"] = {"error": repr(e)[:300]}
        res["heap_preflight_ok"] = False
        staging_ok = flags_ok = False
    if not staging_ok:   # the STAGED legs (push exchange, host heaps) would use it
        res["staging_error"] = ("preflight: a staging-area mapping failed or was not checked; "
                                "the STAGED and push-exchange legs are skipped")
    if not flags_ok:     # the fused one-launch path's barriers live in the flag areas
        res["flags_error"] = ("preflight: a device-barrier flag mapping failed or was not "
                              "checked; the fused path is off for this run")
        L.osgpu_set_fused_max_bytes(0)
    _log(rank, f"preflight ok={res.get('heap_preflight_ok')}")
    if team_ok:
        hsrc = osgpu.device_view(heap_base, seg_bytes)
        htgt = osgpu.device_view(heap_base + seg_bytes, seg_bytes)
        for pe in range(world):
            for s_, off in ((0, 0), (1, seg_bytes)):
                bases[(pe, s_)] = L.osgpu_heap_translate(heap_base + off, rank, pe)
        res["config"]["heap"] = (f"osgpu_heap_create: {heap_bytes} B contiguous per PE "
                                 f"(VMM chunks, dmabuf)")
    else:
        if vmm_err is not None:
            res["heap_error"] = vmm_err
        if heap_base is not None:   # made, but failed its preflight: not used at all
            L.osgpu_heap_destroy(ctypes.c_void_p(heap_base))
            heap_base = None
        hsrc = torch.empty(seg_bytes, dtype=torch.uint8, device=dev)
        htgt = torch.empty(seg_bytes, dtype=torch.uint8, device=dev)
    src = hsrc[: n * 8].view(torch.float64)
    tgt = htgt[: n * 8].view(torch.float64)
    src.uniform_(1.0, 2.0, generator=torch.Generator(device=dev).manual_seed(1000 + rank))
    torch.cuda.synchronize()

    def step():
        fn(tgt.data_ptr(), src.data_ptr(), n, 0, 0, world, wrk, psync)

    if not team_ok:
        state["phase"] = "ipc"
        ok = seg_bytes < (2 << 30)
        handles = []
        for seg in (hsrc, htgt):
            h = (ctypes.c_char * 64)()
            ok = ok and L.osgpu_ipc_get_handle(ctypes.c_void_p(seg.data_ptr()), h) == 0
            handles.append(bytes(h))
        allh = [None] * world
        dist.all_gather_object(allh, handles)
        team_ok = _agree(dist, world, ok)
        if team_ok:
            for pe in range(world):
                for s_, seg in enumerate((hsrc, htgt)):
                    if pe == rank:
                        base = seg.data_ptr()
                    else:
                        base = L.osgpu_ipc_open((ctypes.c_char * 64).from_buffer_copy(allh[pe][s_]))
                        ok = ok and bool(base)
                        if base:
                            mapped.append(base)
                    if base:
                        L.osgpu_heap_register_segment(pe, s_, ctypes.c_void_p(base), seg_bytes)
                        bases[(pe, s_)] = base
            team_ok = _agree(dist, world, ok)
        res["config"]["heap"] = "HIP IPC segments (osgpu_heap_create failed)"
    _log(rank, f"device heaps ready: {team_ok}")

    # ---- primary: exact team kernel over the IPC-mapped heaps
    if team_ok:
        state["phase"] = "team"
        L.osgpu_set_path(osgpu.PATH_P2P)
        t = _timed(step, args.steps, args.warmup, dist, torch)
        res["value"] = args.steps * B / t / GIB
        res["ms_per_step"] = t / args.steps * 1e3
        res["config"]["path"] = "p2p-team (exact owner-computes kernel over the members' mapped heaps, xGMI)"
        res["config"]["algbw_GiBs"] = n * 8 * args.steps / t / GIB
        # the exchange is link-bound: per step GPU g reads shard g of each
        # peer's source (n*8/P bytes per peer) and each peer h writes shard h
        # of g's target: 2*(P-1)*n*8/P bytes arrive at every GPU (and as many
        # leave), 2*n*8/P per link and direction -- the traffic of a
        # reduce-scatter + all-gather over a fully connected fabric
        per_dir = 2 * (world - 1) * (n * 8 // world) * args.steps / t / 1e9
        peak = (world - 1) * XGMI_LINK_GBS
        agg = args.steps * B / t / 1e9
        res["hbm_aggregate"] = {"GBs": agg, "peak_GBs": world * HBM_PEAK_GBS,
                                "frac": agg / (world * HBM_PEAK_GBS),
                                "note": "(P+1)*nreduce*8 bytes per step over all GPUs vs "
                                        "P x 8 TB/s; the exchange is xGMI-bound (roofline)"}
        res["roofline"] = {
            "bound": "xgmi", "achieved": per_dir, "peak": peak, "unit": "GB/s",
            "frac": per_dir / peak, "traffic": None,
            "kernel": (f"osgpu::team_lds_kernel<double, SUM, {world}>"
                       if team_lds(world, remote=res["launch"].get("distinct_gpus", False))
                       else f"osgpu::team_vec_kernel<double, SUM, {world}>"),
            "note": (f"achieved = bytes each GPU receives over its {world - 1} peer link(s) per "
                     f"second: the shard reads from every peer plus every peer's writes of its "
                     f"shard into this GPU's target (it sends as many); peak = {world - 1} x "
                     f"{XGMI_LINK_GBS} GB/s per direction (MI355X xGMI, 153.6 GB/s "
                     f"bidirectional per link)")}
        if ndev < world:  # a rehearsal with ranks sharing GPUs: no xGMI involved
            res["roofline"]["frac"] = None
            res["roofline"]["note"] += "; ranks share a GPU here, so no link is used"
        res["parity_sample"] = _sample_parity(rank, world, src, tgt, n, "sum", dist)
        _log(rank, "team done")
        # ---- the link itself, measured right away (the roofline's peak):
        # every GPU at once copies one chunk per peer with the copy kernel,
        # remote reads and remote writes
        state["phase"] = "xgmi_probe"
        rf = res["roofline"]
        rf["peak_assumed_link_GBs"] = XGMI_LINK_GBS
        try:
            xp = _xgmi_probe(L, torch, dist, rank, world, bases, seg_bytes)
            res["xgmi_probe"] = xp
            link = max(xp["pull_reads_GBs_per_link"], xp["push_writes_GBs_per_link"])
            if ndev >= world:
                # the peak the line's frac is taken against: the measured link
                rf["xgmi_measured"] = {"link_GBs": link, "gpus": "distinct"}
                rf["peak"] = (world - 1) * link
                rf["frac"] = rf["achieved"] / rf["peak"]
                rf["frac_of_assumed_peak"] = rf["achieved"] / ((world - 1) * XGMI_LINK_GBS)
                rf["peak_how"] = ("measured: best of remote reads / remote writes per link per "
                                  "direction, copy kernel, every GPU at once (xgmi_probe)")
            else:  # ranks share a GPU: the probe moved HBM, not a link
                rf["xgmi_measured"] = {"link_GBs": link, "gpus": "shared GPU, not xGMI"}
                rf["peak_how"] = (f"assumed {XGMI_LINK_GBS} GB/s per link per direction; the "
                                  f"probe ran with ranks sharing a GPU (no link)")
            _log(rank, "xgmi probe done")
        except Exception as e:  # the assumed peak stays; reported
            res["xgmi_probe"] = {"error": repr(e)[:300]}
            rf["xgmi_measured"] = None
        # the probe wrote into every target segment: one more call restores
        # the targets the push form below is compared with
        step()
        torch.cuda.synchronize()
        # the push form of the same exchange (remote writes only, staged
        # through the owners' inboxes): same bytes on the links
        state["phase"] = "team_push"
        try:
            if not staging_ok:
                raise RuntimeError("skipped: the staging areas failed their preflight")
            # full-size identity of the two exchange forms: a position-weighted
            # hash of every PE's whole target (verify.hip), before and after
            h_pull = osgpu.checksum("double", osgpu.CK_HASH, tgt.data_ptr(), n)
            L.osgpu_set_team_exchange(1)
            tgt.zero_()
            torch.cuda.synchronize()
            tp = _timed(step, args.steps, args.warmup, dist, torch)
            h_push = osgpu.checksum("double", osgpu.CK_HASH, tgt.data_ptr(), n)
            res["team_push"] = {"value": args.steps * B / tp / GIB,
                                "ms_per_step": tp / args.steps * 1e3,
                                "algbw_GiBs": n * 8 * args.steps / tp / GIB,
                                "xgmi_GBs_per_gpu_per_direction":
                                    2 * (world - 1) * (n * 8 // world) * args.steps / tp / 1e9,
                                "parity_sample": _sample_parity(rank, world, src, tgt, n, "sum",
                                                                dist),
                                "full_target_identical_to_pull_all_ranks":
                                    _agree(dist, world, h_pull == h_push)}
            _log(rank, "team push done")
        except Exception as e:
            res["team_push"] = {"error": repr(e)[:300]}
        finally:
            L.osgpu_set_team_exchange(-1)
    else:
        res["team_error"] = "HIP IPC export/import of the device heaps failed on some rank"

    # ---- the team kernel's two launch shapes over the same heaps (ADVICE
    # r05): every rank launches its shard of the double sum with the local
    # shapes (one-GPU A/Bs: LDS form at 2 members, rounds of 4 at 5-8) and
    # with the remote ones (register form at 2, rounds of 2) that the TEAM
    # path picks when members sit on other GPUs -- kernel only, all ranks at
    # once, max over ranks; bit-identical outputs checked
    if team_ok and not args.no_extra:
        state["phase"] = "team_shapes"
        try:
            res["team_shapes_ab"] = _team_shapes_ab(L, osgpu, torch, dist, rank, world, bases,
                                                    n, tgt)
            _log(rank, "team shapes done")
        except Exception as e:
            res["team_shapes_ab"] = {"error": repr(e)[:300]}

    # ---- the local fold alone on every GPU at once (config 2's kernel: my
    # source + a second resident array, K = 2, NO exchange).  This is not a
    # to_all and earns no scaling credit: it only shows that the per-GPU HBM
    # fold runs at the N = 1 rate while every GPU is busy.  `value` above is
    # the whole to_all, whose exchange is xGMI-bound.
    if not args.no_extra:
        state["phase"] = "local_fold"
        try:
            other = htgt[: n * 8].view(torch.float64)
            other.uniform_(1.0, 2.0, generator=torch.Generator(device=dev).manual_seed(3 + rank))
            lout = torch.empty(n, dtype=torch.float64, device=dev)
            srcs2 = (ctypes.c_void_p * 2)(src.data_ptr(), other.data_ptr())

            def fold_step():
                L.osgpu_combine(5, 0, lout.data_ptr(), srcs2, 2, n, None)

            tl = _timed(fold_step, args.steps, args.warmup, dist, torch)
            ok = bool(torch.equal(lout[:4096], src[:4096] + other[:4096]))
            res["local_fold_no_exchange"] = {
                "GBs_per_gpu": args.steps * 3 * n * 8 / tl / 1e9,
                "frac_of_8TBs_per_gpu": args.steps * 3 * n * 8 / tl / 1e9 / HBM_PEAK_GBS,
                "correct_sample_all_ranks": _agree(dist, world, ok),
                "note": "NOT a to_all (no exchange, no scaling claim): "
                        "combine_lds_kernel<double,SUM,2,2> on every GPU at once, 3*nreduce*8 B "
                        "per GPU per step, max-over-ranks time -- the per-GPU fold rate while "
                        "all GPUs stream"}
            del lout
            torch.cuda.empty_cache()
            _log(rank, "local fold done")
        except Exception as e:
            res["local_fold_no_exchange"] = {"error": repr(e)[:300]}

    # ---- RCCL on the same buffers, then BASELINE config 4 (1 Gi per PE)
    rccl_ok = False
    if not args.no_rccl:
        state["phase"] = "rccl"
        try:
            uid = (ctypes.c_char * 128)()
            if rank == 0:
                assert L.osgpu_rccl_unique_id(uid) == 0
            obj = [bytes(uid)]
            dist.broadcast_object_list(obj, src=0)
            rc = L.osgpu_rccl_init(world, rank, (ctypes.c_char * 128).from_buffer_copy(obj[0]))
            err = L.osgpu_last_error().decode() if rc != 0 else ""
            rccl_ok = _agree(dist, world, rc == 0)
            if not rccl_ok:
                raise RuntimeError(err or "ncclCommInitRank failed on another rank")
            # the communicator as RCCL sees it: ranks and the device of each
            nr, ur, cd = osgpu.rccl_comm_info()
            allc = [None] * world
            dist.all_gather_object(allc, {"rank": ur, "device": cd,
                                          "pci_bus_id": ident.get("pci_bus_id")})
            res["rccl_comm"] = {"nranks": nr, "ranks": allc,
                                "one_rank_per_gpu": len({c["pci_bus_id"] for c in allc}) == nr}
            L.osgpu_set_path(osgpu.PATH_RCCL)
            t2 = _timed(step, args.steps, args.warmup, dist, torch)
            rr = {"value": args.steps * B / t2 / GIB, "ms_per_step": t2 / args.steps * 1e3,
                  "algbw_GiBs": n * 8 * args.steps / t2 / GIB,
                  "path": osgpu.last_path(),
                  "parity_vs_reference_order": _sample_parity(rank, world, src, tgt, n, "sum",
                                                              dist)}
            rr["tolerance"] = _rccl_tolerance(rr["parity_vs_reference_order"], world)
            res["rccl"] = rr
            if res["value"] is None:   # no IPC: RCCL carries the line, flagged
                res["value"], res["ms_per_step"] = rr["value"], rr["ms_per_step"]
                res["config"]["path"] = "rccl (IPC unavailable)"
            _log(rank, "rccl done")
        except Exception as e:  # reported, never hidden
            res["rccl"] = {"error": repr(e)[:300]}
            if 0 < ndev < world:
                res["rccl"]["note"] = ("ranks share a GPU in this run: RCCL refuses more than "
                                       "one rank per GPU, so no RCCL leg can run here")
        # the automatic path's integer dispatch to RCCL, bit-exact vs the oracle
        if rccl_ok:
            state["phase"] = "rccl_integer"
            try:
                res["rccl_integer_auto"] = _rccl_integer_legs(
                    L, osgpu, torch, dist, rank, world, dev, psync, min(n, 16 << 20))
                _log(rank, "rccl integer legs done")
            except Exception as e:  # reported, never hidden
                res["rccl_integer_auto"] = {"error": repr(e)[:300]}
            L.osgpu_set_path(osgpu.PATH_RCCL)
    # ---- BASELINE config 4: double sum, nreduce = 1 Gi (8 GiB per PE) over
    # every GPU.  Exact path: the team kernel over the VMM heaps (each GPU
    # folds its shard of every PE's target in that PE's own order); beside
    # it ncclAllReduce (forced: FP within tolerance, not the reference order).
    if with_c4 and (heap_base is not None or rccl_ok):
        state["phase"] = "config4"
        c4 = {"nreduce": n4, "bytes_per_array": n4 * 8}
        try:
            if heap_base is not None:
                s4 = osgpu.device_view(heap_base + 2 * seg_bytes, n4 * 8).view(torch.float64)
                t4 = osgpu.device_view(heap_base + 2 * seg_bytes + c4_bytes,
                                       n4 * 8).view(torch.float64)
            else:
                s4 = torch.empty(n4, dtype=torch.float64, device=dev)
                t4 = torch.empty(n4, dtype=torch.float64, device=dev)
            s4.uniform_(1.0, 2.0, generator=torch.Generator(device=dev).manual_seed(4000 + rank))
            torch.cuda.synchronize()

            def step4():
                fn(t4.data_ptr(), s4.data_ptr(), n4, 0, 0, world, wrk, psync)

            for name, path, usable in (("team", osgpu.PATH_AUTO, heap_base is not None),
                                       ("rccl", osgpu.PATH_RCCL, rccl_ok)):
                if not usable:
                    continue
                L.osgpu_set_path(path)
                tt = _timed(step4, 3, 1, dist, torch)
                c4[name] = {"path": osgpu.last_path(), "ms_per_call": tt / 3 * 1e3,
                            "value_GiBs": 3 * (world + 1) * n4 * 8 / tt / GIB,
                            "algbw_GiBs": 3 * n4 * 8 / tt / GIB,
                            "xgmi_in_GBs_per_gpu": 3 * 2 * (world - 1) * (n4 * 8 // world) / tt / 1e9,
                            "parity_vs_reference_order":
                                _sample_parity(rank, world, s4, t4, n4, "sum", dist)}
                if name == "rccl":
                    c4[name]["tolerance"] = _rccl_tolerance(
                        c4[name]["parity_vs_reference_order"], world)
                _log(rank, f"config4 {name} done")
            L.osgpu_set_path(osgpu.PATH_AUTO)
            del s4, t4
            torch.cuda.empty_cache()
        except Exception as e:
            c4["error"] = repr(e)[:300]
        res["config4"] = c4

    # ---- BASELINE config 5: float min/max/prod, 128 Mi per PE, sources and
    # targets in pinned HOST memory: H2D + on-GPU exchange + D2H (STAGED path)
    if not args.no_extra:
        state["phase"] = "config5"
        try:
            L.osgpu_set_path(osgpu.PATH_AUTO)
            n5 = args.c5_nreduce
            h5s = torch.empty(n5, dtype=torch.float32).pin_memory()
            h5t = torch.empty(n5, dtype=torch.float32).pin_memory()
            ps = PES.pes_heap(rank) + (1 << 20) - 4096   # symmetric pSync
            g5 = torch.Generator().manual_seed(77 + rank)
            c5 = {"nreduce": n5, "placement": "pinned host memory, STAGED path"}
            if not staging_ok:
                c5["skipped"] = "the staging areas failed their preflight"
            for op, lo, hi in ((("min", -1e3, 1e3), ("max", -1e3, 1e3), ("prod", 0.9, 1.1))
                               if staging_ok else ()):
                h5s.uniform_(lo, hi, generator=g5)
                f5 = getattr(L, f"shmem_float_{op}_to_all")

                def step5():
                    f5(h5t.data_ptr(), h5s.data_ptr(), n5, 0, 0, world, wrk, ps)

                tt = _timed(step5, 3, 1, dist, torch)
                c5[op] = {"ms_per_call": tt / 3 * 1e3,
                          "GiBs_per_PE_incl_H2D_D2H": 3 * n5 * 4 / tt / GIB,
                          "parity": _sample_parity(rank, world, h5s, h5t, n5, op, dist,
                                                   t="float")}
            # the copy-free figure: the same calls on
            # the device heaps, exact team kernel over xGMI
            if team_ok and n5 * 4 <= seg_bytes:
                L.osgpu_set_path(osgpu.PATH_P2P)
                d5s = hsrc[: n5 * 4].view(torch.float32)
                d5t = htgt[: n5 * 4].view(torch.float32)
                gd = torch.Generator(device=dev).manual_seed(97 + rank)
                cf = {"placement": "device heaps (HBM), p2p-team"}
                for op, lo, hi in (("min", -1e3, 1e3), ("max", -1e3, 1e3), ("prod", 0.9, 1.1)):
                    d5s.uniform_(lo, hi, generator=gd)
                    torch.cuda.synchronize()
                    f5 = getattr(L, f"shmem_float_{op}_to_all")

                    def step5d():
                        f5(d5t.data_ptr(), d5s.data_ptr(), n5, 0, 0, world, wrk, psync)

                    tt = _timed(step5d, 3, 1, dist, torch)
                    cf[op] = {"ms_per_call": tt / 3 * 1e3,
                              "GiBs_per_PE": 3 * n5 * 4 / tt / GIB,
                              "parity": _sample_parity(rank, world, d5s, d5t, n5, op, dist,
                                                       t="float")}
                c5["copy_free"] = cf
                L.osgpu_set_path(osgpu.PATH_AUTO)
            res["config5"] = c5
            _log(rank, "config5 done")
        except Exception as e:
            res["config5"] = {"error": repr(e)[:300]}

    # ---- fcollect64 on the same machinery, one PE per
    # GPU -- device heaps over xGMI (COPY path), RCCL allgather, host staging
    if not args.no_extra:
        state["phase"] = "collectives"
        try:
            res["collectives"] = _multi_fcollect(L, osgpu, torch, dist, rank, world, dev, hsrc,
                                                 htgt, n * 8, team_ok, rccl_ok, args, PES,
                                                 staging_ok)
            _log(rank, "collectives done")
        except Exception as e:
            res["collectives"] = {"error": repr(e)[:300]}

    # ---- BASELINE config 1's shape across GPUs: fused one-launch path vs
    # host barriers (DESIGN_HISTORY.md 10)
    if team_ok and not args.no_extra:
        state["phase"] = "small_calls"
        try:
            res["small_calls"] = _multi_small(L, osgpu, torch, dist, rank, world, hsrc, htgt, PES,
                                              flags_ok=flags_ok)
            _log(rank, "small calls done")
        except Exception as e:
            res["small_calls"] = {"error": repr(e)[:300]}

    state["phase"] = "teardown"
    emit()
    L.osgpu_set_path(osgpu.PATH_AUTO)
    dist.barrier()
    for p in mapped:
        L.osgpu_ipc_close(ctypes.c_void_p(p))
    L.osgpu_finalize()
    del hsrc, htgt, src, tgt
    dist.barrier()
    if heap_base is not None:
        L.osgpu_heap_destroy(ctypes.c_void_p(heap_base))
    dist.barrier()
    dist.destroy_process_group()


def device_count_without_hip():
    """GPUs this job may use, counted WITHOUT initialising HIP in this
    process: GPU_MAX_HW_QUEUES (and anything else HIP reads once) must be in
    a rank's environment before its first HIP call, and the launching parent
    must never touch the GPU at all (it only starts and waits for children).
    BENCH_NDEV (set by the launcher for its ranks) wins; otherwise a child
    process asks torch."""
    v = os.environ.get("BENCH_NDEV")
    if v is not None:
        return int(v)
    import subprocess
    r = subprocess.run([sys.executable, "-c",
                        "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=600)
    try:
        return int(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return 0


def hw_queue_cap(world, ndev):
    """Ranks sharing a GPU (a rehearsal on fewer GPUs than ranks): at most
    16 hardware queues on it between them, or its scheduler time-slices
    them in milliseconds (profiles/r02_mp_latency_hwq.jsonl).
    None when every rank has its own GPU (HIP's default stays)."""
    if 0 < ndev < world:
        per_gpu = -(-world // ndev)
        return str(max(1, 16 // per_gpu))
    return None


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv):
    """`python bench.py --gpus N` with no RANK in the environment: start the
    N ranks here, one child process per GPU (the reference's launcher also
    starts its own PEs, src/shmemc/oshrun.in:4), with RANK / LOCAL_RANK /
    WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT set as
    torch.distributed.run would.  This process never touches the GPU (no
    HIP call, no exec after one): it relays rank 0's output and exits with
    the first non-zero rank status, or 1 when no rank printed a JSON line.
    A rank that fails ends the others after a grace period (they may be
    waiting for it in a collective)."""
    import subprocess
    world = max(args.gpus, int(os.environ.get("WORLD_SIZE", "1")))
    ndev = device_count_without_hip()
    env0 = dict(os.environ, WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
                BENCH_NDEV=str(ndev), PYTHONUNBUFFERED="1")
    cap = hw_queue_cap(world, ndev)
    if cap is not None:     # the box may export HIP's default (4): lower it, never raise it
        env0["GPU_MAX_HW_QUEUES"] = str(min(int(cap), int(os.environ.get("GPU_MAX_HW_QUEUES",
                                                                          cap))))
    procs = []
    for r in range(world):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                                      env=env, stdout=subprocess.PIPE, text=True))
    lines = {r: [] for r in range(world)}

    def relay(r, p):
        for line in p.stdout:
            lines[r].append(line)
            if r == 0:                      # rank 0's line is the bench line
                sys.stdout.write(line)
                sys.stdout.flush()
            else:
                sys.stderr.write(f"[bench rank {r} stdout] {line}")
    readers = [threading.Thread(target=relay, args=(r, p), daemon=True)
               for r, p in enumerate(procs)]
    for t in readers:
        t.start()
    limit = time.time() + args.deadline + 300      # the ranks' own watchdog fires first
    grace = float(os.environ.get("BENCH_RANK_GRACE_S", "60"))
    failed_at = None
    while any(p.poll() is None for p in procs):
        now = time.time()
        if failed_at is None and any(p.returncode not in (None, 0) for p in procs):
            failed_at = now
        if now > limit or (failed_at is not None and now - failed_at > grace):
            for p in procs:
                if p.poll() is None:
                    p.kill()
            break
        time.sleep(0.2)
    for p in procs:
        p.wait()
    for t in readers:
        t.join(timeout=10)
    codes = [p.returncode for p in procs]
    bad = [c for c in codes if c != 0]
    has_line = any(l.startswith("{") for l in lines[0])
    if bad or not has_line:
        sys.stderr.write(f"[bench launcher] rank exit codes {codes}; "
                         f"rank 0 printed {'a' if has_line else 'no'} JSON line\n")
    return bad[0] if bad else (0 if has_line else 1)


def dry_rank(args):
    """--dry-ranks: what a rank of launch_ranks() sees, without the GPU:
    join the gloo group through MASTER_ADDR/PORT, gather every rank's
    plumbing, rank 0 prints it as one JSON line (tests/test_bench_contract.py).
    --dry-fail-rank R: rank R exits with status 7 after the gather."""
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    mine = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE",
                                            "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                                            "GPU_MAX_HW_QUEUES", "BENCH_NDEV")}
    mine["pid"] = os.getpid()
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"dry": True, "n_gpus": world, "ranks": allr}), flush=True)
    if rank == args.dry_fail_rank:
        sys.exit(7)


def main():
    args = parse()
    multi = args.gpus > 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1
    if multi and "RANK" not in os.environ:
        sys.exit(launch_ranks(args, sys.argv[1:]))
    if args.dry_ranks:
        dry_rank(args)
    elif multi:
        bench_multi(args)
    else:
        bench_single(args)


if __name__ == "__main__":
    main()
