#!/usr/bin/env python3
"""team_variants.py -- A/B of team-kernel builds over every type at 2, 4
and 8 members.  Not part of the product.

  python tools/team_variants.py build      (here, on the CPU)
      compiles team.hip (and combine.hip) with each variant's -D flags into
      tools/variants/<name>/libosgpu_reduce.so, linked with the tree's other
      objects; "git:<rev>" variants take team.hip/combine.hip/elem_ops.hpp
      from that revision (the baseline before a change)
  python tools/team_variants.py build_copy / run_copy
      the same for copy.hip (COPY_VARIANTS): the collectives' copy kernel
      with P ranges of 64 MiB and 512 MiB (osgpu_copy), interleaved rounds
  python tools/team_variants.py run        (on the GPU box)
      every build loaded into one process, interleaved on the same arrays:
      team_vec_kernel through osgpu_team_combine, one launch over n elements
      per member, HIP-event spans over REPS launches, TV_ROUNDS rounds; one
      JSON line per (variant, type, P) with the median and the fraction of
      8 TB/s for 2*P*n*s bytes.
"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "test-resilient-osss-ucx_amd", "csrc")
VAR = os.path.join(ROOT, "tools", "variants")
VARLIB = os.path.join(ROOT, "tools", "varlib")
FL = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
      "-fno-fast-math"]
VARIANTS = {
    "r03": ("git:5c84853", []),                       # round 3's shipped team kernel
    "tree": (None, ["-DOSGPU_TEAM_PIPE=0", "-DOSGPU_TEAM_PEROUT=0"]),  # r04 shape, r03 order
    "gh1": (None, ["-DOSGPU_TEAM_GH=1", "-DOSGPU_TEAM_PIPE=0", "-DOSGPU_TEAM_PEROUT=0"]),
    "pipe_g1": (None, ["-DOSGPU_TEAM_PIPE=1", "-DOSGPU_TEAM_G8=1", "-DOSGPU_TEAM_GH=1",
                       "-DOSGPU_TEAM_PEROUT=0"]),
    "perout": (None, ["-DOSGPU_TEAM_PEROUT=1", "-DOSGPU_TEAM_PIPE=0"]),
    "tree2": (None, ["-DOSGPU_TEAM_LDS_MIN_P=9"]),    # register form at every P
    "final": (None, []),                              # the tree's defaults
    "final2": (None, []),                             # duplicate build (control)
    "g8_4": (None, ["-DOSGPU_TEAM_G8=4"]),            # 8 members: all 4 x 8 vectors in flight
    # (a two-half LDS tile, OSGPU_TEAM_LDS_SPLIT, measured equal to one and
    # was removed: profiles/r04_team_place_4.jsonl)
    "lds8": (None, ["-DOSGPU_TEAM_LDS_MAX_P=8"]),      # LDS form at 3-8 members
    # (round 4 also measured 2 / 4 members per wave in the LDS form,
    # OSGPU_TEAM_LDS_K, since removed: profiles/r04_team_place_2/3.jsonl)
    # (round 4 also measured a persistent LDS form, OSGPU_TEAM_LDS_PERSIST,
    # since removed: profiles/r04_team_sweep_4.jsonl)
    "lds5": (None, ["-DOSGPU_TEAM_LDS_MIN_P=5"]),
    "lds2": (None, ["-DOSGPU_TEAM_LDS_MIN_P=2"]),
    "lds5u2": (None, ["-DOSGPU_TEAM_LDS_MIN_P=5", "-DOSGPU_TEAM_LDS_U=2"]),
    "lds5u8": (None, ["-DOSGPU_TEAM_LDS_MIN_P=5", "-DOSGPU_TEAM_LDS_U=8"]),
    "u8_pipe_g2": (None, ["-DOSGPU_TEAM_PIPE=1", "-DOSGPU_TEAM_U8=8", "-DOSGPU_TEAM_G8=2",
                          "-DOSGPU_TEAM_GH=1", "-DOSGPU_TEAM_PEROUT=0"]),
}
if os.environ.get("TV_BUILD"):
    VARIANTS = {k: v for k, v in VARIANTS.items() if k in os.environ["TV_BUILD"].split(",")}
COPY_VARIANTS = {
    "blocked": "git:281a986",   # ranges one after another (before round 3's round-robin)
    "roundrobin": None,         # the tree's copy.hip
}
OTHERS = ["fused.o", "verify.o", "longdouble.o", "copy.o", "runtime.o", "heap.o",
          "shmem_reduce.o", "shmem_collect.o"]


def build():
    if not os.environ.get("TV_NO_MAKE"):   # (TV_NO_MAKE: the tree's objects as they are)
        subprocess.run(["make", "-s", "-j8"], cwd=CSRC, check=True)
    procs = []
    for name, (rev, flags) in VARIANTS.items():
        d = os.path.join(VAR, name)
        os.makedirs(d, exist_ok=True)
        src = CSRC
        if rev:
            src = os.path.join(d, "src")
            os.makedirs(src, exist_ok=True)
            for f in ("team.hip", "combine.hip", "elem_ops.hpp", "combine.hpp"):
                txt = subprocess.run(["git", "show", f"{rev[4:]}:test-resilient-osss-ucx_amd/csrc/{f}"],
                                     cwd=ROOT, check=True, capture_output=True).stdout
                open(os.path.join(src, f), "wb").write(txt)
        for f in ("team", "combine"):
            tmp = os.path.join(d, "tmp_" + f)
            os.makedirs(tmp, exist_ok=True)
            procs.append(subprocess.Popen(["/opt/rocm/bin/hipcc"] + FL + flags +
                                          ["--save-temps", "-c", os.path.join(src, f + ".hip"),
                                           "-o", os.path.join(d, f + ".o")], cwd=tmp))
    assert all(p.wait() == 0 for p in procs)
    for name in VARIANTS:   # register table of every team kernel (tools/isa/reg_table.py)
        d = os.path.join(VAR, name)
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "isa", "reg_table.py"),
                        os.path.join(d, "tmp_team", "team-hip-amdgcn-amd-amdhsa-gfx950.s"),
                        "team_vec_kernel", "--json", os.path.join(d, "regs.jsonl")],
                       check=True, capture_output=True)
    for name in VARIANTS:
        d = os.path.join(VAR, name)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                        os.path.join(d, "libosgpu_reduce.so"), os.path.join(d, "team.o"),
                        os.path.join(d, "combine.o")] + [os.path.join(CSRC, o) for o in OTHERS] +
                       ["-lrccl", "-ldl", "-lpthread"], check=True)
        # tools/variants/ stays here (.gpurunignore: the save-temps are
        # hundreds of MB); the library and its register table travel
        lib = os.path.join(VARLIB, name)
        os.makedirs(lib, exist_ok=True)
        for f in ("libosgpu_reduce.so", "regs.jsonl"):
            shutil.copy(os.path.join(d, f), lib)
        print("built", name)


def run():
    """Every variant loaded into ONE process (each build its own module,
    RTLD_LOCAL), the variants interleaved launch block by launch block on the
    same arrays: box and allocation effects hit them alike.  Per (type, P):
    TV_ROUNDS rounds of (for each variant: a HIP-event span over REPS
    launches); the median per variant."""
    import ctypes
    import torch
    torch.cuda.init()
    names = os.environ.get("TV_NAMES", ",".join(VARIANTS)).split(",")
    libs = {}
    for name in names:
        L = ctypes.CDLL(os.path.join(VARLIB, name, "libosgpu_reduce.so"), mode=os.RTLD_LOCAL)
        L.osgpu_team_combine.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        libs[name] = L
    reps = int(os.environ.get("REPS", "10"))
    rounds = int(os.environ.get("TV_ROUNDS", "5"))
    st = torch.cuda.Stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    types = (("double", 5, torch.float64), ("float", 4, torch.float32),
             ("int", 1, torch.int32), ("short", 0, torch.int16), ("long", 2, torch.int64),
             ("complexf", 7, torch.complex64), ("complexd", 8, torch.complex128))
    only = os.environ.get("TV_TYPES")
    nbytes = int(os.environ.get("TV_BYTES", str(512 << 20)))
    for P in (2, 4, 8):
        for t, code, dt in types:
            if only and t not in only.split(","):
                continue
            es = torch.empty(0, dtype=dt).element_size()
            n = nbytes // es
            g = torch.Generator(device="cuda").manual_seed(5)
            xs = []
            for _ in range(P):
                x = torch.empty(n, dtype=dt, device="cuda")
                if dt.is_floating_point or dt.is_complex:
                    x.view(torch.float32 if dt in (torch.float32, torch.complex64)
                           else torch.float64).uniform_(1, 2, generator=g)
                else:
                    x.random_(-100, 100, generator=g)
                xs.append(x)
            ys = [torch.empty(n, dtype=dt, device="cuda") for _ in range(P)]
            S = (ctypes.c_void_p * P)(*[x.data_ptr() for x in xs])
            D = (ctypes.c_void_p * P)(*[y.data_ptr() for y in ys])
            acc = xs[0].clone()
            for x in xs[1:]:
                acc = acc + x
            torch.cuda.synchronize()
            times = {name: [] for name in names}
            exact = {}
            for name, L in libs.items():
                for _ in range(2):
                    assert L.osgpu_team_combine(code, 0, P, D, S, n, sp) == 0
                torch.cuda.synchronize()
                # member 0's result: x0 + x1 + ... in order (complexf: the
                # compiled order adds imaginary parts as b.im + a.im -- same
                # values for these finite inputs)
                exact[name] = bool(torch.equal(ys[0], acc))
            for _ in range(rounds):
                for name, L in libs.items():
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    for _ in range(reps):
                        L.osgpu_team_combine(code, 0, P, D, S, n, sp)
                    e1.record(st)
                    e1.synchronize()
                    times[name].append(e0.elapsed_time(e1) * 1e3 / reps)
            for name in names:
                us = sorted(times[name])[len(times[name]) // 2]
                print(json.dumps({"variant": name, "type": t, "P": P, "n": n, "us": us,
                                  "frac": 2 * P * n * es / us / 8e6,
                                  "spread_us": [min(times[name]), max(times[name])],
                                  "member0_exact": exact[name]}), flush=True)
            del xs, ys, acc
            torch.cuda.empty_cache()


def run_sweep():
    """Every (type, op) at every P in TV_PS, every variant library in
    TV_NAMES loaded into one process and interleaved round by round with
    the same-mix copy ceiling (osgpu_copy: P ranges of n*s bytes in one
    launch, the copy kernel's round-robin tiles -- P read and P write streams
    over the same bytes, nothing folded).  Inputs: products in [0.9, 1.1)
    (no overflow over 8 factors), sums in [-1.5, 1.5), min/max in
    [-1e3, 1e3), integers random bits; no NaN.  Every variant's P outputs
    are compared byte for byte with the first variant's.  One JSON line per
    (type, op, P, variant) on stdout and in gpurun_out/team_sweep.jsonl."""
    import ctypes
    import torch
    torch.cuda.init()
    names = os.environ.get("TV_NAMES", ",".join(VARIANTS)).split(",")
    libs = {}
    for name in names:
        L = ctypes.CDLL(os.path.join(VARLIB, name, "libosgpu_reduce.so"), mode=os.RTLD_LOCAL)
        L.osgpu_team_combine.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.osgpu_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                 ctypes.c_void_p]
        libs[name] = L
    C = libs[names[0]]
    reps = int(os.environ.get("REPS", "5"))
    rounds = int(os.environ.get("TV_ROUNDS", "5"))
    nbytes = int(os.environ.get("TV_BYTES", str(512 << 20)))
    PS = [int(p) for p in os.environ.get("TV_PS", "2,4,5,6,7,8").split(",")]
    types = {"short": (0, 2, "i"), "int": (1, 4, "i"), "long": (2, 8, "i"), "float": (4, 4, "f"),
             "double": (5, 8, "d"), "complexf": (7, 8, "f"), "complexd": (8, 16, "d")}
    ops = {"sum": 0, "prod": 1, "and": 2, "or": 3, "xor": 4, "max": 5, "min": 6}
    only = os.environ.get("TV_TYPES")
    only_ops = os.environ.get("TV_OPS")
    st = torch.cuda.Stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    srcs = [torch.empty(nbytes, dtype=torch.uint8, device="cuda") for _ in range(8)]
    dsts = {k: [torch.empty(nbytes, dtype=torch.uint8, device="cuda") for _ in range(8)]
            for k in ("first", "other")}
    g = torch.Generator(device="cuda").manual_seed(17)
    outf = open(os.path.join(ROOT, "gpurun_out", "team_sweep.jsonl"), "a")
    for t, (code, es, kind) in types.items():
        if only and t not in only.split(","):
            continue
        n = nbytes // es
        for op, oc in ops.items():
            if kind != "i" and op in ("and", "or", "xor"):
                continue
            if t.startswith("complex") and op in ("max", "min"):
                continue
            if only_ops and op not in only_ops.split(","):
                continue
            for b in srcs:
                if kind == "i":
                    b.view(torch.int32).random_(generator=g)
                else:
                    v = b.view(torch.float32 if kind == "f" else torch.float64)
                    lo, hi = {"prod": (0.9, 1.1), "sum": (-1.5, 1.5)}.get(op, (-1e3, 1e3))
                    v.uniform_(lo, hi, generator=g)
            for P in PS:
                S = (ctypes.c_void_p * P)(*[x.data_ptr() for x in srcs[:P]])
                # variants 2.. write into the second output set (compared
                # with the first variant's after their first launches)
                D0 = (ctypes.c_void_p * P)(*[x.data_ptr() for x in dsts["first"][:P]])
                D1 = (ctypes.c_void_p * P)(*[x.data_ptr() for x in dsts["other"][:P]])
                N = (ctypes.c_size_t * P)(*([n * es] * P))
                torch.cuda.synchronize()
                equal = {}
                for i, name in enumerate(names):
                    D = D0 if i == 0 else D1
                    for _ in range(2):
                        assert libs[name].osgpu_team_combine(code, oc, P, D, S, n, sp) == 0
                    st.synchronize()
                    if i > 0:
                        equal[name] = all(torch.equal(dsts["first"][q], dsts["other"][q])
                                          for q in range(P))
                for _ in range(2):
                    assert C.osgpu_copy(D1, S, N, P, sp) == 0
                times = {name: [] for name in names + ["copy"]}
                order = names + ["copy"]
                for rnd in range(rounds):
                    # rotated each round: a fixed order biased identical
                    # kernels by up to 4 % by position (r04_team_place_2)
                    for name in order[rnd % len(order):] + order[:rnd % len(order)]:
                        e0 = torch.cuda.Event(enable_timing=True)
                        e1 = torch.cuda.Event(enable_timing=True)
                        e0.record(st)
                        for _ in range(reps):
                            if name == "copy":
                                C.osgpu_copy(D1, S, N, P, sp)
                            else:
                                libs[name].osgpu_team_combine(code, oc, P, D1, S, n, sp)
                        e1.record(st)
                        e1.synchronize()
                        times[name].append(e0.elapsed_time(e1) * 1e3 / reps)
                B = 2 * P * n * es
                cus = sorted(times["copy"])[rounds // 2]
                for name in names:
                    us = sorted(times[name])[rounds // 2]
                    rec = {"type": t, "op": op, "P": P, "variant": name, "n": n, "us": us,
                           "frac": B / us / 8e6, "copy_us": cus, "copy_frac": B / cus / 8e6,
                           "frac_of_copy": cus / us,
                           "spread_us": [min(times[name]), max(times[name])],
                           "equal_to_" + names[0]: equal.get(name, True)}
                    print(json.dumps(rec), flush=True)
                    outf.write(json.dumps(rec) + "\n")
                outf.flush()


def run_place():
    """The team kernel's form against placement: double sum at P in TV_PS
    (default 4, 8), TV_TRIALS fresh allocations (2P arrays of n = 64 Mi
    doubles, as bench.py's roofline_team_by_members), every variant in
    TV_NAMES and the same-mix copy interleaved on each allocation, TV_ROUNDS
    event spans of REPS launches each.  One JSON line per (P, trial,
    variant); gpurun_out/team_place.jsonl."""
    import ctypes
    import torch
    torch.cuda.init()
    names = os.environ.get("TV_NAMES", "final,tree2").split(",")
    libs = {}
    for name in names:
        L = ctypes.CDLL(os.path.join(VARLIB, name, "libosgpu_reduce.so"), mode=os.RTLD_LOCAL)
        L.osgpu_team_combine.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.osgpu_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                 ctypes.c_void_p]
        libs[name] = L
    C = libs[names[0]]
    reps = int(os.environ.get("REPS", "5"))
    rounds = int(os.environ.get("TV_ROUNDS", "5"))
    trials = int(os.environ.get("TV_TRIALS", "5"))
    n = int(os.environ.get("TV_N", str(64 << 20)))
    st = torch.cuda.Stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    outf = open(os.path.join(ROOT, "gpurun_out", "team_place.jsonl"), "a")
    for P in [int(p) for p in os.environ.get("TV_PS", "4,8").split(",")]:
        for trial in range(trials):
            g = torch.Generator(device="cuda").manual_seed(100 * P + trial)
            srcs = [torch.empty(n, dtype=torch.float64, device="cuda").uniform_(1, 2, generator=g)
                    for _ in range(P)]
            dsts = [torch.empty(n, dtype=torch.float64, device="cuda") for _ in range(P)]
            S = (ctypes.c_void_p * P)(*[x.data_ptr() for x in srcs])
            D = (ctypes.c_void_p * P)(*[x.data_ptr() for x in dsts])
            N = (ctypes.c_size_t * P)(*([n * 8] * P))
            torch.cuda.synchronize()
            for name in names:
                assert libs[name].osgpu_team_combine(5, 0, P, D, S, n, sp) == 0
            assert C.osgpu_copy(D, S, N, P, sp) == 0
            st.synchronize()
            times = {name: [] for name in names + ["copy"]}
            order = names + ["copy"]
            for rnd in range(rounds):
                for name in order[rnd % len(order):] + order[:rnd % len(order)]:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    for _ in range(reps):
                        if name == "copy":
                            C.osgpu_copy(D, S, N, P, sp)
                        else:
                            libs[name].osgpu_team_combine(5, 0, P, D, S, n, sp)
                    e1.record(st)
                    e1.synchronize()
                    times[name].append(e0.elapsed_time(e1) * 1e3 / reps)
            B = 2 * P * n * 8
            cus = sorted(times["copy"])[rounds // 2]
            for name in names:
                us = sorted(times[name])[rounds // 2]
                rec = {"P": P, "trial": trial, "variant": name, "us": us, "frac": B / us / 8e6,
                       "copy_frac": B / cus / 8e6, "frac_of_copy": cus / us}
                print(json.dumps(rec), flush=True)
                outf.write(json.dumps(rec) + "\n")
            outf.flush()
            del srcs, dsts
            torch.cuda.empty_cache()


def build_copy():
    subprocess.run(["make", "-s", "-j8"], cwd=CSRC, check=True)
    others = ["combine.o", "team.o", "fused.o", "verify.o", "longdouble.o", "runtime.o", "heap.o",
              "shmem_reduce.o", "shmem_collect.o"]
    for name, rev in COPY_VARIANTS.items():
        d = os.path.join(VAR, "copy_" + name)
        os.makedirs(d, exist_ok=True)
        src = os.path.join(CSRC, "copy.hip")
        if rev:
            src = os.path.join(d, "copy.hip")
            for f in ("copy.hip", "combine.hpp"):
                txt = subprocess.run(["git", "show", f"{rev[4:]}:test-resilient-osss-ucx_amd/csrc/{f}"],
                                     cwd=ROOT, check=True, capture_output=True).stdout
                open(os.path.join(d, f), "wb").write(txt)
        subprocess.run(["/opt/rocm/bin/hipcc"] + FL + ["-c", src, "-o", os.path.join(d, "copy.o")],
                       check=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                        os.path.join(d, "libosgpu_reduce.so"), os.path.join(d, "copy.o")] +
                       [os.path.join(CSRC, o) for o in others] + ["-lrccl", "-ldl", "-lpthread"],
                       check=True)
        print("built", name)


def run_copy():
    import ctypes
    import torch
    torch.cuda.init()
    libs = {}
    for name in COPY_VARIANTS:
        L = ctypes.CDLL(os.path.join(VAR, "copy_" + name, "libosgpu_reduce.so"), mode=os.RTLD_LOCAL)
        L.osgpu_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                 ctypes.c_void_p]
        libs[name] = L
    reps = int(os.environ.get("REPS", "10"))
    rounds = int(os.environ.get("TV_ROUNDS", "7"))
    st = torch.cuda.Stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    for nb in (64 << 20, 512 << 20):
        for P in (2, 4, 8):
            src = [torch.empty(nb, dtype=torch.uint8, device="cuda").random_(0, 255) for _ in range(P)]
            dst = [torch.empty(nb, dtype=torch.uint8, device="cuda") for _ in range(P)]
            S = (ctypes.c_void_p * P)(*[x.data_ptr() for x in src])
            D = (ctypes.c_void_p * P)(*[x.data_ptr() for x in dst])
            N = (ctypes.c_size_t * P)(*([nb] * P))
            torch.cuda.synchronize()
            times = {name: [] for name in libs}
            for name, L in libs.items():
                for _ in range(2):
                    assert L.osgpu_copy(D, S, N, P, sp) == 0
            torch.cuda.synchronize()
            ok = all(torch.equal(a, b) for a, b in zip(src, dst))
            for _ in range(rounds):
                for name, L in libs.items():
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    for _ in range(reps):
                        L.osgpu_copy(D, S, N, P, sp)
                    e1.record(st)
                    e1.synchronize()
                    times[name].append(e0.elapsed_time(e1) * 1e3 / reps)
            for name in libs:
                us = sorted(times[name])[len(times[name]) // 2]
                print(json.dumps({"variant": name, "ranges": P, "bytes_per_range": nb, "us": us,
                                  "frac": 2 * P * nb / us / 8e6,
                                  "spread_us": [min(times[name]), max(times[name])],
                                  "exact": ok}), flush=True)
            del src, dst
            torch.cuda.empty_cache()


if __name__ == "__main__":
    {"build": build, "run": run, "run_sweep": run_sweep, "run_place": run_place,
     "build_copy": build_copy,
     "run_copy": run_copy}[sys.argv[1]]()
