#!/usr/bin/env python3
"""ld_variants.py -- A/B of long double (x87 soft-float) team-kernel builds:
each variant compiles longdouble.hip against its own x87.hpp into
tools/variants/ld_<name>/libosgpu_reduce.so (linked with the tree's other
objects).  Not part of the product.

  python tools/ld_variants.py build   (here, on the CPU)
      variants: "base" = x87.hpp and longdouble.hip of git HEAD (or
      LDV_BASE=<rev>), "cur" = the tree's, plus any LDV_EXTRA=name=path,...
      (another x87.hpp with the tree's longdouble.hip)
  python tools/ld_variants.py run     (on the GPU box)
      every build loaded into ONE process (RTLD_LOCAL), interleaved launch
      block by launch block on the same arrays (box and allocation effects hit
      them alike): osgpu_team_combine(longdouble, sum|prod, P) over n elements,
      HIP-event spans over REPS launches, LDV_ROUNDS rounds, median per
      variant; HBM bytes 2 * P * n * 16.  Every variant's P outputs must be
      byte-identical to the first variant's (the shipped, GPU-tested build).
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "test-resilient-osss-ucx_amd", "csrc")
VAR = os.path.join(ROOT, "tools", "variants")
FL = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
      "-fno-fast-math"]
OTHERS = ["combine.o", "team.o", "fused.o", "verify.o", "copy.o", "host_fold.o", "runtime.o", "heap.o",
          "shmem_reduce.o", "shmem_collect.o"]


def variants():
    v = {"base": "git:" + os.environ.get("LDV_BASE", "HEAD"), "cur": None}
    for item in filter(None, os.environ.get("LDV_EXTRA", "").split(",")):
        name, path = item.split("=", 1)
        v[name] = path
    return v


def build():
    subprocess.run(["make", "-s", "-j8"], cwd=CSRC, check=True)
    procs = []
    # LDV_BUILD=a,b: build only those (the others' libraries stay as they are)
    only = set(filter(None, os.environ.get("LDV_BUILD", "").split(",")))
    todo = {k: v for k, v in variants().items() if not only or k in only}
    for name, src in todo.items():
        d = os.path.join(VAR, "ld_" + name)
        s = os.path.join(d, "src")
        os.makedirs(s, exist_ok=True)
        for f in ("longdouble.hip", "combine.hpp", "elem_ops.hpp", "x87.hpp"):
            if src is not None and src.startswith("git:") and f in ("longdouble.hip", "x87.hpp"):
                txt = subprocess.run(["git", "show", f"{src[4:]}:test-resilient-osss-ucx_amd/csrc/{f}"],
                                     cwd=ROOT, check=True, capture_output=True).stdout
            elif src is not None and not src.startswith("git:") and f == "x87.hpp":
                txt = open(src, "rb").read()     # a header file; the tree's kernel
            else:
                txt = open(os.path.join(CSRC, f), "rb").read()
            open(os.path.join(s, f), "wb").write(txt)
        procs.append(subprocess.Popen(["/opt/rocm/bin/hipcc"] + FL + ["-c", os.path.join(s, "longdouble.hip"),
                                                                      "-o", os.path.join(d, "longdouble.o")]))
    assert all(p.wait() == 0 for p in procs)
    for name in todo:
        d = os.path.join(VAR, "ld_" + name)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                        os.path.join(d, "libosgpu_reduce.so"), os.path.join(d, "longdouble.o")] +
                       [os.path.join(CSRC, o) for o in OTHERS] + ["-lrccl", "-ldl", "-lpthread"],
                       check=True)
        print("built", name)


def run():
    import ctypes
    import torch
    torch.cuda.init()
    names = os.environ.get("LDV_NAMES", ",".join(variants())).split(",")
    libs = {}
    for name in names:
        L = ctypes.CDLL(os.path.join(VAR, "ld_" + name, "libosgpu_reduce.so"), mode=os.RTLD_LOCAL)
        L.osgpu_team_combine.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        libs[name] = L
    reps = int(os.environ.get("REPS", "10"))
    rounds = int(os.environ.get("LDV_ROUNDS", "5"))
    n = int(os.environ.get("LD_N", str(8 << 20)))
    st = torch.cuda.Stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(5)
    out = open(os.path.join(ROOT, "gpurun_out", "ld_variants.jsonl"), "a")
    for op_name, op in (("sum", 0), ("prod", 1)):
        for dist in ("random", "positive", "ones"):
            for P in (4, 8):
                srcs = []
                for _ in range(P):
                    v = torch.empty((n, 2), dtype=torch.int64, device=dev)
                    if dist == "ones":
                        v[:, 0] = -(1 << 63)
                        v[:, 1] = 0x3fff
                    else:
                        v[:, 0] = torch.randint(-(1 << 62), 1 << 62, (n,), device=dev,
                                                generator=g) | (-(1 << 63))
                        e = 0x3fff + torch.randint(-3, 4, (n,), device=dev, generator=g)
                        sgn = torch.randint(0, 2, (n,), device=dev, generator=g) << 15
                        v[:, 1] = e | (sgn if dist == "random" else 0)
                    srcs.append(v)
                # one set of targets for every variant (the placement of 2P
                # arrays moves the rate by several %)
                outs = [torch.zeros((n, 2), dtype=torch.int64, device=dev) for _ in range(P)]
                S = (ctypes.c_void_p * P)(*[x.data_ptr() for x in srcs])
                D = (ctypes.c_void_p * P)(*[y.data_ptr() for y in outs])
                torch.cuda.synchronize()   # the fills ran on the default stream
                ref, same = None, {}
                for name, L in libs.items():
                    for y in outs:
                        y.zero_()
                    torch.cuda.synchronize()
                    assert L.osgpu_team_combine(6, op, P, D, S, n, sp) == 0
                    torch.cuda.synchronize()
                    # 10 value bytes per element: the significand and the
                    # sign/exponent word
                    got = [torch.stack([y[:, 0], y[:, 1] & 0xffff], 1) for y in outs]
                    if ref is None:
                        ref = got
                    same[name] = all(torch.equal(a, b) for a, b in zip(ref, got))
                del ref, got
                times = {name: [] for name in names}
                for _ in range(rounds):
                    for name, L in libs.items():
                        e0 = torch.cuda.Event(enable_timing=True)
                        e1 = torch.cuda.Event(enable_timing=True)
                        e0.record(st)
                        for _ in range(reps):
                            L.osgpu_team_combine(6, op, P, D, S, n, sp)
                        e1.record(st)
                        e1.synchronize()
                        times[name].append(e0.elapsed_time(e1) * 1e3 / reps)
                for name in names:
                    us = sorted(times[name])[len(times[name]) // 2]
                    line = json.dumps({"variant": name, "op": op_name, "dist": dist, "P": P, "n": n,
                                       "us": us, "frac_of_8TBs": 2 * P * n * 16 / us / 8e6,
                                       "spread_us": [min(times[name]), max(times[name])],
                                       "identical_to_" + names[0]: same[name]})
                    print(line, flush=True)
                    out.write(line + "\n")
                del srcs, outs
                torch.cuda.empty_cache()


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
