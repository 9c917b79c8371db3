#!/usr/bin/env python3
"""combine_variants.py -- A/B of combine-kernel builds (csrc/combine.hip with
different -D flags) loaded into ONE process and interleaved launch block by
launch block on the same arrays.  Not part of the product.

  python tools/combine_variants.py build   (here, on the CPU)
  python tools/combine_variants.py run     (on the GPU box)

Variants: CV_VARIANTS="name=-DFLAG=V -DFLAG2=W;name2=..." (default: the
tree's build vs OSGPU_COMBINE_G8=2 and =1).  Per (type, K): CV_ROUNDS rounds
of (for each variant: a HIP-event span over REPS launches), the median per
variant, (K + 1) * n * s bytes per launch; every variant's output must equal
the first variant's.
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
OTHERS = ["team.o", "fused.o", "verify.o", "longdouble.o", "copy.o", "runtime.o", "heap.o",
          "shmem_reduce.o", "shmem_collect.o"]


def variants():
    spec = os.environ.get("CV_VARIANTS", "base=;g2=-DOSGPU_COMBINE_G8=2;g1=-DOSGPU_COMBINE_G8=1")
    out = {}
    for item in filter(None, spec.split(";")):
        name, flags = item.split("=", 1)
        out[name] = flags.split()
    return out


def build():
    subprocess.run(["make", "-s", "-j8"], cwd=CSRC, check=True)
    procs = []
    for name, flags in variants().items():
        d = os.path.join(VAR, "cv_" + name)
        os.makedirs(d, exist_ok=True)
        procs.append(subprocess.Popen(["/opt/rocm/bin/hipcc"] + FL + flags +
                                      ["-c", os.path.join(CSRC, "combine.hip"), "-o",
                                       os.path.join(d, "combine.o")]))
    assert all(p.wait() == 0 for p in procs)
    for name in variants():
        d = os.path.join(VAR, "cv_" + name)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                        os.path.join(d, "libosgpu_reduce.so"), os.path.join(d, "combine.o")] +
                       [os.path.join(CSRC, o) for o in OTHERS] + ["-lrccl", "-ldl", "-lpthread"],
                       check=True)
        print("built", name)


def run():
    import ctypes
    import torch
    torch.cuda.init()
    names = list(variants())
    libs = {}
    for name in names:
        L = ctypes.CDLL(os.path.join(VAR, "cv_" + name, "libosgpu_reduce.so"), mode=os.RTLD_LOCAL)
        L.osgpu_combine.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
        libs[name] = L
    reps = int(os.environ.get("REPS", "10"))
    rounds = int(os.environ.get("CV_ROUNDS", "7"))
    nbytes = int(os.environ.get("CV_BYTES", str(512 << 20)))
    st = torch.cuda.Stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    out = open(os.path.join(ROOT, "gpurun_out", "combine_variants.jsonl"), "a")
    g = torch.Generator(device="cuda").manual_seed(7)
    bufs = [torch.empty(nbytes, dtype=torch.uint8, device="cuda") for _ in range(9)]
    for b in bufs[:8]:
        b.view(torch.float64).uniform_(1, 2, generator=g)
    o = bufs[8]
    for t, code, es in (("double", 5, 8), ("float", 4, 4), ("int", 1, 4)):
        for K in (2, 4, 6, 7, 8):
            n = nbytes // es
            S = (ctypes.c_void_p * K)(*[bufs[j].data_ptr() for j in range(K)])
            torch.cuda.synchronize()
            ref, same = None, {}
            for name, L in libs.items():
                o.zero_()
                torch.cuda.synchronize()
                assert L.osgpu_combine(code, 0, o.data_ptr(), S, K, n, sp) == 0
                torch.cuda.synchronize()
                if ref is None:
                    ref = o.clone()
                same[name] = bool(torch.equal(o, ref))
            del ref
            times = {name: [] for name in names}
            for _ in range(rounds):
                for name, L in libs.items():
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    for _ in range(reps):
                        L.osgpu_combine(code, 0, o.data_ptr(), S, K, n, sp)
                    e1.record(st)
                    e1.synchronize()
                    times[name].append(e0.elapsed_time(e1) * 1e3 / reps)
            for name in names:
                us = sorted(times[name])[len(times[name]) // 2]
                line = json.dumps({"variant": name, "type": t, "K": K, "n": n, "us": us,
                                   "frac_of_8TBs": (K + 1) * n * es / us / 8e6,
                                   "spread_us": [min(times[name]), max(times[name])],
                                   "identical_to_" + names[0]: same[name]})
                print(line, flush=True)
                out.write(line + "\n")


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
