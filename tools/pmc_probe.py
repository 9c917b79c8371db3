#!/usr/bin/env python3
"""The kernels bench.py's N = 1 line prices, launched bare for a PMC pass.

bench.py runs this as a child process under `rocprofv3 --pmc FETCH_SIZE` and
again under `--pmc WRITE_SIZE` (the two do not fit one pass), so the line's
roofline.traffic is measured in the same run that times the kernels, not
looked up from profiles/.  Every launch goes through the C ABI of the
in-tree library (osgpu_combine / osgpu_team_combine), on the same shapes the
bench times:

  combine  combine_lds_kernel<double, SUM, 2, 2>: 2 sources -> 1 target, n doubles
  team P   the team kernel for P members (double sum, team.hip's form for P),
           P sources -> P targets, n doubles each

No torch: device memory from the HIP runtime the library is linked to.

usage: pmc_probe.py NREDUCE REPS [P ...]      (default P: 2 4 8)
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get("OSGPU_LIB_PATH") or os.path.join(
    ROOT, "test-resilient-osss-ucx_amd", "libosgpu_reduce.so")
T_DOUBLE, OP_SUM = 5, 0


def main():
    n = int(sys.argv[1])
    reps = int(sys.argv[2])
    members = [int(p) for p in sys.argv[3:]] or [2, 4, 8]
    L = ctypes.CDLL(LIB, mode=ctypes.RTLD_GLOBAL)
    H = ctypes.CDLL("libamdhip64.so.7")  # the runtime L is linked to (already loaded)
    vp = ctypes.c_void_p
    H.hipMalloc.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t]
    H.hipMemset.argtypes = [vp, ctypes.c_int, ctypes.c_size_t]
    H.hipFree.argtypes = [vp]
    L.osgpu_combine.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_int,
                                ctypes.c_size_t, vp]
    L.osgpu_team_combine.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp,
                                     ctypes.c_size_t, vp]
    L.osgpu_last_error.restype = ctypes.c_char_p
    nb = n * 8

    def alloc(k, byte0):
        out = []
        for i in range(k):
            p = vp()
            if H.hipMalloc(ctypes.byref(p), nb) != 0:
                sys.exit(f"hipMalloc of {nb} bytes failed")
            # finite positive doubles, a different pattern per array
            # (0x3f3f... ~ 4.8e-4, 0x3e3e... ~ 1.1e-8, ...)
            if H.hipMemset(p, byte0 - i if byte0 else 0, nb) != 0:
                sys.exit("hipMemset failed")
            out.append(p)
        if H.hipDeviceSynchronize() != 0:  # the launches below go to a non-blocking stream
            sys.exit("hipDeviceSynchronize failed")
        return out

    def check(rc):
        if rc != 0:
            sys.exit(L.osgpu_last_error().decode())

    src = alloc(2, 0x3f)
    dst = alloc(1, 0)
    srcs = (vp * 2)(*[p.value for p in src])
    for _ in range(reps):
        check(L.osgpu_combine(T_DOUBLE, OP_SUM, dst[0], srcs, 2, n, None))
    check(H.hipDeviceSynchronize())
    for p in src + dst:
        H.hipFree(p)
    for P in members:
        src = alloc(P, 0x3f)
        dst = alloc(P, 0)
        S = (vp * P)(*[p.value for p in src])
        D = (vp * P)(*[p.value for p in dst])
        for _ in range(reps):
            check(L.osgpu_team_combine(T_DOUBLE, OP_SUM, P, D, S, n, None))
        check(H.hipDeviceSynchronize())
        for p in src + dst:
            H.hipFree(p)
    print(f"pmc_probe: combine + team {members}, n={n}, {reps} launches each", flush=True)


if __name__ == "__main__":
    main()
