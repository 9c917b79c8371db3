#!/usr/bin/env python3
"""In-process A/B of two builds of the team kernel on the SAME arrays:
the shipped library and a variant (argv[1]) are both loaded RTLD_LOCAL, so
every trial (a fresh allocation of P sources and P targets, double sum, n
elements each) times A, B and the same-mix copy interleaved, twice.  One
JSON line per (P, trial): the medians and B/A.  Not part of the product.
    python tools/team_inproc_ab.py tools/ab/<variant>/libosgpu_reduce.so [P,...] [trials]"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
A_PATH = os.path.join(ROOT, "test-resilient-osss-ucx_amd", "libosgpu_reduce.so")
B_PATH = sys.argv[1]
MEMBERS = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "5,6,7,8").split(",")]
TRIALS = int(sys.argv[3]) if len(sys.argv) > 3 else 4
N = 64 << 20
REPS = 10


def lib(path):
    L = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    L.osgpu_team_combine.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    L.osgpu_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                             ctypes.c_void_p]
    return L


LA, LB = lib(A_PATH), lib(B_PATH)
st = torch.cuda.Stream()
sp = ctypes.c_void_p(st.cuda_stream)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def span(f):
    for _ in range(2):
        f()
    torch.cuda.synchronize()
    e0.record(st)
    for _ in range(REPS):
        f()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / REPS


# AB_CASES="type:op,..." (osgpu.TYPES / OPS names; default double:sum): the
# same byte footprint per array (N doubles' worth) for every type
NAMES_T = ["short", "int", "long", "longlong", "float", "double", "longdouble", "complexf",
           "complexd"]
NAMES_O = ["sum", "prod", "and", "or", "xor", "max", "min"]
TORCH_T = {"short": torch.int16, "int": torch.int32, "long": torch.int64,
           "longlong": torch.int64, "float": torch.float32, "double": torch.float64,
           "complexf": torch.complex64, "complexd": torch.complex128}
CASES = [c.split(":") for c in os.environ.get("AB_CASES", "double:sum").split(",")]

for (tname, oname), P in [(c, P) for c in CASES for P in MEMBERS]:
    tcode, ocode = NAMES_T.index(tname), NAMES_O.index(oname)
    dt = TORCH_T[tname]
    esz = torch.empty(0, dtype=dt).element_size()
    NE = N * 8 // esz
    for trial in range(TRIALS):
        def mk():
            if dt.is_floating_point or dt.is_complex:
                return torch.empty(NE, dtype=dt, device="cuda:0").uniform_(1, 2) \
                    if not dt.is_complex else torch.complex(
                        torch.empty(NE, device="cuda:0", dtype=torch.float32 if dt == torch.complex64
                                    else torch.float64).uniform_(0.9, 1.1),
                        torch.empty(NE, device="cuda:0", dtype=torch.float32 if dt == torch.complex64
                                    else torch.float64).uniform_(-0.1, 0.1))
            return torch.randint(-1000, 1000, (NE,), dtype=dt, device="cuda:0")
        xs = [mk() for _ in range(P)]
        ys = [torch.empty(NE, dtype=dt, device="cuda:0") for _ in range(P)]
        S = (ctypes.c_void_p * P)(*[x.data_ptr() for x in xs])
        D = (ctypes.c_void_p * P)(*[y.data_ptr() for y in ys])
        NB = (ctypes.c_size_t * P)(*([N * 8] * P))
        torch.cuda.synchronize()
        ta, tb, tc = [], [], []
        for _ in range(2):
            ta.append(span(lambda: LA.osgpu_team_combine(tcode, ocode, P, D, S, NE, sp)))
            ya = ys[P - 1][12345].item()
            tb.append(span(lambda: LB.osgpu_team_combine(tcode, ocode, P, D, S, NE, sp)))
            yb = ys[P - 1][12345].item()
            tc.append(span(lambda: LA.osgpu_copy(D, S, NB, P, sp)))
        B = 2 * P * N * 8
        a, b, c = min(ta), min(tb), min(tc)
        print(json.dumps({"type": tname, "op": oname, "P": P, "trial": trial,
                          "a_frac": B / a / 8e6, "b_frac": B / b / 8e6,
                          "copy_frac": B / c / 8e6, "a_of_copy": c / a, "b_of_copy": c / b,
                          "b_over_a": a / b, "same_result": ya == yb, "variant": B_PATH}),
              flush=True)
        del xs, ys
        torch.cuda.empty_cache()
