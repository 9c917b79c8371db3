#!/usr/bin/env python3
"""In-process A/B of two builds of the combine kernel (osgpu_combine, the
headline's combine_vec_kernel<double,SUM,2> shape) on the SAME arrays: the
shipped library and a variant (argv[1]) both loaded RTLD_LOCAL; every trial
(fresh K inputs + output, n elements) times A, B and the copy kernel over
the same bytes, interleaved twice; the outputs are compared bit for bit.
One JSON line per (type, op, K, trial).  Not part of the product.
    AB_CASES=double:sum python tools/combine_inproc_ab.py <variant.so> [K,...] [trials]"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
A_PATH = os.path.join(ROOT, "test-resilient-osss-ucx_amd", "libosgpu_reduce.so")
B_PATH = sys.argv[1]
KS = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "2").split(",")]
TRIALS = int(sys.argv[3]) if len(sys.argv) > 3 else 6
N = int(os.environ.get("AB_N", str(64 << 20)))  # doubles' worth of bytes per array
REPS = 20
NAMES_T = ["short", "int", "long", "longlong", "float", "double", "longdouble", "complexf",
           "complexd"]
NAMES_O = ["sum", "prod", "and", "or", "xor", "max", "min"]
TORCH_T = {"short": torch.int16, "int": torch.int32, "long": torch.int64,
           "float": torch.float32, "double": torch.float64}
CASES = [c.split(":") for c in os.environ.get("AB_CASES", "double:sum").split(",")]


def lib(path):
    L = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    L.osgpu_combine.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
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


for (tname, oname), K in [(c, K) for c in CASES for K in KS]:
    tcode, ocode = NAMES_T.index(tname), NAMES_O.index(oname)
    dt = TORCH_T[tname]
    NE = N * 8 // torch.empty(0, dtype=dt).element_size()
    for trial in range(TRIALS):
        if dt.is_floating_point:
            xs = [torch.empty(NE, dtype=dt, device="cuda:0").uniform_(1, 2) for _ in range(K)]
        else:
            xs = [torch.randint(-1000, 1000, (NE,), dtype=dt, device="cuda:0") for _ in range(K)]
        oa = torch.empty(NE, dtype=dt, device="cuda:0")
        ob = torch.empty(NE, dtype=dt, device="cuda:0")
        S = (ctypes.c_void_p * K)(*[x.data_ptr() for x in xs])
        # copy ceiling over the same footprint: (K+1)*N*8 bytes as K/2+... one
        # read + one write stream of (K+1)/2 * N*8 bytes each (bench's form)
        half = (K + 1) * N * 8 // 2
        cbuf = torch.empty(2 * half, dtype=torch.uint8, device="cuda:0")
        CD = (ctypes.c_void_p * 1)(cbuf.data_ptr() + half)
        CS = (ctypes.c_void_p * 1)(cbuf.data_ptr())
        CN = (ctypes.c_size_t * 1)(half)
        torch.cuda.synchronize()
        ta, tb, tc = [], [], []
        for _ in range(2):
            ta.append(span(lambda: LA.osgpu_combine(tcode, ocode, oa.data_ptr(), S, K, NE, sp)))
            tb.append(span(lambda: LB.osgpu_combine(tcode, ocode, ob.data_ptr(), S, K, NE, sp)))
            tc.append(span(lambda: LA.osgpu_copy(CD, CS, CN, 1, sp)))
        torch.cuda.synchronize()
        same = bool(torch.equal(oa, ob))
        B = (K + 1) * N * 8
        a, b, c = min(ta), min(tb), min(tc)
        print(json.dumps({"type": tname, "op": oname, "K": K, "trial": trial,
                          "a_frac": B / a / 8e6, "b_frac": B / b / 8e6, "copy_frac": B / c / 8e6,
                          "b_over_a": a / b, "same_output": same, "variant": B_PATH}), flush=True)
        del xs, oa, ob, cbuf
        torch.cuda.empty_cache()
