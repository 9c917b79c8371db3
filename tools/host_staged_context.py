#!/usr/bin/env python3
"""Which earlier part of the bench process slows the host-staged path?
(44.5 GB/s each way in a fresh process, 27.7 inside the
bench.)  Each setting runs in its own process: the named prefix steps, then
bench.host_staged_time.  One JSON line per setting.  Not part of the product.
    python tools/host_staged_context.py none torch_stream api team_rate"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 64 << 20
ENV = json.loads(os.environ.get("CTX_ENV", "{}"))

STEPS = {
    "none": "pass",
    "torch_init": "torch.zeros(1, device='cuda'); torch.cuda.synchronize()",
    "torch_stream": "s = torch.cuda.Stream(); torch.zeros(1, device='cuda'); torch.cuda.synchronize()",
    "torch_alloc": "x = torch.empty(3 << 30, dtype=torch.uint8, device='cuda'); x.fill_(1); "
                   "del x; torch.cuda.empty_cache()",
    "api": "bench.api_call_time(N)",
    "placements": "L = osgpu.load()\nfor P in (2, 4, 8): bench.team_placements(L, torch, N, 5, P)",
    "headline": "L = osgpu.load(); bench.kernel_rate(L, torch, 5, 0, N, 8, torch.float64, "
                "lambda x, k: x.uniform_(1.0, 2.0))",
    "extra": "L = osgpu.load(); bench.extra_kernel_rates(L, torch)",
    "side_stream": "s = torch.cuda.Stream(); x = torch.ones(1 << 20, device='cuda')\n"
                   "with torch.cuda.stream(s): x.add_(1)\ntorch.cuda.synchronize()",
    "events": "e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)\n"
              "e0.record(); torch.ones(1, device='cuda'); e1.record(); torch.cuda.synchronize()\n"
              "e0.elapsed_time(e1)",
    "events_side": "s = torch.cuda.Stream()\n"
                   "e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)\n"
                   "e0.record(s); e1.record(s); torch.cuda.synchronize(); e0.elapsed_time(e1)",
    "copy_side": "L = osgpu.load(); a = torch.ones(1 << 20, dtype=torch.uint8, device='cuda')\n"
                 "o = torch.empty_like(a); s = torch.cuda.Stream(); torch.cuda.synchronize()\n"
                 "osgpu.copy([o.data_ptr()], [a.data_ptr()], [1 << 20], s.cuda_stream)\n"
                 "torch.cuda.synchronize()",
    "copy_thread": "L = osgpu.load(); a = torch.ones(1 << 20, dtype=torch.uint8, device='cuda')\n"
                   "o = torch.empty_like(a); torch.cuda.synchronize()\n"
                   "osgpu.copy([o.data_ptr()], [a.data_ptr()], [1 << 20], None)\n"
                   "torch.cuda.synchronize()",
    "team_rate": "L = osgpu.load(); bench.team_kernel_rate(L, torch, N, 5)",
    "ceiling": "L = osgpu.load(); bench.stream_ceiling(L, torch, 3 * N * 8 // 2, reps=5)",
}


def run(prefix):
    code = ["import sys, json, ctypes", f"sys.path.insert(0, {ROOT!r})", "import bench",
            "import torch, osgpu", f"N = {N}"]
    code += [STEPS[p] for p in prefix]
    code.append("print('RESULT ' + json.dumps(bench.host_staged_time(N)))")
    r = subprocess.run([sys.executable, "-c", "\n".join(code)], capture_output=True, text=True,
                       timeout=300, cwd=ROOT, env=dict(os.environ, **ENV))
    if os.environ.get("CTX_STDERR"):  # keep the child's stderr (HIP logs)
        with open(os.environ["CTX_STDERR"] + "." + "+".join(prefix), "w") as f:
            f.write(r.stderr)
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
    out = json.loads(line[0][7:]) if line else {"error": r.stderr[-800:]}
    out.pop("note", None)
    return {"prefix": prefix, "env": {k: v for k, v in ENV.items()},
            **{k: (v.get("pcie_GBs_each_way", v) if isinstance(v, dict) else v)
               for k, v in out.items()}}


if __name__ == "__main__":
    for arg in sys.argv[1:] or ["none"]:
        print(json.dumps(run(arg.split("+"))), flush=True)
