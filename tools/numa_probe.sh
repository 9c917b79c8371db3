#!/bin/bash
# host-staged with a 1.5-s warm-up: child without torch vs in a torch
# process, after the bench's team placements.  Not product.
set -e
O=gpurun_out/numa; mkdir -p $O
timeout -k 10 800 python -c "
import sys, json, os; sys.path.insert(0, '.'); import bench, torch, osgpu
L = osgpu.load()
for P in (2, 4, 8): bench.team_placements(L, torch, 64 << 20, 5, P)
for k in range(2):
    print(json.dumps({'child': bench.host_staged_child(64 << 20)}), flush=True)
    print(json.dumps({'in_torch': bench.host_staged_time(64 << 20)}), flush=True)
os.environ['OSGPU_STAGE_COPY'] = 'kout'
print(json.dumps({'child_kout': bench.host_staged_child(64 << 20)}), flush=True)
" > $O/child_vs_torch2.jsonl
