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
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_collectives.py tests/test_collectives.py > $O/pytest_coll.txt 2>&1
timeout -k 10 300 python -c "
import sys, json; sys.path.insert(0, '.'); import bench
print(json.dumps(bench.collectives_single()))" > $O/coll_bench.json
OSGPU_LIB_PATH=$PWD/tools/ab/collold/libosgpu_reduce.so timeout -k 10 300 python -c "
import sys, json; sys.path.insert(0, '.'); import bench
print(json.dumps(bench.collectives_single()))" > $O/coll_bench_old.json
