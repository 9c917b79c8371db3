#!/bin/bash
# the bench's own 4-member placement measurement, repeated: how often does a
# trial collapse, and does the re-timing after the copy agree?  Not product.
set -e
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 700 python -c "
import sys, json; sys.path.insert(0, '.'); import bench, torch, osgpu
L = osgpu.load()
for k in range(12):
    r = bench.team_placements(L, torch, 64 << 20, 20, 4)
    print(json.dumps({'round': k, 'placements': r['placements']}), flush=True)
" > $O/p4_repeat.jsonl
