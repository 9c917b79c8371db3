#!/bin/bash
# heap stagger A/B: 8 and 4 ranks self-launched on one GPU (bench.py N>1
# rehearsal, heaps from osgpu_heap_create).  Not product.
set -e
O=gpurun_out/r05; mkdir -p $O
for st in 1 0; do
  for n in 4 8; do
    OSGPU_HEAP_STAGGER=$st timeout -k 10 400 python bench.py --gpus $n --steps 10 --warmup 3 --no-extra > $O/stagger${st}_n$n.log 2>&1
  done
done
