#!/bin/bash
# One-lease A/B of the host-staged path: stream/queue
# probe, HEAD, HEAD with the copy streams created before the member mapping,
# and the round-2 tree (tools/ab/r02, built from d92c5fe).  Not product.
set -e
mkdir -p gpurun_out
O=gpurun_out/ab
mkdir -p $O
timeout -k 10 180 tools/ab/stream_queue_probe $((256<<20)) 6 > $O/stream_queue.jsonl
SWEEP_SETTINGS='[{}, {"GPU_MAX_HW_QUEUES": "8"}]' timeout -k 10 300 python tools/sweep_host_staged.py > $O/hs_head.jsonl
OSGPU_LIB_PATH=$PWD/tools/ab/order/csrc/libosgpu_reduce.so SWEEP_SETTINGS='[{}]' \
  timeout -k 10 200 python tools/sweep_host_staged.py > $O/hs_order.jsonl
(cd tools/ab/r02 && SWEEP_SETTINGS='[{}]' timeout -k 10 200 python tools/sweep_host_staged.py) > $O/hs_r02.jsonl
