#!/bin/bash
# host-staged in the bench's context (one extra stream before): copy-stream
# creation variants.  Not product.
set -e
O=gpurun_out/numa; mkdir -p $O
for cs in plain prio cumask; do
  CTX_ENV="{\"OSGPU_STAGE_COPY\":\"dma\",\"OSGPU_COPY_STREAMS\":\"$cs\"}" timeout -k 10 300 python tools/host_staged_context.py none side_stream team_rate
done > $O/ctx_streams.jsonl
