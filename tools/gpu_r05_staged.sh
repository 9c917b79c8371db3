#!/bin/bash
# round 5: host-staged copy streams / legs A/B in the bench's context + the
# GPU tests this change touches.  Not product.
set -e
O=gpurun_out/r05; mkdir -p $O
for cs in prio plain cumask; do
  for sc in dma kout; do
    CTX_ENV="{\"OSGPU_STAGE_COPY\":\"$sc\",\"OSGPU_COPY_STREAMS\":\"$cs\"}" timeout -k 10 300 python tools/host_staged_context.py none side_stream
  done
done > $O/staged_streams.jsonl
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "copy_modes or host_staged or copy_streams" \
  tests/test_gpu_team_local.py::test_merge_matches_calls_when_threads_switch \
  tests/test_multiproc.py::test_preflight_more_than_8_members tests/test_multiproc.py::test_preflight_processes \
  tests/test_multiproc.py::test_host_staged_processes tests/test_gpu_collectives.py > $O/pytest_staged.txt 2>&1
