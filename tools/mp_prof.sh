#!/bin/bash
# rocprofv3 kernel statistics of the small-call paths with one process per
# PE: two mp_worker.py ranks in `latency` mode on this GPU, each under its own
# rocprofv3 (the worker starts no other program).  Not part of the product.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 MASTER_PORT=${MASTER_PORT:-29541} WORLD_SIZE=2
export MP_SIZES=${MP_SIZES:-1024,65536} MP_REPS=${MP_REPS:-200}
mkdir -p gpurun_out/mp_prof
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r timeout -k 10 240 rocprofv3 --kernel-trace --stats \
      -d gpurun_out/mp_prof/rank$r -o run --output-format csv -- \
      python3 tests/support/mp_worker.py latency gpurun_out/mp_prof > gpurun_out/mp_prof/rank$r.log 2>&1 &
done
rc=0
for j in $(jobs -p); do wait $j || rc=$?; done
echo "mp_prof rc=$rc"
exit $rc
