#!/bin/bash
# Acquire a GPU box for ONE command: retries only while gpurun reports that
# no box was free or the box was lost before the command ran (nothing
# charged); stops at the first call whose command actually ran, whatever
# its status.  Usage: tools/gpurun_retry.sh LOG TIMEOUT 'COMMAND'
log=$1; to=$2; cmd=$3
for i in $(seq 1 ${RETRIES:-12}); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if grep -q "no free box\|status=transient\|backing off\|taken away by the GPU service\|stopped responding while being prepared\|GPU slot(s) on this pod are busy" "$log" && ! grep -q "all steps done" "$log"; then
    echo "attempt $i: no box ($rc), retrying" >> "$log.attempts"
    sleep ${RETRY_SLEEP:-120}
    continue
  fi
  echo "attempt $i: rc=$rc" >> "$log.attempts"
  exit $rc
done
exit 3
