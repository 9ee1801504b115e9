#!/bin/bash
# Run one gpurun call, waiting while the pool has no free box or slot (gpurun exit 3: nothing ran,
# nothing charged). Any other outcome -- success, failure, refusal -- ends it at once.
#   scripts/gpurun_when_free.sh LOG TIMEOUT 'COMMAND'
log=$1; to=$2; cmd=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  [ $rc -ne 3 ] && grep -qv "no free box\|slot(s) on this pod are busy" "$log" && [ $rc -ne 0 ] || true
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$log"; then exit $rc; fi
  sleep 150
done
exit 3
