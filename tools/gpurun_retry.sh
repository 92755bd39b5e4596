#!/bin/bash
# retry a gpurun call while the pool has no box (infrastructure, nothing ran);
# any call that actually ran (pass or fail) ends the loop.  Log: $1.call
log=$1; shift
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun "$@" > "$log.call" 2>&1
  rc=$?
  if grep -q "no free box\|backing off\|stopped responding while being prepared\|status=transient" "$log.call"; then
    sleep 150
    continue
  fi
  echo "rc=$rc try=$i" >> "$log.call"
  exit $rc
done
