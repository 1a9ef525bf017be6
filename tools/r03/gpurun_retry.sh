#!/bin/bash
# retry gpurun only while the call never ran (infrastructure "transient" status or exit 3)
out=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun "$@" > "$out" 2>&1
  rc=$?
  if grep -q "status=transient\|backing off" "$out" || [ $rc -eq 3 ]; then sleep 45; continue; fi
  exit $rc
done
exit 99
