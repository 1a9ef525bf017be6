#!/bin/bash
# Run one GPU step under its own time limit; stop the whole call (exit 99) on a
# crash-class status (timeout 124/137, abort 134, segfault 139) so no further GPU
# step starts after a fault.  Usage: tools/gpu_step.sh SECONDS LOGFILE cmd...
secs=$1; log=$2; shift 2
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_step] rc=$rc cmd=$*" >> "$log"
case $rc in
  0|1|2|5) exit 0 ;;
  *) echo "[gpu_step] crash-class exit $rc; stopping" | tee -a "$log"; exit 99 ;;
esac
