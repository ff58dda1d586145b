#!/bin/bash
# Run one gpurun call, waiting while nothing could run: no free GPU slot (exit 3), a transient
# box failure before the command started, or the previous call still finishing ("already
# running").  Those charge nothing.  Any other outcome -- including a failed GPU command -- ends it.
#   bash tools/gpurun_wait.sh TIMEOUT 'command'  > log
tmp=$(mktemp)
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$1" -- "$2" 2>&1 | tee "$tmp"
  rc=${PIPESTATUS[0]}
  if [ $rc -ne 3 ] && ! grep -qE "status=transient|already running" "$tmp"; then rm -f "$tmp"; exit $rc; fi
  sleep 90
done
rm -f "$tmp"
exit 3
