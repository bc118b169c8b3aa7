#!/bin/bash
# gpurun with retry ONLY when no box was obtained (transient / exit 3: nothing ran, nothing charged)
TO=$1; shift
for i in 1 2 3 4; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" 2>&1); rc=$?
  echo "$out" | tail -4
  if echo "$out" | grep -q "status=transient\|no box\|slot free" || [ $rc -eq 3 ]; then sleep 45; continue; fi
  exit $rc
done
