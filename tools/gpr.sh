#!/bin/bash
# gpurun wrapper (development tool): re-submits only when the GPU service reports an
# infrastructure event (status=transient: nothing ran, nothing charged); any real
# result, failure included, is returned as is.
#   bash tools/gpr.sh TIMEOUT 'command'
T=$1; shift
for i in 1 2 3 4 5; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
  if echo "$out" | grep -q "status=transient"; then
    echo "[gpr] transient infrastructure event, resubmitting in 100 s ($i)" >&2
    sleep 100
    continue
  fi
  echo "$out" | grep -v "every call sends the whole tree"
  exit 0
done
echo "$out"
