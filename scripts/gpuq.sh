#!/bin/bash
# retry a gpurun call while the pool has no free box (exit 3); any other status ends it
out=$1; shift
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun "$@" > $out 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  sleep 60
done
echo "final rc=$rc" >> $out
