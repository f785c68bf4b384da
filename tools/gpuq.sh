#!/bin/bash
# host-side: retry gpurun only while no box is free (rc 3) or the call was transient; never on a command failure
out=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun "$@" > $out 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" $out; then sleep 60; continue; fi
  echo "rc=$rc" >> $out; exit $rc
done
