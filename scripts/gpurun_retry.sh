#!/bin/bash
# Run one gpurun call, retrying ONLY while gpurun reports "no box or slot free"
# (exit 3: nothing ran, nothing charged).  Usage: gpurun_retry.sh LOG TIMEOUT CMD
log=$1; to=$2; shift 2
for i in $(seq 20); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $log 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  sleep 150
done
echo EXIT $rc >> $log
