#!/bin/bash
# Run one gpurun call, retrying ONLY while gpurun reports that nothing ran
# (exit 3: no free slot / box, or an infrastructure back-off), waiting as long
# as gpurun asks ("retry in Ns"), at most ~4 hours.  Usage: gpurun_retry.sh LOG TIMEOUT CMD
log=$1; to=$2; shift 2
for i in $(seq 200); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $log 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  w=$(grep -o "retry in [0-9]*s" $log | grep -o "[0-9]*" | tail -1)
  sleep $(( ${w:-120} > 60 ? ${w:-120} + 5 : 65 ))
done
echo EXIT $rc >> $log
