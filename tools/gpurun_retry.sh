#!/bin/bash
# (local helper) retry a gpurun call only while it reports "no box/slot free" (exit 3); any other outcome ends it
log=$1; shift
for i in $(seq 1 20); do
  timeout 1800 /usr/local/graft/bin/gpurun "$@" > "$log" 2>&1; rc=$?
  [ $rc -ne 3 ] && { echo "rc=$rc after $i tries" >> "$log"; exit $rc; }
  sleep 150
done
echo "gave up" >> "$log"
