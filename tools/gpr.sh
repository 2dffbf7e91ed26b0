#!/bin/bash
# Local helper: run one gpurun call; retry (after a pause) only when the box never started
# ("status=transient": nothing ran, nothing charged).  Usage: tools/gpr.sh <timeout> '<command>'
T=$1; shift
for i in 1 2 3 4; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
  echo "$out" | tail -15
  echo "$out" | grep -q "status=transient" || exit 0
  sleep 150
done
