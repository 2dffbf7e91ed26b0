#!/bin/bash
# On the box (host only): output-file write strategies into $TMPDIR (tools/wbench.c).
set -uo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
df -T /tmp . | tee gpurun_out/wbench_df.txt
gcc -O2 -pthread -o /tmp/wbench tools/wbench.c && timeout -k 5 200 /tmp/wbench /tmp/wb.bin ${1:-8} ${2:-16} | tee gpurun_out/wbench.txt
