#!/bin/bash
# On the GPU box: kernel-trace stats of a short bench run.  Usage: profiles/scripts/gpu_trace.sh <tag> [extra bench args]
set -uo pipefail
TAG=${1:-t}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_$TAG -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 "$@" > gpurun_out/tr_$TAG.json 2> gpurun_out/tr_$TAG.err || { echo "trace failed: $?"; tail -20 gpurun_out/tr_$TAG.err; exit 1; }
cat gpurun_out/tr_$TAG.json
f=$(find gpurun_out/tr_$TAG -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 "$f"
