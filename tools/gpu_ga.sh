#!/bin/bash
# On the GPU box: GapAssem GPU tests + the cfg5 bench line.  Usage: bash tools/gpu_ga.sh <tag>
set -uo pipefail
TAG=${1:-ga}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "gapassem or cfg5" > gpurun_out/pytest_ga_$TAG.log 2>&1 || { echo "pytest failed: $?"; tail -40 gpurun_out/pytest_ga_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_ga_$TAG.log
timeout -k 10 300 python3 bench.py --config 5 > gpurun_out/bench5_$TAG.json 2> gpurun_out/bench5_$TAG.err || { echo "bench5 failed: $?"; tail -20 gpurun_out/bench5_$TAG.err; exit 1; }
cat gpurun_out/bench5_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_$TAG -o run --output-format csv -- python3 bench.py --config 5 --no-parity --no-cpu-baseline --steps 10 --warmup 2 > /dev/null 2> gpurun_out/tr_$TAG.err || { echo "trace failed"; exit 1; }
f=$(find gpurun_out/tr_$TAG -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f"
