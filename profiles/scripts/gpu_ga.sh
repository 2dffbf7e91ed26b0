#!/bin/bash
# On the GPU box: the GapAssem GPU tests, then the cfg5 bench line and its kernel trace.
# Usage: bash profiles/scripts/gpu_ga.sh <tag>
set -uo pipefail
TAG=${1:-ga}
mkdir -p gpurun_out/prof_${TAG}_c5
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "gapassem or msa or ga_ or consensus or refine or kat" > gpurun_out/pytest_ga_$TAG.log 2>&1 || { echo "ga pytest failed: $?"; tail -40 gpurun_out/pytest_ga_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_ga_$TAG.log
timeout -k 10 300 python3 bench.py --config 5 > gpurun_out/bench5_$TAG.json 2> gpurun_out/bench5_$TAG.err || { echo "bench5 failed: $?"; tail -20 gpurun_out/bench5_$TAG.err; exit 1; }
cat gpurun_out/bench5_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_c5/trace -o run --output-format csv -- python3 bench.py --config 5 --steps 10 --warmup 2 --no-parity --no-cpu-baseline > gpurun_out/prof_${TAG}_c5/bench_trace.json 2> gpurun_out/prof_${TAG}_c5.err || { echo "trace5 failed"; exit 1; }
python3 tools/kstats.py gpurun_out/prof_${TAG}_c5/trace/run_kernel_stats.csv
echo ga done
