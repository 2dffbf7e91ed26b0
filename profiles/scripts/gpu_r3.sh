#!/bin/bash
# On the GPU box: the GPU test suite, then the cfg2 and cfg4 bench lines.
# Usage: bash profiles/scripts/gpu_r3.sh <tag> [extra pytest args...]
set -uo pipefail
TAG=${1:-r3}
shift || true
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread "$@" > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed: $?"; tail -60 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed: $?"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
mkdir -p gpurun_out/prof_${TAG}_c2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_c2/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-parity --no-cpu-baseline > gpurun_out/prof_${TAG}_c2/bench_trace.json 2> gpurun_out/prof_${TAG}_c2.err || { echo "trace failed"; exit 1; }
echo done
