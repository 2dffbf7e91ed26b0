#!/bin/bash
# On the GPU box: the GPU test suite, then the cfg2 and cfg4 bench lines.
# Usage: bash tools/gpu_r3.sh <tag> [pytest -k expr]
set -uo pipefail
TAG=${1:-r3}
K=${2:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed: $?"; tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed: $?"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 python3 bench.py --config 4 --scale 0.102 --steps 10 --warmup 2 > gpurun_out/bench4_$TAG.json 2> gpurun_out/bench4_$TAG.err || { echo "bench4 failed: $?"; tail -20 gpurun_out/bench4_$TAG.err; exit 1; }
cat gpurun_out/bench4_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_c4/trace -o run --output-format csv -- python3 bench.py --config 4 --scale 0.102 --steps 5 --warmup 1 --no-parity --no-cpu-baseline > gpurun_out/prof_${TAG}_c4/bench_trace.json 2> gpurun_out/prof_${TAG}_c4.err || { echo "trace failed"; exit 1; }
echo done
