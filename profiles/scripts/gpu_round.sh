#!/bin/bash
# On the GPU box: GPU parity tests, then the cfg2 and cfg5 bench lines (with parity + CPU baseline).
# Usage: bash profiles/scripts/gpu_round.sh <tag> [pytest -k expr]
set -uo pipefail
TAG=${1:-r2}
K=${2:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed: $?"; tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed: $?"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 python3 bench.py --config 5 > gpurun_out/bench5_$TAG.json 2> gpurun_out/bench5_$TAG.err || { echo "bench5 failed: $?"; tail -20 gpurun_out/bench5_$TAG.err; exit 1; }
cat gpurun_out/bench5_$TAG.json
