#!/bin/bash
# On the GPU box: GPU parity tests then one bench line (no CPU baseline).  Usage: profiles/scripts/gpu_quick.sh <tag> [pytest -k expr]
set -uo pipefail
TAG=${1:-q}
mkdir -p gpurun_out
export TMPDIR=/tmp
K=${2:-}
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed: $?"; tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed: $?"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
