#!/bin/bash
# On the GPU box: GPU parity tests, one bench line (with CPU baseline), then the profile passes.
# Usage: bash profiles/scripts/gpu_check.sh <tag>
set -uo pipefail
TAG=${1:-r1}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed: $?"; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed: $?"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
bash profiles/run_prof.sh $TAG || { echo "prof failed: $?"; exit 1; }
