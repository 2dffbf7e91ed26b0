#!/bin/bash
# On the GPU box (round 5): the GPU test suite, the default bench line, and a two-rank rehearsal of
# `bench.py --gpus 2` (bench.py launches both ranks itself; gloo, both on the one card).
# Usage: bash profiles/scripts/gpu_r5.sh <tag> [skip-tests] [skip-rehearsal]
set -uo pipefail
TAG=${1:-r5}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed: $?"; tail -60 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu_$TAG.log
fi
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed: $?"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
if [ "${3:-}" != "skip-rehearsal" ]; then
  PW_DIST_BACKEND=gloo timeout -k 10 400 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 --cfg3-scale 0.05 \
    > gpurun_out/bench2_$TAG.json 2> gpurun_out/bench2_$TAG.err || { echo "2-rank bench failed: $?"; tail -30 gpurun_out/bench2_$TAG.err; exit 1; }
  cat gpurun_out/bench2_$TAG.json
fi
