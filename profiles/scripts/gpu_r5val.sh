#!/bin/bash
# On the GPU box (round 5): the GPU test suite, the default bench line, and the full cfg3 bench
# (10 M records: the pass, the CLI end to end with CRC-32 parity against the chunked oracle).
# Usage: bash profiles/scripts/gpu_r5val.sh <tag> [skip-tests]
set -uo pipefail
TAG=${1:-r5v}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed: $?"; tail -60 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu_$TAG.log
fi
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed: $?"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 500 python3 -u bench.py --config 3 --steps 5 --warmup 2 > gpurun_out/bench3_$TAG.json 2> gpurun_out/bench3_$TAG.err || { echo "bench cfg3 failed: $?"; tail -20 gpurun_out/bench3_$TAG.err; exit 1; }
cat gpurun_out/bench3_$TAG.json
