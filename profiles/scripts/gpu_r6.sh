#!/bin/bash
# On the GPU box: GPU suite + the default bench line (cfg2 + cfg3 at N=1 + cfg5).
# Usage: bash profiles/scripts/gpu_r6.sh <tag> [skip-tests]
set -uo pipefail
TAG=${1:-r6}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed: $?"; tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu_$TAG.log
fi
T0=$(date +%s)
timeout -k 10 580 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail gpurun_out/bench_$TAG.err; exit 1; }
echo "bench wall $(( $(date +%s) - T0 )) s"
tail -c 600 gpurun_out/bench_$TAG.json
