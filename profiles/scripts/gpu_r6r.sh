#!/bin/bash
# On the GPU box: the mgpu GPU tests (pw_runner and torch paths), then the default bench with the
# host phase lines.  Usage: bash profiles/scripts/gpu_r6r.sh <tag> [rehearse]
set -uo pipefail
TAG=${1:-r6r}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "mgpu or smoke" > gpurun_out/pytest_mgpu_$TAG.log 2>&1 || { echo "pytest failed: $?"; tail -40 gpurun_out/pytest_mgpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_mgpu_$TAG.log
bash profiles/scripts/gpu_r6f.sh $TAG ${2:-}
