#!/bin/bash
# On the GPU box: optional GPU tests (a -k filter), then alternating same-call kernel-trace sweeps of
# experiment builds (tools/abl_build/<variant>) under the bench (BENCH_ARGS).
# Usage: profiles/scripts/gpu_ab.sh <tag> "<pytest -k expr or ->" <rounds> variant...
set -uo pipefail
TAG=$1; K=$2; R=$3; shift 3
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$K" != "-" ]; then
  timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "$K" > gpurun_out/ab_${TAG}_pytest.log 2>&1 || { echo "pytest failed: $?"; tail -40 gpurun_out/ab_${TAG}_pytest.log; exit 1; }
  tail -2 gpurun_out/ab_${TAG}_pytest.log
fi
for i in $(seq 1 $R); do
  bash tools/exp_sweep.sh ${TAG}_$i "$@" || exit 1
done
