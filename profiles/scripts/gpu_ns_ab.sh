#!/bin/bash
set -uo pipefail
export BENCH_ARGS=--no-gapassem
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ns.log 2>&1 || { echo "pytest failed: $?"; tail -30 gpurun_out/pytest_ns.log; exit 1; }
tail -2 gpurun_out/pytest_ns.log
for i in 1 2; do
  PW_NS_SIDE=1 bash tools/exp_sweep.sh ns${i}h head || exit 1
  bash tools/exp_sweep.sh ns${i}c cur || exit 1
done
