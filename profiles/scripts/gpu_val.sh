#!/bin/bash
# On the GPU box: the whole GPU test suite, the default bench line (cfg2 + cfg5 sub-object, CPU
# baseline), then the cfg2 profile (kernel trace + PMC passes).  Usage: bash profiles/scripts/gpu_val.sh <tag>
set -uo pipefail
TAG=${1:-val}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed: $?"; grep -E "FAIL|Error|first difference" gpurun_out/pytest_gpu_$TAG.log | head -20; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed: $?"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
bash profiles/run_prof.sh ${TAG}_c2
