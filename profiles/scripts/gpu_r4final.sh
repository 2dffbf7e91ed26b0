#!/bin/bash
# On the GPU box, end of round 4: the GPU test suite, the default bench line (cfg2 + cfg5), the cfg2
# profile (kernel trace + PMC passes, profiles/run_prof.sh), then the large configs
# (profiles/scripts/gpu_big.sh: full cfg3, cfg4 at the given scale, kernel traces).
# Usage: bash profiles/scripts/gpu_r4final.sh <tag> [cfg4 scale] [skip-tests]
set -uo pipefail
TAG=${1:-r4f}
S4=${2:-0.11}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${3:-}" != "skip-tests" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed: $?"; tail -60 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu_$TAG.log
fi
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed: $?"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
bash profiles/run_prof.sh ${TAG}_c2 || exit 1
bash profiles/run_prof.sh ${TAG}_c5 --config 5 || exit 1
bash profiles/scripts/gpu_big.sh $TAG $S4
