#!/bin/bash
# On the GPU box: the round's judged artefacts in one call — full GPU suite, smoke, the cfg2 and
# cfg5 bench lines, then the cfg2 and cfg5 profiles (trace + PMC passes).
# Usage: bash profiles/scripts/gpu_final.sh <tag>
set -uo pipefail
TAG=${1:-final}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed: $?"; tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail gpurun_out/bench_$TAG.err; exit 1; }
timeout -k 10 300 python3 bench.py --config 5 > gpurun_out/bench5_$TAG.json 2> gpurun_out/bench5_$TAG.err || { echo "bench5 failed"; tail gpurun_out/bench5_$TAG.err; exit 1; }
echo benches done
bash profiles/run_prof.sh ${TAG}_c2 || exit 1
bash profiles/run_prof.sh ${TAG}_c5 --config 5 || exit 1
echo final done
