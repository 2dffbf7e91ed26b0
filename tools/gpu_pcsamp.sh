#!/bin/bash
# On the GPU box: stochastic PC sampling of a short bench run of an experiment build.
# Usage: tools/gpu_pcsamp.sh <tag> <lib>
set -uo pipefail
TAG=${1:-pc}; LIBP=${2:-build_exp/libpwasm_amd_pc_0.so}
mkdir -p gpurun_out/pcs_$TAG
export TMPDIR=/tmp
PWASM_LIB=$PWD/$LIBP timeout -k 10 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 -d gpurun_out/pcs_$TAG -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/pcs_$TAG/bench.json 2> gpurun_out/pcs_$TAG/err.txt
rc=$?
echo "rc=$rc"; tail -5 gpurun_out/pcs_$TAG/err.txt; find gpurun_out/pcs_$TAG -name "*.csv" | head; exit $rc
