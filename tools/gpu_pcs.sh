#!/bin/bash
# On the GPU box: PC sampling (rocprofv3, host_trap, beta) of the report kernels under the cfg2
# bench: which instructions render_kernel's waves sit on.  Usage: tools/gpu_pcs.sh <tag> [method]
set -uo pipefail
TAG=${1:-pcs}
M=${2:-host_trap}
mkdir -p gpurun_out/pcs_$TAG
export TMPDIR=/tmp
timeout -k 5 60 rocprofv3 -L > gpurun_out/pcs_$TAG/avail.txt 2>&1 || echo "list-avail rc $?"
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $M --pc-sampling-unit time --pc-sampling-interval 1 -d gpurun_out/pcs_$TAG/run -o run --output-format csv -- python3 bench.py --steps 30 --warmup 2 --no-parity --no-cpu-baseline --no-gapassem > gpurun_out/pcs_$TAG/bench.json 2> gpurun_out/pcs_$TAG/pcs.err || { echo "pc sampling failed: $?"; tail -20 gpurun_out/pcs_$TAG/pcs.err; exit 1; }
find gpurun_out/pcs_$TAG/run -type f | head
