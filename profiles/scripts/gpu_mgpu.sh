#!/bin/bash
# On the GPU box: multi-rank rehearsals on ONE GPU (gloo collectives; RCCL needs a GPU per rank)
# and the cfg3 per-GPU throughput at N=1.  Usage: bash profiles/scripts/gpu_mgpu.sh <tag>
set -uo pipefail
TAG=${1:-m}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --config 3 --scale 0.1 --no-parity --no-cpu-baseline > gpurun_out/bench3_$TAG.json 2> gpurun_out/bench3_$TAG.err || { echo "bench cfg3 n1 failed: $?"; tail -20 gpurun_out/bench3_$TAG.err; exit 1; }
cat gpurun_out/bench3_$TAG.json
PW_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --scale 0.05 --steps 5 --warmup 2 > gpurun_out/bench3x2_$TAG.json 2> gpurun_out/bench3x2_$TAG.err || { echo "bench cfg3 x2 failed: $?"; tail -20 gpurun_out/bench3x2_$TAG.err; exit 1; }
cat gpurun_out/bench3x2_$TAG.json
