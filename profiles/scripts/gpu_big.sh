#!/bin/bash
# On the GPU box: the large configs on one GPU — cfg3 in full (10M records) and cfg4 (>= 1k
# Mb-contig records) — bench lines with streamed-hash parity + CPU baseline, then a kernel trace of
# each (no parity).  Usage: bash profiles/scripts/gpu_big.sh <tag> [cfg4 scale]
set -uo pipefail
TAG=${1:-r3}
S4=${2:-0.102}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u bench.py --config 3 --steps 10 --warmup 2 > gpurun_out/bench3_$TAG.json 2> gpurun_out/bench3_$TAG.err || { echo "bench3 failed: $?"; tail -20 gpurun_out/bench3_$TAG.err; exit 1; }
cat gpurun_out/bench3_$TAG.json
timeout -k 10 400 python3 -u bench.py --config 4 --scale $S4 --steps 10 --warmup 2 > gpurun_out/bench4_$TAG.json 2> gpurun_out/bench4_$TAG.err || { echo "bench4 failed: $?"; tail -20 gpurun_out/bench4_$TAG.err; exit 1; }
cat gpurun_out/bench4_$TAG.json
for C in 3 4; do
  SC=1.0; [ $C = 4 ] && SC=$S4
  OUT=gpurun_out/prof_${TAG}_c$C
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py --config $C --scale $SC --steps 5 --warmup 1 --no-parity --no-cpu-baseline > "$OUT/bench_trace.json" 2> "$OUT/trace.err" || { echo "trace $C failed"; tail -5 "$OUT/trace.err"; exit 1; }
  echo "trace $C done"
done
