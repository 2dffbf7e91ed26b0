#!/bin/bash
# On the GPU box: bench every build_exp/libpwasm_amd_<n>.so given (timing only).
set -uo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for n in "$@"; do
  PWASM_LIB=$PWD/build_exp/libpwasm_amd_$n.so timeout -k 10 240 python3 bench.py --no-cpu-baseline --steps 20 \
    > gpurun_out/exp_$n.json 2> gpurun_out/exp_$n.err || { echo "variant $n failed: $?"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/exp_$n.json')); print('$n', d['roofline']['kernel_ms'])"
done
