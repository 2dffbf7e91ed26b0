#!/bin/bash
# On the GPU box: the other BASELINE configs' bench lines on the final HEAD (cfg1, cfg4, cfg3 in
# full on one GPU with its CRC-32 parity).  Usage: bash profiles/scripts/gpu_r6cfg.sh <tag>
set -uo pipefail
TAG=${1:-r6cfg}
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in ${CFGS:-1 4 3}; do
  timeout -k 10 400 python3 bench.py --config $c --steps 10 --warmup 2 > gpurun_out/bench_c${c}_$TAG.json 2> gpurun_out/bench_c${c}_$TAG.err || { echo "cfg$c failed"; tail gpurun_out/bench_c${c}_$TAG.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/bench_c${c}_$TAG.json'))
print('cfg$c', d['value'], d['unit'], 'ms', round(d['ms_per_step'], 4), 'frac', d['roofline']['frac'], 'parity', d.get('parity'), 'e2e', (d.get('e2e') or {}).get('cli_wall_s'))"
done
