#!/bin/bash
# On the GPU box: the final HEAD check — full GPU suite, smoke, the default bench line (as the
# driver runs them).  Usage: bash profiles/scripts/gpu_r6z.sh <tag>
set -uo pipefail
TAG=${1:-r6z}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed: $?"; tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 580 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_$TAG.json'))
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'parity', d['parity'])
print('e2e', d['e2e']['cli_wall_s'], 'cfg3', d['scaling_cfg3']['value'], d['scaling_cfg3']['e2e_wall_s'])
print('ga', d['gapassem']['ms_per_step'], d['gapassem']['roofline']['frac'], 'pack', d['gpu_pack']['cs_GB_per_s'])"
