#!/bin/bash
# On the GPU box, during kernel development: a fast parity subset, then the cfg2 bench line and a
# kernel trace.  Usage: profiles/scripts/gpu_dev.sh <tag> [pytest -k expr]
set -uo pipefail
TAG=${1:-dev}
K=${2:-"kat or edge_mix or modes or cfg2 or long_indels or reverse or error_midway"}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed: $?"; grep -E "FAIL|Error|error|first difference|oracle:|hip:" gpurun_out/pytest_$TAG.log | head -30; tail -5 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-gapassem > gpurun_out/prof_$TAG/bench.json 2> gpurun_out/prof_$TAG/bench.err || { echo "bench failed"; tail -5 gpurun_out/prof_$TAG/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/prof_$TAG/bench.json'));print('parity',d['parity'],'kernel_ms',d['roofline']['kernel_ms'],'frac',d['roofline']['frac'])"
python3 tools/kstat.py $(find gpurun_out/prof_$TAG/trace -name "*kernel_stats.csv" | head -1)
if [ "${G5:-0}" = 1 ]; then  # the cfg5 (GapAssem) step too: parity + kernel trace
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG/trace5 -o run --output-format csv -- python3 bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG/bench5.json 2> gpurun_out/prof_$TAG/bench5.err || { echo "bench5 failed"; tail -5 gpurun_out/prof_$TAG/bench5.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/prof_$TAG/bench5.json'));print('cfg5 parity',d.get('parity'),'ms',d['ms_per_step'],'frac',d['roofline']['frac'])"
  python3 tools/kstat.py $(find gpurun_out/prof_$TAG/trace5 -name "*kernel_stats.csv" | head -1)
fi
