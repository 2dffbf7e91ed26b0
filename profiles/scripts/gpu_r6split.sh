#!/bin/bash
# On the GPU box: the split pass A/B (PW_REPORT_SPLIT=0 vs default) on cfg2 — parity-checked bench
# lines and kernel traces, alternating — then the GPU tests of the report path.
# Usage: bash profiles/scripts/gpu_r6split.sh <tag> [pytest -k expr]
set -uo pipefail
TAG=${1:-split}
mkdir -p gpurun_out/split_$TAG
export TMPDIR=/tmp
for i in 1 2; do
  for v in ${MODES:-0 3}; do
    export PW_REPORT_SPLIT=$v
    timeout -k 10 300 python3 bench.py --no-cfg3 --no-gapassem --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/split_$TAG/b_${v}_$i.json 2> gpurun_out/split_$TAG/b_${v}_$i.err || { echo "bench $v failed"; tail -5 gpurun_out/split_$TAG/b_${v}_$i.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/split_$TAG/b_${v}_$i.json'))
print('$v', $i, 'ms', round(d['ms_per_step'], 4), 'value', round(d['value'] / 1e9, 3), 'G/s kernel_ms', d['roofline']['kernel_ms'], 'parity', d['parity'])"
  done
done
unset PW_REPORT_SPLIT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/split_$TAG/trace -o run --output-format csv -- python3 bench.py --no-cfg3 --no-gapassem --no-cpu-baseline --no-parity --steps 10 --warmup 2 > /dev/null 2> gpurun_out/split_$TAG/trace.err || { echo "trace failed"; exit 1; }
f=$(find gpurun_out/split_$TAG/trace -name "*kernel_stats.csv" | head -1); python3 tools/kstat.py $f
if [ -n "${2:-}" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "$2" > gpurun_out/split_$TAG/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/split_$TAG/pytest.log; exit 1; }
  tail -2 gpurun_out/split_$TAG/pytest.log
fi
