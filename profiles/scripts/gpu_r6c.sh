#!/bin/bash
# On the GPU box: GPU tests selected by $2 (- for none), alternating same-call sweeps of the
# variants after $3 ($1 rounds), then the default bench line without cfg3.
# Usage: bash profiles/scripts/gpu_r6c.sh <rounds> "<pytest -k expr or ->" <tag> variant...
set -uo pipefail
R=$1; K=$2; TAG=$3; shift 3
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$K" != "-" ]; then
  timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "$K" > gpurun_out/ab_${TAG}_pytest.log 2>&1 || { echo "pytest failed: $?"; tail -40 gpurun_out/ab_${TAG}_pytest.log; exit 1; }
  tail -2 gpurun_out/ab_${TAG}_pytest.log
fi
for i in $(seq 1 $R); do
  bash tools/exp_sweep.sh ${TAG}_$i "$@" || exit 1
done
timeout -k 10 300 python3 bench.py --no-cfg3 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "bench failed"; tail gpurun_out/bench_${TAG}.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_${TAG}.json'))
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'parity', d['parity'])
print('e2e', d['e2e'])
print('ga', d['gapassem']['ms_per_step'], d['gapassem']['roofline']['frac'])"
