#!/bin/bash
# On the GPU box: the default bench line (cfg2 + cfg3 at N=1 + cfg5) with the mgpu phases of the
# cfg3 e2e leg, then a 2-rank gloo rehearsal of bench.py --gpus 2 (cfg3 at scale 0.05).
set -uo pipefail
TAG=${1:-r6f}
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(date +%s)
PW_PROFILE_HOST=1 timeout -k 10 580 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail gpurun_out/bench_$TAG.err; exit 1; }
echo "bench wall $(( $(date +%s) - S )) s"
grep "mgpu \|e2e\]" gpurun_out/bench_$TAG.err
python3 -c "
import json; d=json.load(open('gpurun_out/bench_$TAG.json'))
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'parity', d['parity'])
print('e2e', json.dumps(d['e2e']))
print('scaling_cfg3', json.dumps(d['scaling_cfg3']))
print('ga', d['gapassem']['ms_per_step'], d['gapassem']['roofline']['frac'])"
if [ "${2:-}" = "rehearse" ]; then
  S=$(date +%s)
  PW_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --cfg3-scale 0.05 --no-cpu-baseline > gpurun_out/bench2_$TAG.json 2> gpurun_out/bench2_$TAG.err || { echo "rehearsal failed"; tail gpurun_out/bench2_$TAG.err; exit 1; }
  echo "rehearsal wall $(( $(date +%s) - S )) s"
  python3 -c "
import json; d=json.load(open('gpurun_out/bench2_$TAG.json'))
print('n', d['n_gpus'], 'value', d['value'], 'keys', sorted(d.keys()))
print('scaling_cfg3', json.dumps(d['scaling_cfg3']))"
fi
